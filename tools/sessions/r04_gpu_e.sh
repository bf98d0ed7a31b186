#!/bin/bash
# Round-4 GPU session E: whole-batch parity at the benchmark sizes, window
# sweeps of the gather configs (C3 / C4 / C6 parse, C5 flows).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_full_shard.py > $O/r04e_tests.txt 2>&1
timeout -k 10 300 python3 tools/c5_same_run.py --reps 8 --variant window_indexed=1058 \
    --variant window_indexed=1066 --variant window_indexed=1068 --variant window_indexed=1048 \
    --out $O/r04_c5_windows2.json > $O/r04_c5_windows2.log 2>&1
for cfg in c3 c4; do
  timeout -k 10 300 python3 tools/abtune.py --config $cfg --rounds 3 --var win_i=25 \
      --var win_i=1035 --var win_i=1026 --var win_i=1036 --var win_i=1028 \
      --out $O/r04_win_ab_$cfg.json > $O/r04_win_ab_$cfg.log 2>&1
done
timeout -k 10 300 python3 tools/abtune.py --config c6 --rounds 3 --var win_i=1069 \
    --var win_i=1068 --var win_i=1089 --var win_i=1059 \
    --out $O/r04_win_ab_c6.json > $O/r04_win_ab_c6.log 2>&1
