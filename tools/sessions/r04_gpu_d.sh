#!/bin/bash
# Round-4 GPU session D: parity after the flows-window / slow-path changes,
# the slow-path A/B again (no scratch), the C5 line, and the world-2 gloo
# rehearsal of the default line with its sub-lines (both ranks on one GPU).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_flows.py tests/test_gpu_parity.py -k "flow or slow_path" > $O/r04d_tests.txt 2>&1
for cfg in c4 c6; do
  timeout -k 10 300 python3 tools/abtune.py --config $cfg --rounds 4 --var slow=0 --var slow=1 \
      --var slow=2 --out $O/r04_slow_ab2_$cfg.json > $O/r04_slow_ab2_$cfg.log 2>&1
  timeout -k 10 400 python3 tools/pmc_kernels.py --sized --out $O/r04_slow_pmc2_$cfg.json -- \
      python3 tools/abtune.py --config $cfg --rounds 1 --steps 3 --var slow=0 --var slow=1 \
      --var slow=2 > $O/r04_slow_pmc2_$cfg.log 2>&1
done
timeout -k 10 200 python3 bench.py --config c5 --steps 200 --warmup 20 > $O/r04d_c5.json 2> $O/r04d_c5.err
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 \
    > $O/r04d_gloo2.json 2> $O/r04d_gloo2.err
