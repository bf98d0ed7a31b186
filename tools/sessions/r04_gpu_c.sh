#!/bin/bash
# Round-4 GPU session C: parity of the new variants, C5 A/B, C4/C6 slow-path
# A/B, sized-request PMC of C2/C3.  Each step under its own time limit.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_flows.py tests/test_gpu_parity.py -k "flow or slow_path" > $O/r04c_tests.txt 2>&1
tools/c5_ab.sh r04_c5ab3 flow_kernel=8 flow_kernel=9 window_indexed=1056
for cfg in c4 c6; do
  timeout -k 10 300 python3 tools/abtune.py --config $cfg --rounds 4 --var slow=0 --var slow=1 \
      --var slow=2 --out $O/r04_slow_ab_$cfg.json > $O/r04_slow_ab_$cfg.log 2>&1
  timeout -k 10 400 python3 tools/pmc_kernels.py --sized --out $O/r04_slow_pmc_$cfg.json -- \
      python3 tools/abtune.py --config $cfg --rounds 1 --steps 3 --var slow=0 --var slow=1 \
      --var slow=2 > $O/r04_slow_pmc_$cfg.log 2>&1
done
for cfg in c2 c3; do
  timeout -k 10 400 python3 tools/pmc_kernels.py --sized --out $O/r04_sized_$cfg.json -- \
      python3 bench.py --config $cfg --streams 1 --steps 20 --warmup 3 --no-cpu-baseline \
      --no-variants --no-host-path --no-sublines > $O/r04_sized_$cfg.log 2>&1
done
