#!/bin/bash
# Round-4 GPU session I: table-in-image flows kernel variants (10/12/13),
# events A/B beside the default and the parse, PMC per variant.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_flows.py -k "without_hashes or ragged" > $O/r04i_tests.txt 2>&1
timeout -k 10 300 python3 tools/c5_same_run.py --reps 10 --variant flow_kernel=10 \
    --variant flow_kernel=12 --variant flow_kernel=13 --out $O/r04_c5ab5_events.json \
    > $O/r04_c5ab5_events.log 2>&1
for v in 10 13; do
  timeout -k 10 400 python3 tools/pmc_kernels.py --out $O/r04_c5ab5_pmc_fk$v.json -- \
      python3 tools/c5_same_run.py --reps 2 --variant flow_kernel=$v --out /tmp/c5_pmc_run.json \
      > $O/r04_c5ab5_pmc_fk$v.log 2>&1
  rm -rf $O/r04_c5ab5_pmc_fk$v
done
