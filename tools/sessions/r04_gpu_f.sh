#!/bin/bash
# Round-4 GPU session F: parse_read lazy chunk bounds (READ_PLAN 17) parity
# and its c3r / c2r A/B against the default first-chunk path.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_parse_read.py > $O/r04f_tests.txt 2>&1
for r in 1 2; do
  for v in "" "--tune read_plan=17"; do
    n=$([ -z "$v" ] && echo def || echo lazy)
    timeout -k 10 200 python3 bench.py --config c3r --steps 200 --warmup 20 --no-cpu-baseline \
        --no-variants $v > $O/r04f_c3r_${n}_$r.json 2> $O/r04f_c3r_${n}_$r.err
  done
done
timeout -k 10 400 python3 tools/pmc_kernels.py --sized --out $O/r04f_c3r_pmc.json -- \
    python3 bench.py --config c3r --steps 5 --warmup 2 --no-cpu-baseline --no-variants \
    --no-gate --tune read_plan=17 > $O/r04f_c3r_pmc.log 2>&1
rm -rf $O/r04f_c3r_pmc
du -sk $O/* 2>/dev/null | sort -n | tail -4; grep -h "is an array" $O/r04f_*.err | sort | uniq -c
