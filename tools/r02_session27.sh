#!/usr/bin/env bash
# Round-2 GPU session 27: parse_read with line-completing chunk-0 windows (plans 7 / 8).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 400 par27 python -u -m pytest tests/test_parse_read.py -x -q --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/par27.log && ! grep -q "failed" gpurun_out/par27.log || exit 3
$S 300 ab27_c3r python tools/abtune.py --config c3r --rounds 3 --var plan=0 --var plan=7 --var plan=8 --out gpurun_out/ab27_c3r.json || exit $?
$S 300 ab27_c2r python tools/abtune.py --config c2r --rounds 3 --var plan=0 --var plan=7 --var plan=8 --out gpurun_out/ab27_c2r.json || exit $?
for p in 7 8; do
  $S 300 pmcr_$p python tools/pmc_traffic.py --config c3r --tag r02w --tune read_plan=$p || exit $?
done
echo done
