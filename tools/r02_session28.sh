#!/usr/bin/env bash
# Round-2 GPU session 28: parse_read with 5-piece line-completing chunk-0 windows (plans 10 / 11).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 400 par28 python -u -m pytest tests/test_parse_read.py -x -q -k "read_plan" --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/par28.log && ! grep -q "failed" gpurun_out/par28.log || exit 3
$S 300 ab28_c3r python tools/abtune.py --config c3r --rounds 3 --var plan=0 --var plan=10 --var plan=11 --out gpurun_out/ab28_c3r.json || exit $?
$S 300 ab28_c2r python tools/abtune.py --config c2r --rounds 3 --var plan=0 --var plan=10 --var plan=11 --out gpurun_out/ab28_c2r.json || exit $?
echo done
