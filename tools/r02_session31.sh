#!/usr/bin/env bash
# Round-2 GPU session 31: parse_read compiled for 8 waves per SIMD (plan 12) vs plan 11.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 400 par31 python -u -m pytest tests/test_parse_read.py tests/test_hostmap.py -x -q --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/par31.log && ! grep -q "failed" gpurun_out/par31.log || exit 3
$S 300 ab31_c3r python tools/abtune.py --config c3r --rounds 4 --var plan=0 --var plan=12 --var plan=1 --out gpurun_out/ab31_c3r.json || exit $?
$S 300 ab31_c2r python tools/abtune.py --config c2r --rounds 4 --var plan=0 --var plan=12 --out gpurun_out/ab31_c2r.json || exit $?
echo done
