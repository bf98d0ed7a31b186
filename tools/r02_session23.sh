#!/usr/bin/env bash
# Round-2 GPU session 23: no LDS slack past the last wave image (8 blocks per CU
# at 5 chunks) — parity, then default vs fixed-3 reference ratios.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 600 par23 python -u -m pytest tests/test_gpu_parity.py tests/test_flows.py tests/test_packed.py tests/test_geneve.py -x -q --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/par23.log && ! grep -q "failed" gpurun_out/par23.log || exit 3
$S 300 ab23_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=0 --var win_i=3 --out gpurun_out/ab23_c3.json || exit $?
$S 300 ab23_c4 python tools/abtune.py --config c4 --rounds 3 --var win_i=0 --var win_i=3 --out gpurun_out/ab23_c4.json || exit $?
$S 300 ab23_c6 python tools/abtune.py --config c6 --rounds 3 --var win_i=0 --var win_i=1068 --var win_i=8 --out gpurun_out/ab23_c6.json || exit $?
$S 300 ab23_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,win_i=5 --out gpurun_out/ab23_c5.json || exit $?
echo done
