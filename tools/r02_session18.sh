#!/usr/bin/env bash
# Round-2 GPU session 18: line-completing windows, second pass (caps, packed, flows).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 400 flow_parity python -u -m pytest tests/test_flows.py -x -q --timeout 300 --timeout-method thread || exit $?
grep -q "passed" gpurun_out/flow_parity.log && ! grep -q "failed" gpurun_out/flow_parity.log || exit 3
$S 300 ab18_c3 python tools/abtune.py --config c3 --rounds 4 --var win_i=0 --var win_i=24 --var win_i=25 --var win_i=26 --out gpurun_out/ab18_c3.json || exit $?
$S 300 ab18_c4 python tools/abtune.py --config c4 --rounds 4 --var win_i=0 --var win_i=24 --var win_i=25 --var win_i=26 --out gpurun_out/ab18_c4.json || exit $?
$S 300 ab18_c3p python tools/abtune.py --config c3p --rounds 3 --var win_i=0 --var win_i=25 --out gpurun_out/ab18_c3p.json || exit $?
$S 300 ab18_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,win_i=25 --var fonly=1,win_i=26 --var fonly=1,win_i=28 --out gpurun_out/ab18_c5.json || exit $?
$S 300 ab18_c6 python tools/abtune.py --config c6 --rounds 3 --var win_i=0 --var win_i=28 --var win_i=29 --out gpurun_out/ab18_c6.json || exit $?
echo done
