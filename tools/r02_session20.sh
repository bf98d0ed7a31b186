#!/usr/bin/env bash
# Round-2 GPU session 20: line-completing windows with a larger minimum (flows, tunnel).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 400 par20 python -u -m pytest tests/test_flows.py tests/test_gpu_parity.py -x -q -k "window or flow" --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/par20.log && ! grep -q "failed" gpurun_out/par20.log || exit 3
$S 300 ab20_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,win_i=1045 --var fonly=1,win_i=1046 --var fonly=1,win_i=1056 --var fonly=1,win_i=1058 --out gpurun_out/ab20_c5.json || exit $?
$S 300 ab20_c6 python tools/abtune.py --config c6 --rounds 3 --var win_i=0 --var win_i=1069 --var win_i=1079 --var win_i=1089 --var win_i=9 --out gpurun_out/ab20_c6.json || exit $?
$S 300 ab20_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=0 --var win_i=1035 --var win_i=1036 --out gpurun_out/ab20_c3.json || exit $?
echo done
