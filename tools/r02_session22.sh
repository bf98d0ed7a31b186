#!/usr/bin/env bash
# Round-2 GPU session 22: flows / tunnel line-completing defaults — GPU suite,
# smoke, default-vs-fixed A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || exit 3
$S 120 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 ab22_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,win_i=5 --out gpurun_out/ab22_c5.json || exit $?
$S 300 ab22_c6 python tools/abtune.py --config c6 --rounds 3 --var win_i=0 --var win_i=8 --out gpurun_out/ab22_c6.json || exit $?
echo done
