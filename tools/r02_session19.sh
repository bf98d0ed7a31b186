#!/usr/bin/env bash
# Round-2 GPU session 19: line-completing record windows as the default — GPU
# suite, smoke, default-vs-old A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || exit 3
$S 120 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 ab19_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=0 --var win_i=2 --var win_i=3 --out gpurun_out/ab19_c3.json || exit $?
$S 300 ab19_c4 python tools/abtune.py --config c4 --rounds 3 --var win_i=0 --var win_i=3 --out gpurun_out/ab19_c4.json || exit $?
echo done
