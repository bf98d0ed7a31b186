#!/usr/bin/env bash
# Round-2 GPU session 13: 2-chunk record window on offset-addressed frames —
# GPU suite at the new default, packed-layout A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
$S 300 ab13_c3p python tools/abtune.py --config c3p --rounds 3 --var win_i=2 --var win_i=3 --out gpurun_out/ab13_c3p.json || exit $?
$S 300 ab13_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=0 --var win_i=3 --out gpurun_out/ab13_c3.json || exit $?
echo done
