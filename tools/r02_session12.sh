#!/usr/bin/env bash
# Round-2 GPU session 12: staged-window size re-checked now that record modes
# start the window at the chunk holding byte 12.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 ab12_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=2 --var win_i=3 --var win_i=4 --out gpurun_out/ab12_c3.json || exit $?
$S 300 ab12_c4 python tools/abtune.py --config c4 --rounds 3 --var win_i=2 --var win_i=3 --var win_i=4 --out gpurun_out/ab12_c4.json || exit $?
$S 300 ab12_c6 python tools/abtune.py --config c6 --rounds 3 --var win_i=5 --var win_i=6 --var win_i=8 --out gpurun_out/ab12_c6.json || exit $?
echo done
