#!/usr/bin/env bash
# Round-2 GPU session 14: flows kernel staged window (C5) re-checked with the byte-12 start.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 ab14_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1,win_i=3 --var fonly=1,win_i=4 --var fonly=1,win_i=5 --var fonly=1,win_i=6 --out gpurun_out/ab14_c5.json || exit $?
$S 300 ab14_c4 python tools/abtune.py --config c4 --rounds 3 --var win_i=0 --var win_i=100 --out gpurun_out/ab14_c4.json || exit $?
echo done
