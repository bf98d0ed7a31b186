#!/usr/bin/env bash
# Round-2 GPU session 21: confirm the flows / tunnel line-completing windows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 ab21_c5 python tools/abtune.py --config c5 --rounds 5 --var fonly=1 --var fonly=1,win_i=1045 --var fonly=1,win_i=1035 --var fonly=1,win_i=1044 --var win_i=0 --var win_i=1045 --out gpurun_out/ab21_c5.json || exit $?
$S 300 ab21_c6 python tools/abtune.py --config c6 --rounds 5 --var win_i=0 --var win_i=1069 --var win_i=1068 --var win_i=1059 --var win_i=1058 --out gpurun_out/ab21_c6.json || exit $?
echo done
