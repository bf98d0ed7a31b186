#!/usr/bin/env bash
# Round-2 GPU session 36: flows kernel grid variants under the line-completing window.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 ab36_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,fk=2 --var fonly=1,fk=1 --var fonly=1,blocks=1792 --out gpurun_out/ab36_c5.json || exit $?
echo done
