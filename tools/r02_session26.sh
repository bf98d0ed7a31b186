#!/usr/bin/env bash
# Round-2 GPU session 26: line floors of the flows kernel (C5) and of C4 records.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 floor_c5 python tools/line_floor.py --config c5 --flows || exit $?
$S 300 floor_c4b python tools/line_floor.py --config c4 || exit $?
$S 300 floor_c3b python tools/line_floor.py --config c3 || exit $?
echo done
