#!/usr/bin/env bash
# Round-2 GPU session 15: the 128-B line floor of the record walk (C3, C4).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 floor_c3 python tools/line_floor.py --config c3 || exit $?
$S 300 floor_c4 python tools/line_floor.py --config c4 || exit $?
echo done
