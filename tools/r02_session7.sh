#!/usr/bin/env bash
# Round-2 GPU session 7: staggered stream starts on C2 (driver's 20 steps).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 stagger_c2 python tools/stagger_ab.py --config c2 --stagger 0 --stagger 2 --stagger 4 --stagger 6 --stagger 8 --stagger 10 --stagger 12 --steps 20 --steps 4 --steps 200 || exit $?
$S 300 stagger_c2_r8 python tools/stagger_ab.py --config c2 --record 8 --stagger 0 --stagger 4 --stagger 6 --stagger 8 --steps 20 || exit $?
echo done
