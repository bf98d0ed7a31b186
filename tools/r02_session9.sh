#!/usr/bin/env bash
# Round-2 GPU session 9: staggered stream starts on the other multi-stream configs.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 stagger_c2m python tools/stagger_ab.py --config c2m --rounds 7 --stagger 0 --stagger 6 --stagger 10 --stagger 14 --steps 20 --steps 200 || exit $?
$S 300 stagger_c2r python tools/stagger_ab.py --config c2r --rounds 7 --stagger 0 --stagger 6 --stagger 10 --stagger 14 --steps 20 --steps 200 || exit $?
$S 300 stagger_c2b python tools/stagger_ab.py --config c2 --rounds 9 --stagger 0 --stagger 5 --stagger 6 --stagger 7 --steps 20 || exit $?
$S 300 stagger_c2_3s python tools/stagger_ab.py --config c2 --streams 3 --rounds 7 --stagger 0 --stagger 4 --stagger 6 --steps 20 --steps 200 || exit $?
echo done
