#!/usr/bin/env bash
# Round-2 GPU session 16: PMC read bytes per frame vs the line floor, per window.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for w in 2 3 5 8 100; do
  $S 300 pmcw_c3_$w python tools/pmc_traffic.py --config c3 --tag r02w --tune window_indexed=$w || exit $?
done
for w in 2 3 8; do
  $S 300 pmcw_c4_$w python tools/pmc_traffic.py --config c4 --tag r02w --tune window_indexed=$w || exit $?
done
echo done
