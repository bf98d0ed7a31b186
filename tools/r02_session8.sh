#!/usr/bin/env bash
# Round-2 GPU session 8: does a longer warm-up change the 20-step region (clock ramp)?
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for w in 5 100 1000 4000; do
  $S 300 warm_$w python tools/stagger_ab.py --config c2 --warmup $w --rounds 5 --stagger 0 --stagger 6 --steps 20 --steps 200 || exit $?
done
echo done
