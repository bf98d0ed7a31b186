#!/usr/bin/env bash
# Round-2 GPU session 34: the driver's exact bench command, three times, on the final tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
for i in 1 2 3; do
  $S 300 driver_$i python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
done
echo done
