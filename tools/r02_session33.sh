#!/usr/bin/env bash
# Round-2 GPU session 33: determinism soak on the final kernels.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 600 soak python -u tools/soak.py --iters 20000 || exit $?
echo done
