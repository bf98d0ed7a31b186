#!/usr/bin/env bash
# Round-2 GPU session 35: strong scaling's one-GPU point (BASELINE configs[3]: 64 M C4 frames) on the final tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 600 c4_strong python bench.py --config c4 --scaling strong --steps 10 --warmup 2 --no-cpu-baseline --no-host-path || exit $?
echo done
