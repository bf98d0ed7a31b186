#!/usr/bin/env bash
# Round-2 GPU session 25: differential fuzz (30 M frames per case) and soak on
# the line-completing-window / device-scope-store kernels.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 1000 bigfuzz python -u tools/bigfuzz.py --frames 30000000 --seed 5150 || exit $?
cp gpurun_out/bigfuzz.json gpurun_out/bigfuzz_30M_s5150.json
echo done
