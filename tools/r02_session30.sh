#!/usr/bin/env bash
# Round-2 GPU session 30: final evidence on the final kernels — every config's
# PMC / kernel-trace / bench line, then the 30 M-frame differential fuzz.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/profile_round.sh r02 || exit $?
S=tools/gpu_step.sh
$S 1000 bigfuzz python -u tools/bigfuzz.py --frames 30000000 --seed 6060 || exit $?
cp gpurun_out/bigfuzz.json gpurun_out/bigfuzz_30M_s6060.json
echo session-done
