#!/usr/bin/env bash
# Round-2 GPU session 32: multi-process paths on the final tree — torchrun at
# world size 1 over RCCL, and bench.py --gpus 2 folding two gloo ranks onto the box's GPU.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 torchrun1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 gpus2_gloo python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 || exit $?
$S 300 c5_gpus2_gloo python bench.py --config c5 --gpus 2 --dist-backend gloo --steps 10 --warmup 2 || exit $?
echo done
