set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows,streams=1 --var mode=flows,streams=2 --var mode=flows,streams=3 --out gpurun_out/ab_c5.json
tools/gpu_step.sh 300 bench_c5 python bench.py --config c5 --steps 200 --warmup 10
tools/gpu_step.sh 300 torchrun2_gloo_c5 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c5 --steps 20 --warmup 2 --dist-backend gloo
