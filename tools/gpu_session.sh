set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 ab_c3 python tools/abtune.py --config c3 --rounds 3 --var streams=1 --var streams=1,blocks=2048 --var streams=1,blocks=4096 --var streams=1,blocks=16384 --out gpurun_out/ab_c3.json
tools/gpu_step.sh 300 ab_c4 python tools/abtune.py --config c4 --rounds 3 --var streams=1 --var streams=1,blocks=2048 --var streams=1,blocks=8192 --out gpurun_out/ab_c4.json
