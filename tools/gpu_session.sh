set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 ab_c2 python tools/abtune.py --config c2 --rounds 5 --var streams=2 --var streams=2,pipe=4 --var streams=2,pipe=16 --var streams=2,depth=3 --var streams=3 --var streams=2,pol=1 --var streams=2,pol=2 --var streams=1 --out gpurun_out/ab_c2.json
