set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows --var mode=parse --out gpurun_out/ab_c5.json
tools/gpu_step.sh 300 ab_c2 python tools/abtune.py --config c2 --rounds 3 --var streams=2 --var streams=1 --out gpurun_out/ab_c2.json
