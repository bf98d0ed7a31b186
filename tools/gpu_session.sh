set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 bench_c2 python bench.py
tools/gpu_step.sh 300 bench_c3s python bench.py --config c3s --steps 200 --warmup 10
