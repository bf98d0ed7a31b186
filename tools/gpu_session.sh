set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_mod python -u -m pytest tests/test_modify.py -x -q -m gpu --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c2m python tools/abtune.py --config c2m --rounds 5 --var pipe=1 --var wb=64 --var wb=64,pol=2 --var wb=64,pol=3 --var wb=32,pol=2 --var streams=2,pipe=1 --var streams=2,wb=64 --var streams=2,wb=64,pol=2 --var streams=2,wb=64,pol=3 --var streams=2,wb=32,pol=2 --out gpurun_out/ab_c2m.json
