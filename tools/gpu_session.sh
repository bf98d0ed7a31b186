set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_flows python -u -m pytest tests/test_flows.py -x -q -m gpu --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows --var mode=flows,blocks=1280 --var mode=flows,blocks=1536 --var mode=flows,win_i=4 --out gpurun_out/ab_c5.json
