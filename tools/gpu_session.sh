set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_flows python -u -m pytest tests/test_flows.py tests/test_gpu_parity.py -x -q -m gpu -k "flow or config5" --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows --var mode=flows,win_i=3 --var mode=flows,win_i=4 --var mode=flows,win_i=2 --var mode=flows,win_i=6 --var mode=parse --out gpurun_out/ab_c5.json
