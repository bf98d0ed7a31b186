set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_max python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k maximum --timeout 120 --timeout-method thread
