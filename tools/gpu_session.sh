set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 600 pytest_gpu python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
