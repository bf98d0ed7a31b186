set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_header python -u -m pytest tests/test_header.py -x -q -m gpu --timeout 120 --timeout-method thread
