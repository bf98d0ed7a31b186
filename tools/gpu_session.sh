set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_hostmap python -u -m pytest tests/test_hostmap.py tests/test_packed.py -x -q -m gpu --timeout 120 --timeout-method thread
