set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_cpp python -u -m pytest tests/test_cpp_mirror.py -x -q -m gpu -s --timeout 120 --timeout-method thread
