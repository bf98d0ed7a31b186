# One gpurun session: the GPU test suite, smoke, and the default bench line.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_session.sh
# Each step runs under its own time limit (tools/gpu_step.sh); a fault,
# abort or timeout ends the session.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 pytest_gpu python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
tools/gpu_step.sh 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
tools/gpu_step.sh 300 bench_c2 python bench.py
