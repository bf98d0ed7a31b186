set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_hostmap python -u -m pytest tests/test_hostmap.py tests/test_pipeline.py -x -q -m gpu --timeout 120 --timeout-method thread
for c in c2 c3 c3s c6; do
tools/gpu_step.sh 200 hp_$c python tools/hostpath.py --config $c --steps 50
tools/gpu_step.sh 200 hpzc_$c python tools/hostpath.py --config $c --steps 50 --zero-copy
done
