set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in c2 c3; do
tools/gpu_step.sh 200 hpzc8_$c python tools/hostpath.py --config $c --steps 50 --zero-copy --rec8
tools/gpu_step.sh 200 hpzc_$c python tools/hostpath.py --config $c --steps 50 --zero-copy
done
