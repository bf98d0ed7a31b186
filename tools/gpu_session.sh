set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 bigfuzz python -u tools/bigfuzz.py --frames 30000000 --seed 777
