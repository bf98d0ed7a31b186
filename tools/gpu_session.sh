set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 200 hdrsplit_128 python tools/hdrsplit.py --head 128
tools/gpu_step.sh 200 hdrsplit_192 python tools/hdrsplit.py --head 192
tools/gpu_step.sh 200 hdrsplit_128_s6 python tools/hdrsplit.py --head 128 --streams 6
