set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 600 pytest_gpu python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
tools/gpu_step.sh 300 ab_c3 python tools/abtune.py --config c3 --rounds 3 --var fb=1 --var fb=2 --out gpurun_out/ab_c3.json
tools/gpu_step.sh 300 ab_c6 python tools/abtune.py --config c6 --rounds 3 --var fb=1 --var fb=2 --out gpurun_out/ab_c6.json
tools/gpu_step.sh 300 ab_c4 python tools/abtune.py --config c4 --rounds 3 --var fb=1 --var fb=2 --out gpurun_out/ab_c4.json
for c in c3 c3s c6; do
for fb in 1 2; do
for w in 3 5 8; do
tools/gpu_step.sh 200 hpzc_${c}_fb${fb}_w$w python tools/hostpath.py --config $c --steps 50 --zero-copy --fb $fb --win $w
done
done
done
