set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_packed python -u -m pytest tests/test_packed.py -x -q -m gpu --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c3p python tools/abtune.py --config c3p --rounds 3 --var mode=packed --var mode=parse --out gpurun_out/ab_c3p.json
tools/gpu_step.sh 200 prof_c3p rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3p -o run -- python3 bench.py --config c3p --steps 30 --warmup 2 --no-cpu-baseline --no-variants
