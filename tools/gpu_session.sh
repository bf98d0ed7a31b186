set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_flows python -u -m pytest tests/test_flows.py -x -q -m gpu --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows --out gpurun_out/ab_c5.json
tools/gpu_step.sh 200 prof_c5 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
