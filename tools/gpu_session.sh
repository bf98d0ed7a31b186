set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pmc_c3s python tools/pmc_traffic.py --config c3s --tag r01
tools/gpu_step.sh 200 prof_c3s rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3s -o run -- python3 bench.py --config c3s --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
