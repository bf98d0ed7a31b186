set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 600 pytest_gpu python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
tools/gpu_step.sh 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
tools/gpu_step.sh 300 bench_c2 python bench.py
for c in c3 c3s c4 c5 c6 c2m c3r; do tools/gpu_step.sh 300 bench_$c python bench.py --config $c --steps 50 --warmup 5; done
mkdir -p gpurun_out/prof_c2 gpurun_out/prof_c2_s1
tools/gpu_step.sh 300 rocprof_c2 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run -- python3 bench.py --no-cpu-baseline
tools/gpu_step.sh 300 rocprof_c2_s1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_s1 -o run -- python3 bench.py --streams 1 --no-cpu-baseline --no-variants
tools/gpu_step.sh 400 pmc_c2 python tools/pmc_traffic.py --config c2 --tag r01
