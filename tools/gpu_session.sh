# Evidence refresh: bench lines for every config, rocprofv3 kernel stats, PMC traffic.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 bench_c2 python bench.py
for c in c2m c3 c3r c3s c4 c5 c6; do
tools/gpu_step.sh 300 bench_$c python bench.py --config $c --steps 200 --warmup 10
done
tools/gpu_step.sh 200 prof_c2_s1 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2_s1 -o run -- python3 bench.py --steps 500 --warmup 20 --no-cpu-baseline --no-variants --streams 1
tools/gpu_step.sh 200 prof_c2 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2 -o run -- python3 bench.py --steps 500 --warmup 20 --no-cpu-baseline --no-variants
for c in c4 c5; do
tools/gpu_step.sh 200 prof_$c rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$c -o run -- python3 bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
done
tools/gpu_step.sh 300 pmc_c5 python tools/pmc_traffic.py --config c5 --tag r01
