set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 200 prof_c5a rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5a -o run -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
cp ingot_amd/lib/libingot_gpu.so /tmp/keep.so
cp tools/alt/libingot_gpu_h256.so ingot_amd/lib/libingot_gpu.so
tools/gpu_step.sh 200 prof_c5b rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5b -o run -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
cp /tmp/keep.so ingot_amd/lib/libingot_gpu.so
tools/gpu_step.sh 200 prof_c5c rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5c -o run -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-variants --streams 1
