set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 120 list_avail rocprofv3 --list-avail
tools/gpu_step.sh 300 segbench python tools/segbench.py
mkdir -p gpurun_out/prof_c2 gpurun_out/prof_c2_s1
tools/gpu_step.sh 300 rocprof_c2 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --no-cpu-baseline
tools/gpu_step.sh 300 rocprof_c2_s1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_s1 -o run -- python3 bench.py --streams 1 --no-cpu-baseline --no-variants
for v in 32x1 64x1 128x1; do
SEG_ONLY=$v SEG_ROUNDS=1 SEG_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_seg_$v -o run -- python3 tools/segbench.py > gpurun_out/pmc_seg_$v.log 2>&1
done
