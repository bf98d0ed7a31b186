# rocprofv3 evidence for one bench config: PMC traffic (FETCH_SIZE / WRITE_SIZE
# passes, tools/pmc_traffic.py) and a kernel-trace --stats summary of a
# single-stream bench run.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/profile_config.sh c5 r01 [nopmc]
set -e
cfg=${1:-c2}; tag=${2:-r01}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "${3:-}" = nopmc ] || tools/gpu_step.sh 400 pmc_$cfg python tools/pmc_traffic.py --config $cfg --tag $tag
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$cfg -o run -- \
    python3 $R/bench.py --config $cfg --streams 1 --steps 100 --warmup 10 --no-cpu-baseline \
    --no-variants --no-gate > $R/gpurun_out/prof_$cfg.log 2>&1
find $R/gpurun_out/prof_$cfg -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/${tag}_${cfg}_streams1_kernel_stats.csv \;
head -5 $R/gpurun_out/${tag}_${cfg}_streams1_kernel_stats.csv
