#!/usr/bin/env bash
# Round evidence for every bench config on the final kernels, one gpurun call:
#   1. PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) -> profiles/<tag>_pmc_<cfg>.json
#      (tools/pmc_traffic.py records the kernel name and the kernel-source digest,
#      which bench.py checks before attaching the file to a line);
#   2. rocprofv3 --kernel-trace --stats of a single-stream bench run
#      -> profiles/<tag>_<cfg>_streams1_kernel_stats.csv (its own JSON line:
#      gpurun_out/prof_<cfg>.log, checked by tools/check_profiles.py);
#   3. the bench line itself (default streams, gated) -> gpurun_out/bench_<cfg>.log.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/profile_round.sh r04 [cfgs...]
set -u
tag=${1:-r02}; shift || true
cfgs=${*:-"c2 c2m c2r c3 c3p c3r c3s c4 c5 c6 c6e"}
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
S=tools/gpu_step.sh
for cfg in $cfgs; do
    $S 300 pmc_$cfg python tools/pmc_traffic.py --config $cfg --tag $tag || exit $?
    cp gpurun_out/${tag}_pmc_$cfg.json profiles/ 2>/dev/null
    case $cfg in c2|c2m|c2r) s=2000 ;; *) s=200 ;; esac
    # the kernel-trace summary of a single-stream bench run: every dispatch
    # of the parse kernel runs alone, so the summary's mean is the
    # per-launch time that run's JSON line (gpurun_out/prof_<cfg>.log) reports
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $R/gpurun_out/prof_$cfg -o run -- python3 $R/bench.py --config $cfg --streams 1 \
        --steps $s --warmup 20 --no-cpu-baseline --no-variants --no-host-path --no-sublines \
        > $R/gpurun_out/prof_$cfg.log 2>&1) || exit $?
    f=$(find $R/gpurun_out/prof_$cfg -name "*kernel_stats.csv" | head -1)
    cp "$f" $R/gpurun_out/${tag}_${cfg}_streams1_kernel_stats.csv
    $S 300 bench_$cfg python bench.py --config $cfg --steps $s --warmup 20 --no-sublines || exit $?
    # raw rocprofv3 output: the JSON / summary above hold the results, and
    # gpurun copies gpurun_out/ back only below 64 MiB
    rm -rf gpurun_out/pmc_$cfg gpurun_out/prof_$cfg
done
echo profile-round-done
