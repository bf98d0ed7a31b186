#!/usr/bin/env bash
# Round-2 GPU session 2: where a 20-step region's fixed cost goes.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 200 region_probe python tools/region_probe.py || exit $?
cp gpurun_out/region_probe.log gpurun_out/region_probe.json
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace20 -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants > $R/gpurun_out/trace20.log 2>&1 || exit $?
echo session-done
