#!/bin/bash
# C5 flows-kernel A/B on the GPU box: the flows variants beside the plain
# parse over the same FLOWS frames (tools/c5_same_run.py), then per-kernel
# HBM bytes (tools/pmc_kernels.py).  Usage: tools/c5_ab.sh TAG VARIANT...
# (VARIANT = KEY=VALUE[,KEY=VALUE], e.g. window_indexed=1056)
set -eo pipefail
tag=$1; shift
args=()
for v in "$@"; do args+=(--variant "$v"); done
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/c5_same_run.py --reps 10 "${args[@]}" \
    --out gpurun_out/${tag}_events.json > gpurun_out/${tag}_events.log 2>&1
timeout -k 10 400 python3 tools/pmc_kernels.py --sized --out gpurun_out/${tag}_pmc.json -- \
    python3 tools/c5_same_run.py --reps 2 "${args[@]}" --out /tmp/c5_pmc_run.json \
    > gpurun_out/${tag}_pmc.log 2>&1
rm -rf gpurun_out/${tag}_pmc  # raw rocprofv3 CSVs: the JSON holds the result
