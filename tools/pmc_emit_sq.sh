#!/usr/bin/env bash
# SQ counters of the emit kernels (one rocprofv3 pass, 8 SQ counters):
#   bash tools/pmc_emit_sq.sh TAG [emit_probe args...]
# -> gpurun_out/pmc_emit_TAG/ (sqlite; read with tools/pmc_db.py)
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmc_emit_$tag -o p -- \
    python3 tools/emit_probe.py --reps 2 --rounds 1 "$@" > gpurun_out/pmc_emit_$tag.log 2>&1
