#!/usr/bin/env bash
# SQ counters of the C2 slot-ring kernel (k_parse_pipe), single stream, two
# passes of at most 8 SQ counters each:
#   bash tools/pmc_c2_sq.sh TAG [bench args...]
# -> gpurun_out/pmc_c2sq_TAG_{a,b}/ (sqlite; read with tools/pmc_db.py)
set -e
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
B="bench.py --config c2 --streams 1 --steps 50 --warmup 5 --no-cpu-baseline --no-variants --no-host-path --no-sublines"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU"
Bc="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --pmc $A -d gpurun_out/pmc_c2sq_${tag}_a -o p -- \
    python3 $B "$@" > gpurun_out/pmc_c2sq_${tag}_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc $Bc -d gpurun_out/pmc_c2sq_${tag}_b -o p -- \
    python3 $B "$@" > gpurun_out/pmc_c2sq_${tag}_b.log 2>&1
