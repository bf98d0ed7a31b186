#!/usr/bin/env bash
# Round-2 GPU session 5: record-store scope variants, second pass (more
# rounds, stream counts, 8-B records, the rewrite ring and C4/C6).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 ab5_c2_s2 python tools/abtune.py --config c2 --rounds 8 --var streams=2 --var streams=2,pol=11 --var streams=2,pol=27 --var streams=2,pol=1 --var streams=3,pol=11 --var streams=4,pol=11 --out gpurun_out/ab5_c2_s2.json || exit $?
$S 300 ab5_c2_s1 python tools/abtune.py --config c2 --rounds 8 --var streams=1 --var streams=1,pol=11 --var streams=1,pol=27 --var streams=1,pol=1 --out gpurun_out/ab5_c2_s1.json || exit $?
$S 300 ab5_c2_r8 python tools/abtune.py --config c2 --rounds 6 --var streams=2,rec=8 --var streams=2,rec=8,pol=11 --var streams=2,rec=8,pol=27 --var streams=1,rec=8 --var streams=1,rec=8,pol=11 --out gpurun_out/ab5_c2_r8.json || exit $?
$S 300 ab5_c2m python tools/abtune.py --config c2m --rounds 6 --var streams=2 --var streams=2,pol=11 --var streams=2,pol=27 --var streams=1 --var streams=1,pol=11 --out gpurun_out/ab5_c2m.json || exit $?
$S 300 ab5_c4 python tools/abtune.py --config c4 --rounds 4 --var pol=2 --var pol=18 --var pol=34 --out gpurun_out/ab5_c4.json || exit $?
$S 300 ab5_c3s python tools/abtune.py --config c3s --rounds 4 --var pol=2 --var pol=18 --var pol=34 --var pol=10 --out gpurun_out/ab5_c3s.json || exit $?
echo done
