#!/usr/bin/env bash
# Round-2 GPU session 4: record-store scope variants (INGOT_TUNE_CACHE_POLICY
# bits 3-5) — parity, then interleaved A/B on C2 (1 and 2 streams) and C3.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 pipe_tests python -u -m pytest tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread || exit $?
$S 300 ab_c2_s1 python tools/abtune.py --config c2 --var streams=1 --var streams=1,pol=11 --var streams=1,pol=19 --var streams=1,pol=27 --var streams=1,pol=35 --var streams=1,pol=43 --var streams=1,pol=1 --out gpurun_out/ab_c2_s1.json || exit $?
$S 300 ab_c2_s2 python tools/abtune.py --config c2 --var streams=2 --var streams=2,pol=11 --var streams=2,pol=19 --var streams=2,pol=27 --var streams=2,pol=35 --var streams=2,pol=43 --out gpurun_out/ab_c2_s2.json || exit $?
$S 300 ab_c3 python tools/abtune.py --config c3 --var pol=2 --var pol=10 --var pol=18 --var pol=26 --var pol=34 --out gpurun_out/ab_c3.json || exit $?
echo done
