#!/usr/bin/env bash
# Round-2 GPU session 11: staging-load cache bits (INGOT_TUNE_CACHE_POLICY bits 6-8).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 pipe_tests python -u -m pytest tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread || exit $?
$S 300 ab11_c2_s2 python tools/abtune.py --config c2 --rounds 6 --var streams=2 --var streams=2,pol=75 --var streams=2,pol=139 --var streams=2,pol=203 --var streams=2,pol=267 --var streams=2,pol=331 --var streams=2,pol=395 --out gpurun_out/ab11_c2_s2.json || exit $?
$S 300 ab11_c2_s1 python tools/abtune.py --config c2 --rounds 6 --var streams=1 --var streams=1,pol=75 --var streams=1,pol=139 --var streams=1,pol=203 --var streams=1,pol=267 --var streams=1,pol=331 --var streams=1,pol=395 --out gpurun_out/ab11_c2_s1.json || exit $?
$S 300 ab11_c3 python tools/abtune.py --config c3 --rounds 3 --var pol=2 --var pol=66 --var pol=130 --var pol=194 --var pol=258 --var pol=322 --var pol=386 --out gpurun_out/ab11_c3.json || exit $?
$S 300 ab11_c4 python tools/abtune.py --config c4 --rounds 3 --var pol=2 --var pol=66 --var pol=194 --var pol=322 --out gpurun_out/ab11_c4.json || exit $?
echo done
