#!/usr/bin/env bash
# Round-2 GPU session 6: the ring kernel's grid / depth re-checked under the
# device-scope record stores; default bench lines (2,000 and 20 steps).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 pipe_tests python -u -m pytest tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread || exit $?
$S 300 ab6_c2 python tools/abtune.py --config c2 --rounds 6 --var streams=2 --var streams=2,pipe=4 --var streams=2,pipe=16 --var streams=2,depth=3 --var streams=2,pol=3 --var streams=1 --var streams=1,pipe=4 --var streams=1,depth=3 --out gpurun_out/ab6_c2.json || exit $?
$S 300 bench python bench.py || exit $?
$S 300 bench20 python bench.py --steps 20 --warmup 5 || exit $?
$S 300 bench20b python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
