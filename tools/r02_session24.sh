#!/usr/bin/env bash
# Round-2 GPU session 24: C5 bench line with the fixed 5-chunk flows window vs the default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 c5_def python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline --no-host-path || exit $?
$S 300 c5_w5 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline --no-host-path --tune window_indexed=5 || exit $?
$S 300 c5_def2 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline --no-host-path || exit $?
$S 300 ab24_c5 python tools/abtune.py --config c5 --rounds 3 --var fonly=1 --var fonly=1,win_i=5 --var win_i=0 --var win_i=5 --out gpurun_out/ab24_c5.json || exit $?
echo done
