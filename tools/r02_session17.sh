#!/usr/bin/env bash
# Round-2 GPU session 17: line-completing windows (INGOT_TUNE_WINDOW_INDEXED 20+k):
# parity, interleaved A/B, PMC read bytes per frame against the line floor.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 300 win_parity python -u -m pytest tests/test_gpu_parity.py -x -q -k "window or compact or packed" --timeout 300 --timeout-method thread || exit $?
grep -q "passed" gpurun_out/win_parity.log && ! grep -q "failed" gpurun_out/win_parity.log || exit 3
$S 300 ab17_c3 python tools/abtune.py --config c3 --rounds 3 --var win_i=0 --var win_i=23 --var win_i=24 --var win_i=25 --var win_i=28 --out gpurun_out/ab17_c3.json || exit $?
$S 300 ab17_c4 python tools/abtune.py --config c4 --rounds 3 --var win_i=0 --var win_i=24 --var win_i=25 --var win_i=28 --out gpurun_out/ab17_c4.json || exit $?
for w in 2 3 8 25 28; do
  $S 300 pmcw_c3_$w python tools/pmc_traffic.py --config c3 --tag r02w --tune window_indexed=$w || exit $?
done
for w in 2 28; do
  $S 300 pmcw_c4_$w python tools/pmc_traffic.py --config c4 --tag r02w --tune window_indexed=$w || exit $?
done
echo done
