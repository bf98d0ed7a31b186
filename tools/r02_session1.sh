#!/usr/bin/env bash
# Round-2 GPU session 1: parity suite, doorbell-gated C2 bench at the
# driver's 20 steps (and ungated / long-run for comparison), the gloo N=2
# rehearsal on one GPU, strong-scaling C4 at N=1, the c2r parse_read shape.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- bash tools/r02_session1.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 300 pytest_gpu python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S 150 bench_c2_20 python bench.py --steps 20 --warmup 5 || exit $?
$S 120 bench_c2_20_nogate python bench.py --steps 20 --warmup 5 --no-gate --no-cpu-baseline || exit $?
$S 120 bench_c2_2000 python bench.py --no-cpu-baseline || exit $?
$S 180 bench_gloo2 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline --no-variants || exit $?
$S 120 bench_c2r python bench.py --config c2r --steps 200 --warmup 10 --no-cpu-baseline || exit $?
$S 300 bench_c4_strong python bench.py --config c4 --scaling strong --steps 10 --warmup 2 --no-cpu-baseline --no-variants || exit $?
echo session-done
