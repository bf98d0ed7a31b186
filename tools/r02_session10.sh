#!/usr/bin/env bash
# Round-2 GPU session 10: full GPU suite, smoke, default bench lines on the
# sc1-record / staggered-stream tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
$S 120 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 bench20 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 bench20b python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 bench python bench.py || exit $?
echo done
