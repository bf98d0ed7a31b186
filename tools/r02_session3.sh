set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
$S 120 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 bench python bench.py || exit $?
$S 300 bench20 python bench.py --steps 20 --warmup 5 || exit $?
echo done
