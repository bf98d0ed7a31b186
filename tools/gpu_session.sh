# Evidence refresh: full GPU suite, smoke, bench lines for every config,
# rocprofv3 kernel stats of the default command.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 pytest_gpu python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
tools/gpu_step.sh 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
tools/gpu_step.sh 300 bench_c2 python bench.py
for c in c2m c3 c3p c3r c3s c4 c5 c6; do
tools/gpu_step.sh 300 bench_$c python bench.py --config $c --steps 200 --warmup 10
done
