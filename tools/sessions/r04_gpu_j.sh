#!/bin/bash
# round 4, session j: global-address-space loads past the window (all
# kernels) + FLOW_KERNEL 15 / 16 (port word read in the walk's L4 step):
# the -m gpu suite, the flows variants beside the default 13 and the plain
# parse (twice), and the C3 / C4 lines against the r04 profile round.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04j_tests.txt 2>&1
tail -2 gpurun_out/r04j_tests.txt
bash tools/c5_ab.sh r04j_a flow_kernel=13 flow_kernel=15 flow_kernel=16
bash tools/c5_ab.sh r04j_b flow_kernel=15 flow_kernel=13 flow_kernel=16
for c in c4 c3; do
  timeout -k 10 300 python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --no-host-path --no-variants > gpurun_out/r04j_bench_$c.json 2> gpurun_out/r04j_bench_$c.log
done
echo done-j
