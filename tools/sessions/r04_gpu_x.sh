#!/bin/bash
# round 4, session x: k_flows_bits with narrower windows (FLOW_KERNEL 16:
# 3..5 chunks, 17: 2..5 — the plain parse's) now that the address block's
# source is chosen per lane, beside 15 and the plain parse, two orders.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_flows.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04x_tests.txt 2>&1
tail -2 gpurun_out/r04x_tests.txt
bash tools/c5_ab.sh r04x_a flow_kernel=15 flow_kernel=16 flow_kernel=17
bash tools/c5_ab.sh r04x_b flow_kernel=17 flow_kernel=16 flow_kernel=15
echo done-x
