#!/bin/bash
# round 4, session k: FLOW_KERNEL 15 (k_flows_bits: the Toeplitz hash bit by
# bit from the key windows in SGPRs, no table) — flows parity, then beside the
# default 13 and the plain parse, two orders.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_flows.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04k_tests.txt 2>&1
tail -2 gpurun_out/r04k_tests.txt
bash tools/c5_ab.sh r04k_a flow_kernel=13 flow_kernel=15
bash tools/c5_ab.sh r04k_b flow_kernel=15 flow_kernel=13
echo done-k
