#!/bin/bash
# round 4, session m: FLOW_KERNEL 17 (k_flows_bits with the key in SGPRs,
# each window one scalar shift) beside 15 and the default 13, two orders.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_flows.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04m_tests.txt 2>&1
tail -2 gpurun_out/r04m_tests.txt
bash tools/c5_ab.sh r04m_a flow_kernel=13 flow_kernel=15 flow_kernel=17
bash tools/c5_ab.sh r04m_b flow_kernel=17 flow_kernel=15 flow_kernel=13
echo done-m
