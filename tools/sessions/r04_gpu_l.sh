#!/bin/bash
# round 4, session l: FLOW_KERNEL 16 (k_flows_bits with the key windows'
# scalar loads one word ahead) beside 15 and the default 13, two orders.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_flows.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04l_tests.txt 2>&1
tail -2 gpurun_out/r04l_tests.txt
bash tools/c5_ab.sh r04l_a flow_kernel=13 flow_kernel=15 flow_kernel=16
bash tools/c5_ab.sh r04l_b flow_kernel=16 flow_kernel=15 flow_kernel=13
echo done-l
