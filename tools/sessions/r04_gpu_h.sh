#!/bin/bash
# Round-4 GPU session H: the table-in-image flows kernel (FLOW_KERNEL 10/11).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_flows.py > $O/r04h_tests.txt 2>&1
tools/c5_ab.sh r04_c5ab4 flow_kernel=10 flow_kernel=11 window_indexed=1045
