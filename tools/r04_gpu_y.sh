#!/bin/bash
# round 4, session y: FLOW_KERNEL 16 (k_flows_bits with the histogram's
# atomics fused in) — flows parity incl. histograms, then the whole C5 step
# (flows + histogram, 2 streams) A/B against 15 + the separate histogram
# pass, and the flows kernel alone beside the plain parse.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_flows.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04y_tests.txt 2>&1
tail -2 gpurun_out/r04y_tests.txt
timeout -k 10 400 python3 tools/abtune.py --config c5 --var fk=15 --var fk=16 --rounds 6 --out gpurun_out/r04y_step_ab.json > gpurun_out/r04y_step_ab.log 2>&1
tail -4 gpurun_out/r04y_step_ab.log
timeout -k 10 400 python3 tools/abtune.py --config c5 --var fk=16 --var fk=15 --rounds 6 --out gpurun_out/r04y_step_ab2.json > gpurun_out/r04y_step_ab2.log 2>&1
tail -4 gpurun_out/r04y_step_ab2.log
echo done-y
