#!/bin/bash
# Round-4 evidence on the k_flows_bits tree, session n: the whole -m gpu suite
# and smoke().
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/r04_gpu_tests_final.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.txt 2>&1
tail -3 $O/r04_gpu_tests_final.txt
