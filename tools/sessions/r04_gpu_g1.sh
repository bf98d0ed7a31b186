#!/bin/bash
# Round-4 final GPU session 1: the whole -m gpu suite and smoke() on the final tree.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/r04_gpu_tests_final.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.txt 2>&1
tail -3 $O/r04_gpu_tests_final.txt
