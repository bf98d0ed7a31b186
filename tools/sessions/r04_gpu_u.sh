#!/bin/bash
# Round-4 closing GPU session on the final sources: the whole -m gpu suite and
# smoke(), then the profile round (PMC + kernel trace + line, every config).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/r04_gpu_tests_final.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.txt 2>&1
tail -2 $O/r04_gpu_tests_final.txt
bash tools/profile_round.sh r04
