#!/bin/bash
# Round-4 final GPU session on the frozen tree: the whole -m gpu suite and
# smoke(), the driver's exact command x2 + once under a kernel trace, and the
# 30 M-frame differential run.  Stops at the first failing step.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
R=$(pwd)
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/r04_gpu_tests_final.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r04_driver_line_$r.json \
      2> $O/r04_driver_line_$r.err
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/$O/r04_driver_prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 \
    > $R/$O/r04_driver_line_traced.json 2> $R/$O/r04_driver_line_traced.err)
f=$(find $O/r04_driver_prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/r04_c2_driver_kernel_stats.csv
rm -rf $O/r04_driver_prof
timeout -k 10 300 python3 tools/cpu_share_probe.py > $O/r04_cpu_share_probe.log 2>&1
timeout -k 10 900 python3 tools/bigfuzz.py --frames 30000000 --seed 7070 > $O/r04_bigfuzz.log 2>&1
cp $O/bigfuzz.json $O/r04_bigfuzz_30M.json
tail -1 $O/r04_gpu_tests_final.txt
