#!/bin/bash
# Round-4 final GPU session 2: the driver's exact command (x2) and its kernel
# trace, then the 30 M-frame differential run over every kernel.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
R=$(pwd)
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
timeout -k 10 900 python3 tools/bigfuzz.py --frames 30000000 --seed 7070 > $O/r04_bigfuzz.log 2>&1
cp $O/bigfuzz.json $O/r04_bigfuzz_30M.json
