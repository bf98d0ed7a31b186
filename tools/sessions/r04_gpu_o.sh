#!/bin/bash
# Round-4 evidence on the k_flows_bits tree, session o: the driver's exact
# command (x3) and once under a kernel trace, the 30 M-frame differential run
# over every kernel, the determinism soak.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
R=$(pwd)
mkdir -p $O
for r in 1 2 3; do
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
timeout -k 10 400 python3 tools/soak.py --iters 2000 > $O/r04_soak.txt 2>&1
echo done-o
