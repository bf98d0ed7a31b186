#!/bin/bash
# Round-4 closing: the driver's exact command x3 on the final sources (the
# lines attach the closing profile round's PMC files) and once under a kernel
# trace.
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
echo done-v
