#!/bin/bash
# Round-4 closing robustness run on the final sources: a second 30 M-frame
# differential run (another seed) and a 10x longer determinism soak.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 tools/bigfuzz.py --frames 30000000 --seed 9090 > $O/r04_bigfuzz_seed9090.log 2>&1
cp $O/bigfuzz.json $O/r04_bigfuzz_30M_seed9090.json
timeout -k 10 600 python3 tools/soak.py --iters 20000 > $O/r04_soak_20k.txt 2>&1
cp $O/soak.json $O/r04_soak_20k.json
tail -1 $O/r04_soak_20k.txt
echo done-z
