set -eo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for a in "20 5" "20 50" "100 5" "20 5"; do set -- $a
  timeout -k 10 200 python3 bench.py --config c5 --steps $1 --warmup $2 --no-cpu-baseline --no-host-path --no-variants > gpurun_out/c5edge_$1_$2.json 2>/dev/null
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c5edge_$1_$2.json').read().splitlines() if x.startswith('{')][-1])
print('steps $1 warmup $2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launch_mean_us'])"
done
