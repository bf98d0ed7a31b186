# Every bench config once on one GPU, one JSON line each, collected into
# gpurun_out/bench_all.json (-> profiles/rNN_bench_all_configs.json).
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/bench_all.sh [steps]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=${1:-200}
mkdir -p gpurun_out
for c in c2 c2m c3 c3p c3r c3s c4 c5 c6; do
    case $c in c2|c2m) s=2000 ;; *) s=$STEPS ;; esac
    tools/gpu_step.sh 300 bench_$c python bench.py --config $c --steps $s --warmup 20
done
python - <<'EOF'
import json
from pathlib import Path
out = {}
for c in "c2 c2m c3 c3p c3r c3s c4 c5 c6".split():
    lines = [l for l in Path(f"gpurun_out/bench_{c}.log").read_text().splitlines()
             if l.startswith("{")]
    out[c] = json.loads(lines[-1])
Path("gpurun_out/bench_all.json").write_text(json.dumps(out, indent=1))
for c, v in out.items():
    print(c, v["value"], v["ms_per_step"], v["roofline"]["frac"])
EOF
