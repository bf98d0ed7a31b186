set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 -Iinclude tools/c2_loop.cpp -Lingot_amd/lib -lingot_gpu -Wl,-rpath,$GRAFT_REPO_ROOT/ingot_amd/lib -o /tmp/c2_loop 2>/dev/null
for s in 1 2 3; do tools/gpu_step.sh 120 c2loop_s$s /tmp/c2_loop $s 2000; done
tools/gpu_step.sh 300 ab_c2 python tools/abtune.py --config c2 --rounds 3 --var streams=1 --var streams=2 --var streams=3 --out gpurun_out/ab_c2.json
