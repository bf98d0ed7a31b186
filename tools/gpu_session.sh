set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 pytest_flows python -u -m pytest tests/test_flows.py -x -q -m gpu --timeout 120 --timeout-method thread
tools/gpu_step.sh 300 ab_c5 python tools/abtune.py --config c5 --rounds 3 --var mode=flows --var mode=flows,blocks=1280 --var mode=flows,blocks=768 --var mode=flows,blocks=2048 --var mode=parse --out gpurun_out/ab_c5.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU --output-format csv -d gpurun_out/sq2_c5b -o run -- python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-variants --streams 1 > gpurun_out/sq2_c5b.log 2>&1
