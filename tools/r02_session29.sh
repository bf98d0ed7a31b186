#!/usr/bin/env bash
# Round-2 GPU session 29: parse_read default = line-completing chunk-0 window —
# GPU suite, smoke, A/B vs the round-1 plan.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S 900 gputests python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || exit 3
$S 120 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 ab29_c3r python tools/abtune.py --config c3r --rounds 4 --var plan=0 --var plan=1 --out gpurun_out/ab29_c3r.json || exit $?
$S 300 ab29_c2r python tools/abtune.py --config c2r --rounds 4 --var plan=0 --var plan=1 --out gpurun_out/ab29_c2r.json || exit $?
$S 300 pmcr_11 python tools/pmc_traffic.py --config c3r --tag r02w --tune read_plan=11 || exit $?
echo done
