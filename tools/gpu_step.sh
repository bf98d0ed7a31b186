#!/usr/bin/env bash
# Run one GPU step under its own time limit; log its exit code.  Exit 0/1
# (pass / ordinary test failure) lets the session continue; anything else
# (fault, abort, segfault, timeout) stops the session: run nothing more.
# usage: tools/gpu_step.sh SECONDS LOGNAME cmd...
set -u
secs=$1; name=$2; shift 2
mkdir -p "${GRAFT_REPO_ROOT:-.}/gpurun_out"
out="${GRAFT_REPO_ROOT:-.}/gpurun_out/$name.log"
echo "[gpu_step] $(date +%T) start $name: $*" | tee -a "${GRAFT_REPO_ROOT:-.}/gpurun_out/steps.log"
timeout -k 10 "$secs" "$@" > "$out" 2>&1
rc=$?
echo "[gpu_step] $(date +%T) end $name rc=$rc" | tee -a "${GRAFT_REPO_ROOT:-.}/gpurun_out/steps.log"
tail -5 "$out"
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
exit 0
