#!/bin/bash
# Run one GPU step under its own time limit; log to gpurun_out/<name>.log.
# Usage: tools/gpu_step.sh NAME SECONDS cmd...   Exit codes: passes through
# test failures (1) so later independent steps still run from the caller, but
# the caller must stop on 124/137 (time limit), 134/139 (abort/segv).
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc"
tail -n 30 "gpurun_out/$name.log"
exit $rc
