#!/bin/bash
# bench (default + larger batch) then a rocprofv3 kernel-trace pass of the default bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/gpu_step.sh bench_default 500 python bench.py ${BENCH_ARGS} || exit $?
tools/gpu_step.sh bench_f256 500 python bench.py --frames 256 --steps 3 --no-cpu-baseline || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -5 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
