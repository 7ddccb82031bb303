#!/bin/bash
# bench (default config) then a rocprofv3 kernel-trace pass of a shorter bench run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/gpu_step.sh bench_default 600 python bench.py ${BENCH_ARGS} || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
