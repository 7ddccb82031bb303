#!/bin/bash
# Full GPU tests, then a one-lane rocprofv3 kernel trace of a short bench
# (kernel averages without the two lanes' overlap).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit $?
ZW_PIPE_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o one -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof1.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '^{' gpurun_out/prof1.log | cut -c1-200; exit $rc
