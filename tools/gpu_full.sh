#!/bin/bash
# Full round check: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace of a short bench.
# Stops at the first time-limit / fault exit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh bench 400 python bench.py ${BENCH_ARGS}; rc=$?
fatal $rc && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
exit $rc
