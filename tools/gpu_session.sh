#!/bin/bash
# One GPU session: smoke -> GPU tests -> bench -> (optional) encode PMC.
# Every step has its own time limit (tools/gpu_step.sh); the session stops at
# the first time-limit / fault exit and at the first test failure.
#   BENCH_ARGS   extra bench.py arguments      PMC=1  run tools/gpu_pmc_encode.sh
#   TESTS        pytest selection (default: tests -m gpu)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -ne 0 ] && exit $rc
tools/gpu_step.sh pytest_gpu 600 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread; rc=$?
[ $rc -ne 0 ] && exit $rc
tools/gpu_step.sh bench 500 python bench.py ${BENCH_ARGS}; rc=$?
fatal $rc && exit $rc
if [ -n "$PMC" ]; then
  tools/gpu_pmc_encode.sh 256 > gpurun_out/pmc_enc.log 2>&1; rc=$?
  echo "[pmc] rc=$rc"; tail -40 gpurun_out/pmc_enc.log
fi
exit $rc
