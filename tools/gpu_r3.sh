#!/bin/bash
# Round-3 GPU session: smoke -> GPU parity tests -> k_xform_mb leg -> bench.
# Stops at the first time-limit / fault exit (no GPU step after one).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh pytest_gpu 900 python -u -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} --timeout 300 --timeout-method thread; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh xmb 240 python -u tools/xmb_bench.py; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh bench 500 python -u bench.py ${BENCH_ARGS}; rc=$?
exit $rc
