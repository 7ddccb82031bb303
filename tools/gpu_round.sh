#!/bin/bash
# GPU session script: smoke -> parity tests -> bench.  Stops at the first
# time-limit / fault exit; plain test failures (rc 1) continue to the bench.
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh pytest_gpu 700 python -m pytest tests -m gpu -q ${PYTEST_ARGS:--x}; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh bench 400 python bench.py ${BENCH_ARGS}; rc=$?
exit $rc
