#!/bin/bash
# Iteration check: GPU parity tests, the phase-cycle profile (profiling build,
# make -C image-webp_amd prof) and a short bench (encode only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh pytest_gpu 500 python -u -m pytest ${TESTS:-tests -m gpu} -q -x --timeout 300 --timeout-method thread; rc=$?
[ $rc -ne 0 ] && exit $rc
tools/gpu_step.sh phase 200 python tools/phase_prof.py ${PHASE_FRAMES:-256}; rc=$?
fatal $rc && exit $rc
tools/gpu_step.sh bench 300 python bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-extras; rc=$?
exit $rc
