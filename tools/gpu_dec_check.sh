#!/bin/bash
# Decoder check: RGB / decode GPU tests, then the decode-path line of the bench
# (extras only) and the per-phase host timing of a single-frame decode.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh dec_tests 300 python -u -m pytest tests/test_gpu_rgb.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "decode or rgb or loop_filter" || exit $?
ZW_DEC_TIMING=1 tools/gpu_step.sh dec_bench 300 python tools/dec_rgba_bench.py 256 || exit $?
tools/gpu_step.sh dec_single 200 python tools/dec_bench.py || exit $?
