#!/bin/bash
# encoder parity tests (all encode + quantiser tests) -> short one-lane verified bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh enc_tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -k "encode or quant" || exit $?
ZW_PIPE_LANES=1 bash tools/gpu_variants.sh ${LIBS:-libzwebp.so}
