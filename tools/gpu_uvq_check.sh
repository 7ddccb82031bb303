#!/bin/bash
# encode parity tests (both kernel shapes) -> short verified bench -> small-batch sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh enc_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -k "encode" || exit $?
ZW_PIPE_LANES=1 bash tools/gpu_variants.sh libzwebp.so || exit $?
tools/gpu_step.sh small_batch 300 python tools/small_batch.py 1920 1080 ${SB_SIZES:-1,8,32}
