#!/bin/bash
# k_xform_mb A/B on one box: the product library against a variant build
# (VARIANT=<exp name>, image-webp_amd/zwebp/libzwebp_<exp>.so from `make exp`),
# interleaved, after the k_xform_mb parity tests (run against the variant too).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=${VARIANT:-full}
tools/gpu_step.sh xmbtest 300 python -u -m pytest tests/test_xmb.py -m gpu -q -x --timeout 120 --timeout-method thread || exit $?
ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$V.so tools/gpu_step.sh xmbtest_$V 300 python -u -m pytest tests/test_xmb.py -m gpu -q -x --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  tools/gpu_step.sh xmb_base$i 240 python -u tools/xmb_bench.py || exit $?
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$V.so tools/gpu_step.sh xmb_$V$i 240 python -u tools/xmb_bench.py || exit $?
done
