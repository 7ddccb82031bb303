#!/bin/bash
# k_yuv2rgb: the RGB/RGBA decode tests, then the 256-frame RGBA timing for the
# library variants in Y2R_LIBS ("_" = the product library).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh y2rtest 300 python -u -m pytest tests/test_gpu_rgb.py -m gpu -q -x --timeout 120 --timeout-method thread; rc=$?; fatal $rc && exit $rc
for v in ${Y2R_LIBS:-_}; do
  lib=$PWD/image-webp_amd/zwebp/libzwebp.so; [ "$v" != "_" ] && lib=$PWD/image-webp_amd/zwebp/libzwebp$v.so
  ZWEBP_LIB=$lib ZW_DEC_CHUNK=128 tools/gpu_step.sh y2r$v 240 python -u tools/yuv2rgb_bench.py; rc=$?; fatal $rc && exit $rc
done
exit 0
