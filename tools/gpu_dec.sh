#!/bin/bash
# Decode kernels: parity tests, then timing of the batch shape (256 1080p
# frames, one workgroup per frame) for the library variants in DEC_LIBS
# ("" = the product library) with and without ZW_DEC_FUSE.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
if [ -z "$NO_TEST" ]; then
  tools/gpu_step.sh dectest 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rgb.py -m gpu -q -x -k "decode or loop_filter or roundtrip or rgb" --timeout 200 --timeout-method thread; rc=$?; fatal $rc && exit $rc
fi
for v in ${DEC_LIBS:-_}; do
  lib=$PWD/image-webp_amd/zwebp/libzwebp.so; [ "$v" != "_" ] && lib=$PWD/image-webp_amd/zwebp/libzwebp$v.so
  for fu in ${DEC_FUSE:-0}; do
    if [ "$fu" = 1 ]; then export ZW_DEC_FUSE=1; else unset ZW_DEC_FUSE; fi
    ZWEBP_LIB=$lib ZW_DEC_CHUNK=256 ZW_DEC_ROWS=0 tools/gpu_step.sh dec${v}_f$fu 240 python -u tools/dec_bench.py 256 3; rc=$?; fatal $rc && exit $rc
  done
done
exit 0
