#!/bin/bash
# Decode-kernel check + timing (ZW_DEC_RECON4 1 / 0), then the xmb variants.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh dectest 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "decode or loop_filter or roundtrip" --timeout 200 --timeout-method thread; rc=$?; fatal $rc && exit $rc
for r4 in 1 0; do
  ZW_DEC_RECON4=$r4 ZW_DEC_CHUNK=256 ZW_DEC_ROWS=0 tools/gpu_step.sh dec_r4_$r4 240 python -u tools/dec_bench.py 256 3; rc=$?; fatal $rc && exit $rc
done
for v in ${XMB_VARIANTS:-}; do
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp$v.so tools/gpu_step.sh xmb$v 240 python -u tools/xmb_bench.py; rc=$?; fatal $rc && exit $rc
done
exit 0
