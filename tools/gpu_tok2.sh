#!/bin/bash
# Two-stage device token parse (k_dec_tok1 + k_dec_tok2): decode tests with both
# parsers (TOK2_TESTS=0 skips), stage-1 cycles per step from the profiling builds
# (TOK2_PROF="tokprof ..."), host / device / auto rates at 1024 1080p frames over
# TOK2_DISTINCT distinct frames (4) per library (TOK2_LIBS="'' exp ...").
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=${TOK2_DISTINCT:-4}
if [ "${TOK2_TESTS:-1}" = 1 ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q -k "decode or golden or token or tokl" --timeout 200 --timeout-method thread > gpurun_out/tok2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tok2_tests.log
[ $rc -ne 0 ] && exit $rc
fi
for L in ${TOK2_PROF:-tokprof}; do
ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$L.so timeout -k 10 200 python -u tools/dec_tokens.py 64 1 device $D > gpurun_out/tok2_prof_$L.log 2>&1 || { tail -20 gpurun_out/tok2_prof_$L.log; exit 1; }
echo "== $L"; grep -E "k_dec_tok1|tokens=" gpurun_out/tok2_prof_$L.log | head -3
done
for L in ${TOK2_LIBS:-main}; do
if [ "$L" = main ]; then LIB=$PWD/image-webp_amd/zwebp/libzwebp.so; else LIB=$PWD/image-webp_amd/zwebp/libzwebp_$L.so; fi
ZWEBP_LIB=$LIB timeout -k 10 300 python -u tools/dec_tokens.py ${TOK2_FRAMES:-1024} 2 ${TOK2_MODES:-host,device,auto} $D > gpurun_out/tok2_b_$L.log 2>&1 || { tail -20 gpurun_out/tok2_b_$L.log; exit 1; }
echo "== $L"; cat gpurun_out/tok2_b_$L.log
done
