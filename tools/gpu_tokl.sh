# lane-parallel device token parse (k_dec_tokl): records equal to the host parse on a
# 64-frame batch, cycles per step from the profiling build, 1024-frame rates, decode tests
mkdir -p gpurun_out
ZW_DEC_TOKENS_DUMP=gpurun_out/tok timeout -k 10 200 python -u tools/dec_tokens.py 64 1 host,device > gpurun_out/tokl_a.log 2>&1 || { tail -20 gpurun_out/tokl_a.log; exit 1; }
cat gpurun_out/tokl_a.log
python tools/cmp_recs.py gpurun_out/tok 8160 | head -8
for L in ${TOKL_LIBS:-tokprof}; do
ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$L.so timeout -k 10 200 python -u tools/dec_tokens.py 64 1 device > gpurun_out/tokl_prof_$L.log 2>&1 || { tail -20 gpurun_out/tokl_prof_$L.log; exit 1; }
echo "== $L"; grep -E "k_dec_tokl|tokens=" gpurun_out/tokl_prof_$L.log | head -4
done
[ -n "$TOKL_QUICK" ] && exit 0
timeout -k 10 300 python -u tools/dec_tokens.py 1024 2 host,device,mixed > gpurun_out/tokl_b.log 2>&1 || { tail -20 gpurun_out/tokl_b.log; exit 1; }
cat gpurun_out/tokl_b.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rgb.py -m gpu -x -q -k "decode or golden or lossy" --timeout 200 --timeout-method thread > gpurun_out/tokl_tests.log 2>&1; tail -5 gpurun_out/tokl_tests.log
