# device token parse: records equal to the host parse, a profiling build, 1024-frame rates
# (host / device / mixed splits, download parts 1 and 4), decode tests
mkdir -p gpurun_out && ZW_DEC_TOKENS_DUMP=gpurun_out/tok timeout -k 10 200 python -u tools/dec_tokens.py 64 1 host,device && \
ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_tokprof.so timeout -k 10 200 python -u tools/dec_tokens.py 64 1 device > gpurun_out/tokprof.log 2>&1 && grep k_dec_tokens gpurun_out/tokprof.log | head -4 && \
timeout -k 10 300 python -u tools/dec_tokens.py 1024 2 && \
ZW_DEC_DL_PARTS=4 timeout -k 10 300 python -u tools/dec_tokens.py 1024 2 && \
ZW_DEC_TOKENS_HOST=0.25 timeout -k 10 200 python -u tools/dec_tokens.py 1024 2 mixed && \
ZW_DEC_TOKENS_HOST=0.75 timeout -k 10 200 python -u tools/dec_tokens.py 1024 2 mixed && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "decode" --timeout 200 --timeout-method thread > gpurun_out/tok_tests.log 2>&1; tail -3 gpurun_out/tok_tests.log
