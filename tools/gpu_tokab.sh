# token-parse A/B: per profiling build, 64 frames (device tokens: cycles per decision) and 1024 frames (host vs mixed)
mkdir -p gpurun_out
for L in ${LIBS:-tokprof toksmem tokw4 tokw8}; do
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$L.so timeout -k 10 200 python -u tools/dec_tokens.py 64 1 device > gpurun_out/tokab_$L.log 2>&1 || exit 1
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/libzwebp_$L.so timeout -k 10 300 python -u tools/dec_tokens.py 1024 2 host,mixed,device >> gpurun_out/tokab_$L.log 2>&1 || exit 1
  echo "== $L"; grep -E "k_dec_tokens|tokens=" gpurun_out/tokab_$L.log | grep -v "frame 0:" | head -6
done
