# device token parse vs host at batch sizes 1024 / 2048 / 4096 (1080p), host shares of a split
mkdir -p gpurun_out
grep -o -w -E "avx512f|avx512cd|avx512bw|avx512vl|avx512_vbmi2|avx2|bmi2" /proc/cpuinfo | sort | uniq -c > gpurun_out/cpuflags.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/cpuflags.txt; cat gpurun_out/cpuflags.txt
for F in 1024 2048 4096; do
  timeout -k 10 400 python -u tools/dec_tokens.py $F 1 host,device >> gpurun_out/tokl_sizes.log 2>&1 || { tail -5 gpurun_out/tokl_sizes.log; exit 1; }
  for H in 0.25 0.4; do
    ZW_DEC_TOKENS_HOST=$H timeout -k 10 400 python -u tools/dec_tokens.py $F 1 mixed >> gpurun_out/tokl_sizes.log 2>&1 || { tail -5 gpurun_out/tokl_sizes.log; exit 1; }
  done
done
cat gpurun_out/tokl_sizes.log
