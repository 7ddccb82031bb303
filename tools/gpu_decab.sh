# batch decode (host parse) chunk size x download parts sweep on 1024 1080p frames, interleaved rounds
mkdir -p gpurun_out
for round in 1 2 3; do for C in 128 256 512; do for P in 2 4; do
  echo -n "r$round chunk $C parts $P: "
  ZW_DEC_CHUNK=$C ZW_DEC_DL_PARTS=$P timeout -k 10 120 python -u tools/dec_tokens.py 1024 3 host 2>&1 | grep -o "[0-9]* decodes/s" || exit 1
done; done; done
