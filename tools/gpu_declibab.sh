# batch decode (host parse, 1024 1080p frames) per library variant, interleaved rounds;
# an argument lib@VAR=VALUE runs lib with that environment variable set
mkdir -p gpurun_out
for round in 1 2 3; do for arg in "$@"; do
  lib=${arg%%@*}; envs=""; [ "$arg" != "$lib" ] && envs=${arg#*@}
  echo -n "r$round $arg: "
  env $envs ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 120 python -u tools/dec_tokens.py 1024 3 host 2>&1 | grep -o "[0-9]* decodes/s.*" || exit 1
done; done
