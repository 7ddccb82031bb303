# headline-only bench per library variant, alternating (verified digests in every line)
mkdir -p gpurun_out
for r in 1 2; do for lib in "$@"; do
  echo -n "$lib: "
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 300 python -u bench.py --steps 10 --no-extras --no-cpu-baseline 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value'],1), d['verified'], {k: round(v,2) for k,v in d.get('kernel_ms_per_step', {}).items()})" || exit 1
done; done
