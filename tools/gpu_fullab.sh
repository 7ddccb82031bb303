# full bench per library variant, alternating; prints the headline and the host-heavy legs
mkdir -p gpurun_out
for r in 1 2; do for lib in "$@"; do
  echo -n "$lib: "
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline 2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print(round(d['value'], 1), d['verified'], 'container', round(d['container_rgba']['container_rgba_encodes_per_s'], 1),
      'host_resident', round(d['host_resident']['encodes_per_s'], 1), 'seam16', round(d['seam_threads']['threads']['16']['encodes_per_s'], 1),
      'decode', round(d['decode_path']['batch_decodes_per_s'], 1), 'emit_ms', round(d['host_ms_per_step']['emit'], 1))" || exit 1
done; done
