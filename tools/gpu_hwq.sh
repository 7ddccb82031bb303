# headline-only bench at GPU_MAX_HW_QUEUES 4 / 8 / 16, alternating (verified digests in every line)
mkdir -p gpurun_out
for r in 1 2; do for q in 8 4 16; do
  echo -n "hwq $q: "
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 10 --no-extras --no-cpu-baseline 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value'],1), d['verified'])" || exit 1
done; done
