# headline-only bench per pipeline lane count, alternating
mkdir -p gpurun_out
for r in 1 2; do for L in 2 3 4; do
  echo -n "lanes $L: "
  ZW_PIPE_LANES=$L timeout -k 10 300 python -u bench.py --steps 10 --no-extras --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' || exit 1
done; done
