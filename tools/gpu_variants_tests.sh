#!/bin/bash
# Per library variant: a parity test subset (TESTS_K pattern), then a short verified bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  n=$(basename $lib .so)
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -k "${TESTS_K:-encode}" > gpurun_out/t_$n.log 2>&1 || { echo "tests $n failed"; tail -5 gpurun_out/t_$n.log; exit 1; }
  echo "tests $n: $(tail -1 gpurun_out/t_$n.log)"
done
STEPS=${STEPS:-10} bash tools/gpu_variants.sh "$@" "$@"
