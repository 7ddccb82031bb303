#!/bin/bash
# Decode kernels: row-parallel (ZW_DEC_ROWS=1) vs one workgroup per frame (0)
# over batch sizes; picks the default threshold in zw_dec_host.cpp.
mkdir -p gpurun_out
for n in 1 8 32 64 256; do
  for r in 1 0; do
    echo "== frames $n rows $r"
    ZW_DEC_ROWS=$r timeout -k 10 120 python tools/dec_bench.py $n 3 || exit $?
  done
done
