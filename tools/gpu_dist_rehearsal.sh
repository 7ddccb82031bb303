#!/bin/bash
# N=2 rehearsal of bench.py's distributed path on one GPU (gloo, both ranks on device 0)
mkdir -p gpurun_out
ZW_BENCH_BACKEND=gloo ZW_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --frames 256 --no-cpu-baseline \
  > gpurun_out/dist2.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "^\{" gpurun_out/dist2.log | cut -c1-300; tail -3 gpurun_out/dist2.log; exit $rc
