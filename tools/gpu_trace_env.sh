#!/bin/bash
# pipeline timeline under different copy-engine settings
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" ZW_PIPE_TRACE=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tr.log 2>&1 || return $?; grep -E "^lane|chunk [0-3]: p1 fetched" gpurun_out/tr.log | tail -5; }
run X=0 || exit $?
run GPU_FORCE_BLIT_COPY_SIZE=0 || exit $?
run HSA_ENABLE_SDMA=1 || exit $?
run GPU_BLIT_ENGINE_TYPE=1 || exit $?
run GPU_BLIT_ENGINE_TYPE=2 || exit $?
