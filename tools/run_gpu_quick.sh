#!/bin/bash
# local: build everything, then run the quick GPU iteration (tests + phase profile)
set -e
make -s -C /root/repo/image-webp_amd
make -s -C /root/repo/image-webp_amd prof
make -s -C /root/repo/oracle
timeout 1500 /usr/local/graft/bin/gpurun --timeout 900 -- tools/gpu_quick.sh "$@"
