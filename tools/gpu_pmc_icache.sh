#!/bin/bash
# Instruction-fetch PMC passes for the encode kernels (each pass its own rocprofv3 run,
# kernel-trace only). usage: tools/gpu_pmc_icache.sh [frames] [lib]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmci
F=${1:-64}
[ -n "$2" ] && export ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$2
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmci/p$i -o run -- python3 tools/enc_once.py $F > gpurun_out/pmci/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/pmci/p$i.log && exit $rc
done
exit 0
