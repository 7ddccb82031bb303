#!/bin/bash
# Decode kernels (k_dec_recon, k_loopfilter; 256 1080p frames, one workgroup per
# frame): kernel trace + SQ counter passes over tools/dec_bench.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcdec
export ZW_DEC_CHUNK=256 ZW_DEC_ROWS=0 DEC_BATCH_ONLY=1
run() {  # name, rocprofv3 args...
  local n=$1; shift
  timeout -k 10 150 rocprofv3 "$@" --output-format csv -d gpurun_out/pmcdec/$n -o $n -- python3 tools/dec_bench.py 256 2 > gpurun_out/pmcdec/$n.log 2>&1
  local rc=$?; echo "[$n] rc=$rc"; tail -1 gpurun_out/pmcdec/$n.log | cut -c1-300; return $rc
}
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
run trace --kernel-trace --stats; rc=$?; fatal $rc && exit $rc
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES; rc=$?; fatal $rc && exit $rc
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE; rc=$?; fatal $rc && exit $rc
python3 tools/xmb_pmc_summary.py gpurun_out/pmcdec "dec_recon|loopfilter" $((256 * 8160)) > gpurun_out/pmcdec/summary.json; echo "[summary] rc=$?"
