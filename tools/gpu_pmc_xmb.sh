#!/bin/bash
# k_xform_mb (+ k_xform_mb_i4): kernel trace + PMC passes (one counter group
# per run) over tools/xmb_bench.py (RGBA-fused and Y/U/V forms, 256 1080p frames).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
run() {  # name, rocprofv3 args...
  local n=$1; shift
  timeout -k 10 150 rocprofv3 "$@" --output-format csv -d gpurun_out/pmc/$n -o $n -- python3 tools/xmb_bench.py --reps 3 > gpurun_out/pmc/$n.log 2>&1
  local rc=$?; echo "[$n] rc=$rc"; tail -1 gpurun_out/pmc/$n.log | cut -c1-300; return $rc
}
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
run trace --kernel-trace --stats; rc=$?; fatal $rc && exit $rc
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES; rc=$?; fatal $rc && exit $rc
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE; rc=$?; fatal $rc && exit $rc
run sq3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC; rc=$?; fatal $rc && exit $rc
run fetch --pmc FETCH_SIZE; rc=$?; fatal $rc && exit $rc
run write --pmc WRITE_SIZE; rc=$?; fatal $rc && exit $rc
python3 tools/xmb_pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json; echo "[summary] rc=$?"
