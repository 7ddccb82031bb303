#!/bin/bash
# k_dec_tokl (lane-parallel token parse, 64 1080p frames = one wave): SQ counter
# passes, summed per kernel by tools/pmc_summary.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmctok
export ZW_DEC_TOKENS=device
run() {  # name, rocprofv3 args...
  local n=$1; shift
  timeout -k 10 150 rocprofv3 "$@" --output-format csv -d gpurun_out/pmctok/$n -o $n -- python3 tools/dec_tokens.py 64 1 device > gpurun_out/pmctok/$n.log 2>&1
  local rc=$?; echo "[$n] rc=$rc"; return $rc
}
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH; rc=$?; fatal $rc && exit $rc
run p2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE; rc=$?; fatal $rc && exit $rc
run p3 --pmc SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VALU; rc=$?; fatal $rc && exit $rc
python3 tools/pmc_summary.py gpurun_out/pmctok | grep -A40 k_dec_tokl
