#!/bin/bash
# VALU-issue PMC of the encode kernels: two rocprofv3 --pmc passes (kernel-trace
# only, each its own run, within the SQ / GRBM slot limits), then
# tools/encode_pmc_summary.py -> gpurun_out/pmc_enc/summary.json.  One lane of F
# frames: with F = 512 (the default) its two 256-frame chunks take each pass in
# one frame-pair launch (k_encode_pass1_fp / k_encode_pass2_fp), as the headline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_enc
F=${1:-512}
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  ZW_PIPE_LANES=1 timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_enc/p$i -o run -- python3 tools/enc_once.py $F > gpurun_out/pmc_enc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/pmc_enc/p$i.log && exit $rc
done
python3 tools/encode_pmc_summary.py gpurun_out/pmc_enc $F > gpurun_out/pmc_enc/summary.json && cat gpurun_out/pmc_enc/summary.json
