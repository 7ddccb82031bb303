#!/bin/bash
# HBM traffic of the frame-pair encode kernels: FETCH_SIZE and WRITE_SIZE, one
# rocprofv3 --pmc pass each (kernel-trace only), over one lane of F frames
# (512: each pass one frame-pair launch, as the headline), then
# tools/pmc_enc_traffic.py -> gpurun_out/pmc_enc_t/summary.json.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_enc_t
F=${1:-512}
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  ZW_PIPE_LANES=1 timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_enc_t/p$i -o run -- python3 tools/enc_once.py $F > gpurun_out/pmc_enc_t/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/pmc_enc_t/p$i.log && exit $rc
done
python3 tools/pmc_enc_traffic.py gpurun_out/pmc_enc_t $F > gpurun_out/pmc_enc_t/summary.json && cat gpurun_out/pmc_enc_t/summary.json
