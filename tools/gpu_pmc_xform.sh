#!/bin/bash
# HBM traffic of k_fdct_quant: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
# (they do not fit one TCC pass), kernel-trace only.  Summary -> gpurun_out/pmc_xform/summary.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_xform
F=${1:-256}
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_xform/p$i -o run -- python3 tools/xform_bench.py $F > gpurun_out/pmc_xform/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; tail -1 gpurun_out/pmc_xform/p$i.log; [ $rc -ne 0 ] && tail -5 gpurun_out/pmc_xform/p$i.log && exit $rc
done
python3 tools/pmc_traffic.py gpurun_out/pmc_xform k_fdct_quant $F > gpurun_out/pmc_xform/summary.json && cat gpurun_out/pmc_xform/summary.json
