#!/bin/bash
# k_fdct_quant: parity of the LDS-coalesced variants, then a variant sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 6 7 8; do
  ZW_XFORM_VARIANT=$v tools/gpu_step.sh xform_par_$v 200 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "fdct or transform_quant or xform" || exit $?
done
bash tools/gpu_xform_sweep.sh "${SWEEP:-5:1048576 6:1048576 7:1048576 8:1048576 99:1048576 98:1048576 5:1048576 6:1048576}"
