#!/bin/bash
# k_xform_mb variants: parity (tests/test_xmb.py under ZW_XMB_VARIANT=$PFV) and
# alternating timings of the default (0) and $PFV (default 1) forms.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PFV=${PFV:-1}
ZW_XMB_VARIANT=$PFV timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xmb.py \
  > gpurun_out/xpf_test.log 2>&1; rc=$?
tail -4 gpurun_out/xpf_test.log
[ $rc -eq 0 ] || exit $rc
for v in 0 $PFV 0 $PFV; do
  ZW_XMB_VARIANT=$v timeout -k 10 200 python tools/xmb_bench.py --reps 10 > gpurun_out/xpf_b$v.log 2>&1 || exit $?
  echo "variant $v"; grep '^{' gpurun_out/xpf_b$v.log
done
