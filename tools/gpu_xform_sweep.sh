#!/bin/bash
# sweep k_fdct_quant variants/grids: tools/gpu_xform_sweep.sh "v:g v:g ..."
mkdir -p gpurun_out
list=${1:-"0:16 2:100000 3:100000 4:256"}
for vg in $list; do
  v=${vg%%:*}; g=${vg##*:}
  ZW_XFORM_VARIANT=$v ZW_XFORM_GRID=$g timeout -k 10 120 python tools/xform_bench.py 256 2>/dev/null | tail -1 || exit $?
done | tee gpurun_out/xform_sweep.log
