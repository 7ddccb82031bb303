#!/bin/bash
# One-lane rocprofv3 kernel stats of a short bench for each library variant:
#   tools/gpu_kprof.sh libA.so libB.so ...  -> gpurun_out/kp_<lib>/k_kernel_stats.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib ZW_PIPE_LANES=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$n -o k -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/kp_$n.log 2>&1
  rc=$?; echo "== $n rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
  python3 tools/prof_summary.py gpurun_out/kp_$n/k_kernel_stats.csv | head -14
done
exit 0
