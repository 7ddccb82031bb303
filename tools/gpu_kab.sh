#!/bin/bash
# Alternating one-lane encode-kernel timing of library variants:
#   tools/gpu_kab.sh reps libA.so libB.so [libC.so ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
reps=$1; shift
for r in $(seq 1 $reps); do
  for lib in "$@"; do
    ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 200 python -u tools/kab.py 3 >> gpurun_out/kab.log 2>&1; rc=$?
    tail -n 1 gpurun_out/kab.log
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
