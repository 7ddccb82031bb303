#!/bin/bash
# A/B of library variants: parity tests on each variant library, then a short
# bench of each.  usage: tools/gpu_ab.sh libA.so libB.so ...  (paths under image-webp_amd/zwebp)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for lib in "$@"; do
  n=$(basename $lib .so)
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib tools/gpu_step.sh test_$n 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -q -x --timeout 300 --timeout-method thread; rc=$?
  [ $rc -ne 0 ] && exit $rc
done
for lib in "$@"; do
  n=$(basename $lib .so)
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib tools/gpu_step.sh bench_$n 300 python bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-extras; rc=$?
  fatal $rc && exit $rc
done
exit 0
