#!/bin/bash
# Parity tests of the default library (TESTS, -k KSEL), then REPS rounds of
# short verified benches over the given libraries (alternating):
#   tools/gpu_abn.sh libA.so libB.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
tools/gpu_step.sh ab_tests 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_batch.py} -q -x --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} || exit $?
for r in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/ab_${n}_$r.log 2>&1; rc=$?
    echo "== $n rep $r rc=$rc"
    fatal $rc && exit $rc
  done
done
python3 tools/ab_summary.py gpurun_out/ab_*_[0-9].log
exit 0
