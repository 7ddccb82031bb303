#!/bin/bash
# Short verified bench of each library variant (no extras, no CPU baseline).
# usage: tools/gpu_variants.sh libA.so libB.so ...  (under image-webp_amd/zwebp)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for lib in "$@"; do
  n=$(basename $lib .so)
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/var_$n.log 2>&1; rc=$?
  echo "== $n rc=$rc"; grep '^{' gpurun_out/var_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), d['verified'], {k: round(v,2) for k,v in d['kernel_ms_per_step'].items()})"
  fatal $rc && exit $rc
done
exit 0
