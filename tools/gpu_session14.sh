#!/bin/bash
# smoke + GPU tests + full bench, then the headline with 8 vs 16 HW queues (A/B)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS="smoke pytest bench" bash tools/gpu_r4.sh || exit $?
for r in 1 2; do
  for q in 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 10 --no-extras --no-cpu-baseline > gpurun_out/hwq_${q}_$r.log 2>&1 || exit $?
    grep '^{' gpurun_out/hwq_${q}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hwq $q', round(d['value'],1), d['verified'])"
  done
done
