#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS="ptest" PTEST="tests/test_gpu_batch.py tests/test_partitions.py tests/test_gpu_parity.py" bash tools/gpu_r4.sh || exit $?
for r in 1 2; do
  for e in 0 1; do
    ZW_EMIT_PAIRS=$e timeout -k 10 300 python -u bench.py --steps 10 --no-extras --no-cpu-baseline > gpurun_out/emit_${e}_$r.log 2>&1 || exit $?
    grep '^{' gpurun_out/emit_${e}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pairs=$e', round(d['value'],1), d['verified'], 'emit ms/batch', round(d['host_ms_per_step']['emit'],1), 'per core', round(d['host_emit_frames_per_s_per_core'],1))"
  done
done
