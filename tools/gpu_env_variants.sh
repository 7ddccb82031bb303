#!/bin/bash
# Short verified bench under several environment settings.
# usage: tools/gpu_env_variants.sh "NAME:VAR=1 VAR2=2" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for spec in "$@"; do
  n=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/env_$n.log 2>&1; rc=$?
  echo "== $n ($vars) rc=$rc"; grep '^{' gpurun_out/env_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), d['verified'], round(d['ms_per_step'],1), {k: round(v,2) for k,v in d['kernel_ms_per_step'].items()})"
  fatal $rc && exit $rc
done
exit 0
