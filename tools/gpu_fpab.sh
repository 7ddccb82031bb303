#!/bin/bash
# Pipeline shape A/B of the headline (bench.py --no-extras): CFGS entries are
# env settings, BFR=<frames> sets --frames.
for cfg in ${CFGS:-"ZW_ENC_FP=0" "X=1" "ZW_PIPE_LANES=1" "ZW_PIPE_LANES=3" "ZW_PIPE_LANES=4" "BFR=2048"}; do
  fr=1024; case "$cfg" in *BFR=*) fr=${cfg##*BFR=};; esac
  echo -n "[$cfg] "
  env $cfg timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --frames $fr --steps 10 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v,2) for k,v in d.get('kernel_ms_per_step', {}).items()}, {k: round(v,1) for k,v in d.get('host_ms_per_step', {}).items()})" || exit 1
done
