for cfg in "ZW_ENC_FP=0" "ZW_PIPE_LANES=1" "ZW_ENC_FP=0 BFR=2048" "BFR=2048" "ZW_PIPE_LANES=1 BFR=2048"; do
  fr=1024; case "$cfg" in *BFR=2048*) fr=2048;; esac
  echo -n "[$cfg] "
  env $cfg timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --frames $fr --steps 10 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v,2) for k,v in d.get('kernel_ms_per_step', {}).items()})" || exit 1
done
