cd "$GRAFT_REPO_ROOT"
for cfg in "" "ZW_DEC_CHUNK=256" "ZW_DEC_DL_PARTS=8" "ZW_DEC_CHUNK=64" "ZW_DEC_FAN_THREADS=8"; do
  echo "== cfg [$cfg]"
  env $cfg timeout -k 10 200 python -u tools/dec_tokens.py 1024 3 auto 4 2>&1 | tail -1 || exit 1
done
