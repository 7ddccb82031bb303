#!/bin/bash
# Round-4 evidence refresh at HEAD: encode VALU-issue PMC, k_xform_mb trace +
# PMC, k_fdct_quant HBM traffic, and a rocprofv3 kernel trace of the bench.
# Stops at the first time-limit / fault exit.  STEPS selects.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for st in ${STEPS:-enc xmb xform prof}; do
  case $st in
    enc) bash tools/gpu_pmc_encode.sh 256 > gpurun_out/pmc_enc.log 2>&1; rc=$?; echo "[enc] rc=$rc"; tail -3 gpurun_out/pmc_enc.log;;
    xmb) bash tools/gpu_pmc_xmb.sh > gpurun_out/pmc_xmb.log 2>&1; rc=$?; echo "[xmb] rc=$rc"; tail -3 gpurun_out/pmc_xmb.log | cut -c1-200;;
    xform)
      mkdir -p gpurun_out/pmc_xf; rc=0
      i=0
      for c in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_xf/p$i -o run -- python3 tools/xform_bench.py 256 > gpurun_out/pmc_xf/p$i.log 2>&1
        rc=$?; echo "[xform $c] rc=$rc"; [ $rc -ne 0 ] && break
      done
      [ $rc -eq 0 ] && python3 tools/pmc_traffic.py gpurun_out/pmc_xf k_fdct_quant_t 256 > gpurun_out/pmc_xf/traffic.json && cat gpurun_out/pmc_xf/traffic.json;;
    prof) mkdir -p gpurun_out/benchprof && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o bench -- python3 -u bench.py > gpurun_out/benchprof/bench.log 2>&1; rc=$?; echo "[prof] rc=$rc"; tail -1 gpurun_out/benchprof/bench.log | cut -c1-200;;
  esac
  fatal $rc && exit $rc
done
exit 0
