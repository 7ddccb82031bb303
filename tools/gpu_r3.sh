#!/bin/bash
# Round-3 GPU session: smoke -> GPU parity tests -> k_xform_mb leg (+ no-I4,
# PMC passes) -> bench -> kernel trace of the bench (prof).  Stops at the
# first time-limit / fault exit (no GPU
# step after one).  STEPS overrides the list (e.g. STEPS="xmb bench").
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for st in ${STEPS:-smoke pytest xmb pmc bench}; do
  case $st in
    smoke) tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()";;
    pytest) tools/gpu_step.sh pytest_gpu 600 python -u -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} --timeout 300 --timeout-method thread;;
    xmbtest) tools/gpu_step.sh xmbtest 300 python -u -m pytest tests/test_xmb.py -m gpu -q -x --timeout 120 --timeout-method thread;;
    xmb) tools/gpu_step.sh xmb 240 python -u tools/xmb_bench.py && tools/gpu_step.sh xmb_noi4 240 python -u tools/xmb_bench.py --no-i4;;
    pmc) bash tools/gpu_pmc_xmb.sh > gpurun_out/pmc.log 2>&1; r=$?; echo "[pmc] rc=$r"; tail -20 gpurun_out/pmc.log; (exit $r);;
    bench) tools/gpu_step.sh bench 600 python -u bench.py ${BENCH_ARGS};;
    prof) mkdir -p gpurun_out/benchprof && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o bench -- python3 -u bench.py ${BENCH_ARGS} > gpurun_out/benchprof/bench.log 2>&1; r=$?; echo "[prof] rc=$r"; tail -2 gpurun_out/benchprof/bench.log | cut -c1-400; (exit $r);;
  esac
  rc=$?
  fatal $rc && exit $rc
done
exit 0
