#!/bin/bash
# Round-6 GPU session steps (each under its own time limit; stops at the first
# time-limit / fault exit).  STEPS selects, e.g. STEPS="smoke pytest bench".
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|137|134|139|135|132) return 0;; *) return 1;; esac; }
for st in ${STEPS:-smoke pytest bench}; do
  case $st in
    smoke) tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()";;
    pytest) tools/gpu_step.sh pytest_gpu 900 python -u -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} --timeout 300 --timeout-method thread;;
    ptest) tools/gpu_step.sh ptest 600 python -u -m pytest ${PTEST:-tests} -m gpu -q -x --timeout 200 --timeout-method thread;;
    dec) tools/gpu_step.sh dec 300 python -u tools/dec_bench.py 256 3 && tools/gpu_step.sh dec_rgba 300 python -u tools/dec_rgba_bench.py 256;;
    bench) tools/gpu_step.sh bench 900 python -u bench.py ${BENCH_ARGS};;
    prof) mkdir -p gpurun_out/benchprof && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o bench -- python3 -u bench.py ${BENCH_ARGS} > gpurun_out/benchprof/bench.log 2>&1; r=$?; echo "[prof] rc=$r"; tail -2 gpurun_out/benchprof/bench.log | cut -c1-400; (exit $r);;
    cmd) tools/gpu_step.sh cmd ${CMD_SECS:-300} bash -c "$CMD";;
  esac
  rc=$?
  fatal $rc && exit $rc
done
exit 0
