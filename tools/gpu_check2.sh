#!/bin/bash
# smoke -> all GPU tests -> bench -> small-batch sweep (one time limit per step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh bench 500 python bench.py ${BENCH_ARGS} || exit $?
tools/gpu_step.sh small_batch 300 python tools/small_batch.py 1920 1080 ${SB_SIZES:-24,48,64}
