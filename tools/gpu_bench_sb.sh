cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh bench 500 python bench.py || exit $?
tools/gpu_step.sh small_batch 300 python tools/small_batch.py 1920 1080 24,48,64
