cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh smoke 240 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh rows_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "encode" || exit $?
tools/gpu_step.sh small_batch 300 python tools/small_batch.py 1920 1080 1,2,4,8,16,32
