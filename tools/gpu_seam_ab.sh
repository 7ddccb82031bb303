# seam batching knobs vs per-call encodes (tools/seam_threads.py, 1080p RGBA Q75 m4)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
run() { echo "== $1" >> gpurun_out/seam_ab.log; shift; env "$@" timeout -k 10 200 python -u tools/seam_threads.py 3 16 32 64 >> gpurun_out/seam_ab.log 2>&1 || exit 1; tail -1 gpurun_out/seam_ab.log; }
rm -f gpurun_out/seam_ab.log
run solo16 ZW_SEAM_SOLO=16
run solo8 ZW_SEAM_SOLO=8
run solo0 ZW_SEAM_SOLO=0
run solo24 ZW_SEAM_SOLO=24
