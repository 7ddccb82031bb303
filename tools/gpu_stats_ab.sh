cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sab
for lib in libzwebp.so libzwebp_s64c4.so libzwebp_s128c2.so libzwebp_s256c4.so libzwebp_h256.so libzwebp_h1024.so; do
  n=${lib%.so}
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sab/$n -o k -- python3 tools/kab.py 3 > gpurun_out/sab/$n.log 2>&1 || exit 1
  python3 - "$n" << 'PY'
import csv, sys
n = sys.argv[1]
rows = {r['Name']: r for r in csv.DictReader(open(f'gpurun_out/sab/{n}/k_kernel_stats.csv'))}
d = tail = open(f'gpurun_out/sab/{n}.log').read().strip().splitlines()[-1]
print(n, {k: round(float(rows[k]['AverageNs'])/1e6, 3) for k in ('k_stats_hist', 'k_stats_final', 'k_stats_flags') if k in rows}, d[-60:])
PY
done
