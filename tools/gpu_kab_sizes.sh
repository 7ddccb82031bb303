# one-lane encode-kernel times of library variants at 1080p, 4K and 768x512 (alternating)
mkdir -p gpurun_out
for r in 1 2; do for sz in "1920 1080" "3840 2160" "768 512"; do for lib in "$@"; do
  ZWEBP_LIB=$PWD/image-webp_amd/zwebp/$lib timeout -k 10 200 python -u tools/kab.py 2 $sz >> gpurun_out/kabsz.log 2>&1 || exit 1
  tail -n 1 gpurun_out/kabsz.log
done; done; done
