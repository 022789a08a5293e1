# A/B of the fused colour path (tools/fused_colour.patch applied: k_fdct reading the decoder's
# planes, VF_JPEG_FUSE=1) against the k_color pass (VF_JPEG_FUSE=0) and tools/libv_head.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
rm -f gpurun_out/fuse_*.jsonl
for rep in 1 2; do
for v in head fuse1 fuse0; do
  unset VFILTER_LIB VF_JPEG_FUSE
  case $v in head) export VFILTER_LIB=$PWD/tools/libv_head.so ;; fuse1) export VF_JPEG_FUSE=1 ;; fuse0) export VF_JPEG_FUSE=0 ;; esac
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes ${AB_SIZES:-480p,1080p,4k} --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/fuse_$v.jsonl > gpurun_out/fuse_$v.log 2>&1 || { echo JPEG_BENCH_FAILED $v; tail -30 gpurun_out/fuse_$v.log; exit 1; }
done
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/fuse_*.jsonl')):
    for l in open(f):
        d=json.loads(l); s=d.get('stages_ms',{}); print(f.split('_')[-1][:-6], d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], 'colour', s.get('color_invert'), 'fdct', s.get('fdct_huffman'))"
