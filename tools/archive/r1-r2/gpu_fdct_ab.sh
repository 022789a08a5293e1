# A/B of k_fdct workgroup counts (VF_FDCT_WGS) against tools/libv_head.so on the JPEG-mode bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
rm -f gpurun_out/fab_*.jsonl
for rep in 1 2; do
for v in head ${FAB_WGS:-0 2048 4096 8192}; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; unset VF_FDCT_WGS; else unset VFILTER_LIB; export VF_FDCT_WGS=$v; fi
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes ${AB_SIZES:-480p,1080p,4k} --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/fab_$v.jsonl > gpurun_out/fab_$v.log 2>&1 || { echo JPEG_BENCH_FAILED $v; tail -30 gpurun_out/fab_$v.log; exit 1; }
done
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/fab_*.jsonl')):
    for l in open(f):
        d=json.loads(l); print(f.split('_')[-1][:-6], d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], 'fdct', d.get('stages_ms',{}).get('fdct_huffman'))"
