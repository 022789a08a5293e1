# A/B of two library builds on the JPEG-mode bench (tools/libv_head.so = last commit, in-tree = working tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
rm -f gpurun_out/ab_*.jsonl
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes ${AB_SIZES:-480p,1080p,4k} --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/ab_$v.jsonl > gpurun_out/ab_$v.log 2>&1 || { echo JPEG_BENCH_FAILED $v; tail -30 gpurun_out/ab_$v.log; exit 1; }
done
done
python -c "
import json
for v in ('head','new'):
    for l in open('gpurun_out/ab_%s.jsonl'%v):
        d=json.loads(l); print(v, d['size'], d['gpu_resident_fps'], 'h2h', d.get('host_to_host_fps'), d.get('host_to_host_2threads_fps'), d['parity_vs_oracle'], d.get('stages_ms'))"
