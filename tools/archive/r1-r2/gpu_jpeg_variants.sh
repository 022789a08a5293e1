# JPEG-mode bench of every tools/variants/libv_*.so (interleaved, 2 rounds); prints per-stage ms
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/var_*.jsonl
for rep in 1 2; do
for lib in tools/variants/libv_*.so; do
  v=$(basename $lib .so); v=${v#libv_}
  VFILTER_LIB=$PWD/$lib timeout -k 10 120 python -u tools/jpeg_bench.py --sizes ${VAR_SIZES:-1080p} --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/var_$v.jsonl > gpurun_out/var_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/var_$v.log; exit 1; }
done
done
python3 -c "
import json, glob
for f in sorted(glob.glob('gpurun_out/var_*.jsonl')):
    for l in open(f):
        d=json.loads(l); s=d['stages_ms']; print(f[15:-6], d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], s)"
