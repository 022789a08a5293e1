# Huffman write stage: shipped vs no coefficient stores (timing only), 1080p and 4K
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/wabl_*.jsonl
for rep in 1 2; do
for v in base nocoef; do
  if [ $v = base ]; then unset VFILTER_LIB; else export VFILTER_LIB=$PWD/tools/libv_abl_$v.so; fi
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 1080p,4k --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/wabl_$v.jsonl > gpurun_out/wabl_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/wabl_$v.log; exit 1; }
done
done
unset VFILTER_LIB
python3 -c "
import json
for v in ('base','nocoef'):
    for l in open('gpurun_out/wabl_%s.jsonl'%v):
        d=json.loads(l); print(v, d['size'], d['gpu_resident_fps'], d['stages_ms']['huffman_write'], d['stages_ms']['dc_idct'])"
