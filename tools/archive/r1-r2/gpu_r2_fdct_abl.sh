# k_fdct time split: the shipped kernel vs timing-only ablations (tools/build_fdct_ablations.sh)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/abl_*.jsonl
for rep in 1 2; do
for v in base nopix noac; do
  if [ $v = base ]; then unset VFILTER_LIB; else export VFILTER_LIB=$PWD/tools/libv_abl_$v.so; fi
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/abl_$v.jsonl > gpurun_out/abl_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/abl_$v.log; exit 1; }
done
done
unset VFILTER_LIB
python3 -c "
import json
for v in ('base','nopix','noac'):
    for l in open('gpurun_out/abl_%s.jsonl'%v):
        d=json.loads(l); print(v, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d['stages_ms']['fdct_huffman'])"
