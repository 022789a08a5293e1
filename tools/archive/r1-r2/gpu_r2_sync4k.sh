# Speculative vs pass-based Huffman sync at 4K (and 1080p) on the current build, interleaved
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/sync4k_*.jsonl
for rep in 1 2; do
for m in spec pass; do
  VF_JPEG_SYNC=$m timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 4k,1080p --batch 32 --iters 10 --cpu-seconds 0 --out gpurun_out/sync4k_$m.jsonl > gpurun_out/sync4k_$m.log 2>&1 || { echo BENCH_FAILED $m; tail -30 gpurun_out/sync4k_$m.log; exit 1; }
done
done
python3 -c "
import json
for m in ('spec','pass'):
    for l in open('gpurun_out/sync4k_%s.jsonl'%m):
        d=json.loads(l); print(m, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d['stages_ms']['huffman_sync'], d.get('huffman_sync_mode'))"
