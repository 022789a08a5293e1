# Speculative vs span sync (G = 1, 2, 4) on 480p / 1080p / 4K scenes, resident stages, 2 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for m in "spec 0" "pass 1" "pass 2" "pass 4"; do
  set -- $m
  VF_JPEG_SYNC=$1 VF_JPEG_SYNC_G=$2 timeout -k 10 200 python3 tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 10 --cpu-seconds 0 --resident-only > gpurun_out/sm.jsonl 2> gpurun_out/sm.log || { echo RUN_FAILED; tail -20 gpurun_out/sm.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/sm.jsonl'):
    d = json.loads(l); s = d['stages_ms']
    print('rep $rep $1 G$2', d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], 'sync', s['huffman_sync'], 'write', s['huffman_write'])"
done
done
