# 4K JPEG: resident rate and stage times by batch size (the coefficient buffer is 32 MB per frame)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/b4k.jsonl
for b in 4 8 16 32; do
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 4k --batch $b --iters 20 --cpu-seconds 0 --out gpurun_out/b4k.jsonl > gpurun_out/b4k.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/b4k.log; exit 1; }
done
for m in "4k async3 8" "4k async3 16" "4k async4 16" "4k async3 32"; do
  timeout -k 10 120 python -u tools/jpeg_modes.py $m >> gpurun_out/b4k_modes.jsonl 2>> gpurun_out/b4k.log || { echo MODES_FAILED; tail -20 gpurun_out/b4k.log; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/b4k.jsonl'):
    d=json.loads(l); print(d['batch'], d['gpu_resident_fps'], d['stages_ms'])
for l in open('gpurun_out/b4k_modes.jsonl'): print(l.strip())"
