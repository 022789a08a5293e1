# JPEG GPU parity + plumbing + 480p / 1080p / 4K JPEG-mode bench (no CPU reference)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
rm -f gpurun_out/jpeg_q.jsonl
timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/jpeg_q.jsonl > gpurun_out/jpeg_q.log 2>&1 || { echo JPEG_BENCH_FAILED; tail -30 gpurun_out/jpeg_q.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/jpeg_q.jsonl'):
    d=json.loads(l); print(d['size'], d['gpu_resident_fps'], d['host_to_host_fps'], d['host_to_host_2threads_fps'], d['parity_vs_oracle'], d.get('stages_ms'))"
