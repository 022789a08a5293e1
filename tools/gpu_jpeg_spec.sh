# speculative sync: JPEG parity (default = speculative, then the pass-based path forced),
# fallback statistics, bench + kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
VF_JPEG_SYNC=pass timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg_pass.log 2>&1 || { echo PYTEST_PASS_FAILED; tail -40 gpurun_out/pytest_jpeg_pass.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg_pass.log
for sz in 480p 1080p 4k; do
VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python -u tools/jpeg_host_trace.py $sz > gpurun_out/syncstats_$sz.log 2>&1 || { echo FAILED; tail -20 gpurun_out/syncstats_$sz.log; exit 1; }
echo $sz; grep "sync:" gpurun_out/syncstats_$sz.log | tail -1
done
rm -f gpurun_out/jpeg_q.jsonl
timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/jpeg_q.jsonl > gpurun_out/jpeg_q.log 2>&1 || { echo JPEG_BENCH_FAILED; tail -30 gpurun_out/jpeg_q.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/jpeg_q.jsonl'):
    d=json.loads(l); print(d['size'], d['gpu_resident_fps'], d['host_to_host_fps'], d['host_to_host_2threads_fps'], d['parity_vs_oracle'], d['stages_ms'])"
