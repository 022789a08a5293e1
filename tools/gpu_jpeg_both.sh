# JPEG: tests (spec default + pass-forced), then 480p/1080p/4K resident rates for both sync paths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
VF_JPEG_SYNC=pass timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg_pass.log 2>&1 || { echo PYTEST_PASS_FAILED; tail -40 gpurun_out/pytest_jpeg_pass.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg_pass.log
for mode in auto spec pass; do
rm -f gpurun_out/jb_$mode.jsonl
VF_JPEG_SYNC=$mode timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/jb_$mode.jsonl > gpurun_out/jb_$mode.log 2>&1 || { echo JB_FAILED; tail gpurun_out/jb_$mode.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/jb_$mode.jsonl'):
    d=json.loads(l); st=d['stages_ms']; print('$mode', d['size'], d['gpu_resident_fps'], d['host_to_host_2threads_fps'], d['parity_vs_oracle'], 'sync', st['huffman_sync'], 'write', st['huffman_write'])"
done
