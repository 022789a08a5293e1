# JPEG kernel change: JPEG tests, stage times, kernel stats, worker form
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_jk_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_jk_tests.log; exit 1; }
tail -1 gpurun_out/r2_jk_tests.log
for size in 1080p 4k; do timeout -k 10 120 python -u tools/jpeg_bench.py --sizes $size --batch 32 --iters 20 --cpu-seconds 0 2>&1 | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['size'], d['gpu_resident_fps'], d['stages_ms'])
"; done
bash tools/gpu_jpeg_stats.sh 1080p | head -8
timeout -k 10 100 python -u tools/jpeg_modes.py 1080p async3
