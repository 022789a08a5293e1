# Huffman table cache in the host parse: JPEG tests, worker form and system rates
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tc_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_tc_tests.log; exit 1; }
tail -1 gpurun_out/r2_tc_tests.log
rm -f gpurun_out/r2_tc.jsonl
for size in 480p 1080p; do
  VF_JPEG_TRACE=1 timeout -k 10 100 python -u tools/jpeg_modes.py $size async3 >> gpurun_out/r2_tc.jsonl 2> gpurun_out/r2_tc_trace_$size.err || { echo FAILED; tail -20 gpurun_out/r2_tc_trace_$size.err; exit 1; }
  grep "submit codec" gpurun_out/r2_tc_trace_$size.err | tail -3
done
cat gpurun_out/r2_tc.jsonl
rm -f gpurun_out/r2_tc_pipe.jsonl
for size in 480p 1080p; do
timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size $size --batch 32 --frames 16384 --policy pull --out gpurun_out/r2_tc_pipe.jsonl > gpurun_out/r2_tc_pipe.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_tc_pipe.log; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/r2_tc_pipe.jsonl'):
    d = json.loads(l); print(d['size'], d['fps'], d['n_errors'])
"
