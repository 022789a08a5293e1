# zero-copy kernel with tiles numbered across ranges: parity, then configs[3] mixed + configs[2]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tiles_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_tiles_tests.log; exit 1; }
tail -1 gpurun_out/r2_tiles_tests.log
rm -f gpurun_out/r2_tiles_pipe.jsonl
for i in 1 2; do
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --size mixed --batch 16 --frames 768 --policy pull --producer copy --out gpurun_out/r2_tiles_pipe.jsonl > gpurun_out/r2_tiles_pipe.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_tiles_pipe.log; exit 1; }
done
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer copy --out gpurun_out/r2_tiles_pipe.jsonl > gpurun_out/r2_tiles_pipe.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_tiles_pipe.log; exit 1; }
timeout -k 10 120 python -u tools/e2e_probe.py > gpurun_out/r2_tiles_e2e.jsonl 2> gpurun_out/r2_tiles_e2e.err || { echo E2E_FAILED; tail -20 gpurun_out/r2_tiles_e2e.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r2_tiles_pipe.jsonl'):
    d = json.loads(l); print(d['size'], d['fps'], d['GBps_each_way'], d['n_errors'])
for l in open('gpurun_out/r2_tiles_e2e.jsonl'):
    d = json.loads(l); print(d['size'], d['pinned_GBps_each_way'], d['pinned_pipelined_GBps_each_way'])
"
