# distributor-level pipeline runs (configs[2]/[3]) on the 1-GPU box, + host->host sweep
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/pipeline.jsonl gpurun_out/pipeline.log
run() { timeout -k 10 240 python -u tools/pipeline_bench.py --out gpurun_out/pipeline.jsonl "$@" >> gpurun_out/pipeline.log 2>&1 || { echo "PIPELINE_FAILED $*"; tail -30 gpurun_out/pipeline.log; exit 1; }; }
run --workers 1 --size 1080p --frames 2048 --batch 16 --inflight 1
run --workers 1 --size 1080p --frames 2048 --batch 16 --inflight 2
run --workers 1 --size 1080p --frames 2048 --batch 16 --inflight 3
run --workers 1 --size 4k --frames 512 --batch 16
run --workers 2 --size 4k --frames 512 --batch 16
run --workers 2 --size mixed --frames 1536 --batch 16 --policy pull
run --workers 1 --size 480p --frames 4096 --batch 32
run --workers 1 --size 1080p --frames 2048 --batch 16 --producer copy
cat gpurun_out/pipeline.jsonl
timeout -k 10 200 python -u tools/sweep.py --e2e-only --out gpurun_out/e2e_engine.jsonl > gpurun_out/e2e_engine.log 2>&1 && cat gpurun_out/e2e_engine.jsonl
