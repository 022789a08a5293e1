# bench N=1 (with the slot-ring e2e beside zero-copy), then an N=2 one-card rehearsal
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench7.json 2> gpurun_out/r2_bench7.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench7.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_bench7.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['end_to_end'], {k: v for k, v in d['jpeg_mode'].items() if 'fps' in k})"
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 100 --warmup 10 --no-sweep > gpurun_out/r2_bench_n2b.json 2> gpurun_out/r2_bench_n2b.log || { echo N2_FAILED; tail -30 gpurun_out/r2_bench_n2b.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_bench_n2b.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'], list(d['distributor'].keys()))"
