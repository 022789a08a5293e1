# N=4 rehearsal of the bench on ONE card after the round-2 changes (4 ranks + 4 workers share GPU 0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 800 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 4 --steps 100 --warmup 10 --no-sweep > gpurun_out/r2_bench_n4c.json 2> gpurun_out/r2_bench_n4c.log || { echo N4_FAILED; tail -30 gpurun_out/r2_bench_n4c.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_bench_n4c.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'], {k: (v.get('fps'), v.get('error')) for k, v in d['distributor'].items() if isinstance(v, dict)})"
