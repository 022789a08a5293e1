# The JPEG system leg (one GPU worker) and the 8-worker control plane with VF_TCP_READER=thread
# and select, alternating, three reps.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for r in thread select; do
    VF_TCP_READER=$r timeout -k 10 150 python -u tools/pipeline_bench.py --jpeg --size 1080p --batch 32 --policy pull --frames 16384 > gpurun_out/rs_pipe.json 2> gpurun_out/rs_pipe.err || { echo PIPE_FAILED; tail -20 gpurun_out/rs_pipe.err; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/rs_pipe.json').read().splitlines()[-1]); print('rep $rep $r system jpeg', r['fps'], r['latency_ms_mean'], r['n_errors'])"
    VF_TCP_READER=$r timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers 8 --policy pull --bytes 181876 --batch 32 --frames 64000 --group 16 --out gpurun_out/rs_cp.jsonl > /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/rs_cp.jsonl').read().splitlines()[-1]); print('rep $rep $r cp8 jpeg', d['fps'], d['distributor_cpu_us_per_frame'])"
  done
done
