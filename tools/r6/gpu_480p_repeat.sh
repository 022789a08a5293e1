# The 480p / 512x512 JPEG system legs, 5 runs each, interleaved (the bench's distributor form).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3 4 5; do
for sz in 480p 512sq; do
  timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch 64 --policy pull \
      --frames 98304 > gpurun_out/r6_rep_${sz}_$rep.json 2> gpurun_out/r6_rep_${sz}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_rep_${sz}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6_rep_${sz}_$rep.json') if l.startswith('{')][-1]); print('$sz rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'])"
done
done
