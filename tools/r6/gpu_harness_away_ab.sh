# (needs the --harness-away option, built for this A/B and reverted) tools/pipeline_bench.py placing its own threads on the CPUs of NUMA nodes that hold no worker GPU
# (--harness-away 1, the default) vs leaving them to the scheduler (0): the small JPEG legs and 1080p,
# 4 reps interleaved, and the raw configs[2] leg once each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3 4; do
for sz in 512sq 480p 1080p; do
for a in 0 1; do
  b=64; n=98304
  [ $sz = 1080p ] && { b=32; n=24576; }
  timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch $b --policy pull \
      --frames $n --harness-away $a > gpurun_out/r6_ha_${sz}_${a}_$rep.json 2> gpurun_out/r6_ha_${sz}_${a}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_ha_${sz}_${a}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('gpurun_out/r6_ha_${sz}_${a}_$rep.json') if x.startswith('{')][-1]); print('$sz away $a rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'p99', d['latency_ms_p99'], 'errors', d['n_errors'], '|', d.get('harness_cpus'))"
done
done
done
for a in 0 1; do
  timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --size 4k --batch 16 --policy shard --producer copy \
      --frames 768 --harness-away $a > gpurun_out/r6_ha_c2_${a}.json 2> gpurun_out/r6_ha_c2_${a}.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_ha_c2_${a}.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('gpurun_out/r6_ha_c2_${a}.json') if x.startswith('{')][-1]); print('configs2 away $a', d['fps'], 'errors', d['n_errors'], '|', d.get('harness_cpus'))"
done
