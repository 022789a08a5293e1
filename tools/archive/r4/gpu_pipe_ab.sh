# Round-4 A/B of the JPEG-through-distributor leg: the round-3 producer
# (tools/_pb_r3.py, per-frame node-pool submit) against the inline copy of small frames, and
# --numa-local 0, alternating, plus the 4K configs[2] leg to check the large-frame path.
# (tools/_pb_r3.py = `git show 178ea10:tools/pipeline_bench.py`, written before the call, not kept in the tree)
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/pipe_ab.jsonl
rm -f $OUT
for rep in 1 2 3; do
  for v in r3 new; do
    for nl in 1 0; do
      T=tools/pipeline_bench.py; [ $v = r3 ] && T=tools/_pb_r3.py
      echo "== $v numa_local=$nl rep $rep"
      timeout -k 10 150 python -u $T --jpeg --size 1080p --batch 32 --policy pull --frames 16384 --numa-local $nl > gpurun_out/pipe_ab_one.json 2> gpurun_out/pipe_ab.err || { echo FAILED; tail -20 gpurun_out/pipe_ab.err; exit 1; }
      python -c "import json,sys; r=json.loads(open('gpurun_out/pipe_ab_one.json').read().splitlines()[-1]); r['ab']='$v'; r['numa_local']=$nl; print(json.dumps({k:r[k] for k in ('ab','numa_local','fps','latency_ms_mean','n_errors')})); open('$OUT','a').write(json.dumps(r)+'\n')"
    done
  done
done
for v in r3 new; do
  T=tools/pipeline_bench.py; [ $v = r3 ] && T=tools/_pb_r3.py
  timeout -k 10 150 python -u $T --size 4k --batch 16 --policy shard --producer copy --frames 256 > gpurun_out/pipe_ab_one.json 2> gpurun_out/pipe_ab.err || { echo FAILED; tail -20 gpurun_out/pipe_ab.err; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/pipe_ab_one.json').read().splitlines()[-1]); r['ab']='$v'; print(json.dumps({k:r[k] for k in ('ab','size','fps','n_errors')})); open('$OUT','a').write(json.dumps(r)+'\n')"
done
echo AB_OK
