# Is the small legs' run-to-run swing CPU co-scheduling?  The 512x512 system leg 4 times with the harness
# process (distributor, producer, checks) left to the scheduler vs pinned to the CPUs of a NUMA node other
# than the GPU's (the worker pins itself to the GPU's node either way, so the two never share a core),
# interleaved.  Prints the topology first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd distributed-video-filter_amd && OTHER=$(python3 -c "
from vfilter.numa import gpu_numa_node, node_cpus, node_count
g = gpu_numa_node(0); n = node_count()
print('gpu node', g, 'nodes', n, 'gpu node cpus', len(node_cpus(g)), file=__import__('sys').stderr)
o = [c for k in range(n) if k != g for c in node_cpus(k)]
print(','.join(map(str, o)))") && cd .. || exit 1
[ -n "$OTHER" ] || { echo NO_OTHER_NODE; exit 1; }
for rep in 1 2 3 4; do
for mode in free other; do
  if [ $mode = other ]; then PRE="taskset -c $OTHER"; else PRE=""; fi
  timeout -k 10 150 $PRE python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size 512sq --batch 64 --policy pull \
      --frames 98304 > gpurun_out/r6_hc_${mode}_$rep.json 2> gpurun_out/r6_hc_${mode}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_hc_${mode}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('gpurun_out/r6_hc_${mode}_$rep.json') if x.startswith('{')][-1]); print('512sq harness $mode rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'p99', d['latency_ms_p99'], 'errors', d['n_errors'])"
done
done
