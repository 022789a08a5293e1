#!/bin/bash
# JPEG hard 1080p through distributor + worker: the tree against tools/exp/libvf_notg.so (6 tables, G = 4), 3 reps.
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_hardsys.jsonl; rm -f $P
for rep in 1 2 3; do
for lib in distributed-video-filter_amd/vfilter/libvfilter_hip.so tools/exp/libvf_notg.so; do
  VFILTER_LIB=$PWD/$lib timeout -k 10 200 python tools/pipeline_bench.py --workers 1 --jpeg --content hard --size 1080p --batch 32 --policy pull --frames 3072 --out $P > /dev/null 2>> gpurun_out/r5_hardsys.err || { echo FAILED; tail -20 gpurun_out/r5_hardsys.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$P')][-1]; print('$lib'.split('/')[-1], d['fps'], d['n_errors'])"
done
done
