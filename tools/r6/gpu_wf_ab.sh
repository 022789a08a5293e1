#!/bin/bash
# JPEG worker form at 512 x 512 and 480p (batches of 64): the last commit's library
# (tools/libv_head.so) against the working tree, interleaved, 4 reps each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3 4; do
for v in head tree; do
  L=distributed-video-filter_amd/vfilter/libvfilter_hip.so; [ $v = head ] && L=tools/libv_head.so
  for sz in 512sq 480p; do
    r=$(VFILTER_LIB=$L timeout -k 10 120 python3 tools/r6/worker_form_phases.py $sz 64) || { echo FAILED; exit 1; }
    echo "$v rep $rep $r"
  done
done
done
