#!/bin/bash
# The JPEG codec's host preparation: DecFrames built in page-locked memory by the parse tasks
# (this tree) against the round's previous build (tools/exp/libvf_t4.so: built in a vector,
# then copied).  JPEG GPU tests, the host phase trace, and the 512² / 480p system legs, 2 reps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r5_prep_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r5_prep_pytest.log; exit 1; }
tail -1 gpurun_out/r5_prep_pytest.log
for lib in tools/exp/libvf_t4.so distributed-video-filter_amd/vfilter/libvfilter_hip.so; do
  VFILTER_LIB=$PWD/$lib VF_JPEG_TRACE=1 timeout -k 10 120 python3 tools/jpeg_host_trace.py 512sq > gpurun_out/htrace_ab.log 2>&1 || exit 1
  echo "$lib: $(grep submit gpurun_out/htrace_ab.log | tail -1 | sed 's/.*prep_dec/prep_dec/')  $(grep 'python wall' gpurun_out/htrace_ab.log | tail -1)"
done
P=gpurun_out/r5_prep_pipe.jsonl; rm -f $P
for rep in 1 2; do
for lib in tools/exp/libvf_t4.so distributed-video-filter_amd/vfilter/libvfilter_hip.so; do
for sz in 512sq 480p; do
  VFILTER_LIB=$PWD/$lib timeout -k 10 200 python tools/pipeline_bench.py --workers 1 --jpeg --size $sz --batch 32 --policy pull --frames 32768 --out $P > /dev/null 2>> gpurun_out/r5_prep_pipe.err || { echo FAILED; tail -20 gpurun_out/r5_prep_pipe.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$P')][-1]; print('$lib'.split('/')[-1], d['size'], d['fps'], d['n_errors'])"
done
done
done
