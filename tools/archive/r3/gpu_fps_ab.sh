# Round 3: resident JPEG frames/s without a profiler attached, libraries alternating
# ($LIBS "name=path ...", "new" = the working tree's; $REPS rounds; AB_SIZE, AB_CONTENT).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-4}); do
for nv in ${LIBS:-head=tools/libv_head.so new=}; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export VFILTER_LIB=$PWD/$lib; else unset VFILTER_LIB; fi
  rm -f gpurun_out/fps_$v.jsonl
  timeout -k 10 200 python3 tools/jpeg_bench.py --sizes ${AB_SIZE:-1080p} --batch 32 --iters ${ITERS:-100} --cpu-seconds 0 --content ${AB_CONTENT:-scene} --resident-only --out gpurun_out/fps_$v.jsonl > gpurun_out/fps_$v.log 2>&1 || { echo FPS_FAILED $v; tail -30 gpurun_out/fps_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/fps_$v.jsonl').readline()); print('rep', $rep, '$v', d['size'], d['gpu_resident_fps'], d['gpu_resident_ms_per_batch'], d['parity_vs_oracle'])"
done
done
unset VFILTER_LIB
