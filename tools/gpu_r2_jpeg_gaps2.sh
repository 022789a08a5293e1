# JPEG worker form: device timeline + HIP API timeline + the library's own phase trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_jh
VF_JPEG_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/prof_jh -o jh -- python3 tools/jpeg_modes.py 1080p async > gpurun_out/jh.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/jh.log; exit 1; }
grep -v "^W20\|rocprofv3" gpurun_out/jh.log | tail -12
ls gpurun_out/prof_jh
# the two codec streams share one hardware queue (Queue_Id 4 for both in the kernel trace):
# worker-form rate with more hardware queues and / or without the compute gate
rm -f gpurun_out/r2_jpeg_hwq.jsonl
for q in 4 8; do
  for g in 1 0; do
    echo "{\"GPU_MAX_HW_QUEUES\": $q, \"VF_JPEG_GATE\": $g}" >> gpurun_out/r2_jpeg_hwq.jsonl
    GPU_MAX_HW_QUEUES=$q VF_JPEG_GATE=$g timeout -k 10 100 python -u tools/jpeg_modes.py 1080p async >> gpurun_out/r2_jpeg_hwq.jsonl 2>> gpurun_out/r2_jpeg_hwq.err || { echo HWQ_FAILED; tail -20 gpurun_out/r2_jpeg_hwq.err; exit 1; }
  done
done
cat gpurun_out/r2_jpeg_hwq.jsonl
