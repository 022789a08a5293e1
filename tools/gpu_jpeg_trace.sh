set -o pipefail
mkdir -p gpurun_out
VF_JPEG_TRACE=1 timeout -k 10 120 python -u tools/jpeg_host_trace.py 4k 2threads > gpurun_out/jtrace.log 2>&1 || { echo TRACE_FAILED; tail -30 gpurun_out/jtrace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/jtrace.log
