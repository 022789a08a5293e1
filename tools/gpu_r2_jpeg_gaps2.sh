# JPEG worker form: device timeline + HIP API timeline + the library's own phase trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_jh
VF_JPEG_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/prof_jh -o jh -- python3 tools/jpeg_modes.py 1080p async > gpurun_out/jh.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/jh.log; exit 1; }
grep -v "^W20\|rocprofv3" gpurun_out/jh.log | tail -12
ls gpurun_out/prof_jh
