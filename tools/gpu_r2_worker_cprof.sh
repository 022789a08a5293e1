# the JPEG worker's main thread under cProfile, 480p through the distributor
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/wprof*
VF_CPROFILE=1 timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size 480p --batch 32 --frames 32768 --policy pull --profile gpurun_out/wprof > gpurun_out/wprof.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/wprof.log; exit 1; }
grep -o '"fps": [0-9.]*' gpurun_out/wprof.log
head -60 gpurun_out/wprof.*.cprofile
