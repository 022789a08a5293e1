# where the JPEG system path spends its host time: sampled distributor and worker threads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/sampler_*
VF_JPEG_TRACE=1 timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size 480p --batch 32 --frames 16384 --policy pull --profile gpurun_out/sampler_480 > gpurun_out/r2_pipe_prof.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_prof.log; exit 1; }
tail -1 gpurun_out/r2_pipe_prof.log | cut -c1-300
ls gpurun_out/ | grep sampler
head -30 gpurun_out/sampler_480.distributor
for f in gpurun_out/sampler_480.[0-9]*; do echo "== $f"; head -30 $f; done
for f in gpurun_out/sampler_480.*.stderr; do echo "== $f"; grep "submit codec" $f | tail -12; grep "wait codec" $f | tail -5; done
