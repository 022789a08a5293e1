# JPEG 1080p through distributor + worker with the plumbing sampler on both sides (where the
# system rate goes, against the worker form's), plus the same run unprofiled.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --jpeg --size 1080p --batch 32 --frames 2048 --policy pull > gpurun_out/pp_plain.jsonl 2> gpurun_out/pp_plain.log || { echo PIPE_FAILED; tail -20 gpurun_out/pp_plain.log; exit 1; }
cut -c1-400 gpurun_out/pp_plain.jsonl
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --jpeg --size 1080p --batch 32 --frames 2048 --policy pull --profile gpurun_out/pp > gpurun_out/pp_prof.jsonl 2> gpurun_out/pp_prof.log || { echo PIPE_PROF_FAILED; tail -20 gpurun_out/pp_prof.log; exit 1; }
cut -c1-300 gpurun_out/pp_prof.jsonl
ls gpurun_out/pp*
