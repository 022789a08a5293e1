# HBM ceilings by direction (read-only, write-only, copy) for the roofline discussion
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/hbm_ceiling 199065600 12 5 > gpurun_out/r2_hbm_ceiling.jsonl 2> gpurun_out/r2_hbm_ceiling.err || { echo FAILED; tail gpurun_out/r2_hbm_ceiling.err; exit 1; }
cat gpurun_out/r2_hbm_ceiling.jsonl
