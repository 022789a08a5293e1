# Round-4 wait analysis of the JPEG kernels: rocprofv3 kernel stats, then two per-dispatch PMC
# passes (issue / wait cycles) over tools/jpeg_bench.py --resident-only at 1080p x 32 on the
# given content; tools/pmc_waits.py prints per kernel (summed over the last batch) the wave
# cycles, the fraction of them waiting on anything / on issue, and VALU / LDS active cycles.
#   bash tools/r4/gpu_jpeg_pmc_waits.sh [hard|scene] [size]
set -o pipefail
CONTENT=${1:-hard}; SIZE=${2:-1080p}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 tools/jpeg_bench.py --sizes $SIZE --batch 32 --iters 3 --cpu-seconds 0 --resident-only --content $CONTENT"
rm -rf gpurun_out/pmcw_stats gpurun_out/pmcw_a gpurun_out/pmcw_b
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcw_stats -o ks -- $B --out gpurun_out/pmcw_stats.jsonl > gpurun_out/pmcw_stats.log 2>&1 || { echo STATS_FAILED; tail -20 gpurun_out/pmcw_stats.log; exit 1; }
cat gpurun_out/pmcw_stats.jsonl
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcw_a -o pmc -- $B > gpurun_out/pmcw_a.log 2>&1 || { echo PMC_A_FAILED; tail -20 gpurun_out/pmcw_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcw_b -o pmc -- $B > gpurun_out/pmcw_b.log 2>&1 || { echo PMC_B_FAILED; tail -20 gpurun_out/pmcw_b.log; exit 1; }
python3 tools/pmc_waits.py gpurun_out/pmcw_a gpurun_out/pmcw_b gpurun_out/pmcw_stats
