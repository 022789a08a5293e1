# Round 3: the GPU suite (with the configs[4] 4096-frame parity test and the run_now race
# test), smoke, the gfx950 counter list, then one per-dispatch PMC pass over the 1080p JPEG
# batch with the kernel trace beside it (durations per dispatch for the issue fractions).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
grep -E "batch4096|async_in_flight" gpurun_out/r3_pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3_counters.txt 2>&1 || echo LIST_FAILED
grep -cE "SQ_|GRBM_" gpurun_out/r3_counters.txt
rm -rf gpurun_out/pmc_a
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_a -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 3 --cpu-seconds 0 > gpurun_out/pmc_a.log 2>&1 || { echo PMC_A_FAILED; tail -20 gpurun_out/pmc_a.log; exit 1; }
ls gpurun_out/pmc_a/*/ 2>/dev/null | head
