set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --no-traffic --cpu-seconds 0 --no-e2e > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -30 gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof_bench -name "*stats*" | head
timeout -k 10 120 ./tools/pcie_probe > gpurun_out/pcie.txt 2>&1 && cat gpurun_out/pcie.txt
HSA_ENABLE_SDMA=0 timeout -k 10 120 ./tools/pcie_probe > gpurun_out/pcie_nosdma.txt 2>&1 && cat gpurun_out/pcie_nosdma.txt
timeout -k 10 300 python -u tools/sweep.py --out gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1; tail -20 gpurun_out/sweep.log
