# host->host (PCIe-inclusive) rate vs slot size and host copy threads
set -o pipefail
mkdir -p gpurun_out
for cfg in "16777216 4" "16777216 8" "8388608 8" "33554432 8"; do
  set -- $cfg
  VF_SLOT_BYTES=$1 VF_HOST_THREADS=$2 timeout -k 10 120 python -u tools/sweep.py --e2e-only --out gpurun_out/e2e_$1_$2.jsonl > gpurun_out/e2e_$1_$2.log 2>&1 || { echo E2E_FAILED; tail -20 gpurun_out/e2e_$1_$2.log; exit 1; }
  echo "slot=$1 threads=$2"; cat gpurun_out/e2e_$1_$2.jsonl
done
