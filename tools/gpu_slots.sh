set -o pipefail
mkdir -p gpurun_out; : > gpurun_out/slots.txt
for ns in 4 6 8; do
  VF_SLOTS=$ns timeout -k 10 150 python -u tools/sweep.py --e2e-only --out gpurun_out/e2e_s$ns.jsonl > /dev/null 2>&1 || exit 1
  sed "s/^{/{\"slots\": $ns, /" gpurun_out/e2e_s$ns.jsonl >> gpurun_out/slots.txt
  VF_SLOTS=$ns timeout -k 10 150 python -u tools/async_probe.py --size 4k --batches 24 2>&1 | sed "s/^{/{\"slots\": $ns, /" >> gpurun_out/slots.txt || exit 1
done
cat gpurun_out/slots.txt
