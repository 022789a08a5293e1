mkdir -p gpurun_out; : > gpurun_out/async2.txt
P="timeout -k 10 120 python -u tools/async_probe.py --batches 48"
$P --ring 1 >> gpurun_out/async2.txt 2>&1 || exit 1
VF_SLOTS=8 $P --ring 8 >> gpurun_out/async2.txt 2>&1 || exit 1
VF_SLOT_BYTES=67108864 $P --ring 8 >> gpurun_out/async2.txt 2>&1 || exit 1
VF_SLOTS=8 VF_SLOT_BYTES=33554432 $P --ring 8 >> gpurun_out/async2.txt 2>&1 || exit 1
cat gpurun_out/async2.txt
