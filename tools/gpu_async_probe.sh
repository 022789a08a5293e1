mkdir -p gpurun_out; : > gpurun_out/async4.txt
timeout -k 10 150 ./tools/pcie_probe 1073741824 16777216 > gpurun_out/pcie4.txt 2>&1 || exit 1
tail -6 gpurun_out/pcie4.txt
timeout -k 10 120 python -u tools/async_probe.py >> gpurun_out/async4.txt 2>&1 || exit 1
VF_WAIT_POLL=1 timeout -k 10 120 python -u tools/async_probe.py >> gpurun_out/async4.txt 2>&1 || exit 1
cat gpurun_out/async4.txt
