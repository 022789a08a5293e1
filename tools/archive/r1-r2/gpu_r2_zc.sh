#!/bin/bash
# zero-copy (kernel reads/writes page-locked host memory over PCIe) vs SDMA ceilings
set -e
mkdir -p gpurun_out
timeout -k 10 240 tools/zerocopy_probe 199065600 5 > gpurun_out/r2_zerocopy_probe2.jsonl 2> gpurun_out/r2_zerocopy_probe2.err
