# configs[4] dip probe: rate of one launch vs the same bytes cut into sub-launches of
# 64 MiB ... 1 GiB, at 1.6 / 3.2 / 6.4 / 12.7 GB (each size a fresh process, dst pad 0).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pad.txt
for b in 1592524800 3185049600 6370099200 12740198400; do
  timeout -k 10 60 tools/tune_invert large $b 9 0 >> gpurun_out/pad.txt 2>&1 || { echo PAD_FAILED; tail gpurun_out/pad.txt; exit 1; }
done
cat gpurun_out/pad.txt
