set -o pipefail
mkdir -p gpurun_out
for sz in 480p 1080p 4k; do
VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python -u tools/jpeg_host_trace.py $sz > gpurun_out/syncstats_$sz.log 2>&1 || { echo FAILED; tail -20 gpurun_out/syncstats_$sz.log; exit 1; }
echo $sz; grep "spec:" gpurun_out/syncstats_$sz.log | tail -2
done
