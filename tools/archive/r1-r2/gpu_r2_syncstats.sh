# k_spec phase counters (tools/libv_stats.so: tools/build_stats_lib.sh, the sync_stats.patch build; round 3 dropped the k_resolve ones: its serial walk is one LDS read per workgroup now) at 480p and
# 1080p, plus the custom-table JPEG GPU test on the in-tree library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q -k custom_tables --timeout 120 --timeout-method thread > gpurun_out/pytest_custom.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_custom.log; exit 1; }
tail -1 gpurun_out/pytest_custom.log
for sz in 480p 1080p; do
VFILTER_LIB=$PWD/tools/libv_stats.so VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python -u tools/jpeg_host_trace.py $sz > gpurun_out/syncstats_$sz.log 2>&1 || { echo FAILED; tail -20 gpurun_out/syncstats_$sz.log; exit 1; }
echo $sz; grep "spec\|kcycles" gpurun_out/syncstats_$sz.log | tail -3
done
