set -o pipefail
mkdir -p gpurun_out
for b in 256 512 1024; do
cp tools/libv_$b.so distributed-video-filter_amd/vfilter/libvfilter_hip.so
for sz in 1080p 4k; do
VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python -u tools/jpeg_host_trace.py $sz > gpurun_out/ss.log 2>&1 || { echo FAILED; tail -20 gpurun_out/ss.log; exit 1; }
echo "bits $b $sz: $(grep 'spec unres' gpurun_out/ss.log | tail -1) $(grep 'python wall' gpurun_out/ss.log | tail -1)"
done
timeout -k 10 200 python -u tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/jb.log 2>&1 || { echo JB_FAILED; tail gpurun_out/jb.log; exit 1; }
grep -o '"gpu_resident_fps": [0-9.]*\|"huffman_sync": [0-9.]*\|"huffman_write": [0-9.]*' gpurun_out/jb.log | tr '\n' ' '; echo
done
