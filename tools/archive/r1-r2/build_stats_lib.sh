# Builds tools/libv_stats.so: the working tree's library with tools/sync_stats.patch applied
# (k_spec / k_resolve shader-clock phase counters, -DVF_SYNC_STATS=1), from a temp copy; the
# product source never carries the diagnostics.  Used by tools/gpu_r2_syncstats.sh.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cp -r "$ROOT/distributed-video-filter_amd" "$ROOT/include" "$T/"
cd "$T"
patch -s -p1 < "$ROOT/tools/sync_stats.patch"
C=distributed-video-filter_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Iinclude -shared \
  -DVF_SYNC_STATS=1 -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -pthread $C/vf_kernels.hip $C/vf_engine.hip \
  $C/vf_api.hip $C/vf_jpeg_kernels.hip $C/vf_jpeg_host.hip -o "$ROOT/tools/libv_stats.so"
rm -rf "$T"
