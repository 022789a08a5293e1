# Builds the library of the last commit into tools/libv_head.so (the "head" side of tools/gpu_jpeg_ab.sh)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive ${HEAD_REF:-HEAD} distributed-video-filter_amd/csrc include | tar -x -C "$T"
cd "$T"
C=distributed-video-filter_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Iinclude -shared \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip \
  $C/vf_jpeg_kernels.hip $C/vf_jpeg_host.hip -o "$ROOT/tools/libv_head.so"
rm -rf "$T"
