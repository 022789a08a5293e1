# Build library variants of the working tree with extra -D flags for A/B timing on the GPU box:
#   tools/build_variants.sh name1:"-DFOO=1" name2:"-DBAR=2" ...   -> tools/variants/libv_<name>.so
set -e
C=distributed-video-filter_amd/csrc
mkdir -p tools/variants
rm -f tools/variants/*.so
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -I$C $flags -shared \
    -Wl,-rpath,/opt/rocm/lib -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip $C/vf_jpeg_kernels.hip \
    $C/vf_jpeg_host.hip -o tools/variants/libv_$name.so &
done
wait
ls tools/variants
