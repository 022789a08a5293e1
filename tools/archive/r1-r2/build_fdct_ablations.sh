# Timing-only ablations of k_fdct / k_write (ABL_VARIANTS: nopix noac nocoef), built from patched copies in a temp dir (the product source
# is not touched): tools/libv_abl_{nopix,noac,nopack}.so.  Outputs are NOT valid JPEGs.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for v in ${ABL_VARIANTS:-nopix noac}; do
  T=$(mktemp -d)
  mkdir -p "$T/distributed-video-filter_amd"
  cp -r "$ROOT/distributed-video-filter_amd/csrc" "$T/distributed-video-filter_amd/"
  cp -r "$ROOT/include" "$T/"
  python3 - "$T/distributed-video-filter_amd/csrc/vf_jpeg_kernels.hip" "$v" <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]
s = open(p).read()
if v == "nopix":   # pass 1 without pixel loads / colour conversion: a synthetic row
    a = "    const Ycc q = ycc_coefs((int)k, bgr != 0);\n    if (ve == 1 && he <= 2) {"
    b = "    const Ycc q = ycc_coefs((int)k, bgr != 0);\n#pragma unroll\n    for (int j = 0; j < 8; ++j) v[j] = (int)((bx * 8 + j + sy * 3 + k) & 255);\n    if (true) {\n    } else if (ve == 1 && he <= 2) {"
    assert s.count(a) == 1; s = s.replace(a, b)
if v == "noac":    # no AC coding: DC and an empty AC stream per block
    a = "  // AC Huffman coding; every lane of the wave takes part in the 8-lane shuffles\n"
    b = a + "  if (real && r == 0) { dcq[F.blk0 + b] = qo[slot][qo_at(slot, 0)]; acbits[F.blk0 + b] = 0; }\n  return;\n"
    assert s.count(a) == 1; s = s.replace(a, b)
if v == "nocoef":  # Huffman write without the coefficient stores (DC sequence still written)
    a = "        if (WRITE) coef[(uint64_t)blk * 64 + (z < 63 ? z : 63)] = (int16_t)v;"
    b = "        if (WRITE && v == 0x7fffffff) coef[(uint64_t)blk * 64 + (z < 63 ? z : 63)] = (int16_t)v;"
    assert s.count(a) == 1; s = s.replace(a, b)
open(p, "w").write(s)
PY
  C=$T/distributed-video-filter_amd/csrc
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -I$T/include -shared \
    -Wl,-rpath,/opt/rocm/lib -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip $C/vf_jpeg_kernels.hip \
    $C/vf_jpeg_host.hip -o "$ROOT/tools/libv_abl_$v.so"
  rm -rf "$T"
done
