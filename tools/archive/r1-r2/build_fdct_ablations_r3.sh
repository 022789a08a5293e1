# Timing-only ablations of k_fdct (round 3 form), built from patched copies of the working tree
# into tools/variants/libv_<name>.so; the product source is never modified.  Results of these
# libraries are wrong by construction: only their kernel times mean anything.
#   base    unchanged
#   noac    no AC coding rounds (the ranked list is still built)
#   nolist  neither the list nor the rounds
#   nofdct  both DCT passes skipped
#   noquant quantisation replaced by a truncation
#   nopix   pass 1 reads no pixels and converts no colour (a constant ramp per row)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/variants"
for v in ${ABL_VARIANTS:-base noac nolist nofdct noquant nopix}; do
  T=$(mktemp -d)
  cp -r "$ROOT/distributed-video-filter_amd" "$ROOT/include" "$T/"
  python3 - "$T/distributed-video-filter_amd/csrc/vf_jpeg_kernels.hip" "$v" <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]
s = open(p).read()
def rep(a, b):
    global s
    assert a in s, (v, a[:60])
    s = s.replace(a, b)
if v in ("noac", "nolist"):
    rep("for (uint32_t q0 = 0; __ballot(q0 < nnz) != 0; q0 += 8) {", "for (uint32_t q0 = 0; __ballot(q0 < nnz) != 0 && q0 > 1000; q0 += 8) {")
if v == "nolist":
    rep("      if ((m8 >> j) & 1) {\n        lst[at++]", "      if (((m8 >> j) & 1) && kk > 1000) {\n        lst[at++]")
if v == "nofdct":
    rep("    else fdct_islow_line(v, 0);", "    else {}")
    rep("    else fdct_islow_line(v, 1);", "    else {}")
if v == "noquant":
    rep("= quantize(v[i], q.x & 0xFFFF, q.x >> 16, (int32_t)(int16_t)(q.y & 0xFFFF));", "= (int16_t)(v[i] + (q.x & 1));")
if v == "nopix":
    rep("    if (ve == 1 && he <= 2) {  // he == 1: full-resolution line; he == 2: h2v1_downsample",
        "    if (false) {")
    rep("    } else if (he == 2 && ve == 2) {  // h2v2_downsample", "    } else if (false) {")
    rep("v[j] = enc_sample(g, img, (int)k, (int)(bx * 8 + j), sy, ro, bo) - 128;", "v[j] = (int)(j * 7 + r + ro) - 64;")
open(p, "w").write(s)
PY
  cd "$T"
  C=distributed-video-filter_amd/csrc
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Iinclude -shared \
    -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip \
    $C/vf_jpeg_kernels.hip $C/vf_jpeg_host.hip -o "$ROOT/tools/variants/libv_$v.so" &
  cd "$ROOT"
done
wait
ls -la "$ROOT/tools/variants/"
