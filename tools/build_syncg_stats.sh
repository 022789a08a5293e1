# Builds tools/variants/libv_syncg_stats.so: the working tree's library with k_syncg counters
# (rounds per workgroup: max and sum; symbols decoded; shader cycles inside sync_span, summed over
# decodes), printed and cleared by dec_syncg after each pass when VF_SYNCG_STATS is set.
# Diagnostics only, from a patched temp copy; the product source never carries them.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/variants"
T=$(mktemp -d)
cp -r "$ROOT/distributed-video-filter_amd" "$ROOT/include" "$T/"
python3 - "$T/distributed-video-filter_amd/csrc/vf_jpeg_kernels.hip" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
def rep(a, b):
    global s
    assert a in s, a[:80]
    s = s.replace(a, b, 1)
rep("__device__ __forceinline__ uint64_t sync_span(", "__device__ unsigned long long g_sg[8];\n__device__ __forceinline__ uint64_t sync_span(")
# count steps and cycles per decode
rep("""  SyncLane d;
  d.init(words, woff, X, hg);""", """  const long long c0_ = clock64();
  uint32_t steps_ = 0;
  struct Done_ { long long c0; uint32_t *st; __device__ ~Done_() { atomicAdd(&g_sg[2], (unsigned long long)*st); atomicAdd(&g_sg[3], (unsigned long long)(clock64() - c0)); atomicAdd(&g_sg[4], 1ull); } } done_{c0_, &steps_};
  SyncLane d;
  d.init(words, woff, X, hg);""")
rep("""    while (d.pos < mk) d.step(tabs);""", """    while (d.pos < mk) { d.step(tabs); ++steps_; }""")
rep("""  bool check = pass > 0;  // records are valid from the first decode on
  for (;;) {""", """  bool check = pass > 0;  // records are valid from the first decode on
  uint32_t rounds_ = 0;
  const long long w0_ = clock64();
  for (;;) {
    ++rounds_;""")
rep("""  if (t == T - 1 && live && i0 + G < nsub && (pass == 0 || last != last_old)) atomicOr(changed + pass, 1u);""",
    """  if (t == T - 1 && live && i0 + G < nsub && (pass == 0 || last != last_old)) atomicOr(changed + pass, 1u);
  if (t == 0) { atomicMax(&g_sg[0], (unsigned long long)rounds_); atomicAdd(&g_sg[1], (unsigned long long)rounds_); atomicAdd(&g_sg[5], 1ull); atomicAdd(&g_sg[6], (unsigned long long)(clock64() - w0_)); atomicMax(&g_sg[7], (unsigned long long)(clock64() - w0_)); }""")
rep("""  VF_SYNCG(8)
#undef VF_SYNCG
  return hipErrorInvalidValue;""", """  VF_SYNCG(8)
#undef VF_SYNCG
  return hipErrorInvalidValue;
}
static int syncg_stats_dummy = 0;
hipError_t syncg_stats_print(int pass, hipStream_t s) {
  if (!std::getenv("VF_SYNCG_STATS")) return hipSuccess;
  unsigned long long h[8];
  (void)hipStreamSynchronize(s);
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sg), sizeof h);
  const double wg = h[5] ? (double)h[5] : 1.0, dec = h[4] ? (double)h[4] : 1.0;
  std::fprintf(stderr, "[syncg] pass %d  WGs %llu rounds max %llu mean %.2f  decodes %llu symbols/decode %.0f cycles/decode %.0f cycles/symbol %.0f  WG cycles mean %.0f max %llu\\n",
               pass, h[5], h[0], h[1] / wg, h[4], h[2] / dec, h[3] / dec, h[2] ? (double)h[3] / h[2] : 0.0, h[6] / wg, h[7]);
  unsigned long long z[8] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sg), z, sizeof z);
  (void)syncg_stats_dummy;
  return hipSuccess;""")
# call the print after each launch
rep("""                       0, s, sg, fr, us, us_len, exits, cnts, used, ck, ckrem, changed, pass);                    \\
    return hipGetLastError();""", """                       0, s, sg, fr, us, us_len, exits, cnts, used, ck, ckrem, changed, pass);                    \\
    syncg_stats_print(pass, s);                                                                                   \\
    return hipGetLastError();""")
rep("hipError_t dec_syncg(", "hipError_t syncg_stats_print(int pass, hipStream_t s);\nhipError_t dec_syncg(")
if "#include <cstdio>" not in s:
    s = s.replace("#include <stdint.h>", "#include <stdint.h>\n#include <cstdio>\n#include <cstdlib>", 1)
open(p, "w").write(s)
PY
cd "$T"
C=distributed-video-filter_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Iinclude -shared \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip \
  $C/vf_jpeg_kernels.hip $C/vf_jpeg_host.hip -o "$ROOT/tools/variants/libv_syncg_stats.so"
cd "$ROOT"
rm -rf "$T"
ls -la tools/variants/libv_syncg_stats.so
