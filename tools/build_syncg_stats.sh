# Builds tools/variants/libv_syncg_stats.so: the working tree's library with k_syncg counters,
# printed and cleared by dec_syncg after each pass when VF_SYNCG_STATS is set:
#   per workgroup (thread 0's clock): cycles of round 0 (warm-up + first decode) and of the
#   whole pass; rounds; per re-decode: lanes active per round; per lane: warm-up and decode
#   steps.  Diagnostics only, from a patched temp copy; the product source never carries them.
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
rep("template <bool CHECK, uint32_t NDC>\n__device__ __forceinline__ uint64_t sync_span(",
    "__device__ unsigned long long g_sg[16];\ntemplate <bool CHECK, uint32_t NDC>\n__device__ __forceinline__ uint64_t sync_span(")
rep("""  last_old = last;
  bool check = pass > 0;  // records are valid from the first decode on
  for (;;) {
    if (need) {""", """  last_old = last;
  bool check = pass > 0;  // records are valid from the first decode on
  __syncthreads();
  const long long w0_ = clock64();
  long long r0_ = 0;
  uint32_t rounds_ = 0;
  for (;;) {
    if (need && rounds_ > 0) atomicAdd(&g_sg[8], 1ull);
    const long long d0_ = clock64();
    if (need) {""")
rep("""      used[gi0] = entry;
    }
    s_exit[t] = live ? rel(last) : 0u;
    __syncthreads();""", """      used[gi0] = entry;
    }
    if (need && rounds_ > 0) atomicAdd(&g_sg[9], (unsigned long long)(clock64() - d0_));
    s_exit[t] = live ? rel(last) : 0u;
    __syncthreads();
    if (rounds_ == 0) r0_ = clock64() - w0_;
    ++rounds_;""")
rep("""  if (t == T - 1 && live && i0 + G < nsub && (pass == 0 || last != last_old)) atomicOr(changed + pass, 1u);
}""", """  if (t == T - 1 && live && i0 + G < nsub && (pass == 0 || last != last_old)) atomicOr(changed + pass, 1u);
  if (t == 0 && live) {
    const unsigned long long tot_ = (unsigned long long)(clock64() - w0_);
    atomicAdd(&g_sg[0], 1ull);
    atomicAdd(&g_sg[1], (unsigned long long)r0_);
    atomicAdd(&g_sg[2], tot_);
    atomicMax(&g_sg[3], tot_);
    atomicAdd(&g_sg[4], (unsigned long long)rounds_);
    atomicMax(&g_sg[5], (unsigned long long)rounds_);
  }
}""")
rep("""      if (i0 > 0 && warm > 0) {
        const uint32_t b = i0 * kSubBits, w0 = b > warm ? b - warm : 0u;
        SpanLane<SyncTab32, NDC> d;
        d.init(s_w, wb32, pack_state(w0, 0, 0), hg);
        d.run(tabs, b);
        entry = d.state();
      }""", """      if (i0 > 0 && warm > 0) {
        const uint32_t b = i0 * kSubBits, w0 = b > warm ? b - warm : 0u;
        SpanLane<SyncTab32, NDC> d;
        d.init(s_w, wb32, pack_state(w0, 0, 0), hg);
        const long long c0_ = clock64();
        d.run(tabs, b);
        atomicAdd(&g_sg[6], (unsigned long long)(clock64() - c0_));
        atomicAdd(&g_sg[7], 1ull);
        entry = d.state();
      }""")
rep("""  __device__ __forceinline__ void step(const Tab *tabs, int32_t qs) {
    const uint32_t *p = wl + (-(q >> 5) - 1);""", """  uint32_t steps_ = 0;
  __device__ __forceinline__ void step(const Tab *tabs, int32_t qs) {
    ++steps_;
    const uint32_t *p = wl + (-(q >> 5) - 1);""")
rep("""        atomicAdd(&g_sg[7], 1ull);""", """        atomicAdd(&g_sg[7], 1ull);
        atomicAdd(&g_sg[10], (unsigned long long)d.steps_);
        atomicAdd(&g_sg[11], (unsigned long long)(d.pos() - w0));""")
rep("""  for (;;) {
    d.run(tabs, mk);
    const uint64_t st = d.state();""", """  struct Fin_ { SpanLane<SyncTab32, NDC> *d; uint32_t p0; __device__ ~Fin_() { if (CHECK) { atomicAdd(&g_sg[12], (unsigned long long)d->steps_); atomicAdd(&g_sg[13], (unsigned long long)(d->pos() - p0)); } else { atomicAdd(&g_sg[14], (unsigned long long)d->steps_); atomicAdd(&g_sg[15], (unsigned long long)(d->pos() - p0)); } } } fin_{&d, d.pos()};
  for (;;) {
    d.run(tabs, mk);
    const uint64_t st = d.state();""")
rep("hipError_t dec_syncg(", """hipError_t syncg_stats_print(int pass, hipStream_t s) {
  if (!std::getenv("VF_SYNCG_STATS")) return hipSuccess;
  unsigned long long h[16];
  (void)hipStreamSynchronize(s);
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sg), sizeof h);
  const double wg = h[0] ? (double)h[0] : 1.0;
  std::fprintf(stderr, "[syncg] pass %d WGs %llu | WG cycles mean %.0f max %llu | round0 mean %.0f | rounds mean %.2f max %llu | "
               "warm-up lane cycles mean %.0f | re-decodes %llu (%.1f per WG), lane cycles mean %.0f\\n",
               pass, h[0], h[2] / wg, h[3], h[1] / wg, h[4] / wg, h[5], h[7] ? (double)h[6] / h[7] : 0.0, h[8],
               h[8] / wg, h[8] ? (double)h[9] / h[8] : 0.0);
  std::fprintf(stderr, "[syncg]   warm-up steps %llu bits %llu (%.2f bits/step, %.0f cycles/step) | checked decodes steps %llu bits %llu | first decodes steps %llu bits %llu\\n",
               h[10], h[11], h[10] ? (double)h[11] / h[10] : 0.0, h[10] ? (double)h[6] / h[10] : 0.0, h[12], h[13], h[14], h[15]);
  unsigned long long z[16] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sg), z, sizeof z);
  return hipSuccess;
}
hipError_t dec_syncg(""")
rep("""                       pass, warm);                                                                               \\
    return hipGetLastError();""", """                       pass, warm);                                                                               \\
    syncg_stats_print(pass, s);                                                                                   \\
    return hipGetLastError();""")
if "#include <cstdio>" not in s:
    s = "#include <cstdio>\n#include <cstdlib>\n" + s
open(p, "w").write(s)
PY
cd "$T"
C=distributed-video-filter_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -I$C -shared \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -pthread $C/vf_kernels.hip $C/vf_engine.hip $C/vf_api.hip \
  $C/vf_jpeg_kernels.hip $C/vf_jpeg_host.hip -o "$ROOT/tools/variants/libv_syncg_stats.so"
cd "$ROOT"
rm -rf "$T"
ls -la tools/variants/libv_syncg_stats.so
