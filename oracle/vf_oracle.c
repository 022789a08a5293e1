/*
 * vf_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's per-frame filter, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the CHECKER.  It is never
 * linked into, loaded by or called from the product path (libvfilter_hip.so and the
 * vfilter package), which fails loudly when its HIP library is missing.
 *
 * Algorithm restated: OpenCV `bitwise_not`, called at inverter.py:41 as
 *     inverted = cv2.bitwise_not(frame)
 * on the uint8 H x W x 3 frame produced at inverter.py:32/34.  OpenCV (opencv-python,
 * unpinned in requirements.txt:1, not vendored, not installed here) defines it as the
 * per-element bitwise inversion dst(I) = ~src(I); for CV_8U data that is per byte, and it
 * is independent of channel order and shape.  Pinning: tests/golden (all-256-values KAT,
 * tail/alignment KATs, seeded-frame sha256s, and outputs captured from the reference's own
 * worker.py/distributor.py run in the survey container) — see DESIGN.md "Oracle".
 */
#include <stddef.h>
#include <stdint.h>

/* dst[i] = ~src[i] for i in [0, n).  In place (src == dst) is allowed. */
void vfo_invert(const uint8_t *src, uint8_t *dst, size_t n) {
  for (size_t i = 0; i < n; ++i) dst[i] = (uint8_t)~src[i];
}

/* The same over n separately stored frames (sizes may differ). */
void vfo_invert_frames(const uint8_t *const *srcs, uint8_t *const *dsts, const size_t *nbytes,
                       int n) {
  for (int f = 0; f < n; ++f) vfo_invert(srcs[f], dsts[f], nbytes[f]);
}

/* FNV-1a 64 over a byte range: a cheap size-independent digest for large-frame checks. */
uint64_t vfo_fnv1a64(const uint8_t *p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
