// vf_internal.h — shared between the kernel TU and the C-ABI TU (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace vf {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Kernel variants selectable at run time (VF_VARIANT env) for A/B tuning; the default is
// the one tools/tune_invert.hip measured fastest on MI355X.
// Un = n independent 16-B loads in flight per lane; NT = nontemporal loads and stores
// (`global_load/store_dwordx4 ... nt`), NTL / NTS = nontemporal on one side only.
enum Variant : int {
  kVariantU4NT = 0,  // default: 6.32 TB/s at 32 blocks/CU (profiles/r01_tune_sweep2.txt)
  kVariantU2NT = 1,
  kVariantU8NT = 2,
  kVariantU1NT = 3,
  kVariantU4NTL = 4,
  kVariantU4NTS = 5,
  kVariantU4 = 6,
  kVariantU2 = 7,
  kVariantU8 = 8,
  kVariantU1 = 9,
  kVariantCount = 10,
};

const char *variant_name(int v);

struct LaunchCfg {
  int variant = kVariantU4NT;
  int max_blocks = 8192;  // grid cap: 32 workgroups per CU on 256 CUs
};

hipError_t launch_invert(const void *dsrc, void *ddst, size_t nbytes, const LaunchCfg &cfg,
                         hipStream_t stream);

hipError_t launch_invert_frames(const void *const *dsrcs, void *const *ddsts,
                                const size_t *nbytes, int n, size_t total_bytes,
                                const LaunchCfg &cfg, hipStream_t stream);

}  // namespace vf
