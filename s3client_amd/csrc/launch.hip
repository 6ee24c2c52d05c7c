// launch.hip -- the only translation unit with device code: the gfx950 kernels of
// sha256_kernels.hip and the launches that pick among them.  Everything around the launches --
// plans, the host pipeline, streams, routing -- is host C++ in the other units (internal.hpp).
#include <hip/hip_runtime.h>

#include "internal.hpp"
#include "sha256_kernels.hip"

namespace s3h::host {

// Dynamic LDS added to a grid with solo workgroups: 72 KiB of groups + 12 KiB > half of the
// CU's 160 KiB, so one workgroup per CU and a solo group never shares its CU.
constexpr uint32_t kSoloLdsPad = 12 * 1024;
// sha256_md5_group_mixed_kernel: 66 KiB of skewp LDS + this > half of the CU's 160 KiB.
constexpr uint32_t kMixedLdsPad = 16 * 1024;
static_assert(sizeof(s3h::SkewLds<1, true>) + kMixedLdsPad > 80 * 1024, "one mixed workgroup per CU");

hipError_t launch_plan_kernel(const s3h_plan_s* P, int cus, uint64_t range, const s3h::LaunchArgs& A,
                              hipStream_t stream) {
  if (P->algo == S3H_ALGO_MD5 && P->grid <= uint64_t(cus))
    hipLaunchKernelGGL(s3h::md5_pc_kernel<s3h::kMd5Bps>, dim3(P->grid), dim3(s3h::kPcThreads), 0,
                       stream, A);
  else if (P->algo == S3H_ALGO_MD5)  // more workgroups than CUs: the 32 KiB form, several per CU
    hipLaunchKernelGGL(s3h::md5_pc_kernel<1>, dim3(P->grid), dim3(s3h::kPcThreads), 0, stream, A);
  // The skew kernel counts a launch's blocks in 32 bits: a range of 2^31 blocks (128 GiB of
  // one part) or more runs on the quad kernel (same plan geometry, 64-bit counters).
  else if (P->kernel == S3H_KERNEL_SKEW && range >= (1ull << 31) && P->quad_waves == 1)
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<1>, dim3(P->grid), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEW && range >= (1ull << 31))
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<2>, dim3(P->grid), dim3(192), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWS && range >= (1ull << 31))
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<1>, dim3(uint32_t((P->n + 7) / 8)), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWS)
    hipLaunchKernelGGL(s3h::sha256_skew_shared_kernel, dim3(P->grid), dim3(512), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWP && range >= (1ull << 31))
    hipLaunchKernelGGL(s3h::sha256_pair_kernel, dim3(P->grid), dim3(s3h::kPairThreads), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWP)
    hipLaunchKernelGGL((s3h::sha256_skew_kernel<1, true>), dim3(P->grid), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEW && P->quad_waves == 1)
    hipLaunchKernelGGL(s3h::sha256_skew_kernel<1>, dim3(P->grid), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEW)  // two flag-synchronised groups per workgroup
    hipLaunchKernelGGL(s3h::sha256_skew_pairs_kernel, dim3(P->grid), dim3(256),
                       P->solo ? kSoloLdsPad : 0, stream, A);
  else if (P->kernel == S3H_KERNEL_PC)
    hipLaunchKernelGGL(s3h::sha256_pc_kernel, dim3(P->grid), dim3(s3h::kPcThreads), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_QUAD && P->quad_waves == 1)
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<1>, dim3(P->grid), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_QUAD)
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<2>, dim3(P->grid), dim3(192), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_PAIR)
    hipLaunchKernelGGL(s3h::sha256_pair_kernel, dim3(P->grid), dim3(s3h::kPairThreads), 0, stream, A);
  else
    hipLaunchKernelGGL(s3h::sha256_lane_kernel, dim3(P->grid), dim3(256), 0, stream, A);
  return hipGetLastError();
}

hipError_t launch_dual_kernel(DualMode mode, const s3h_plan_s* S, const s3h_plan_s* M,
                              const s3h::LaunchArgs& A, const s3h::LaunchArgs& B, uint64_t* progress,
                              uint32_t epoch, hipStream_t stream) {
  if (mode == kDualGroup) {
    hipLaunchKernelGGL(s3h::sha256_md5_group_kernel<true>, dim3(uint32_t((S->n + 31) / 32)),
                       dim3(192), 0, stream, A, B);
  } else if (mode == kDualGroupMixed) {  // the LDS pad keeps one workgroup per CU
    const uint32_t F = S->dual_solo, G = uint32_t((S->n - 8ull * F + 31) / 32);
    const uint32_t lead = S->dual_apart ? s3h::mixed_lead_wgs(F) : 0;
    hipLaunchKernelGGL(s3h::sha256_md5_group_mixed_kernel, dim3(F + G + lead), dim3(192),
                       kMixedLdsPad, stream, A, B, F, G, lead, progress, epoch);
  } else if (mode == kDualGroupSkew) {
    hipLaunchKernelGGL(s3h::sha256_md5_group_kernel<false>, dim3(uint32_t((S->n + 7) / 8)),
                       dim3(192), 0, stream, A, B);
  } else {
    hipLaunchKernelGGL(s3h::sha256_md5_dual_kernel<false>,
                       dim3(S->grid + s3h::split_md5_wgs(S->grid, S->n)), dim3(128), 0, stream, A, B,
                       uint32_t(S->grid), progress, epoch);
  }
  return hipGetLastError();
}

hipError_t launch_stream_init(uint32_t* state, uint64_t n, int md5, hipStream_t s) {
  hipLaunchKernelGGL(s3h::stream_init_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s, state, n, md5);
  return hipGetLastError();
}

hipError_t launch_stream_splice(const uint8_t* base, const s3h::SpliceJob* jobs, uint8_t* carry,
                                uint8_t* head, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(s3h::stream_splice_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s,
                     base, jobs, carry, head, n);
  return hipGetLastError();
}

hipError_t launch_compare_digests(const uint32_t* got, const uint32_t* want, uint64_t n, uint32_t words,
                                  uint8_t* mismatch, unsigned long long* count, hipStream_t s) {
  hipLaunchKernelGGL(s3h::compare_digests_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s,
                     got, want, n, words, mismatch, count);
  return hipGetLastError();
}

hipError_t launch_generate(uint8_t* base, const s3h::GenPart* parts, uint32_t nparts, uint32_t gx,
                           uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(s3h::generate_kernel, dim3(gx, nparts), dim3(256), 0, s, base, parts, seed);
  return hipGetLastError();
}

}  // namespace s3h::host
