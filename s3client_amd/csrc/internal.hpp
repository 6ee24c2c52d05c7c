// internal.hpp -- what the HIP-facing translation units of libs3hash.so share: the plan object,
// its build / launch / check functions (plan.cpp), the kernel launchers (launch.hip, the only
// unit with device code), pinned host memory and device placement (pinned.cpp), and the
// stream units' hooks.  The C-ABI itself is include/s3hash.h.
//
//   launch.hip    sha256_kernels.hip + the hipLaunchKernelGGL calls (device code)
//   plan.cpp      plans: kernel choice, slot sorting, launches, error words; device-resident C-ABI
//   pinned.cpp    NUMA-placed pinned host memory, device placement, s3h_host_alloc / _numa
//   host_path.cpp host-resident pipeline (slices, groups), per-device contexts, the merge queue
//   stream.cpp    multi-object streams (s3h_stream_*)
//   route.cpp     size-aware routing (model measurement, observed rates, routed entry points)
//   HIP-free: status.cpp, topology.cpp, route_plan.cpp (+ copy_pool.hpp, host_queue.hpp)
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "../../include/s3hash.h"
#include "host_limits.hpp"
#include "kernel_abi.hpp"
#include "status.hpp"
#include "topology.hpp"

// A failed call also clears the thread's last HIP error: a later hipGetLastError after a
// launch must report that launch, not an allocation that failed (and was reported) before.
#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      (void)hipGetLastError();                                                             \
      return ::s3h::host::fail(e_ == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP,           \
                               "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,   \
                               __LINE__);                                                  \
    }                                                                                      \
  } while (0)

struct s3h_plan_s {
  int device = 0;
  int algo = S3H_ALGO_SHA256;
  int kernel = S3H_KERNEL_PC;
  uint64_t n = 0;
  uint64_t cap = 0;             // parts the device arrays hold (host path: reused plans)
  uint64_t total_blocks = 0;
  uint64_t max_blocks = 0;
  uint32_t grid = 0;
  s3h::Slot* d_slots = nullptr;
  uint32_t* d_out_idx = nullptr;
  uint32_t* d_state = nullptr;  // n*8 chaining words, allocated on first ranged launch
  uint8_t* d_zero = nullptr;    // 256 zero bytes: load target for out-of-range lanes
  int quad_waves = 1;           // skew / quad kernels: consumer waves per workgroup (1-2)
  uint32_t solo = 0;            // two-group skew grid: leading one-group workgroups (plan_solo)
  uint32_t dual_solo = 0;       // SHA-256 + MD5 of a ragged batch: skew groups of the mixed grid
  bool dual_apart = false;      // ... whose MD5 chains run on workgroups of their own
  uint64_t* d_clocks = nullptr; // clock probe buffer (caller-owned), see s3h_plan_set_clock_probe
  uint32_t* d_err = nullptr;    // device error word (s3h::kErr* bits), read by plan_check
  // mixed dual grid, apart form: per skew group the producer's step count tagged with the
  // launch epoch (pacing of the MD5 waves on other workgroups); allocated on first use
  uint64_t* d_progress = nullptr;
  uint32_t progress_epoch = 0;
};

namespace s3h::host {

int check_device(int device);

struct DeviceGuard {  // restores the calling thread's current device
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// ------------------------------------------------------------------ plans (plan.cpp)
constexpr uint64_t kMaxParts = 1ull << 31;
int device_cus(int device);  // cached CU count (0 if unknown)
double device_power_cap_w(int device);  // cached board power cap in W (0 if unknown)
uint64_t sort_slots(const uint64_t* offsets, const uint64_t* lengths, uint64_t n, bool nopad,
                    s3h::Slot* slots, uint32_t* order);
uint32_t dual_mixed_solo(const s3h::Slot* slots, uint64_t n, uint64_t cus, bool* apart);
int plan_alloc(int device, int algo, uint64_t cap, s3h_plan_s** out);
int plan_geometry(s3h_plan_s* P, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                  int kernel, s3h::Slot* h_slots, uint32_t* h_order, hipStream_t s);
int plan_build(int device, int algo, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
               int kernel, s3h_plan_s** out);
int plan_refill(s3h_plan_s* P, const uint64_t* offsets, const uint64_t* lengths, bool nopad,
                s3h::Slot* h_slots, uint32_t* h_order, hipStream_t s);
// one launch over blocks [b0, b1) with explicit state / flags / bit lengths
int launch_args(s3h_plan_s* P, const void* d_base, uint32_t* d_digests, uint32_t* d_state,
                uint64_t b0, uint64_t b1, uint64_t origin, uint32_t flags, const uint64_t* d_bits,
                hipStream_t stream);
int plan_launch(s3h_plan_s* P, const void* d_base, uint32_t* d_digests, uint64_t b0, uint64_t b1,
                uint64_t origin, hipStream_t stream, bool ranged);
int plan_check(s3h_plan_s* P, hipStream_t s);

// SHA-256 (plan S) and MD5 (plan M, same parts in the same order) from one grid:
// kDualSplit = sha256_md5_dual_kernel (skew workgroups then MD5 workgroups, one per CU);
// kDualGroup = sha256_md5_group_kernel<true> (skewp group + self-fed MD5 wave per workgroup);
// kDualGroupSkew = sha256_md5_group_kernel<false> (skew group + MD5 wave); kDualGroupMixed =
// sha256_md5_group_mixed_kernel (ragged 2,049-8,192 parts); kDualNone = two launches.
enum DualMode { kDualNone = 0, kDualSplit = 1, kDualGroup = 2, kDualGroupSkew = 3, kDualGroupMixed = 4 };
DualMode dual_mode(const s3h_plan_s* S, const s3h_plan_s* M, uint64_t b0, uint64_t b1);
int dual_launch(s3h_plan_s* S, s3h_plan_s* M, const void* d_base, uint32_t* d_sha,
                uint32_t* d_md5, uint64_t b0, uint64_t b1, uint64_t origin, bool ranged,
                hipStream_t stream);

// ------------------------------------------------------------------ kernel launchers (launch.hip)
// Each returns the launch's hipGetLastError (the caller cleared the thread's error before).
hipError_t launch_plan_kernel(const s3h_plan_s* P, int cus, uint64_t range_blocks,
                              const s3h::LaunchArgs& A, hipStream_t s);
// `progress` / `epoch`: the mixed grid's apart form (F step counts, tagged with this launch's
// epoch; plan.cpp dual_launch); unused by the other forms.
hipError_t launch_dual_kernel(DualMode mode, const s3h_plan_s* S, const s3h_plan_s* M,
                              const s3h::LaunchArgs& A, const s3h::LaunchArgs& B, uint64_t* progress,
                              uint32_t epoch, hipStream_t s);
hipError_t launch_stream_init(uint32_t* state, uint64_t n, int md5, hipStream_t s);
hipError_t launch_stream_splice(const uint8_t* base, const s3h::SpliceJob* jobs, uint8_t* carry,
                                uint8_t* head, uint64_t n, hipStream_t s);
hipError_t launch_compare_digests(const uint32_t* got, const uint32_t* want, uint64_t n,
                                  uint32_t words, uint8_t* mismatch, unsigned long long* count,
                                  hipStream_t s);
hipError_t launch_generate(uint8_t* base, const s3h::GenPart* parts, uint32_t nparts, uint32_t gx,
                           uint64_t seed, hipStream_t s);

// ------------------------------------------------------------------ host memory (pinned.cpp)
// Pinned host memory whose pages live on `node` (< 0: the runtime's hipHostMalloc).
// `strict`: the pages must be on that node (MPOL_BIND, s3h_host_alloc); otherwise the node is
// preferred and the kernel falls back to another when it is short (staging buffers).
hipError_t pinned_alloc(void** out, uint64_t bytes, int node, bool strict = false);
void pinned_free(void* p);
// Placement of device `device` (its PCI address -> sysfs) under the current NUMA policy.
Place device_place(int device);
// Every non-empty part idx[k] is page-locked host memory (hipPointerGetAttributes).
bool all_pinned(const uint8_t* const* parts, const uint64_t* lengths, const uint64_t* idx, uint64_t n);
// [p, p + bytes) lies inside ONE registered / pinned host allocation.
bool pinned_range(const void* p, uint64_t bytes);

// ------------------------------------------------------------------ streams (stream.cpp)
void staging_trim();  // frees the staging that destroyed stream objects left for reuse

}  // namespace s3h::host
