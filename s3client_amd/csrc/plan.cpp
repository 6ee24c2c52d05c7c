// plan.cpp -- plans (the part geometry of one batch, sorted by block count, on a device), the
// kernel choice by part count, launches, device error words, and the device-resident C-ABI
// entry points of include/s3hash.h.  No entry point ever computes a digest on the CPU: with no
// HIP device every call fails with S3H_ENODEV.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "internal.hpp"

namespace s3h::host {

int check_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(S3H_ENODEV, "no HIP device visible (the batched SHA-256 path has no CPU fallback)");
  if (device < 0 || device >= count) return fail(S3H_EINVAL, "device %d out of range [0,%d)", device, count);
  return S3H_OK;
}

namespace {

// Kernel choice by part count (profiles/r01_sweep_skew*.jsonl, r01_sweep_parts_256KiB.jsonl):
// while every consumer wave can own a SIMD, per-chain latency rules and the skewed lane-octet
// kernel (8 VALU/round, 8 chains per wave) wins -- one consumer wave per workgroup up to 2,048
// parts, two up to 4,096 (256 workgroups = one per CU); then the skewed lane-pair kernel
// (9 VALU/round, 32 chains per wave: 1.17x the pair kernel at 8K parts, 1.97x at 16K), then
// the pair kernel until consumer+producer waves fill every SIMD and total instruction count
// rules: producer/consumer up to 64K parts, then the fused one-lane-per-part kernel.
constexpr uint64_t kQuadMaxParts = 4096;   // skew (lane octets), 1-2 consumer waves per WG
constexpr uint64_t kSkewpMaxParts = 28672; // skewp (lane pairs, 32 chains per consumer wave)
constexpr uint64_t kPairMaxParts = 32768;
constexpr uint64_t kPcMaxParts = 65536;

// Skew / quad kernels: consumer waves per workgroup -- the fewest that keep the grid within
// one workgroup per CU (256): one up to 2,048 parts, two up to 4,096 (kQuadMaxParts).
int quad_waves(uint64_t n) {
#ifdef S3H_EXP_FORCE_NC  // tools/ experiment builds only
  return S3H_EXP_FORCE_NC;
#endif
  return n <= 256ull * s3h::kQuadChainsPerWave ? 1 : 2;
}

// Two-group skew grid (2,049-4,096 parts): how many leading workgroups run ONE group.  With
// all four SIMDs of a CU busy each wave issues 2-3 % slower than with two (C3: 2,280 vs 2,228
// cycles/block, profiles/r02_exp_c3_solo.jsonl), and a ragged batch's time is set by its
// longest parts, which sort first.  So the groups of the longest parts get a CU of their own
// (the launch's LDS pad admits one workgroup per CU) when that shortens the estimated
// makespan: group g takes (its first slot's blocks) x (1 alone | kPairSlow paired), and
// workgroups start in grid order on the first CU to free.  Equal-length batches keep 0.
// kPairSlow: measured 1.023 (C3: 2,280 paired vs 2,228 solo cycles/block) plus a margin, so
// that the boundary group (the longest paired one) does not become the new critical path.
constexpr double kPairSlow = 1.04;
uint32_t plan_solo(const s3h::Slot* slots, uint64_t n, uint64_t cus) {
  const uint64_t groups = (n + s3h::kQuadChainsPerWave - 1) / s3h::kQuadChainsPerWave;
  if (cus == 0 || groups < 2) return 0;
  std::vector<double> gb(groups);
  for (uint64_t g = 0; g < groups; ++g)
    gb[g] = double(s3h::nblocks(slots[g * s3h::kQuadChainsPerWave].len));
  std::vector<double> ends;
  ends.reserve(cus);
  auto makespan = [&](uint64_t F) {
    const uint64_t wgs = F + (groups - F + 1) / 2;
    auto dur = [&](uint64_t w) { return w < F ? gb[w] : gb[F + 2 * (w - F)] * kPairSlow; };
    ends.clear();
    double span = 0;
    for (uint64_t w = 0; w < wgs && w < cus; ++w) ends.push_back(dur(w));
    std::make_heap(ends.begin(), ends.end(), std::greater<double>());
    for (uint64_t w = cus; w < wgs; ++w) {  // later workgroups start as the first CU frees
      std::pop_heap(ends.begin(), ends.end(), std::greater<double>());
      ends.back() += dur(w);
      std::push_heap(ends.begin(), ends.end(), std::greater<double>());
    }
    for (double e : ends) span = std::max(span, e);
    return span;
  };
  // Candidate: the fewest solo groups after which no paired group outlasts the longest solo
  // one (durations descend, so a binary search); halved while workgroups beyond one per CU
  // (the grid's shortest) would end later than that.  A few simulations instead of one per F:
  // this runs on every host-path call.
  const uint64_t lim = std::min<uint64_t>(groups, cus);
  uint64_t lo = 1, hi = lim;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (mid < groups && gb[mid] * kPairSlow > gb[0]) lo = mid + 1;
    else hi = mid;
  }
  const double base = makespan(0);
  for (uint64_t F = lo; F >= 1; F /= 2)
    if (makespan(F) < base * 0.995) return uint32_t(F);  // a clear gain only
  return 0;
}

// `cus`: the device's CUs.  Above 4,096 parts, while one 32-chain workgroup per CU holds the
// batch (8,192 parts on MI355X: the C4 shard), the shared-SIMD skew kernel runs every chain
// at the skew kernel's 8 VALU per round with its producer on the same SIMD: C4 shard 492.8 vs
// 468.9 GiB/s for skewp (BENCH_r05 configs.c4.kernels), at 1.26 kW against 0.77 kW
// (2.57 vs 1.65 J/GiB): skewp has the lower energy-delay product (J/GiB x s/GiB: 3.5e-3 vs
// 5.2e-3).  The policy (s3h_kernel_policy) decides in that range:
//   S3H_POLICY_THROUGHPUT  skews, always;
//   S3H_POLICY_EFFICIENCY  skewp, always (env S3H_PREFER_EFFICIENCY=1);
//   S3H_POLICY_POWER       (default) skews only where the board may draw what skews needs to
//                          hold its full clock, else skewp.  Round 6's attribution
//                          (profiles/r06_power_attribution.json, one lease, two rounds): idle
//                          board 245 W; the consumers alone on stale W+K 1,098 W at 2.38 GHz
//                          (+853 W); the producers alone 977 W at 2.32 GHz running 1.66x the
//                          product's block rate (+732 W, ~441 W at the product's rate); the
//                          product 1,344 W at 2.28 GHz against the 1.4 kW cap.  The consumers'
//                          round stream owns two thirds of the dynamic power, and skews at
//                          2.35 GHz would need ~245 + 1,294 x 2.35 / 2.38 = ~1.52 kW.  Under
//                          a cap below kSkewsFullClockW skews runs ~5 % faster than skewp for
//                          ~1.5x its energy (the higher energy-delay product), so POWER picks
//                          skewp; a board allowed 1.5 kW or more keeps skews.
// Outside 4,097 - 32 x CUs parts every policy chooses the same kernel.
constexpr double kSkewsFullClockW = 1500.0;
std::atomic<int> g_kernel_policy{[] {
  const char* e = std::getenv("S3H_PREFER_EFFICIENCY");
  if (e && std::atoi(e) == 1) return int(S3H_POLICY_EFFICIENCY);
  const char* k = std::getenv("S3H_KERNEL_POLICY");
  if (k && std::strcmp(k, "throughput") == 0) return int(S3H_POLICY_THROUGHPUT);
  if (k && std::strcmp(k, "efficiency") == 0) return int(S3H_POLICY_EFFICIENCY);
  return int(S3H_POLICY_POWER);
}()};

int resolve_kernel(int algo, uint64_t n, int kernel, uint64_t cus, int device) {
  if (algo == S3H_ALGO_MD5) return S3H_KERNEL_PC;  // MD5 has one kernel (4 VALU per step)
  if (kernel != S3H_KERNEL_AUTO) return kernel;
  const int policy = g_kernel_policy.load();
  const bool efficient = policy == S3H_POLICY_EFFICIENCY ||
                         (policy == S3H_POLICY_POWER && n > kQuadMaxParts && n <= 32 * cus &&
                          device_power_cap_w(device) > 0 && device_power_cap_w(device) < kSkewsFullClockW);
  return n <= kQuadMaxParts    ? S3H_KERNEL_SKEW
         : n <= 32 * cus       ? (efficient ? S3H_KERNEL_SKEWP : S3H_KERNEL_SKEWS)
         : n <= kSkewpMaxParts ? S3H_KERNEL_SKEWP
         : n <= kPairMaxParts  ? S3H_KERNEL_PAIR
         : n <= kPcMaxParts    ? S3H_KERNEL_PC
                               : S3H_KERNEL_LANE;
}

int check_plan_args(int device, int algo, uint64_t n, int kernel) {
  if (algo != S3H_ALGO_SHA256 && algo != S3H_ALGO_MD5)
    return fail(S3H_EINVAL, "plan: unknown algorithm %d", algo);
  if (n == 0 || n > kMaxParts)
    return fail(S3H_EINVAL, "plan: need 0 < n <= 2^31 (n=%llu)", (unsigned long long)n);
  if (algo == S3H_ALGO_MD5 && kernel != S3H_KERNEL_AUTO && kernel != S3H_KERNEL_PC)
    return fail(S3H_EINVAL, "plan: MD5 supports only the producer/consumer kernel");
  if (kernel < S3H_KERNEL_AUTO || kernel > S3H_KERNEL_SKEWS)
    return fail(S3H_EINVAL, "plan: unknown kernel %d", kernel);
  return check_device(device);
}

s3h::LaunchArgs make_args(s3h_plan_s* P, const void* d_base, uint32_t* d_digests,
                          uint32_t* d_state, uint64_t b0, uint64_t b1, uint64_t origin,
                          uint32_t flags, const uint64_t* d_bits) {
  s3h::LaunchArgs A;
  A.base = static_cast<const uint8_t*>(d_base);
  A.slots = P->d_slots;
  A.out_idx = P->d_out_idx;
  A.state = d_state;
  A.digests = d_digests;
  A.zero = P->d_zero;
  A.bits = d_bits;
  A.blk_begin = b0;
  A.blk_end = b1;
  A.blk_origin = origin;
  A.n = uint32_t(P->n);
  A.flags = flags;
  A.clocks = P->d_clocks;
  A.solo = P->solo;
  A.err = P->d_err;
  return A;
}

const char* kernel_name(const s3h_plan_s* P) {
  static const char* const names[] = {"auto", "lane", "pc", "pair", "quad", "skew", "skewp", "skews"};
  if (P->algo == S3H_ALGO_MD5) return "md5";
  return P->kernel >= 0 && P->kernel <= S3H_KERNEL_SKEWS ? names[P->kernel] : "?";
}

}  // namespace

double device_power_cap_w(int device) {  // cached per device (sysfs hwmon power1_cap)
  constexpr int kMaxDev = 64;
  static std::atomic<double> cap[kMaxDev];
  static std::atomic<bool> have[kMaxDev];
  if (device < 0 || device >= kMaxDev) return 0;
  if (!have[device].load(std::memory_order_acquire)) {
    char bdf[32] = {0};
    double w = 0;
    if (hipDeviceGetPCIBusId(bdf, sizeof bdf, device) == hipSuccess) w = pci_power_cap_w(bdf);
    else (void)hipGetLastError();
    cap[device].store(w, std::memory_order_relaxed);
    have[device].store(true, std::memory_order_release);
  }
  return cap[device].load(std::memory_order_relaxed);
}

int device_cus(int device) {  // cached: the host pipeline asks once per slice
  constexpr int kMaxDev = 64;
  static std::atomic<int> cus[kMaxDev] = {};
  if (device < 0 || device >= kMaxDev) return 0;
  int c = cus[device].load(std::memory_order_relaxed);
  if (c == 0) {
    hipDeviceProp_t prop;
    c = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : -1;
    cus[device].store(c, std::memory_order_relaxed);
  }
  return c > 0 ? c : 0;
}

// Both digests of 2,049-8,192 parts (sha256_md5_group_kernel) run every chain at skewp's rate
// beside a self-fed MD5 wave: ~2,550 cycles per block on the C4 shard's equal parts (457 GiB/s
// for both), planned at 2,650 for ragged groups (exp_config.hpp S3H_EXP_DUAL_SKEWP_CYC).  A
// ragged batch is timed by its longest parts, so sha256_md5_group_mixed_kernel gives the
// longest F x 8 slots skew groups and the rest skewp groups: F = the fewest 8-slot groups
// after which every remaining part, at the skewp rate, ends before the longest part does at
// the skew rate.  Preferred form (`apart`): the skew groups' MD5 chains run on workgroups of
// their own after the skewp ones (64 chains each), so each skew group runs its SHA-256 alone
// at ~2,224 cycles per block -- C3 both digests 136.0 -> 141.5 GiB/s, the SHA-256-alone rate
// (profiles/r04_exp_dual_mixed_apart.jsonl); when that grid does not fit one workgroup per
// CU, each skew group keeps its MD5 wave (~2,280 cycles per block; round 3's form).  0 (the
// plain group kernel) when neither fits (e.g. equal lengths) or there is nothing to gain.
uint32_t dual_mixed_solo(const s3h::Slot* slots, uint64_t n, uint64_t cus, bool* apart) {
  constexpr uint64_t kSkew = 8, kSkewp = 32;
  *apart = false;
  if (n <= 2048 || cus == 0 || (n + kSkewp - 1) / kSkewp > cus) return 0;
  const double longest = double(s3h::nblocks(slots[0].len));
  for (int a = S3H_EXP_MIXED_MD5_APART; a >= 0; --a) {
    const double ratio = a ? double(S3H_EXP_DUAL_SKEWP_CYC) / S3H_EXP_DUAL_SKEW_CYC_APART
                           : double(S3H_EXP_DUAL_SKEWP_CYC) / S3H_EXP_DUAL_SKEW_CYC_INGROUP;
    uint64_t lo = 0, hi = n;  // first slot whose part ends in time at the skewp rate
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (double(s3h::nblocks(slots[mid].len)) * ratio > longest) lo = mid + 1;
      else hi = mid;
    }
    const uint64_t F = (lo + kSkew - 1) / kSkew;
    if (F == 0) return 0;  // the smaller ratio below gives no more skew groups
    // every part would need a skew group at the apart form's ratio: round 3's ratio may
    // still leave some to the skewp groups (advisor r4)
    if (F * kSkew >= n) continue;
    const uint64_t wgs = F + (n - F * kSkew + kSkewp - 1) / kSkewp + (a ? s3h::mixed_lead_wgs(F) : 0);
    if (wgs <= cus) {
      *apart = a != 0;
      return uint32_t(F);
    }
  }
  return 0;
}

// Slots in descending length order (so block counts descend too, padded or not: the kernels
// bound a workgroup's loop by its first slot); returns the total compressions.
uint64_t sort_slots(const uint64_t* offsets, const uint64_t* lengths, uint64_t n, bool nopad,
                    s3h::Slot* slots, uint32_t* order) {
  std::iota(order, order + n, 0u);
  std::stable_sort(order, order + n, [&](uint32_t a, uint32_t b) { return lengths[a] > lengths[b]; });
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    slots[i] = {offsets[order[i]], lengths[order[i]]};
    total += nopad ? lengths[order[i]] >> 6 : s3h::nblocks(lengths[order[i]]);
  }
  return total;
}

// Device arrays of a plan for up to `cap` parts (no geometry yet).  Caller holds the guard.
int plan_alloc(int device, int algo, uint64_t cap, s3h_plan_s** out) {
  auto* P = new s3h_plan_s();
  P->device = device;
  P->algo = algo;
  P->cap = cap;
  const char* what = "slots";
  hipError_t e = hipMalloc(&P->d_slots, cap * sizeof(s3h::Slot));
  if (e == hipSuccess) e = hipMalloc(&P->d_out_idx, cap * sizeof(uint32_t)), what = "output order";
  if (e == hipSuccess) e = hipMalloc(&P->d_zero, 256), what = "zero page";
  if (e == hipSuccess) e = hipMemset(P->d_zero, 0, 256);
  if (e == hipSuccess) e = hipMalloc(&P->d_err, sizeof(uint32_t)), what = "error word";
  if (e == hipSuccess) e = hipMemset(P->d_err, 0, sizeof(uint32_t));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(P->d_slots);
    (void)hipFree(P->d_out_idx);
    (void)hipFree(P->d_zero);
    (void)hipFree(P->d_err);
    delete P;
    *out = nullptr;
    return fail(e == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP,
                "plan alloc (%llu parts: %llu B of slots + %llu B of output order in HBM; failed at "
                "the %s): %s", (unsigned long long)cap, (unsigned long long)(cap * sizeof(s3h::Slot)),
                (unsigned long long)(cap * 4), what, hipGetErrorString(e));
  }
  *out = P;
  return S3H_OK;
}

// Set n parts of geometry: kernel (AUTO by n), grid and the slots sorted by block count into
// h_slots / h_order (n entries each), then copy them to the device on `s` (asynchronous when
// the host arrays are pinned; the caller keeps them alive until `s` passes the copy).
int plan_geometry(s3h_plan_s* P, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                  int kernel, s3h::Slot* h_slots, uint32_t* h_order, hipStream_t s) {
  if (n > P->cap) return fail(S3H_EINVAL, "plan: %llu parts exceed capacity %llu",
                              (unsigned long long)n, (unsigned long long)P->cap);
  P->n = n;
  P->kernel = resolve_kernel(P->algo, n, kernel, uint64_t(device_cus(P->device)), P->device);
  P->total_blocks = sort_slots(offsets, lengths, n, false, h_slots, h_order);
  P->max_blocks = s3h::nblocks(h_slots[0].len);
  P->quad_waves = quad_waves(n);
  P->solo = 0;
  if (P->kernel == S3H_KERNEL_SKEW && P->quad_waves == 2) {
#ifdef S3H_EXP_SOLO  // tools/ experiment builds only: force the solo count
    P->solo = uint32_t(std::min<uint64_t>(S3H_EXP_SOLO, (n + 7) / 8));
#else
    P->solo = plan_solo(h_slots, n, uint64_t(device_cus(P->device)));
#endif
  }
  P->dual_solo = P->algo == S3H_ALGO_SHA256
                     ? dual_mixed_solo(h_slots, n, uint64_t(device_cus(P->device)), &P->dual_apart) : 0;
  P->grid = P->solo ? P->solo + uint32_t(((n + 7) / 8 - P->solo + 1) / 2)
            : P->kernel == S3H_KERNEL_PC ? uint32_t((n + 63) / 64)
            : P->kernel == S3H_KERNEL_PAIR || P->kernel == S3H_KERNEL_SKEWP
                ? uint32_t((n + s3h::kPairParts - 1) / s3h::kPairParts)
            : P->kernel == S3H_KERNEL_QUAD || P->kernel == S3H_KERNEL_SKEW
                ? uint32_t((n + 8 * P->quad_waves - 1) / (8 * P->quad_waves))
            : P->kernel == S3H_KERNEL_SKEWS ? uint32_t((n + 31) / 32)
                : uint32_t((n + 255) / 256);
  HIP_TRY(hipMemcpyAsync(P->d_slots, h_slots, n * sizeof(s3h::Slot), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(P->d_out_idx, h_order, n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  return S3H_OK;
}

int plan_build(int device, int algo, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
               int kernel, s3h_plan_s** out) {
  *out = nullptr;
  if (!offsets || !lengths) return fail(S3H_EINVAL, "plan: need offsets and lengths");
  if (int rc = check_plan_args(device, algo, n, kernel)) return rc;
  DeviceGuard g(device);
  s3h_plan_s* P = nullptr;
  if (int rc = plan_alloc(device, algo, n, &P)) return rc;
  std::vector<uint32_t> order(n);
  std::vector<s3h::Slot> slots(n);
  int rc = plan_geometry(P, offsets, lengths, n, kernel, slots.data(), order.data(), nullptr);
  if (rc == S3H_OK && hipStreamSynchronize(nullptr) != hipSuccess)  // pageable sources
    rc = fail(S3H_EHIP, "plan upload failed");
  if (rc) {
    s3h_plan_destroy(P);
    return rc;
  }
  *out = P;
  return S3H_OK;
}

// Re-sort a plan's slots for new lengths (same n) and upload them asynchronously from
// pinned staging (the caller keeps the staging alive until `s` passes the copy).
int plan_refill(s3h_plan_s* P, const uint64_t* offsets, const uint64_t* lengths, bool nopad,
                s3h::Slot* h_slots, uint32_t* h_order, hipStream_t s) {
  P->total_blocks = sort_slots(offsets, lengths, P->n, nopad, h_slots, h_order);
  P->max_blocks = nopad ? h_slots[0].len >> 6 : s3h::nblocks(h_slots[0].len);
  if (P->kernel == S3H_KERNEL_SKEW && P->quad_waves == 2) {  // two-group grid: re-plan solos
    P->solo = plan_solo(h_slots, P->n, uint64_t(device_cus(P->device)));
    const uint64_t groups = (P->n + 7) / 8;
    P->grid = uint32_t(P->solo + (groups - P->solo + 1) / 2);
  }
  P->dual_apart = false;
  P->dual_solo = P->algo == S3H_ALGO_SHA256 && !nopad
                     ? dual_mixed_solo(h_slots, P->n, uint64_t(device_cus(P->device)), &P->dual_apart) : 0;
  HIP_TRY(hipMemcpyAsync(P->d_slots, h_slots, P->n * sizeof(s3h::Slot), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(P->d_out_idx, h_order, P->n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  return S3H_OK;
}

// Reads, and clears, plan P's device error word once `s` has run everything launched on it
// before.  S3H_EHIP when a launch reported a fault (a producer/consumer wait that timed out,
// sha256_kernels.hip flag_wait_ge): that launch's digests are not the parts' digests, so the
// call must not succeed -- lib/hash's sha256() never returns a wrong digest.
int plan_check(s3h_plan_s* P, hipStream_t s) {
  uint32_t h = 0;
  HIP_TRY(hipMemcpyAsync(&h, P->d_err, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h == 0) return S3H_OK;
  HIP_TRY(hipMemsetAsync(P->d_err, 0, sizeof h, s));
  HIP_TRY(hipStreamSynchronize(s));
  return fail(S3H_EHIP, "%s kernel: synchronisation timeout (device error word 0x%x): a producer/"
              "consumer wait timed out, the launch's digests are invalid", kernel_name(P), h);
}

int launch_args(s3h_plan_s* P, const void* d_base, uint32_t* d_digests, uint32_t* d_state,
                uint64_t b0, uint64_t b1, uint64_t origin, uint32_t flags, const uint64_t* d_bits,
                hipStream_t stream) {
  const s3h::LaunchArgs A = make_args(P, d_base, d_digests, d_state, b0, b1, origin, flags, d_bits);
  (void)hipGetLastError();  // the check below must see this launch, not an older failure
  HIP_TRY(launch_plan_kernel(P, device_cus(P->device), b1 - b0, A, stream));
  return S3H_OK;
}

int plan_launch(s3h_plan_s* P, const void* d_base, uint32_t* d_digests, uint64_t b0, uint64_t b1,
                uint64_t origin, hipStream_t stream, bool ranged) {
  if (!P || !d_base || !d_digests) return fail(S3H_EINVAL, "launch: null plan/base/digests");
  if (b1 <= b0) return S3H_OK;
  DeviceGuard g(P->device);
  if (ranged && !P->d_state) HIP_TRY(hipMalloc(&P->d_state, P->cap * 8 * sizeof(uint32_t)));
  return launch_args(P, d_base, d_digests, ranged ? P->d_state : nullptr, b0, b1, origin, 0,
                     nullptr, stream);
}

// SHA-256 (plan S) and MD5 (plan M, same parts) in ONE grid when one of the dual forms holds
// the batch; kDualNone otherwise (the caller then launches the two plans itself: one after the
// other on the device-resident path, on the two hash streams of a slice on the host path).
// Every fused grid must fit one workgroup per CU: beyond that its MD5 workgroups (the grid's
// tail) would only start as SHA-256 ones retire, i.e. run after them.
DualMode dual_mode(const s3h_plan_s* S, const s3h_plan_s* M, uint64_t b0, uint64_t b1) {
  if (M->algo != S3H_ALGO_MD5 || S->algo != S3H_ALGO_SHA256 || b1 - b0 >= (1ull << 31) ||
      S->n != M->n)
    return kDualNone;
  const uint64_t cus = uint64_t(device_cus(S->device));
#ifdef S3H_EXP_GROUP_SKEW  // tools/ experiment builds only: skew-layout group kernel
  if (S->kernel == S3H_KERNEL_SKEW && S->quad_waves == 1 && S->grid <= cus) return kDualGroupSkew;
#endif
#ifndef S3H_EXP_NO_SPLIT  // tools/ experiment builds only: never the split grid
  if (S->kernel == S3H_KERNEL_SKEW && S->quad_waves == 1 &&
      S->grid + s3h::split_md5_wgs(S->grid, S->n) <= cus)
    return kDualSplit;
#endif
  // skew plans whose split grid does not fit (1,817-2,048 parts on 256 CUs): each skew group
  // with a self-fed MD5 wave over the same 8 parts, one workgroup per CU -- both digests in
  // ~125 ms for 8 MiB parts vs 140 on the skewp group kernel (profiles/r02_exp_dual_group_skew.jsonl)
  if (S->kernel == S3H_KERNEL_SKEW && S->quad_waves == 1 && S->grid <= cus) return kDualGroupSkew;
  // the group kernel runs skewp geometry (32 parts per workgroup) whatever S's own kernel:
  // the skewp / shared-SIMD ranges and the two-group skew range (2,049-4,096 parts, whose
  // two-stream form runs MD5 workgroups on CUs already running SHA-256 ones)
  const bool group_ok = S->kernel == S3H_KERNEL_SKEWP || S->kernel == S3H_KERNEL_SKEWS ||
                        S->kernel == S3H_KERNEL_SKEW;
#ifdef S3H_EXP_NO_GROUP_NC2  // tools/ experiment builds only: round-2 behaviour
  if (S->kernel == S3H_KERNEL_SKEW) return kDualNone;
#endif
#ifndef S3H_EXP_NO_DUAL_MIXED  // tools/ experiment builds only: round-2/3 behaviour
  if (group_ok && S->dual_solo > 0) return kDualGroupMixed;
#endif
#ifdef S3H_EXP_GROUP_ANY  // tools/ experiment builds only: the group kernel at any grid size
  if (group_ok || S->kernel == S3H_KERNEL_PAIR || S->kernel == S3H_KERNEL_PC) return kDualGroup;
#endif
  if (group_ok && (S->n + 31) / 32 <= cus) return kDualGroup;
  return kDualNone;
}

int dual_launch(s3h_plan_s* S, s3h_plan_s* M, const void* d_base, uint32_t* d_sha,
                uint32_t* d_md5, uint64_t b0, uint64_t b1, uint64_t origin, bool ranged,
                hipStream_t stream) {
  const DualMode mode = dual_mode(S, M, b0, b1);
  if (mode == kDualNone) return S3H_EINVAL;
  if (b1 <= b0) return S3H_OK;
  DeviceGuard g(S->device);
  if (ranged && !S->d_state) HIP_TRY(hipMalloc(&S->d_state, S->cap * 8 * sizeof(uint32_t)));
  if (ranged && !M->d_state) HIP_TRY(hipMalloc(&M->d_state, M->cap * 8 * sizeof(uint32_t)));
  const s3h::LaunchArgs A = make_args(S, d_base, d_sha, ranged ? S->d_state : nullptr, b0, b1,
                                      origin, 0, nullptr);
  const s3h::LaunchArgs B = make_args(M, d_base, d_md5, ranged ? M->d_state : nullptr, b0, b1,
                                      origin, 0, nullptr);
  uint64_t* progress = nullptr;
  uint32_t epoch = 0;
  if (s3h::kMd5XcdPace && ((mode == kDualGroupMixed && S->dual_apart) || mode == kDualSplit)) {
    // the skew groups' producer step counts (F <= CUs groups in the mixed grid, sha_grid <= CUs
    // in the split grid; slot (g % 8) * 128 + g / 8); zeroed once, then every launch tags its
    // counts with a new epoch
    constexpr uint64_t kProgressSlots = 1024;
    const uint64_t groups = mode == kDualSplit ? S->grid : S->dual_solo;
    if (groups > kProgressSlots)
      return fail(S3H_EINVAL, "dual grid: %llu skew groups", (unsigned long long)groups);
    if (!S->d_progress) {
      HIP_TRY(hipMalloc(&S->d_progress, kProgressSlots * sizeof(uint64_t)));
      HIP_TRY(hipMemsetAsync(S->d_progress, 0, kProgressSlots * sizeof(uint64_t), stream));
    }
    if (++S->progress_epoch == 0) S->progress_epoch = 1;
    progress = S->d_progress;
    epoch = S->progress_epoch;
  }
  (void)hipGetLastError();
  HIP_TRY(launch_dual_kernel(mode, S, M, A, B, progress, epoch, stream));
  return S3H_OK;
}

}  // namespace s3h::host

using namespace s3h::host;

namespace {

// Consumer waves (= groups) of a skew/skewp grid; 0 for the kernels without a clock probe.
uint32_t consumer_groups(const s3h_plan_s* P) {
  if (P->algo == S3H_ALGO_MD5) return P->grid;  // md5_pc_kernel: one consumer wave per workgroup
  return (P->kernel == S3H_KERNEL_SKEW && P->quad_waves == 2) || P->kernel == S3H_KERNEL_SKEWS
             ? uint32_t((P->n + 7) / 8)
         : P->kernel == S3H_KERNEL_SKEW || P->kernel == S3H_KERNEL_SKEWP ? P->grid
                                                                          : 0u;
}

int batch_device(int device, int algo, const void* d_base, const uint64_t* offsets,
                 const uint64_t* lengths, uint64_t n, uint32_t* d_digests, void* stream) {
  s3h_plan_s* P = nullptr;
  if (int rc = plan_build(device, algo, offsets, lengths, n, S3H_KERNEL_AUTO, &P)) return rc;
  int rc = plan_launch(P, d_base, d_digests, 0, P->max_blocks, 0, static_cast<hipStream_t>(stream), false);
  if (rc == S3H_OK) {
    DeviceGuard g(device);
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) rc = fail(S3H_EHIP, "batch_device sync: %s", hipGetErrorString(e));
    else rc = plan_check(P, static_cast<hipStream_t>(stream));
  }
  s3h_plan_destroy(P);
  return rc;
}

}  // namespace

extern "C" {

int s3h_kernel_policy(int policy, int* previous) {
  if (policy != S3H_POLICY_THROUGHPUT && policy != S3H_POLICY_EFFICIENCY && policy != S3H_POLICY_POWER)
    return fail(S3H_EINVAL, "kernel policy: unknown policy %d", policy);
  const int prev = g_kernel_policy.exchange(policy);
  if (previous) *previous = prev;
  return S3H_OK;
}

int s3h_device_power_cap(int device, double* watts) {
  if (!watts) return fail(S3H_EINVAL, "device power cap: null argument");
  *watts = 0;
  if (int rc = check_device(device)) return rc;
  *watts = device_power_cap_w(device);
  return S3H_OK;
}

int s3h_device_count(int* count) {
  if (!count) return fail(S3H_EINVAL, "null count");
  *count = 0;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return fail(S3H_ENODEV, "no HIP device visible");
  *count = c;
  return S3H_OK;
}

int s3h_device_pci_bus_id(int device, char* out, int len) {
  if (!out || len < 13) return fail(S3H_EINVAL, "need a buffer of at least 13 bytes");
  out[0] = 0;
  if (int rc = check_device(device)) return rc;
  HIP_TRY(hipDeviceGetPCIBusId(out, len, device));
  for (char* c = out; *c; ++c) *c = char(tolower(*c));
  return S3H_OK;
}

int s3h_plan_create(int device, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                    int kernel, s3h_plan_t* plan) {
  if (!plan) return fail(S3H_EINVAL, "null plan out-pointer");
  return plan_build(device, S3H_ALGO_SHA256, offsets, lengths, n, kernel, plan);
}

int s3h_plan_create_ex(int device, int algo, const uint64_t* offsets, const uint64_t* lengths,
                       uint64_t n, int kernel, s3h_plan_t* plan) {
  if (!plan) return fail(S3H_EINVAL, "null plan out-pointer");
  return plan_build(device, algo, offsets, lengths, n, kernel, plan);
}

int s3h_plan_algo(s3h_plan_t P) { return P ? P->algo : S3H_EINVAL; }

int s3h_plan_destroy(s3h_plan_t P) {
  if (!P) return S3H_OK;
  DeviceGuard g(P->device);
  (void)hipFree(P->d_slots);
  (void)hipFree(P->d_out_idx);
  (void)hipFree(P->d_state);
  (void)hipFree(P->d_zero);
  (void)hipFree(P->d_err);
  (void)hipFree(P->d_progress);
  delete P;
  return S3H_OK;
}

int s3h_plan_status(s3h_plan_t P, void* stream) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  DeviceGuard g(P->device);
  return plan_check(P, static_cast<hipStream_t>(stream));
}

int s3h_plan_launch(s3h_plan_t P, const void* d_base, uint32_t* d_digests, void* stream) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  return plan_launch(P, d_base, d_digests, 0, P->max_blocks, 0, static_cast<hipStream_t>(stream), false);
}

int s3h_plan_launch_range(s3h_plan_t P, const void* d_base, uint32_t* d_digests, uint64_t b0,
                          uint64_t b1, uint64_t origin, void* stream) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  if (origin > b0) return fail(S3H_EINVAL, "blk_origin (%llu) > blk_begin (%llu)",
                               (unsigned long long)origin, (unsigned long long)b0);
  return plan_launch(P, d_base, d_digests, b0, b1, origin, static_cast<hipStream_t>(stream), true);
}

int s3h_plan_set_clock_probe(s3h_plan_t P, uint64_t* d_clocks, uint32_t* waves) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  P->d_clocks = d_clocks;
  if (waves) *waves = consumer_groups(P);
  return S3H_OK;
}

int s3h_plan_groups(s3h_plan_t P, uint32_t* groups, uint32_t* solo) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  if (groups) *groups = consumer_groups(P);
  if (solo) *solo = P->solo;
  return S3H_OK;
}

int s3h_plan_dual_solo(s3h_plan_t P, uint32_t* solo) {
  if (!P || !solo) return fail(S3H_EINVAL, "plan dual solo: null argument");
  *solo = P->dual_solo;
  return S3H_OK;
}

int s3h_plan_dual_layout(s3h_plan_t P, uint32_t* solo, int* apart) {
  if (!P) return fail(S3H_EINVAL, "plan dual layout: null plan");
  if (solo) *solo = P->dual_solo;
  if (apart) *apart = P->dual_apart ? 1 : 0;
  return S3H_OK;
}

int s3h_dual_layout(const uint64_t* lengths, uint64_t n, int cus, uint32_t* solo, int* apart) {
  if (!lengths || n == 0 || n > kMaxParts || cus <= 0 || !solo || !apart)
    return fail(S3H_EINVAL, "dual layout: bad argument");
  std::vector<uint64_t> offs(n, 0);
  std::vector<s3h::Slot> slots(n);
  std::vector<uint32_t> order(n);
  sort_slots(offs.data(), lengths, n, false, slots.data(), order.data());
  bool a = false;
  *solo = dual_mixed_solo(slots.data(), n, uint64_t(cus), &a);
  *apart = a ? 1 : 0;
  return S3H_OK;
}

int s3h_plan_info(s3h_plan_t P, uint64_t* n, uint64_t* total_blocks, uint64_t* max_blocks,
                  int* kernel, uint32_t* grid) {
  if (!P) return fail(S3H_EINVAL, "null plan");
  if (n) *n = P->n;
  if (total_blocks) *total_blocks = P->total_blocks;
  if (max_blocks) *max_blocks = P->max_blocks;
  if (kernel) *kernel = P->kernel;
  if (grid) *grid = P->grid;
  return S3H_OK;
}

int s3h_sha256_batch_device(int device, const void* d_base, const uint64_t* offsets,
                            const uint64_t* lengths, uint64_t n, uint32_t* d_digests,
                            void* stream) {
  return batch_device(device, S3H_ALGO_SHA256, d_base, offsets, lengths, n, d_digests, stream);
}

int s3h_md5_batch_device(int device, const void* d_base, const uint64_t* offsets,
                         const uint64_t* lengths, uint64_t n, uint32_t* d_digests, void* stream) {
  return batch_device(device, S3H_ALGO_MD5, d_base, offsets, lengths, n, d_digests, stream);
}

int s3h_sha256_md5_batch_device(int device, const void* d_base, const uint64_t* offsets,
                                const uint64_t* lengths, uint64_t n, uint32_t* d_sha256,
                                uint32_t* d_md5, void* stream) {
  if (!d_base || !d_sha256 || !d_md5) return fail(S3H_EINVAL, "dual batch: null pointer");
  s3h_plan_s* P[2] = {};
  struct Cleanup {
    s3h_plan_s** P;
    ~Cleanup() {
      s3h_plan_destroy(P[0]);
      s3h_plan_destroy(P[1]);
    }
  } C{P};
  if (int rc = plan_build(device, S3H_ALGO_SHA256, offsets, lengths, n, S3H_KERNEL_AUTO, &P[0])) return rc;
  if (int rc = plan_build(device, S3H_ALGO_MD5, offsets, lengths, n, S3H_KERNEL_AUTO, &P[1])) return rc;
  DeviceGuard g(device);
  hipStream_t main_s = static_cast<hipStream_t>(stream);
  if (dual_mode(P[0], P[1], 0, P[0]->max_blocks) != kDualNone) {  // one grid: both digests
    if (int rc = dual_launch(P[0], P[1], d_base, d_sha256, d_md5, 0, P[0]->max_blocks, 0, false,
                             main_s))
      return rc;
    HIP_TRY(hipStreamSynchronize(main_s));
    return plan_check(P[0], main_s);  // the one grid reports into S's word
  }
  // Otherwise (more parts than the one-grid forms hold: > 32 x CUs) both kernels fill the chip
  // on their own, and run one after the other on the caller's stream.  Round 1-3 ran MD5 on a
  // side stream beside SHA-256; measured on one box (256 KiB parts, both digests, GiB/s):
  // 9,000 parts 294 two streams -> 315 in order, 12,288 397 -> 420, 16,384 515 -> 543,
  // 32,768 523 -> 609, 65,536 692 -> 796 (profiles/r04_exp_dual_serial.jsonl): concurrent
  // grids only contend for the same SIMDs.
  if (int rc = plan_launch(P[0], d_base, d_sha256, 0, P[0]->max_blocks, 0, main_s, false)) return rc;
  if (int rc = plan_launch(P[1], d_base, d_md5, 0, P[1]->max_blocks, 0, main_s, false)) return rc;
  HIP_TRY(hipStreamSynchronize(main_s));
  if (int rc = plan_check(P[0], main_s)) return rc;
  return plan_check(P[1], main_s);
}

int s3h_verify_batch_device(int device, int algo, const void* d_base, const uint64_t* offsets,
                            const uint64_t* lengths, uint64_t n, const uint32_t* d_expected,
                            uint8_t* d_mismatch, uint64_t* mismatches, void* stream) {
  if (!d_expected || !d_mismatch || !mismatches) return fail(S3H_EINVAL, "verify: null argument");
  s3h_plan_s* P = nullptr;
  if (int rc = plan_build(device, algo, offsets, lengths, n, S3H_KERNEL_AUTO, &P)) return rc;
  struct Cleanup {
    s3h_plan_s* P;
    ~Cleanup() { s3h_plan_destroy(P); }
  } cleanup{P};
  DeviceGuard g(device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t dw = digest_words(algo);
  uint32_t* d_dig = nullptr;
  unsigned long long* d_count = nullptr;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d_dig), n * dw * 4, s));
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d_count), 8, s));
  HIP_TRY(hipMemsetAsync(d_count, 0, 8, s));
  int rc = plan_launch(P, d_base, d_dig, 0, P->max_blocks, 0, s, false);
  if (rc == S3H_OK) {
    unsigned long long c = 0;
    hipError_t e = launch_compare_digests(d_dig, d_expected, n, dw, d_mismatch, d_count, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&c, d_count, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) rc = fail(S3H_EHIP, "verify: %s", hipGetErrorString(e));
    else rc = plan_check(P, s);  // a faulted launch verifies nothing
    *mismatches = c;
  }
  (void)hipFreeAsync(d_dig, s);
  (void)hipFreeAsync(d_count, s);
  (void)hipStreamSynchronize(s);
  return rc;
}

int s3h_generate_parts(int device, void* d_base, const uint64_t* offsets, const uint64_t* lengths,
                       const uint64_t* part_ids, uint64_t n, uint64_t seed, void* stream) {
  if (!d_base || !offsets || !lengths || !part_ids || n == 0 || n > 65535)
    return fail(S3H_EINVAL, "generate: bad arguments (n must be in [1, 65535] per call)");
  if (int rc = check_device(device)) return rc;
  std::vector<s3h::GenPart> g(n);
  uint64_t maxlen = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i] % 8) return fail(S3H_EINVAL, "generate: offsets must be 8-byte aligned");
    g[i] = {offsets[i], lengths[i], part_ids[i]};
    maxlen = std::max(maxlen, lengths[i]);
  }
  DeviceGuard dg(device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  s3h::GenPart* d_g = nullptr;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d_g), n * sizeof(s3h::GenPart), s));
  HIP_TRY(hipMemcpyAsync(d_g, g.data(), n * sizeof(s3h::GenPart), hipMemcpyHostToDevice, s));
  const uint64_t words = (maxlen + 7) / 8;
  const uint32_t gx = uint32_t(std::min<uint64_t>(std::max<uint64_t>((words + 255) / 256, 1), 256));
  (void)hipGetLastError();
  HIP_TRY(launch_generate(static_cast<uint8_t*>(d_base), d_g, uint32_t(n), gx, seed, s));
  HIP_TRY(hipFreeAsync(d_g, s));
  // the host vector `g` must outlive the async copy
  HIP_TRY(hipStreamSynchronize(s));
  return S3H_OK;
}

}  // extern "C"
