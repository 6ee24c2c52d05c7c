// capi.hip -- host side of the C-ABI in include/s3hash.h.
//
// Everything here is plumbing around the kernels of sha256_kernels.hip: plan building
// (host-side sort by block count), launches, the host-resident streaming path and the
// multi-GPU sharding.  No entry point ever computes a digest on the CPU for the batched API:
// with no HIP device every call fails with S3H_ENODEV.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/s3hash.h"
#include "sha256_kernels.hip"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// A failed call also clears the thread's last HIP error: a later hipGetLastError after a
// launch must report that launch, not an allocation that failed (and was reported) before.
#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      (void)hipGetLastError();                                                             \
      return fail(e_ == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "%s: %s (%s:%d)",     \
                  #expr, hipGetErrorString(e_), __FILE__, __LINE__);                       \
    }                                                                                      \
  } while (0)

int check_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(S3H_ENODEV, "no HIP device visible (the batched SHA-256 path has no CPU fallback)");
  if (device < 0 || device >= count) return fail(S3H_EINVAL, "device %d out of range [0,%d)", device, count);
  return S3H_OK;
}

struct DeviceGuard {  // restores the calling thread's current device
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

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
};

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
constexpr uint64_t kMaxParts = 1ull << 31;

uint32_t digest_words(int algo) { return algo == S3H_ALGO_MD5 ? 4u : 8u; }

// Skew / quad kernels: consumer waves per workgroup -- the fewest that keep the grid within
// one workgroup per CU (256): one up to 2,048 parts, two up to 4,096 (kQuadMaxParts).
int quad_waves(uint64_t n) {
#ifdef S3H_EXP_FORCE_NC  // tools/ experiment builds only
  return S3H_EXP_FORCE_NC;
#endif
  return n <= 256ull * s3h::kQuadChainsPerWave ? 1 : 2;
}

// Slots in descending length order (so block counts descend too, padded or not: the kernels
// bound a workgroup's loop by its first slot); returns the total compressions.
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

// Both digests of 2,049-8,192 parts (sha256_md5_group_kernel) run every chain at skewp's rate
// beside a self-fed MD5 wave: ~2,550 cycles per block (C4 shard, 457 GiB/s for both).  A
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
    const double ratio = a ? 2550.0 / 2224.0 : 2550.0 / 2280.0;
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
    const uint64_t wgs = F + (n - F * kSkew + kSkewp - 1) / kSkewp + (a ? (8 * F + 63) / 64 : 0);
    if (wgs <= cus) {
      *apart = a != 0;
      return uint32_t(F);
    }
  }
  return 0;
}

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

// `cus`: the device's CUs.  Above 4,096 parts, while one 32-chain workgroup per CU holds the
// batch (8,192 parts on MI355X: the C4 shard), the shared-SIMD skew kernel runs every chain
// at the skew kernel's 8 VALU per round with its producer on the same SIMD: C4 shard 500 vs
// 469 GiB/s for skewp on one box (profiles/r02_bench_c4_skews_mulf.jsonl), at about twice the
// board power (r02_smi_c4_power.txt; INTEGRATION.md: pass S3H_KERNEL_SKEWP to trade it back).
// Under S3H_POLICY_EFFICIENCY (s3h_kernel_policy; env S3H_PREFER_EFFICIENCY=1) AUTO keeps
// skewp in that range: the C4 shard runs 8.6 % slower (464 vs 504 GiB/s) but at 1.66 instead
// of 2.44 J/GiB (board 0.77 vs 1.23 kW, BENCH_r04 configs.c4.kernels) --
// the lower energy-delay product (J/GiB x s/GiB: 3.6e-3 vs 4.9e-3).  Outside 4,097 - 32 x CUs
// parts both policies choose the same kernel.
std::atomic<int> g_kernel_policy{[] {
  const char* e = std::getenv("S3H_PREFER_EFFICIENCY");
  return e && std::atoi(e) == 1 ? S3H_POLICY_EFFICIENCY : S3H_POLICY_THROUGHPUT;
}()};

int resolve_kernel(int algo, uint64_t n, int kernel, uint64_t cus) {
  if (algo == S3H_ALGO_MD5) return S3H_KERNEL_PC;  // MD5 has one kernel (4 VALU per step)
  if (kernel != S3H_KERNEL_AUTO) return kernel;
  const bool efficient = g_kernel_policy.load() == S3H_POLICY_EFFICIENCY;
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
  P->kernel = resolve_kernel(P->algo, n, kernel, uint64_t(device_cus(P->device)));
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

// One launch of P's kernel over blocks [b0, b1) (caller holds the device guard).
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

// Dynamic LDS added to a grid with solo workgroups: 72 KiB of groups + 12 KiB > half of the
// CU's 160 KiB, so one workgroup per CU and a solo group never shares its CU.
constexpr uint32_t kSoloLdsPad = 12 * 1024;
// sha256_md5_group_mixed_kernel: 66 KiB of skewp LDS + this > half of the CU's 160 KiB.
constexpr uint32_t kMixedLdsPad = 16 * 1024;
static_assert(sizeof(s3h::SkewLds<1, true>) + kMixedLdsPad > 80 * 1024, "one mixed workgroup per CU");

int launch_args(s3h_plan_s* P, const void* d_base, uint32_t* d_digests, uint32_t* d_state,
                uint64_t b0, uint64_t b1, uint64_t origin, uint32_t flags, const uint64_t* d_bits,
                hipStream_t stream) {
  const s3h::LaunchArgs A = make_args(P, d_base, d_digests, d_state, b0, b1, origin, flags, d_bits);
  (void)hipGetLastError();  // the check below must see this launch, not an older failure
  if (P->algo == S3H_ALGO_MD5 && P->grid <= uint64_t(device_cus(P->device)))
    hipLaunchKernelGGL(s3h::md5_pc_kernel<s3h::kMd5Bps>, dim3(P->grid), dim3(s3h::kPcThreads), 0,
                       stream, A);
  else if (P->algo == S3H_ALGO_MD5)  // more workgroups than CUs: the 32 KiB form, several per CU
    hipLaunchKernelGGL(s3h::md5_pc_kernel<1>, dim3(P->grid), dim3(s3h::kPcThreads), 0, stream, A);
  // The skew kernel counts a launch's blocks in 32 bits: a range of 2^31 blocks (128 GiB of
  // one part) or more runs on the quad kernel (same plan geometry, 64-bit counters).
  else if (P->kernel == S3H_KERNEL_SKEW && b1 - b0 >= (1ull << 31) && P->quad_waves == 1)
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<1>, dim3(P->grid), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEW && b1 - b0 >= (1ull << 31))
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<2>, dim3(P->grid), dim3(192), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWS && b1 - b0 >= (1ull << 31))
    hipLaunchKernelGGL(s3h::sha256_quad_kernel<1>, dim3(uint32_t((P->n + 7) / 8)), dim3(128), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWS)
    hipLaunchKernelGGL(s3h::sha256_skew_shared_kernel, dim3(P->grid), dim3(512), 0, stream, A);
  else if (P->kernel == S3H_KERNEL_SKEWP && b1 - b0 >= (1ull << 31))
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
  HIP_TRY(hipGetLastError());
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

// SHA-256 (plan S) and MD5 (plan M, same parts) in ONE grid (sha256_md5_dual_kernel) when S
// runs a 128-thread skew body; returns S3H_EINVAL without launching otherwise (the caller
// then launches the two plans itself: one after the other on the device-resident path, on the
// two hash streams of a slice on the host path).
// The fused grid must fit one workgroup per CU: beyond that its MD5 workgroups (the grid's
// tail) would only start as SHA-256 ones retire, i.e. run after them.

// How one grid can produce both digests of plan S (SHA-256) and plan M (MD5, same parts in
// the same order): kDualSplit = sha256_md5_dual_kernel (skew with one consumer per workgroup:
// S's workgroups then M's, all within one workgroup per CU); kDualGroup =
// sha256_md5_group_kernel (skewp: each workgroup runs a SHA-256 group and a self-fed MD5 wave
// over the same 32 parts, S->grid <= one per CU); kDualNone = two separate launches.
// kDualGroupMixed = sha256_md5_group_mixed_kernel (ragged 2,049-8,192 parts: the longest
// parts in skew groups, the rest as kDualGroup; S->dual_solo skew workgroups).
enum DualMode { kDualNone = 0, kDualSplit = 1, kDualGroup = 2, kDualGroupSkew = 3, kDualGroupMixed = 4 };

DualMode dual_mode(const s3h_plan_s* S, const s3h_plan_s* M, uint64_t b0, uint64_t b1) {
  if (M->algo != S3H_ALGO_MD5 || S->algo != S3H_ALGO_SHA256 || b1 - b0 >= (1ull << 31) ||
      S->n != M->n)
    return kDualNone;
  const uint64_t cus = uint64_t(device_cus(S->device));
#ifdef S3H_EXP_GROUP_SKEW  // tools/ experiment builds only: skew-layout group kernel
  if (S->kernel == S3H_KERNEL_SKEW && S->quad_waves == 1 && S->grid <= cus) return kDualGroupSkew;
#endif
#ifndef S3H_EXP_NO_SPLIT  // tools/ experiment builds only: never the split grid
  if (S->kernel == S3H_KERNEL_SKEW && S->quad_waves == 1 && S->grid + M->grid <= cus)
    return kDualSplit;
#endif
  // skew plans whose split grid does not fit (1,821-2,048 parts on 256 CUs): each skew group
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
  if (mode == kDualGroup)
    hipLaunchKernelGGL(s3h::sha256_md5_group_kernel<true>, dim3(uint32_t((S->n + 31) / 32)),
                       dim3(192), 0, stream, A, B);
  else if (mode == kDualGroupMixed) {  // the LDS pad keeps one workgroup per CU
    const uint32_t F = S->dual_solo, G = uint32_t((S->n - 8ull * F + 31) / 32);
    const uint32_t lead = S->dual_apart ? (8 * F + 63) / 64 : 0;
    hipLaunchKernelGGL(s3h::sha256_md5_group_mixed_kernel, dim3(F + G + lead), dim3(192),
                       kMixedLdsPad, stream, A, B, F, G, lead);
  }
  else if (mode == kDualGroupSkew)
    hipLaunchKernelGGL(s3h::sha256_md5_group_kernel<false>, dim3(uint32_t((S->n + 7) / 8)),
                       dim3(192), 0, stream, A, B);
  else
    hipLaunchKernelGGL(s3h::sha256_md5_dual_kernel<false>, dim3(S->grid + M->grid), dim3(128), 0,
                       stream, A, B, uint32_t(S->grid));
  HIP_TRY(hipGetLastError());
  return S3H_OK;
}

// ------------------------------------------------------------------ host streaming path
// CPUs this process may use: its affinity mask, capped by a cgroup CPU quota (v2 cpu.max, v1
// cfs_quota_us / cfs_period_us), at least 1.  The reference's jobs run as std::async threads
// on whatever the host grants (lib/src/upload.cpp:136-140); hardware_concurrency() counts the
// machine's CPUs instead -- 256 on the GPU box, whose container quota is 16, where
// over-subscribed copy threads halved the staging rate (BENCH_r02 cpu_baseline.GiBps_by_threads).
double cgroup_cpu_quota() {
  double q = 0, per = 0;
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char a[32] = {0};
    const int got = std::fscanf(f, "%31s %lf", a, &per);
    std::fclose(f);
    if (got == 2 && std::strcmp(a, "max") != 0 && per > 0) return std::atof(a) / per;
    if (got >= 1) return 0;  // "max": unlimited
  }
  FILE* fq = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r");
  FILE* fp = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r");
  if (fq && fp && std::fscanf(fq, "%lf", &q) == 1 && std::fscanf(fp, "%lf", &per) == 1 && q > 0 &&
      per > 0) {
    std::fclose(fq);
    std::fclose(fp);
    return q / per;
  }
  if (fq) std::fclose(fq);
  if (fp) std::fclose(fp);
  return 0;
}

unsigned host_cpus() {
  static const unsigned cpus = [] {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) n = unsigned(CPU_COUNT(&set));
    const double quota = cgroup_cpu_quota();
    if (quota > 0) n = std::min(n, std::max(1u, unsigned(std::ceil(quota))));
    return n;
  }();
  return cpus;
}

// Host threads (the calling thread included) each of `ndevices` concurrent device shards may
// use to stage its parts: the process's CPUs split evenly, at least 1, at most 16.
unsigned host_threads_per_device(int ndevices) {
  return std::min(16u, std::max(1u, host_cpus() / unsigned(std::max(1, ndevices))));
}

// ------------------------------------------------------------------ NUMA placement
// MI355X nodes are dual-socket hosts with four GPUs behind each socket (the GPU box: devices
// on node 1, CPUs 64-127,192-255 local to them).  A device's DMA reads host memory through
// its socket's root complex, so the pinned staging it copies from and the threads that fill
// that staging (memcpy / pread) belong on the device's node: the sysfs numa_node and
// local_cpulist of its PCI function.  The reference's jobs run wherever the host schedules
// them (lib/src/upload.cpp:136-140 std::async, ReadFile lib/src/webclient.cpp:105-116).
// S3H_SYSFS_ROOT (tests) replaces /sys.  Placement policy: s3h_host_numa (env S3H_HOST_NUMA
// = local | off | <node>) -- device-local by default.
constexpr int kMpolBind = 2;
constexpr int kMpolFNode = 1, kMpolFAddr = 2;
constexpr unsigned kMaxNumaNodes = 1024;

std::string sysfs_root() {
  const char* e = std::getenv("S3H_SYSFS_ROOT");
  return e && *e ? std::string(e) : std::string("/sys");
}

bool read_line(const std::string& path, std::string* out) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const bool ok = std::fgets(buf, sizeof buf, f) != nullptr;
  std::fclose(f);
  if (!ok) return false;
  *out = buf;
  while (!out->empty() && std::isspace(static_cast<unsigned char>(out->back()))) out->pop_back();
  return true;
}

// "0-63,128-191" -> set; false when malformed (an empty list is a valid empty set)
bool parse_cpulist(const std::string& s, cpu_set_t* set) {
  CPU_ZERO(set);
  const char* p = s.c_str();
  while (*p) {
    char* end = nullptr;
    const long a = std::strtol(p, &end, 10);
    if (end == p || a < 0) return false;
    long b = a;
    p = end;
    if (*p == '-') {
      b = std::strtol(p + 1, &end, 10);
      if (end == p + 1 || b < a) return false;
      p = end;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(int(c), set);
    if (*p == ',') ++p;
    else if (*p) return false;
  }
  return true;
}

// sysfs NUMA record of one PCI function: node (-1 when the platform gives none) and the
// CPUs local to it.  S3H_EINVAL when <root>/bus/pci/devices/<bdf> does not exist.
int pci_numa(const char* bdf, int* node, std::string* cpulist) {
  if (!bdf || !*bdf) return fail(S3H_EINVAL, "pci numa: empty PCI address");
  std::string b(bdf);
  for (char& c : b) c = char(std::tolower(static_cast<unsigned char>(c)));
  const std::string dir = sysfs_root() + "/bus/pci/devices/" + b;
  std::string v;
  if (!read_line(dir + "/numa_node", &v))
    return fail(S3H_EINVAL, "pci numa: cannot read %s/numa_node", dir.c_str());
  *node = std::atoi(v.c_str());
  if (*node < 0) *node = -1;
  if (!read_line(dir + "/local_cpulist", cpulist)) cpulist->clear();
  return S3H_OK;
}

// CPUs of a NUMA node (<root>/devices/system/node/node<k>/cpulist)
bool node_cpulist(int node, std::string* cpulist) {
  return node >= 0 && read_line(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", cpulist);
}

// Node of the page holding p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR); -1 if unknown.
int mem_node(const void* p) {
  int node = -1;
  if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0, p, kMpolFNode | kMpolFAddr) != 0) return -1;
  return node;
}

// Pinned host memory whose pages live on `node`: anonymous pages bound there (mbind
// MPOL_BIND), touched, then page-locked for DMA with hipHostRegister.  node < 0: the
// runtime's own hipHostMalloc.  pinned_free releases either kind.
std::mutex g_reg_mu;
std::vector<std::pair<void*, size_t>>& registered_bufs() {
  static auto* v = new std::vector<std::pair<void*, size_t>>();
  return *v;
}

hipError_t pinned_alloc(void** out, uint64_t bytes, int node) {
  *out = nullptr;
  if (node < 0 || node >= int(kMaxNumaNodes)) return hipHostMalloc(out, bytes, hipHostMallocDefault);
  const size_t len = std::max<size_t>(size_t(bytes), 1);
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return hipErrorOutOfMemory;
  unsigned long mask[kMaxNumaNodes / 64] = {};
  mask[node / 64] = 1ul << (node % 64);
  if (syscall(SYS_mbind, p, len, kMpolBind, mask, kMaxNumaNodes + 1, 0) != 0) {
    munmap(p, len);  // node not allowed (cpuset mems) or absent: the runtime's placement
    return hipHostMalloc(out, bytes, hipHostMallocDefault);
  }
  // first touch under the binding (large buffers: 8 threads, ~0.2 s for 8 GiB instead of ~2)
  const unsigned toucher = len >= (64u << 20) ? std::min(8u, host_cpus()) : 1u;
  std::vector<std::thread> ts;
  const size_t per = (len / toucher + 4095) & ~size_t(4095);
  for (unsigned t = 1; t < toucher; ++t)
    if (t * per < len)
      ts.emplace_back([=] { std::memset(static_cast<char*>(p) + t * per, 0, std::min(per, len - t * per)); });
  std::memset(p, 0, std::min(per, len));
  for (auto& th : ts) th.join();
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, len);
    return e;
  }
  std::lock_guard<std::mutex> l(g_reg_mu);
  registered_bufs().push_back({p, len});
  *out = p;
  return hipSuccess;
}

void pinned_free(void* p) {
  if (!p) return;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> l(g_reg_mu);
    auto& v = registered_bufs();
    for (auto it = v.begin(); it != v.end(); ++it)
      if (it->first == p) {
        len = it->second;
        v.erase(it);
        break;
      }
  }
  if (len) {
    (void)hipHostUnregister(p);
    munmap(p, len);
  } else {
    (void)hipHostFree(p);
  }
}

// Placement policy: kNumaLocal (the device's node), kNumaOff (no binding), or a forced node
// (measurements: the remote-node side of an A/B).  Changing it re-places the next contexts.
constexpr int kNumaLocal = -1, kNumaOff = -2;
std::atomic<int> g_numa_mode{[] {
  const char* e = std::getenv("S3H_HOST_NUMA");
  if (!e || !*e || std::strcmp(e, "local") == 0) return kNumaLocal;
  if (std::strcmp(e, "off") == 0) return kNumaOff;
  return std::isdigit(static_cast<unsigned char>(e[0])) ? std::atoi(e) : kNumaLocal;
}()};

// Where the host path puts device `device`'s pinned staging and copy threads under the
// current policy: target node (-1 = none) and the CPUs to bind to (the node's CPUs within
// this thread's affinity mask; empty = unbound).
struct Place {
  int dev_node = -1;  // sysfs numa_node of the device (-1: unknown)
  int node = -1;      // staging target
  cpu_set_t cpus;
  int ncpus = 0;
  Place() { CPU_ZERO(&cpus); }
};

Place device_place(int device) {
  Place P;
  char bdf[32] = {0};
  std::string local;
  if (hipDeviceGetPCIBusId(bdf, sizeof bdf, device) == hipSuccess) {
    if (pci_numa(bdf, &P.dev_node, &local) != S3H_OK) {
      P.dev_node = -1;
      local.clear();
    }
  } else {
    (void)hipGetLastError();
  }
  const int mode = g_numa_mode.load();
  if (mode == kNumaOff) return P;
  P.node = mode == kNumaLocal ? P.dev_node : mode;
  if (P.node < 0) return P;
  std::string list = mode == kNumaLocal ? local : std::string();
  if (list.empty()) node_cpulist(P.node, &list);
  cpu_set_t want, mine;
  if (!parse_cpulist(list, &want) || sched_getaffinity(0, sizeof mine, &mine) != 0) return P;
  (void)CPU_AND(&P.cpus, &want, &mine);
  P.ncpus = CPU_COUNT(&P.cpus);
  return P;
}

void bind_self(const Place& P) {
  if (P.ncpus > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof P.cpus, &P.cpus);
}

// Host threads that fill a pinned staging slot from pageable part memory (one task per part
// slice).  DMA straight from pageable memory goes through the runtime's bounce buffer and
// serialises with the host; staging keeps the copy engine fed from pinned memory.
class CopyPool {
 public:
  // Workers bound to place.cpus (the device's node) when that set is non-empty.
  CopyPool(unsigned workers, const Place& place) : bound_(place.ncpus > 0 ? place.node : -1) {
    for (unsigned i = 0; i < workers; ++i)
      threads_.emplace_back([this, place] {
        bind_self(place);
        loop();
      });
  }
  int bound_node() const { return bound_; }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  unsigned size() const { return unsigned(threads_.size()); }
  // fn(i) for every i in [0, n), on the workers and the calling thread; returns when done.
  void run(uint64_t n, const std::function<void(uint64_t)>& fn) {
    {
      std::lock_guard<std::mutex> l(m_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      busy_ = threads_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (uint64_t i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> l(m_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  int bound_ = -1;
  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(uint64_t)>* fn_ = nullptr;
  std::atomic<uint64_t> next_{0};
  uint64_t n_ = 0, gen_ = 0;
  size_t busy_ = 0;
  bool stop_ = false;
};

// ------------------------------------------------------------------ host-path context
// Everything one host-path call needs on a device -- streams, ring events, the copy-thread
// pool, plans, digest buffers, the pinned geometry staging, the HBM ring and the pinned
// staging ring -- is cached per device and reused by the next call (an uploader hashes file
// after file; creating and freeing these per call cost ~8 ms of a 27 ms call on a 512 MiB
// file, profiles/r01_app_upload_hash.txt).  Buffers only grow; an HBM ring above
// kKeepRingBytes is freed when the call returns, so a cached context holds at most
// kKeepRingBytes of HBM plus its staging; s3h_trim() frees idle contexts.
constexpr int kHostRing = 3;
// Host-form stream updates (s3h_stream_update_host): pinned host pieces of the staged copy
// (two, filled alternately); pinned ragged chunks DMA'd one by one only up to this many per
// update (more: staged -- a DMA per 1 MiB chunk costs more than a memcpy); updates above
// 2 x kStreamSubBytes are split into sub-updates of ~kStreamSubBytes (>= kStreamSubMin of
// every chunk) whose copies overlap the hash of the one before.
constexpr uint64_t kStreamPiece = 64ull << 20;
constexpr uint64_t kStreamDmaChunks = 64;
constexpr uint64_t kStreamSubBytes = 128ull << 20;
constexpr uint64_t kStreamSubMin = 64ull << 10;
constexpr int kHostMaxAlgo = 2;
constexpr uint64_t kStageSlot = 32ull << 20;     // pinned staging bytes per ring slot
// Group mode (run_host_groups) for many small parts: parts of at most kGroupMaxPart; a group's
// copy must outlast its longest part's chain (~69 MB/s per chain vs ~52 GB/s of PCIe: 750 x),
// groups between kGroupMin and kGroupMax bytes.
constexpr uint64_t kGroupMaxPart = 1ull << 20;
// Groups of 1,536 x the longest part where two of them fit the HBM ring a context keeps
// between calls (release_large), else 768 x: 20,000 / 100,000 pinned parts of <= 128 KiB at
// 768 x 40.9 / 46.8 GiB/s, at 1,536 x 46.7 / 49.6 (profiles/r05_group_sweep.log).
constexpr uint64_t kGroupCopyPerChain = 1536, kGroupCopyPerChainMin = 768;
constexpr uint64_t kGroupMin = 64ull << 20, kGroupMax = 1ull << 30;
constexpr uint64_t kKeepRingBytes = 1ull << 30;  // largest HBM ring kept between calls
constexpr uint64_t kGroupChunk = 64ull << 20;    // group mode: pinned staging per packed chunk
constexpr uint64_t kPinnedStageMin = 256;        // ragged pinned parts beyond this are staged
// Staged slices are at least 32 KiB up to 4,096 parts per device (slots of up to 128 MiB),
// 128 MiB / n beyond: a file range's pread costs more than it moves below ~32 KiB, and each
// slice of memory parts costs a copy-thread dispatch and a launch (4,000 parts of U[256 KiB,
// 4 MiB] in 8 KiB slices: 512 slices, 26.6 GiB/s).
constexpr uint64_t kFileStageSlot = 128ull << 20;

// One part of a merged batch (concurrent callers, below): host memory or a file range.
struct PartRef {
  const uint8_t* mem;
  int fd;
  uint64_t off;
};

// Where a shard's part bytes come from: host memory (pinned or pageable), byte ranges of an
// open file (read with pread straight into the pinned staging ring), or per-part references
// (a batch merged from concurrent calls whose sources differ).
struct PartSource {
  const uint8_t* const* parts = nullptr;  // memory parts, or null for a file / refs
  int fd = -1;                            // file parts: part i = [file_off[i], +lengths[i])
  const uint64_t* file_off = nullptr;
  const PartRef* refs = nullptr;
  PartRef ref(uint64_t i) const {
    if (parts) return {parts[i], -1, 0};
    if (refs) return refs[i];
    return {nullptr, fd, file_off[i]};
  }
  bool fill(uint64_t i, uint64_t byte0, uint64_t cnt, uint8_t* dst) const {
    const PartRef r = ref(i);
    if (r.mem) {
      std::memcpy(dst, r.mem + byte0, cnt);
      return true;
    }
    for (uint64_t done = 0; done < cnt;) {
      const ssize_t r2 = pread(r.fd, dst + done, cnt - done, off_t(r.off + byte0 + done));
      if (r2 < 0 && errno == EINTR) continue;
      if (r2 <= 0) return false;  // error or a part past the end of the file
      done += uint64_t(r2);
    }
    return true;
  }
};

struct HostCtx {
  int device = 0;
  Place place;  // NUMA node of the pinned staging and CPUs of the copy threads (device_place)
  hipStream_t copy_s = nullptr, hash_s[kHostMaxAlgo] = {};
  hipEvent_t copied[kHostRing] = {}, hashed[kHostRing][kHostMaxAlgo] = {};
  hipEvent_t chunk_copied[kHostRing] = {};  // group mode: a staging chunk's DMA has run
  std::unique_ptr<CopyPool> pool;
  s3h_plan_s* plan[kHostMaxAlgo] = {};
  uint32_t* d_dig[kHostMaxAlgo] = {};
  uint64_t dig_bytes[kHostMaxAlgo] = {};
  uint8_t* pin = nullptr;    // pinned slot/order staging of both plans' geometry
  uint64_t pin_bytes = 0;
  uint8_t* ring = nullptr;   // HBM ring: kHostRing slots of n * slice bytes
  uint64_t ring_bytes = 0;
  uint8_t* stage = nullptr;  // pinned staging ring (pageable and file sources)
  uint64_t stage_bytes = 0;
  // group mode (run_host_groups): two plans per algorithm (group k uses set k & 1) and their
  // pinned geometry staging
  s3h_plan_s* gplan[2][kHostMaxAlgo] = {};
  uint8_t* gpin = nullptr;
  uint64_t gpin_bytes = 0;

  hipError_t ensure_streams() {
    hipError_t e = hipSuccess;
    if (!copy_s) e = hipStreamCreateWithFlags(&copy_s, hipStreamNonBlocking);
    for (hipStream_t& st : hash_s)
      if (e == hipSuccess && !st) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int r = 0; r < kHostRing && e == hipSuccess; ++r) {
      if (!copied[r]) e = hipEventCreateWithFlags(&copied[r], hipEventDisableTiming);
      if (e == hipSuccess && !chunk_copied[r]) e = hipEventCreateWithFlags(&chunk_copied[r], hipEventDisableTiming);
      for (hipEvent_t& h : hashed[r])
        if (e == hipSuccess && !h) e = hipEventCreateWithFlags(&h, hipEventDisableTiming);
    }
    return e;
  }
  static hipError_t grow_dev(uint8_t** p, uint64_t* have, uint64_t want) {
    if (*have >= want) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    const hipError_t e = hipMalloc(p, want);
    if (e == hipSuccess) *have = want;
    return e;
  }
  // pinned host buffers on the context's NUMA node (place.node; < 0: the runtime's choice)
  hipError_t grow_pinned(uint8_t** p, uint64_t* have, uint64_t want) {
    if (*have >= want) return hipSuccess;
    pinned_free(*p);
    *p = nullptr;
    *have = 0;
    const hipError_t e = pinned_alloc(reinterpret_cast<void**>(p), want, place.node);
    if (e == hipSuccess) *have = want;
    return e;
  }
  hipError_t ensure_digests(int a, uint64_t bytes) {
    return grow_dev(reinterpret_cast<uint8_t**>(&d_dig[a]), &dig_bytes[a], bytes);
  }
  CopyPool* ensure_pool(unsigned workers) {  // exactly `workers` threads beside the caller
    if (!pool || pool->size() != workers) pool.reset(new CopyPool(workers, place));
    return pool.get();
  }
  // plan[a] for algorithm `algo` with room for n parts (reallocated only to grow)
  int ensure_plan(int a, int algo, uint64_t n) {
    if (plan[a] && plan[a]->algo == algo && plan[a]->cap >= n) return S3H_OK;
    s3h_plan_destroy(plan[a]);
    plan[a] = nullptr;
    return plan_alloc(device, algo, std::max<uint64_t>(n, 1024), &plan[a]);
  }
  // pinned geometry staging for plan a: cap slots + cap order entries
  s3h::Slot* h_slots(int a) {
    return reinterpret_cast<s3h::Slot*>(pin) + uint64_t(a) * pin_cap();
  }
  uint32_t* h_order(int a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<s3h::Slot*>(pin) + kHostMaxAlgo * pin_cap()) +
           uint64_t(a) * pin_cap();
  }
  uint64_t pin_cap() const { return pin_bytes / (kHostMaxAlgo * (sizeof(s3h::Slot) + 4)); }
  int ensure_gplan(int q, int a, int algo, uint64_t n) {
    s3h_plan_s*& P = gplan[q][a];
    if (P && P->algo == algo && P->cap >= n) return S3H_OK;
    s3h_plan_destroy(P);
    P = nullptr;
    return plan_alloc(device, algo, std::max<uint64_t>(n, 1024), &P);
  }
  uint64_t gpin_cap() const { return gpin_bytes / (2 * kHostMaxAlgo * (sizeof(s3h::Slot) + 4)); }
  hipError_t ensure_gpin(uint64_t n) {
    return grow_pinned(&gpin, &gpin_bytes, 2 * kHostMaxAlgo * std::max<uint64_t>(n, 1024) * (sizeof(s3h::Slot) + 4));
  }
  s3h::Slot* gslots(int q, int a) {
    return reinterpret_cast<s3h::Slot*>(gpin) + uint64_t(q * kHostMaxAlgo + a) * gpin_cap();
  }
  uint32_t* gorder(int q, int a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<s3h::Slot*>(gpin) + 2 * kHostMaxAlgo * gpin_cap()) +
           uint64_t(q * kHostMaxAlgo + a) * gpin_cap();
  }
  hipError_t ensure_pin(uint64_t n) {
    return grow_pinned(&pin, &pin_bytes, kHostMaxAlgo * std::max<uint64_t>(n, 1024) * (sizeof(s3h::Slot) + 4));
  }
  void sync() {
    if (copy_s) (void)hipStreamSynchronize(copy_s);
    for (hipStream_t st : hash_s)
      if (st) (void)hipStreamSynchronize(st);
  }
  void release_large() {  // after a call: do not keep a large HBM ring or staging ring
    if (ring_bytes > kKeepRingBytes) {
      (void)hipFree(ring);
      ring = nullptr;
      ring_bytes = 0;
    }
    if (stage_bytes > kHostRing * kFileStageSlot) {
      pinned_free(stage);
      stage = nullptr;
      stage_bytes = 0;
    }
  }
  ~HostCtx() {
    DeviceGuard g(device);
    sync();
    pool.reset();
    for (hipEvent_t e : copied)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : chunk_copied)
      if (e) (void)hipEventDestroy(e);
    for (auto& row : hashed)
      for (hipEvent_t e : row)
        if (e) (void)hipEventDestroy(e);
    if (copy_s) (void)hipStreamDestroy(copy_s);
    for (hipStream_t st : hash_s)
      if (st) (void)hipStreamDestroy(st);
    for (uint32_t* d : d_dig)
      if (d) (void)hipFree(d);
    for (s3h_plan_s* p : plan)
      if (p) s3h_plan_destroy(p);
    for (auto& row : gplan)
      for (s3h_plan_s* p : row)
        if (p) s3h_plan_destroy(p);
    if (ring) (void)hipFree(ring);
    pinned_free(stage);
    pinned_free(pin);
    pinned_free(gpin);
  }
};

// One cached context per device.  Host calls on a device run one batch at a time (the
// device queue below merges concurrent callers), so the context is normally free; a call that
// still finds it busy gets a private one.
struct HostCtxCache {
  std::mutex m;
  std::vector<HostCtx*> v;  // indexed by device
  std::vector<bool> busy;
  HostCtx* acquire(int device) {
    std::lock_guard<std::mutex> l(m);
    if (v.size() <= size_t(device)) {
      v.resize(device + 1, nullptr);
      busy.resize(device + 1, false);
    }
    if (busy[device]) {
      auto* p = new HostCtx();
      p->device = device;
      p->place = device_place(device);
      return p;
    }
    if (!v[device]) {
      v[device] = new HostCtx();
      v[device]->device = device;
      v[device]->place = device_place(device);
    }
    busy[device] = true;
    return v[device];
  }
  // ok: the call succeeded (keep the cached context); a failed call drops its context.
  void release(HostCtx* c, bool ok) {
    {
      DeviceGuard g(c->device);
      c->release_large();
    }
    {
      std::lock_guard<std::mutex> l(m);
      if (v[c->device] == c) {
        busy[c->device] = false;
        if (ok) return;
        v[c->device] = nullptr;
      }
    }
    delete c;
  }
  // NUMA record of device's cached context (false: none, or busy in a call right now)
  bool numa_of(int device, s3h_host_numa_t* info) {
    std::lock_guard<std::mutex> l(m);
    if (device < 0 || size_t(device) >= v.size() || !v[device] || busy[device]) return false;
    const HostCtx* c = v[device];
    info->staging_node = c->stage ? mem_node(c->stage) : -1;
    info->threads_node = c->pool ? c->pool->bound_node() : -1;
    info->copy_threads = c->pool ? int(c->pool->size()) : 0;
    return true;
  }
  void trim() {
    std::vector<HostCtx*> idle;
    {
      std::lock_guard<std::mutex> l(m);
      for (size_t d = 0; d < v.size(); ++d)
        if (v[d] && !busy[d]) {
          idle.push_back(v[d]);
          v[d] = nullptr;
        }
    }
    for (HostCtx* c : idle) delete c;
  }
};

HostCtxCache& host_ctx_cache() {
  static HostCtxCache* c = new HostCtxCache();  // never destroyed: HIP may be gone at exit
  return *c;
}

// S3H_TRACE_HOST=1: per-shard phase times of the host path on stderr (setup, pipeline, drain).
bool trace_host() {
  static const bool on = [] {
    const char* e = std::getenv("S3H_TRACE_HOST");
    return e && std::atoi(e) == 1;
  }();
  return on;
}

double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool all_pinned(const uint8_t* const* parts, const uint64_t* lengths,
                const std::vector<uint64_t>& idx) {
  for (uint64_t i : idx) {
    if (!lengths[i]) continue;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, parts[i]) != hipSuccess || a.type != hipMemoryTypeHost) {
      (void)hipGetLastError();  // an unregistered pointer may leave a sticky error
      return false;
    }
  }
  return true;
}

struct HostShard {
  int device;
  int ndevices;  // shards running concurrently (host threads are split between them)
  std::vector<uint64_t> parts;  // global part indices on this device
  unsigned threads = 0;  // staging threads cap (0: host_threads_per_device); the split route's
                         // GPU side leaves the rest of the CPUs to its CPU side
};

// The calling thread's staging-thread cap for the host batches it starts (the split route
// sets it around its GPU side; batch_host_on copies it into the shards).
thread_local unsigned g_stage_threads_cap = 0;

unsigned shard_threads(const HostShard& sh) {
  unsigned t = host_threads_per_device(sh.ndevices);
  if (const char* e = std::getenv("S3H_STAGE_THREADS"))  // measurements: cap every shard
    if (std::atoi(e) > 0) t = std::min(t, unsigned(std::atoi(e)));
  return sh.threads ? std::max(1u, std::min(sh.threads, t)) : t;
}

// Many small parts: slicing every part (run_host_shard) would cut them into slices of a few
// hundred bytes (the staging slot holds n slices) or issue one DMA per part and slice, so
// instead the parts go in GROUPS of consecutive parts (~kGroupCopyPerChain x the longest part,
// in [kGroupMin, kGroupMax] bytes): each group is packed into pinned staging by the copy
// threads (memcpy / pread; pinned parts that are one contiguous range of a buffer are DMA'd as
// that range instead), copied by one DMA into one of two HBM group buffers, and hashed WHOLE
// by one launch per algorithm while the next group is packed and copied.
int run_host_groups(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                    const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                    bool pinned) {
  const uint64_t n = sh.parts.size();
  std::vector<uint64_t> lens(n), poff(n);
  uint64_t longest = 0;
  for (uint64_t j = 0; j < n; ++j) {
    lens[j] = lengths[sh.parts[j]];
    longest = std::max(longest, lens[j]);
  }
  // the two group buffers stay within a quarter of the free HBM, as the slice ring does
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const uint64_t budget = std::min<uint64_t>(16ull << 30, (free_b + C.ring_bytes) / 4);
  const uint64_t longest64 = std::max<uint64_t>(64, (longest + 63) & ~uint64_t(63));
  uint64_t per_chain = kGroupCopyPerChain;
  if (const char* e = std::getenv("S3H_GROUP_COPY_PER_CHAIN"))  // measurements only
    if (std::atoll(e) > 0) per_chain = uint64_t(std::atoll(e));
  // beyond 768 x only while two groups fit the HBM ring a context keeps between calls
  // (release_large) -- reallocating it per call costs more than the overlap gains
  const uint64_t keep = kKeepRingBytes / 2;
  const uint64_t want = std::max(kGroupCopyPerChainMin * longest64, std::min(per_chain * longest64, keep));
  const uint64_t G = std::max(longest64, std::min({kGroupMax, std::max(kGroupMin, want), budget / 2 / 64 * 64}));
  std::vector<uint64_t> gstart{0}, gbytes;
  uint64_t acc = 0;
  for (uint64_t j = 0; j < n; ++j) {
    const uint64_t a = (lens[j] + 63) & ~uint64_t(63);
    if (acc + a > G && acc > 0) {
      gbytes.push_back(acc);
      gstart.push_back(j);
      acc = 0;
    }
    poff[j] = acc;
    acc += a;
  }
  gbytes.push_back(acc);
  gstart.push_back(n);
  const uint64_t ngroups = gbytes.size();
  uint64_t maxb = 64, maxparts = 1;
  for (uint64_t k = 0; k < ngroups; ++k) {
    maxb = std::max(maxb, gbytes[k]);
    maxparts = std::max(maxparts, gstart[k + 1] - gstart[k]);
  }
  // pinned parts that form one increasing range of a buffer with small gaps: DMA'd as is
  const uint8_t* const* parts = src.parts;
  auto contiguous = [&](uint64_t j0, uint64_t j1, uint64_t* span) {
    if (!pinned || !parts) return false;
    const uint8_t* lo = nullptr;
    const uint8_t* hi = nullptr;
    for (uint64_t j = j0; j < j1; ++j) {
      if (!lens[j]) continue;
      const uint8_t* p = parts[sh.parts[j]];
      if (hi && p < hi) return false;
      if (!lo) lo = p;
      hi = p + lens[j];
    }
    *span = lo ? uint64_t(hi - lo) : 0;
    return *span <= maxb;
  };
  HIP_TRY(C.ensure_streams());
  hipError_t ce = HostCtx::grow_dev(&C.ring, &C.ring_bytes, 2 * maxb);
  if (ce != hipSuccess) {
    (void)hipGetLastError();
    return fail(S3H_ENOMEM, "host group buffers (2 x %llu B of HBM): %s", (unsigned long long)maxb,
                hipGetErrorString(ce));
  }
  bool any_staged = false;
  for (uint64_t k = 0; k < ngroups && !any_staged; ++k) {
    uint64_t span = 0;
    any_staged = !contiguous(gstart[k], gstart[k + 1], &span);
  }
  // packed groups go through kHostRing pinned chunks of kGroupChunk bytes (a part always fits
  // one): the staging is sized for the copy in flight, not for the group the GPU hashes
  const uint64_t chunk = std::max(kGroupChunk, longest64);
  if (any_staged) {
    ce = C.grow_pinned(&C.stage, &C.stage_bytes, kHostRing * chunk);
    if (ce != hipSuccess) {
      (void)hipGetLastError();
      return fail(S3H_ENOMEM, "pinned group staging (%d x %llu B): %s", kHostRing,
                  (unsigned long long)chunk, hipGetErrorString(ce));
    }
  }
  bool chunk_used[kHostRing] = {};
  uint64_t chunk_next = 0;
  HIP_TRY(C.ensure_gpin(maxparts));
  for (int q = 0; q < 2; ++q)
    for (int a = 0; a < nalgo; ++a) {
      if (int rc = C.ensure_gplan(q, a, algos[a], maxparts)) return rc;
      HIP_TRY(hipMemsetAsync(C.gplan[q][a]->d_err, 0, sizeof(uint32_t), C.copy_s));
    }
  for (int a = 0; a < nalgo; ++a)
    HIP_TRY(C.ensure_digests(a, n * digest_words(algos[a]) * sizeof(uint32_t)));
  CopyPool* pool = any_staged ? C.ensure_pool(shard_threads(sh) - 1) : nullptr;
  std::vector<uint64_t> offs;
  for (uint64_t k = 0; k < ngroups; ++k) {
    const int q = int(k & 1);
    const uint64_t j0 = gstart[k], j1 = gstart[k + 1], ng = j1 - j0;
    uint8_t* const dgrp = C.ring + uint64_t(q) * maxb;
    // group k-2 used set q: its DMAs (host staging and geometry staging) must have run, and
    // its hashes (the HBM group buffer and the plans' device slots) before the copy stream
    // overwrites them
    if (k >= 2) {
      HIP_TRY(hipEventSynchronize(C.copied[q]));
      for (int a = 0; a < nalgo; ++a) HIP_TRY(hipStreamWaitEvent(C.copy_s, C.hashed[q][a], 0));
    }
    uint64_t span = 0;
    const bool direct = contiguous(j0, j1, &span);
    offs.assign(ng, 0);
    const uint8_t* base = nullptr;
    for (uint64_t t = 0; t < ng && direct; ++t)
      if (lens[j0 + t] && !base) base = parts[sh.parts[j0 + t]];
    for (uint64_t t = 0; t < ng; ++t)
      offs[t] = direct ? (lens[j0 + t] ? uint64_t(parts[sh.parts[j0 + t]] - base) : 0) : poff[j0 + t];
    for (int a = 0; a < nalgo; ++a)
      if (int rc = plan_geometry(C.gplan[q][a], offs.data(), lens.data() + j0, ng, S3H_KERNEL_AUTO,
                                 C.gslots(q, a), C.gorder(q, a), C.copy_s))
        return rc;
    if (direct) {
      if (span) HIP_TRY(hipMemcpyAsync(dgrp, base, span, hipMemcpyHostToDevice, C.copy_s));
    } else {  // packed chunk by chunk: parts [ja, jb) whose packed bytes fit one chunk
      for (uint64_t ja = j0, jb; ja < j1; ja = jb) {
        jb = ja + 1;
        while (jb < j1 && poff[jb] + ((lens[jb] + 63) & ~uint64_t(63)) - poff[ja] <= chunk) ++jb;
        const uint64_t bytes = (jb < j1 ? poff[jb] : gbytes[k]) - poff[ja];
        const int c = int(chunk_next++ % kHostRing);
        if (chunk_used[c]) HIP_TRY(hipEventSynchronize(C.chunk_copied[c]));  // its last DMA ran
        uint8_t* const hst = C.stage + uint64_t(c) * chunk;
        std::atomic<bool> bad{false};
        pool->run(jb - ja, [&](uint64_t t) {
          const uint64_t j = ja + t;
          if (lens[j] && !src.fill(sh.parts[j], 0, lens[j], hst + (poff[j] - poff[ja])))
            bad.store(true, std::memory_order_relaxed);
        });
        if (bad.load()) return fail(S3H_EINVAL, "reading a part failed (file shorter than a part?)");
        if (bytes) HIP_TRY(hipMemcpyAsync(dgrp + poff[ja], hst, bytes, hipMemcpyHostToDevice, C.copy_s));
        HIP_TRY(hipEventRecord(C.chunk_copied[c], C.copy_s));
        chunk_used[c] = true;
      }
    }
    HIP_TRY(hipEventRecord(C.copied[q], C.copy_s));
    for (int a = 0; a < nalgo; ++a) {
      s3h_plan_s* P = C.gplan[q][a];
      HIP_TRY(hipStreamWaitEvent(C.hash_s[a], C.copied[q], 0));
      if (int rc = plan_launch(P, dgrp, C.d_dig[a] + j0 * digest_words(algos[a]), 0, P->max_blocks, 0,
                               C.hash_s[a], false))
        return rc;
      HIP_TRY(hipEventRecord(C.hashed[q][a], C.hash_s[a]));
    }
  }
  int rc = S3H_OK;
  for (int a = 0; a < nalgo && rc == S3H_OK; ++a) {
    const uint32_t dw = digest_words(algos[a]);
    std::vector<uint32_t> local(n * dw);
    hipError_t e = hipMemcpyAsync(local.data(), C.d_dig[a], n * dw * 4, hipMemcpyDeviceToHost, C.hash_s[a]);
    if (e == hipSuccess) e = hipStreamSynchronize(C.hash_s[a]);
    if (e != hipSuccess) {
      rc = fail(S3H_EHIP, "D2H digests: %s", hipGetErrorString(e));
      break;
    }
    for (int q = 0; q < 2 && rc == S3H_OK; ++q) rc = plan_check(C.gplan[q][a], C.hash_s[a]);
    if (rc) break;
    for (uint64_t j = 0; j < n; ++j) std::memcpy(digests[a] + dw * sh.parts[j], &local[dw * j], dw * 4);
  }
  C.sync();
  if (trace_host())
    std::fprintf(stderr, "[s3h host] dev %d: %llu parts in %llu groups of <= %llu B (%s)\n", sh.device,
                 (unsigned long long)n, (unsigned long long)ngroups, (unsigned long long)maxb,
                 any_staged ? "staged" : "pinned ranges");
  return rc;
}

// Streams one device's parts through a 3-slot HBM ring; every slice is copied ONCE and
// hashed by each requested algorithm (SHA-256 and/or MD5) on its own stream, so a dual
// digest costs one PCIe pass.  digests[a] receives algo[a]'s digests (global part order).
// Copy modes per slice: pinned parts at a constant stride -> one 2-D DMA; other pinned parts
// -> one DMA per part; pageable parts and file ranges -> host threads fill a pinned staging
// slot (memcpy / pread) and one DMA moves it; more than kStageSlot/64 pageable parts (or no
// pinned memory) -> one pageable DMA per part.
int run_host_shard(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                   const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                   uint64_t slice) {
  if (nalgo < 1 || nalgo > kHostMaxAlgo) return fail(S3H_EINVAL, "host shard: %d algorithms", nalgo);
  const uint64_t n = sh.parts.size();
  if (n == 0) return S3H_OK;
  DeviceGuard g(sh.device);
  const double t_start = wall_s();
  std::vector<uint64_t> offs(n), lens(n);
  for (uint64_t j = 0; j < n; ++j) lens[j] = lengths[sh.parts[j]];
  const uint8_t* const* parts = src.parts;
  bool staged = !parts || !all_pinned(parts, lengths, sh.parts);
  bool uniform = false;
  intptr_t stride = 0;
  if (!staged && n > 1) {  // equal-length parts at a constant positive host stride (file chunks)
    stride = parts[sh.parts[1]] - parts[sh.parts[0]];
    uniform = stride >= intptr_t(lens[0]) && lens[0] > 0;
    for (uint64_t j = 1; j < n && uniform; ++j)
      uniform = lens[j] == lens[0] && parts[sh.parts[j]] - parts[sh.parts[j - 1]] == stride;
  }
  // Many small parts (<= kGroupMaxPart): whole parts in groups instead of slices of every part
  // (run_host_groups) -- when staging would cut slices below 16 KiB (> 2,048 parts), or pinned
  // ragged parts would each take their own DMA per slice (> 64 parts: 4,000 pinned parts of
  // U[1 B, 1 MiB] spent 0.49 s draining 56,000 per-part DMAs for 1.9 GiB).  A caller's
  // explicit slice size keeps the slice pipeline.  Large parts beside them (an object's parts
  // batched with many small objects) run through the slice pipeline afterwards, on their own.
  if (slice == 0) {
    std::vector<uint64_t> small, large;
    for (uint64_t j = 0; j < n; ++j) (lens[j] <= kGroupMaxPart ? small : large).push_back(sh.parts[j]);
    const uint64_t ns = small.size();
    if ((staged && ns > 2048) || (!staged && !uniform && ns > 64)) {
      if (large.empty()) return run_host_groups(C, sh, algos, nalgo, src, lengths, digests, !staged);
      const HostShard hs{sh.device, sh.ndevices, std::move(small), sh.threads};
      const HostShard hl{sh.device, sh.ndevices, std::move(large), sh.threads};
      if (int rc = run_host_groups(C, hs, algos, nalgo, src, lengths, digests, !staged)) return rc;
      return run_host_shard(C, hl, algos, nalgo, src, lengths, digests, 0);
    }
  }
  // Many ragged pinned parts: packing them into staging (memcpy, one DMA per slice) beats one
  // DMA per part per slice (4,000 parts of U[256 KiB, 4 MiB]: 18.0 -> 30.2 GiB/s; 1,024 of
  // U[1, 8] MiB: 24.3 -> 27.8).
  if (!staged && !uniform && n > kPinnedStageMin) staged = true;
  // Too many pageable parts for the staging cap even at 64 B per slice: pageable DMAs.
#ifdef S3H_EXP_PAGEABLE_DIRECT  // tools/ experiment builds only: pageable DMAs, no staging
  bool direct_pageable = staged && parts;
#else
  bool direct_pageable = staged && parts && n * 64 > kStageSlot;
#endif
  if (direct_pageable) staged = false;
  if (slice == 0)
    slice = staged ? std::max<uint64_t>(std::max<uint64_t>(64, kStageSlot / n / 64 * 64),
                                        std::min<uint64_t>(32 << 10, kFileStageSlot / n / 64 * 64))
            : uniform ? (256ull << 10) : (2ull << 20);
  const uint64_t longest = *std::max_element(lens.begin(), lens.end());
  slice = std::min(slice, std::max<uint64_t>(64, (longest + 63) / 64 * 64));  // no idle slot bytes
  // The ring holds kHostRing*n*slice bytes of HBM: keep it within min(16 GiB, free/4).
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const uint64_t budget = std::min<uint64_t>(16ull << 30, (free_b + C.ring_bytes) / 4);
  if (kHostRing * n * slice > budget) slice = std::max<uint64_t>(64, budget / (kHostRing * n) / 64 * 64);
  for (uint64_t j = 0; j < n; ++j) offs[j] = j * slice;
  const uint64_t slot_bytes = n * slice;

  HIP_TRY(C.ensure_streams());
  hipError_t ce = hipSuccess;
  if (staged) {
    ce = C.grow_pinned(&C.stage, &C.stage_bytes, kHostRing * slot_bytes);
    if (ce != hipSuccess) {
      (void)hipGetLastError();
      if (!parts) return fail(S3H_ENOMEM, "pinned staging (%llu B): %s",
                              (unsigned long long)(kHostRing * slot_bytes), hipGetErrorString(ce));
      staged = false;  // memory parts: fall back to pageable DMAs
      direct_pageable = true;
    }
  }
  ce = HostCtx::grow_dev(&C.ring, &C.ring_bytes, kHostRing * slot_bytes);
  if (ce != hipSuccess) return fail(S3H_ENOMEM, "host ring (%llu B): %s",
                                    (unsigned long long)(kHostRing * slot_bytes), hipGetErrorString(ce));
  HIP_TRY(C.ensure_pin(n));
  uint64_t max_blocks = 0;
  for (int a = 0; a < nalgo; ++a) {
    if (int rc = C.ensure_plan(a, algos[a], n)) return rc;
    HIP_TRY(hipMemsetAsync(C.plan[a]->d_err, 0, sizeof(uint32_t), C.copy_s));  // before any launch
    HIP_TRY(C.ensure_digests(a, n * digest_words(algos[a]) * sizeof(uint32_t)));
    // geometry upload on the copy stream: every launch waits for a later copy on it
    if (int rc = plan_geometry(C.plan[a], offs.data(), lens.data(), n, S3H_KERNEL_AUTO,
                               C.h_slots(a), C.h_order(a), C.copy_s))
      return rc;
    max_blocks = std::max(max_blocks, C.plan[a]->max_blocks);
  }
  CopyPool* pool = nullptr;
  const unsigned threads = shard_threads(sh);  // the caller + workers
  if (staged) pool = C.ensure_pool(threads - 1);
  const uint64_t bps = slice / 64;  // blocks per slice
  s3h_plan_s* P0 = C.plan[0];
  s3h_plan_s* P1 = nalgo == 2 ? C.plan[1] : nullptr;
  const bool fused = nalgo == 2 && P0->max_blocks == P1->max_blocks &&
                     dual_mode(P0, P1, 0, bps) != kDualNone;
  int rc = S3H_OK;
  uint64_t k = 0;
  const double t_setup = wall_s();
  // Slices of bps blocks, then a geometric tail: the copies set the pace (PCIe; C2: a full
  // slice copies in ~4.7 ms and hashes in ~3.8) and slice k's hash runs beside slice k+1's
  // copy, so the hash keeps up only while hash(k) <= copy(k+1).  Once fewer than D slices are
  // left each slice takes 1/D of the rest (sizes shrink by (D-1)/D >= the hash/copy ratio,
  // ~0.81), down to bps/16, so the hash exposed after the last copy is one small slice's
  // (~0.24 ms).  Halving (D = 2) broke the condition at the first tail slice: 3.8 ms of
  // full-slice hash ran past the copies (tools/host_timeline.py trace).
  auto slice_blocks = [&](uint64_t b0) -> uint64_t {
    const uint64_t left = max_blocks - b0;
#ifndef S3H_EXP_NO_TAIL_RAMP  // tools/ experiment builds only: round-3 fixed slices
    constexpr uint64_t D = S3H_EXP_TAIL_RAMP_DIV;
    if (bps >= 256 && left < D * bps)
      return std::min(left, std::max<uint64_t>(bps / 16, (left + D - 1) / D));
#endif
    return std::min(left, bps);
  };
  for (uint64_t b0 = 0, step = 0; b0 < max_blocks && rc == S3H_OK; b0 += step, ++k) {
    step = slice_blocks(b0);
    const uint64_t sbytes = step * 64;  // bytes of each part this slice carries (<= slice)
    const int r = int(k % kHostRing);
    uint8_t* slot_base = C.ring + uint64_t(r) * slot_bytes;
    hipError_t e = hipSuccess;
    for (int a = 0; a < nalgo && k >= kHostRing && e == hipSuccess; ++a)
      e = hipStreamWaitEvent(C.copy_s, C.hashed[r][a], 0);  // slot reusable once all hashed it
    if (e != hipSuccess) { rc = fail(S3H_EHIP, "wait: %s", hipGetErrorString(e)); break; }
    const uint64_t byte0 = b0 * 64;
    if (staged) {
      // host slot r is free once the DMA that last read it (copied[r]) has finished
      uint8_t* hslot = C.stage + uint64_t(r) * slot_bytes;
      if (k >= kHostRing) e = hipEventSynchronize(C.copied[r]);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "stage wait: %s", hipGetErrorString(e)); break; }
      std::atomic<bool> bad{false};
      pool->run(n, [&](uint64_t j) {
        const uint64_t len = lens[j];
        if (byte0 < len && !src.fill(sh.parts[j], byte0, std::min(sbytes, len - byte0), hslot + j * slice))
          bad.store(true, std::memory_order_relaxed);
      });
      if (bad.load()) { rc = fail(S3H_EINVAL, "reading a part failed (file shorter than a part?)"); break; }
      e = step == bps ? hipMemcpyAsync(slot_base, hslot, slot_bytes, hipMemcpyHostToDevice, C.copy_s)
                      : hipMemcpy2DAsync(slot_base, slice, hslot, slice, sbytes, n,
                                         hipMemcpyHostToDevice, C.copy_s);
      if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D staged: %s", hipGetErrorString(e));
    } else if (uniform) {
      if (byte0 < lens[0]) {
        const uint64_t cnt = std::min(sbytes, lens[0] - byte0);
        e = hipMemcpy2DAsync(slot_base, slice, parts[sh.parts[0]] + byte0, stride, cnt, n,
                             hipMemcpyHostToDevice, C.copy_s);
        if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D 2D: %s", hipGetErrorString(e));
      }
    } else {
      for (uint64_t j = 0; j < n && rc == S3H_OK; ++j) {
        const uint64_t len = lens[j];
        if (byte0 >= len) continue;
        const uint64_t cnt = std::min(sbytes, len - byte0);
        e = hipMemcpyAsync(slot_base + j * slice, parts[sh.parts[j]] + byte0, cnt,
                           hipMemcpyHostToDevice, C.copy_s);
        if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D: %s", hipGetErrorString(e));
      }
    }
    if (rc) break;
    e = hipEventRecord(C.copied[r], C.copy_s);
    if (fused) {  // both digests from one grid on one stream
      if (e == hipSuccess) e = hipStreamWaitEvent(C.hash_s[0], C.copied[r], 0);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e)); break; }
      rc = dual_launch(P0, P1, slot_base, C.d_dig[0], C.d_dig[1], b0, b0 + step, b0, true,
                       C.hash_s[0]);
      if (rc == S3H_OK) e = hipEventRecord(C.hashed[r][0], C.hash_s[0]);
      if (e == hipSuccess) e = hipEventRecord(C.hashed[r][1], C.hash_s[0]);
    }
    for (int a = 0; a < nalgo && rc == S3H_OK && !fused; ++a) {
      if (e == hipSuccess) e = hipStreamWaitEvent(C.hash_s[a], C.copied[r], 0);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e)); break; }
      if (b0 < C.plan[a]->max_blocks)  // both pad 9 B, so equal block counts; guard anyway
        rc = plan_launch(C.plan[a], slot_base, C.d_dig[a], b0, b0 + step, b0, C.hash_s[a], true);
      if (rc == S3H_OK) e = hipEventRecord(C.hashed[r][a], C.hash_s[a]);
    }
    if (rc == S3H_OK && e != hipSuccess) rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e));
  }
  const double t_issue = wall_s();
  for (int a = 0; a < nalgo && rc == S3H_OK; ++a) {
    const uint32_t dw = digest_words(algos[a]);
    std::vector<uint32_t> local(n * dw);
    hipStream_t hs = C.hash_s[fused ? 0 : a];
    hipError_t e = hipMemcpyAsync(local.data(), C.d_dig[a], n * dw * 4, hipMemcpyDeviceToHost, hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    if (e != hipSuccess) { rc = fail(S3H_EHIP, "D2H digests: %s", hipGetErrorString(e)); break; }
    if ((rc = plan_check(C.plan[a], hs)) != S3H_OK) break;  // every slice's launch reported in
    for (uint64_t j = 0; j < n; ++j)
      std::memcpy(digests[a] + dw * sh.parts[j], &local[dw * j], dw * 4);
  }
  C.sync();  // nothing of this call may still run when the context is handed on
  if (trace_host())
    std::fprintf(stderr,
                 "[s3h host] dev %d: %llu parts, slice %llu B, %s, %llu slices: setup %.2f ms, "
                 "issue %.2f ms, drain %.2f ms; copy threads %u (%u CPUs over %d devices); "
                 "numa: device node %d, staging node %d, copy threads on %d CPUs of node %d\n",
                 sh.device, (unsigned long long)n, (unsigned long long)slice,
                 !parts ? "staged (file pread)" : staged ? "staged (pageable)"
                 : direct_pageable ? "pageable per-part" : uniform ? "pinned 2-D" : "pinned per-part",
                 (unsigned long long)k, 1e3 * (t_setup - t_start), 1e3 * (t_issue - t_setup),
                 1e3 * (wall_s() - t_issue), staged ? threads : 0u, host_cpus(), sh.ndevices,
                 C.place.dev_node, staged ? mem_node(C.stage) : -1, C.place.ncpus, C.place.node);
  return rc;
}

// File ranges and merged part references have no pageable-DMA fallback, and their staging
// slot is n x slice bytes with slices of at least 64 B: a shard of more than
// kMaxStagedRefs such parts runs in passes of that many, so the pinned staging ring never
// exceeds kHostRing x kFileStageSlot (384 MiB).
constexpr uint64_t kMaxStagedRefs = kFileStageSlot / 64;  // 2,097,152 parts

int run_host_shard_passes(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                          const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                          uint64_t slice) {
  if (src.parts || sh.parts.size() <= kMaxStagedRefs)
    return run_host_shard(C, sh, algos, nalgo, src, lengths, digests, slice);
  for (uint64_t s = 0; s < sh.parts.size(); s += kMaxStagedRefs) {
    const uint64_t e = std::min<uint64_t>(sh.parts.size(), s + kMaxStagedRefs);
    HostShard sub{sh.device, sh.ndevices,
                  std::vector<uint64_t>(sh.parts.begin() + s, sh.parts.begin() + e), sh.threads};
    if (int rc = run_host_shard(C, sub, algos, nalgo, src, lengths, digests, slice)) return rc;
  }
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

}  // namespace

// Multi-object stream (include/s3hash.h "multi-object streams").  Host bookkeeping: per
// message carry length (< 64) and total bytes.  Device: chaining state (message order),
// 64-B carry and head-block buffers, the splice jobs, three re-sortable plans.
struct s3h_stream_s {
  int device = 0, algo = 0;
  uint64_t n = 0;
  s3h_plan_s *head = nullptr, *body = nullptr, *fin = nullptr;
  uint32_t* d_state = nullptr;
  uint8_t* d_carry = nullptr;
  uint8_t* d_head = nullptr;
  s3h::SpliceJob* d_jobs = nullptr;
  uint64_t* d_bits = nullptr;
  // Host-form updates (s3h_stream_update_host): each update's chunks are packed at 64-B
  // aligned offsets into device staging set hb -- two sets, so update k+1's copy (on copy_s)
  // overlaps update k's hash (on own) -- by DMA straight from pinned chunks, or, for pageable
  // chunks, through pinned host pieces (two, kStreamPiece bytes) that copy threads on the
  // device's NUMA node fill while the previous piece's DMA runs.
  uint8_t* d_hs[2] = {nullptr, nullptr};
  uint64_t d_hs_cap[2] = {0, 0};
  uint8_t* h_piece[2] = {nullptr, nullptr};
  uint64_t h_piece_cap = 0;
  hipEvent_t hs_copied[2] = {nullptr, nullptr}, hs_hashed[2] = {nullptr, nullptr};
  hipEvent_t piece_copied[2] = {nullptr, nullptr};
  hipStream_t copy_s = nullptr;
  unsigned hs_set = 0, piece_next = 0;
  uint32_t* d_dig = nullptr;   // host-form final
  // Pinned staging of an update / final in two sets used alternately: set b is rewritten
  // only once the call that used it two calls ago has completed (staged[b]), so the host
  // prepares update k+1 while update k's kernels run (one set made every update wait for the
  // previous one's kernels: the GPU idled ~45 us per update, -4.7 % at 64 KiB chunks).
  uint8_t* h_pin = nullptr;
  s3h::SpliceJob* h_jobs[2] = {nullptr, nullptr};
  s3h::Slot* h_slots[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  uint32_t* h_order[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  uint64_t* h_bits[2] = {nullptr, nullptr};
  hipEvent_t staged[2] = {nullptr, nullptr};
  hipEvent_t done = nullptr;  // end of the last update / final: the next call's stream waits on it
  hipStream_t done_on = nullptr;  // the stream `done` was recorded on (same stream: no wait)
  bool done_set = false;
  unsigned set = 0;
  bool used_stage = false;  // this call copied from staging set `set ^ 1` (else no staged[] record)
  // What the head / body plans' device slots hold: an update whose lengths equal them and
  // whose offsets are them plus one constant (equal chunks appended in place) reuses the
  // slots with the launch base moved by that constant -- no re-sort, no copies.
  std::vector<uint64_t> up_offs[2], up_lens[2];
  bool up_valid[2] = {false, false};
  uint64_t slot_reuses = 0, slot_refills = 0;  // s3h_stream_stats: how updates found their slots
  // A call that failed after it started queueing work leaves the messages' host bookkeeping
  // (carries, totals) ahead of or behind the device state: the object refuses further calls.
  std::string failed;
  hipStream_t own = nullptr;
  std::vector<uint64_t> total;
  std::vector<uint32_t> carry;
  std::vector<uint64_t> offs, lens, offs2, lens2;
};

namespace {

// Host-form staging of destroyed stream objects, kept per device for the next object (an
// uploader creates one per batch of objects: allocating, first-touching and registering 2 x 64
// MiB of pinned pieces plus the device sets cost ~35 ms per object, ~20 % of a C2-sized batch;
// profiles/r05_stream_vs_batch_ab.json).  At most kStagingKeep entries per device; s3h_trim
// frees them.
struct StreamStaging {
  uint8_t* d_hs[2] = {nullptr, nullptr};
  uint64_t d_hs_cap[2] = {0, 0};
  uint8_t* h_piece[2] = {nullptr, nullptr};
  uint64_t h_piece_cap = 0;
};
constexpr size_t kStagingKeep = 2;
struct StagingCache {
  std::mutex m;
  std::map<int, std::vector<StreamStaging>> free;
};
StagingCache& staging_cache() {
  static auto* c = new StagingCache();
  return *c;
}

void staging_release(int device, const StreamStaging& st) {
  DeviceGuard g(device);
  for (uint8_t* p : st.d_hs) (void)hipFree(p);
  pinned_free(st.h_piece[0]);
  pinned_free(st.h_piece[1]);
}

void staging_trim() {
  std::map<int, std::vector<StreamStaging>> all;
  {
    std::lock_guard<std::mutex> l(staging_cache().m);
    all.swap(staging_cache().free);
  }
  for (auto& kv : all)
    for (auto& st : kv.second) staging_release(kv.first, st);
}

void stream_free(s3h_stream_s* S) {
  DeviceGuard g(S->device);
  if (S->own) (void)hipStreamSynchronize(S->own);
  if (S->copy_s) (void)hipStreamSynchronize(S->copy_s);
  for (hipEvent_t e : {S->staged[0], S->staged[1], S->done})
    if (e) (void)hipEventSynchronize(e);
  s3h_plan_destroy(S->head);
  s3h_plan_destroy(S->body);
  s3h_plan_destroy(S->fin);
  for (void* p : {(void*)S->d_state, (void*)S->d_carry, (void*)S->d_head, (void*)S->d_jobs,
                  (void*)S->d_bits, (void*)S->d_dig})
    (void)hipFree(p);
  pinned_free(S->h_pin);
  if (S->d_hs[0] || S->d_hs[1] || S->h_piece[0]) {  // idle now: keep it for the next object
    StreamStaging st;
    std::copy(S->d_hs, S->d_hs + 2, st.d_hs);
    std::copy(S->d_hs_cap, S->d_hs_cap + 2, st.d_hs_cap);
    std::copy(S->h_piece, S->h_piece + 2, st.h_piece);
    st.h_piece_cap = S->h_piece_cap;
    bool kept = false;
    {
      std::lock_guard<std::mutex> l(staging_cache().m);
      auto& v = staging_cache().free[S->device];
      if (v.size() < kStagingKeep) {
        v.push_back(st);
        kept = true;
      }
    }
    if (!kept) staging_release(S->device, st);
  }
  for (hipEvent_t e : {S->staged[0], S->staged[1], S->done, S->hs_copied[0], S->hs_copied[1],
                       S->hs_hashed[0], S->hs_hashed[1], S->piece_copied[0], S->piece_copied[1]})
    if (e) (void)hipEventDestroy(e);
  if (S->own) (void)hipStreamDestroy(S->own);
  if (S->copy_s) (void)hipStreamDestroy(S->copy_s);
  delete S;
}

int stream_reset(s3h_stream_s* S, hipStream_t s) {
  std::fill(S->total.begin(), S->total.end(), 0);
  std::fill(S->carry.begin(), S->carry.end(), 0u);
  hipLaunchKernelGGL(s3h::stream_init_kernel, dim3(uint32_t((S->n + 255) / 256)), dim3(256), 0, s,
                     S->d_state, S->n, int(S->algo == S3H_ALGO_MD5));
  HIP_TRY(hipGetLastError());
  return S3H_OK;
}

// Claims the next staging set for a call on stream `s`: waits (host) until the set's previous
// use has completed, and orders `s` after the previous call's work on any stream (on the
// same stream, stream order does it; a handle reused after hipStreamDestroy is safe too, as
// destroying a stream waits for its work).
int stream_begin(s3h_stream_s* S, hipStream_t s, unsigned* b) {
  *b = S->set;
  S->set ^= 1u;
  S->used_stage = false;
  HIP_TRY(hipEventSynchronize(S->staged[*b]));
  if (!S->done_set || s != S->done_on) HIP_TRY(hipStreamWaitEvent(s, S->done, 0));
  return S3H_OK;
}

// staged[b] is recorded only when the call copied from set b (an update that reused the
// device slots copied nothing; the set's previous record still bounds its last use).
int stream_end(s3h_stream_s* S, hipStream_t s, unsigned b) {
  if (S->used_stage) HIP_TRY(hipEventRecord(S->staged[b], s));
  HIP_TRY(hipEventRecord(S->done, s));
  S->done_on = s;
  S->done_set = true;
  return S3H_OK;
}

// Launch base of update plan `which` (0 head, 1 body) for these slots: the device's slots
// moved by a constant when they fit (see up_offs), else after a refill from staging set b.
int stream_plan_base(s3h_stream_s* S, int which, s3h_plan_s* P, const uint8_t* base,
                     const std::vector<uint64_t>& offs, const std::vector<uint64_t>& lens,
                     unsigned b, hipStream_t s, const uint8_t** launch_base) {
  if (S->up_valid[which] && lens == S->up_lens[which]) {
    bool same = true, have = false;
    uint64_t delta = 0;
    for (uint64_t i = 0; i < S->n && same; ++i) {
      if (!lens[i]) continue;  // an empty slot is never read
      const uint64_t d = offs[i] - S->up_offs[which][i];
      if (!have) {
        delta = d;
        have = true;
      } else {
        same = d == delta;
      }
    }
    if (same) {  // base + off_now == (base + delta) + off_uploaded, modulo 2^64 like the slots
      *launch_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(base) + delta);
      ++S->slot_reuses;
      return S3H_OK;
    }
  }
  ++S->slot_refills;
  S->up_valid[which] = false;
  S->used_stage = true;
  if (int rc = plan_refill(P, offs.data(), lens.data(), true, S->h_slots[b][which], S->h_order[b][which], s))
    return rc;
  S->up_offs[which] = offs;
  S->up_lens[which] = lens;
  S->up_valid[which] = true;
  *launch_base = base;
  return S3H_OK;
}

// Runs one update / final body between stream_begin and stream_end.  stream_end runs on
// every exit after stream_begin succeeded -- staged[b] and `done` are recorded even when the
// body failed midway, so a later call never rewrites a staging set a queued copy still reads,
// nor skips waiting for partly queued work -- and a failed body marks the object failed.
template <typename Body>
int stream_call(s3h_stream_s* S, hipStream_t s, Body body) {
  if (!S->failed.empty())
    return fail(S3H_EINVAL, "stream object failed earlier (%s): destroy it", S->failed.c_str());
  unsigned b = 0;
  if (int rc = stream_begin(S, s, &b)) return rc;
  const int rc = body(b);
  const std::string err = g_err;
  const int rc_end = stream_end(S, s, b);
  if (rc) {
    S->failed = err;
    g_err = err;
    return rc;
  }
  if (rc_end) S->failed = g_err;
  return rc_end;
}

int stream_update_body(s3h_stream_s* S, const uint8_t* base, const uint64_t* offsets,
                       const uint64_t* lengths, hipStream_t s, unsigned b) {
  const uint64_t n = S->n;
  s3h::SpliceJob* const h_jobs = S->h_jobs[b];
  bool any_splice = false, any_head = false, any_body = false;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t L = lengths[i], off = L ? offsets[i] : 0;
    const uint32_t c = S->carry[i];
    s3h::SpliceJob j = {off, 0, c, 0, 0, 0};
    uint64_t body_off = off, B = 0;
    if (L == 0) {
    } else if (c > 0 && c + L < 64) {  // still inside one block: buffer it
      j.h = uint32_t(L);
      j.mode = s3h::kSpliceGrow;
      S->carry[i] = c + uint32_t(L);
    } else {
      j.h = c > 0 ? 64 - c : 0;  // bytes that complete the carried block
      body_off = off + j.h;
      B = (L - j.h) & ~uint64_t(63);
      j.r = uint32_t(L - j.h - B);
      j.tail = body_off + B;
      j.mode = (c > 0 ? s3h::kSpliceHead : 0) | (j.r ? s3h::kSpliceReset : 0);
      S->carry[i] = j.r;
    }
    S->total[i] += L;
    h_jobs[i] = j;
    any_splice |= j.mode != 0;
    any_head |= (j.mode & s3h::kSpliceHead) != 0;
    any_body |= B != 0;
    S->offs[i] = 64 * i;
    S->lens[i] = (j.mode & s3h::kSpliceHead) ? 64 : 0;
    S->offs2[i] = body_off;
    S->lens2[i] = B;
  }
  if (any_splice) {
    S->used_stage = true;
    HIP_TRY(hipMemcpyAsync(S->d_jobs, h_jobs, n * sizeof(s3h::SpliceJob), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(s3h::stream_splice_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s,
                       base, S->d_jobs, S->d_carry, S->d_head, n);
    HIP_TRY(hipGetLastError());
  }
  constexpr uint32_t kAppend = s3h::kNoPad | s3h::kResume;
  if (any_head) {  // the blocks straddling the previous update and this one come first
    const uint8_t* hb = nullptr;
    if (int rc = stream_plan_base(S, 0, S->head, S->d_head, S->offs, S->lens, b, s, &hb)) return rc;
    if (int rc = launch_args(S->head, hb, nullptr, S->d_state, 0, 1, 0, kAppend, nullptr, s)) return rc;
  }
  if (any_body) {
    const uint8_t* bb = nullptr;
    if (int rc = stream_plan_base(S, 1, S->body, base, S->offs2, S->lens2, b, s, &bb)) return rc;
    if (int rc = launch_args(S->body, bb, nullptr, S->d_state, 0, S->body->max_blocks, 0, kAppend, nullptr, s)) return rc;
  }
  return S3H_OK;
}

int stream_update(s3h_stream_s* S, const uint8_t* base, const uint64_t* offsets,
                  const uint64_t* lengths, hipStream_t s) {
  return stream_call(S, s, [&](unsigned b) { return stream_update_body(S, base, offsets, lengths, s, b); });
}

// The error words of the stream's three plans (head / body / final launches), once `s` has
// run everything before: plan_check.  Every plan's word is read and cleared (a fault of one
// must not be reported again by a later check), then the first failure is returned.
int stream_check(s3h_stream_s* S, hipStream_t s) {
  int first = S3H_OK;
  std::string msg;
  for (s3h_plan_s* P : {S->head, S->body, S->fin})
    if (int rc = plan_check(P, s); rc && !first) {
      first = rc;
      msg = g_err;
    }
  if (first) g_err = msg;
  return first;
}

int stream_final_body(s3h_stream_s* S, uint32_t* d_digests, hipStream_t s, unsigned b) {
  const uint64_t n = S->n;
  for (uint64_t i = 0; i < n; ++i) {
    S->offs[i] = 64 * i;
    S->lens[i] = S->carry[i];
    S->h_bits[b][i] = S->total[i] << 3;
  }
  S->used_stage = true;
  HIP_TRY(hipMemcpyAsync(S->d_bits, S->h_bits[b], n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  if (int rc = plan_refill(S->fin, S->offs.data(), S->lens.data(), false, S->h_slots[b][0], S->h_order[b][0], s)) return rc;
  // one or two padded blocks per message, starting from the appended state
  if (int rc = launch_args(S->fin, S->d_carry, d_digests, S->d_state, 0, S->fin->max_blocks, 0,
                           s3h::kResume, S->d_bits, s)) return rc;
  return stream_reset(S, s);
}

int stream_final(s3h_stream_s* S, uint32_t* d_digests, hipStream_t s) {
  return stream_call(S, s, [&](unsigned b) { return stream_final_body(S, d_digests, s, b); });
}

}  // namespace

namespace {

// ------------------------------------------------------------------ concurrent callers
// upload.cpp:136-140 hashes from cfg.jobs std::async threads, each call covering only its own
// job's parts.  Run as they come, 16 such calls of 32 parts put 16 small grids on the
// process's few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), which run them a few at a
// time: 4 GiB in 16 x 32 parts of 8 MiB took 1.3-1.4 s against 0.124 s for one call with all
// 512 parts.  So the calls of one device meet in a queue: the first caller (the leader) takes
// every pending request with the same algorithms and slice size and runs them as ONE shard --
// parts from memory and file ranges mixed -- then scatters the digests back; calls that arrive
// meanwhile form the next batch.  Once calls have been seen to overlap (within the last
// second), a leader first gathers the rest of the burst: it waits until no call has arrived
// for kGatherQuiet (at most kGatherMax).
struct HostReq {
  const int* algos;
  int nalgo;
  const PartSource* src;
  const uint64_t* lengths;
  uint32_t* const* digests;
  const HostShard* sh;
  uint64_t slice;
  int rc = S3H_OK;
  std::string err;
  bool done = false;
};

struct DevQueue {
  std::mutex m;
  std::condition_variable cv;
  std::vector<HostReq*> pending;
  bool leader = false;
  double last_overlap = -1e9;  // when a call last found another one on this device
};

constexpr double kGatherQuiet = 300e-6, kGatherMax = 3e-3;

DevQueue& dev_queue(int device) {
  static std::mutex m;
  static std::vector<std::unique_ptr<DevQueue>>* qs = new std::vector<std::unique_ptr<DevQueue>>();
  std::lock_guard<std::mutex> l(m);
  if (qs->size() <= size_t(device)) qs->resize(device + 1);
  if (!(*qs)[device]) (*qs)[device].reset(new DevQueue());
  return *(*qs)[device];
}

bool same_work(const HostReq& a, const HostReq& b) {
  if (a.nalgo != b.nalgo || a.slice != b.slice) return false;
  for (int k = 0; k < a.nalgo; ++k)
    if (a.algos[k] != b.algos[k]) return false;
  return true;
}

// One context, one shard: a single request as it is, several merged into one part list.
int run_merged(HostCtx* C, const std::vector<HostReq*>& batch) {
  const HostReq& f = *batch[0];
  int rc;
  if (batch.size() == 1) {
    rc = run_host_shard_passes(*C, *f.sh, f.algos, f.nalgo, *f.src, f.lengths, f.digests, f.slice);
  } else {
    uint64_t m = 0;
    bool mem = true;
    HostShard sh{f.sh->device, 1, {}, f.sh->threads};
    for (const HostReq* r : batch) {
      m += r->sh->parts.size();
      mem = mem && r->src->parts;
      sh.ndevices = std::max(sh.ndevices, r->sh->ndevices);
      sh.threads = sh.threads && r->sh->threads ? std::max(sh.threads, r->sh->threads) : 0;  // 0 = no cap
    }
    std::vector<uint64_t> lens(m);
    std::vector<const uint8_t*> ptrs(mem ? m : 0);
    std::vector<PartRef> refs(mem ? 0 : m);
    sh.parts.resize(m);
    uint64_t k = 0;
    for (const HostReq* r : batch)
      for (uint64_t g : r->sh->parts) {
        lens[k] = r->lengths[g];
        if (mem) ptrs[k] = r->src->parts[g];
        else refs[k] = r->src->ref(g);
        sh.parts[k] = k;
        ++k;
      }
    PartSource src;
    if (mem) src.parts = ptrs.data();
    else src.refs = refs.data();
    std::vector<uint32_t> out[kHostMaxAlgo];
    uint32_t* outp[kHostMaxAlgo] = {};
    for (int a = 0; a < f.nalgo; ++a) {
      out[a].resize(m * digest_words(f.algos[a]));
      outp[a] = out[a].data();
    }
    rc = run_host_shard_passes(*C, sh, f.algos, f.nalgo, src, lens.data(), outp, f.slice);
    k = 0;
    for (const HostReq* r : batch) {
      for (uint64_t g : r->sh->parts) {
        for (int a = 0; a < f.nalgo && rc == S3H_OK; ++a) {
          const uint32_t dw = digest_words(f.algos[a]);
          std::memcpy(r->digests[a] + dw * g, outp[a] + dw * k, dw * 4);
        }
        ++k;
      }
    }
  }
  return rc;
}

// Runs a batch on the device's context; nothing escapes.
int run_guarded(const std::vector<HostReq*>& batch, std::string* err) {
  HostCtx* C = nullptr;
  int rc;
  try {
    C = host_ctx_cache().acquire(batch[0]->sh->device);
    rc = run_merged(C, batch);
  } catch (const std::bad_alloc&) {
    rc = fail(S3H_ENOMEM, "host batch: out of host memory");
  } catch (...) {
    rc = fail(S3H_EHIP, "host batch: unexpected exception");
  }
  *err = rc ? g_err : std::string();
  if (C) host_ctx_cache().release(C, rc == S3H_OK);
  return rc;
}

// Runs a batch and hands every request its status, so the device queue's leader always gets
// to mark the batch done.  A merged batch that fails is re-run one request at a time: one
// caller's unreadable file range or allocation failure must not fail the other callers,
// and each caller gets its own status and message.
void run_batch(const std::vector<HostReq*>& batch) {
  std::string err;
  const int rc = run_guarded(batch, &err);
  if (rc != S3H_OK && batch.size() > 1) {
    for (HostReq* r : batch) r->rc = run_guarded({r}, &r->err);
    return;
  }
  for (HostReq* r : batch) {
    r->rc = rc;
    r->err = err;
  }
}

// Runs `r` (in a batch with the device's other pending calls); returns when it is done.
void submit(HostReq& r) {
  DevQueue& q = dev_queue(r.sh->device);
  std::unique_lock<std::mutex> l(q.m);
  q.pending.push_back(&r);
  if (q.leader || q.pending.size() > 1) q.last_overlap = wall_s();
  q.cv.notify_all();  // a gathering leader counts arrivals
  q.cv.wait(l, [&] { return r.done || !q.leader; });
  if (r.done) return;
  q.leader = true;
  const double t0 = wall_s();
  for (double t_arr = t0; t0 - q.last_overlap < 1.0;) {
    const size_t had = q.pending.size();
    q.cv.wait_for(l, std::chrono::duration<double>(kGatherQuiet / 3));
    const double t = wall_s();
    if (q.pending.size() != had) t_arr = t;
    if (t - t_arr > kGatherQuiet || t - t0 > kGatherMax) break;
  }
  while (!r.done && !q.pending.empty()) {
    std::vector<HostReq*> batch;
    HostReq* first = q.pending.front();
    for (auto it = q.pending.begin(); it != q.pending.end();) {
      if (same_work(*first, **it)) {
        batch.push_back(*it);
        it = q.pending.erase(it);
      } else {
        ++it;
      }
    }
    l.unlock();
    run_batch(batch);
    l.lock();
    for (HostReq* b : batch) b->done = true;
    q.cv.notify_all();
  }
  q.leader = false;  // a waiting caller takes over what is still pending
  q.cv.notify_all();
}

}  // namespace

extern "C" {

const char* s3h_last_error(void) { return g_err.c_str(); }
int s3h_api_version(void) { return S3H_API_VERSION; }

int s3h_trim(void) {
  host_ctx_cache().trim();
  staging_trim();
  return S3H_OK;
}

int s3h_kernel_policy(int policy, int* previous) {
  if (policy != S3H_POLICY_THROUGHPUT && policy != S3H_POLICY_EFFICIENCY)
    return fail(S3H_EINVAL, "kernel policy: unknown policy %d", policy);
  const int prev = g_kernel_policy.exchange(policy);
  if (previous) *previous = prev;
  return S3H_OK;
}

int s3h_host_threads(int ndevices, int* cpus) {
  if (cpus) *cpus = int(host_cpus());
  return int(host_threads_per_device(ndevices));
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

int s3h_pci_numa(const char* pci_bus_id, int* node, char* cpulist, int len, int* usable_cpus) {
  if (!node) return fail(S3H_EINVAL, "pci numa: null node");
  *node = -1;
  if (cpulist && len > 0) cpulist[0] = 0;
  if (usable_cpus) *usable_cpus = 0;
  std::string local;
  if (int rc = pci_numa(pci_bus_id, node, &local)) return rc;
  if (cpulist && len > 0) std::snprintf(cpulist, size_t(len), "%s", local.c_str());
  cpu_set_t want, mine, both;
  if (usable_cpus && parse_cpulist(local, &want) && sched_getaffinity(0, sizeof mine, &mine) == 0) {
    (void)CPU_AND(&both, &want, &mine);
    *usable_cpus = CPU_COUNT(&both);
  }
  return S3H_OK;
}

int s3h_device_numa_node(int device, int* node, char* cpulist, int len) {
  if (!node) return fail(S3H_EINVAL, "device numa: null node");
  *node = -1;
  char bdf[32];
  if (int rc = s3h_device_pci_bus_id(device, bdf, sizeof bdf)) return rc;
  return s3h_pci_numa(bdf, node, cpulist, len, nullptr);
}

int s3h_host_numa(int mode, int* previous) {
  if (mode < kNumaOff || mode >= int(kMaxNumaNodes))
    return fail(S3H_EINVAL, "host numa: mode %d (want -1 local, -2 off, or a node)", mode);
  const int prev = g_numa_mode.exchange(mode);
  if (previous) *previous = prev;
  if (prev != mode) host_ctx_cache().trim();  // idle contexts re-place on their next call
  return S3H_OK;
}

int s3h_host_numa_info(int device, s3h_host_numa_t* info) {
  if (!info) return fail(S3H_EINVAL, "host numa info: null argument");
  *info = s3h_host_numa_t{-1, -1, 0, -1, -1, 0};
  if (int rc = check_device(device)) return rc;
  const Place P = device_place(device);
  info->device_node = P.dev_node;
  info->target_node = P.node;
  info->bound_cpus = P.ncpus;
  (void)host_ctx_cache().numa_of(device, info);
  return S3H_OK;
}

int s3h_host_alloc(int node, uint64_t bytes, void** out) {
  if (!out || bytes == 0) return fail(S3H_EINVAL, "host alloc: null out-pointer or 0 bytes");
  *out = nullptr;
  if (node < -1 || node >= int(kMaxNumaNodes)) return fail(S3H_EINVAL, "host alloc: bad node %d", node);
  const hipError_t e = pinned_alloc(out, bytes, node);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(e == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "host alloc (%llu B on node %d): %s",
                (unsigned long long)bytes, node, hipGetErrorString(e));
  }
  return S3H_OK;
}

int s3h_host_free(void* p) {
  pinned_free(p);
  return S3H_OK;
}

int s3h_mem_node(const void* p, int* node) {
  if (!p || !node) return fail(S3H_EINVAL, "mem node: null argument");
  *node = mem_node(p);
  return *node >= 0 ? S3H_OK : fail(S3H_EINVAL, "mem node: get_mempolicy failed (%s)", std::strerror(errno));
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

// Consumer waves (= groups) of a skew/skewp grid; 0 for the kernels without a clock probe.
static uint32_t consumer_groups(const s3h_plan_s* P) {
  if (P->algo == S3H_ALGO_MD5) return P->grid;  // md5_pc_kernel: one consumer wave per workgroup
  return (P->kernel == S3H_KERNEL_SKEW && P->quad_waves == 2) || P->kernel == S3H_KERNEL_SKEWS
             ? uint32_t((P->n + 7) / 8)
         : P->kernel == S3H_KERNEL_SKEW || P->kernel == S3H_KERNEL_SKEWP ? P->grid
                                                                          : 0u;
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

static int batch_device(int device, int algo, const void* d_base, const uint64_t* offsets,
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

int s3h_sha256_batch_device(int device, const void* d_base, const uint64_t* offsets,
                            const uint64_t* lengths, uint64_t n, uint32_t* d_digests,
                            void* stream) {
  return batch_device(device, S3H_ALGO_SHA256, d_base, offsets, lengths, n, d_digests, stream);
}

int s3h_md5_batch_device(int device, const void* d_base, const uint64_t* offsets,
                         const uint64_t* lengths, uint64_t n, uint32_t* d_digests, void* stream) {
  return batch_device(device, S3H_ALGO_MD5, d_base, offsets, lengths, n, d_digests, stream);
}

// Shard s (of nshards) gets parts i with i % nshards == s and runs on device devs[s]; a device
// may appear more than once (its shards run concurrently, each on its own context).

static int batch_host_on(const int* algos, int nalgo, const PartSource& src,
                         const uint64_t* lengths, uint64_t n, uint32_t* const* digests,
                         const std::vector<int>& devs, uint64_t slice_bytes) {
  if (!lengths || n == 0) return fail(S3H_EINVAL, "batch_host: bad arguments");
  for (int a = 0; a < nalgo; ++a)
    if (!digests[a]) return fail(S3H_EINVAL, "batch_host: null digest array");
  int count = 0;
  if (int rc = s3h_device_count(&count)) return rc;
  if (devs.empty()) return fail(S3H_EINVAL, "batch_host: no devices");
  for (int d : devs)
    if (d < 0 || d >= count) return fail(S3H_EINVAL, "batch_host: device %d out of range [0,%d)", d, count);
  if (slice_bytes % 64) return fail(S3H_EINVAL, "slice_bytes must be a multiple of 64");
  if (src.parts)
    for (uint64_t i = 0; i < n; ++i)
      if (!src.parts[i] && lengths[i]) return fail(S3H_EINVAL, "batch_host: part %llu is null", (unsigned long long)i);
  const int nshards = int(std::min<uint64_t>(devs.size(), n));
  std::vector<HostShard> shards(nshards);
  for (int k = 0; k < nshards; ++k) shards[k] = {devs[k], nshards, {}, g_stage_threads_cap};
  for (uint64_t i = 0; i < n; ++i) shards[i % nshards].parts.push_back(i);
  std::vector<int> rcs(nshards, S3H_OK);
  std::vector<std::string> errs(nshards);
  auto run = [&](int k) {
    HostReq r{algos, nalgo, &src, lengths, digests, &shards[k], slice_bytes};
    submit(r);
    rcs[k] = r.rc;
    errs[k] = r.err;
  };
  if (nshards == 1) {
    run(0);  // the caller's own thread: its affinity is the caller's business
  } else {   // one thread per device shard, on that device's node (it stages and issues DMAs)
    std::vector<std::thread> pool;
    for (int k = 0; k < nshards; ++k)
      pool.emplace_back([&run, k, place = device_place(shards[k].device)] {
        bind_self(place);
        run(k);
      });
    for (auto& t : pool) t.join();
  }
  for (int k = 0; k < nshards; ++k)
    if (rcs[k]) return fail(rcs[k], "device %d: %s", shards[k].device, errs[k].c_str());
  return S3H_OK;
}

// ndevices GPUs 0..ndevices-1 (0 or more than visible = all visible).
static int batch_host(const int* algos, int nalgo, const PartSource& src,
                      const uint64_t* lengths, uint64_t n, uint32_t* const* digests, int ndevices,
                      uint64_t slice_bytes) {
  int count = 0;
  if (int rc = s3h_device_count(&count)) return rc;
  if (ndevices <= 0 || ndevices > count) ndevices = count;
  std::vector<int> devs(ndevices);
  std::iota(devs.begin(), devs.end(), 0);
  return batch_host_on(algos, nalgo, src, lengths, n, digests, devs, slice_bytes);
}

static int batch_host(int algo, const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                      uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  if (!parts) return fail(S3H_EINVAL, "batch_host: null parts");
  uint32_t* const out[1] = {digests};
  PartSource src;
  src.parts = parts;
  return batch_host(&algo, 1, src, lengths, n, out, ndevices, slice_bytes);
}

int s3h_sha256_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                          uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  return batch_host(S3H_ALGO_SHA256, parts, lengths, n, digests, ndevices, slice_bytes);
}

int s3h_md5_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                       uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  return batch_host(S3H_ALGO_MD5, parts, lengths, n, digests, ndevices, slice_bytes);
}

int s3h_sha256_md5_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                              uint32_t* sha256_digests, uint32_t* md5_digests, int ndevices,
                              uint64_t slice_bytes) {
  static const int algos[2] = {S3H_ALGO_SHA256, S3H_ALGO_MD5};
  uint32_t* const out[2] = {sha256_digests, md5_digests};
  if (!parts) return fail(S3H_EINVAL, "batch_host: null parts");
  PartSource src;
  src.parts = parts;
  return batch_host(algos, 2, src, lengths, n, out, ndevices, slice_bytes);
}

int s3h_sha256_batch_host_on(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                             uint32_t* digests, const int* devices, int ndevices,
                             uint64_t slice_bytes) {
  if (!parts || !devices || ndevices <= 0) return fail(S3H_EINVAL, "batch_host_on: bad arguments");
  static const int algo = S3H_ALGO_SHA256;
  uint32_t* const out[1] = {digests};
  PartSource src;
  src.parts = parts;
  return batch_host_on(&algo, 1, src, lengths, n, out, std::vector<int>(devices, devices + ndevices),
                       slice_bytes);
}

// Open `path` and check that every range lies inside it -- before the call can be merged
// with other callers' (a batch fails as a whole).  Returns the descriptor or -1 (error set).
static int open_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                           uint64_t n) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    fail(S3H_EINVAL, "file_parts: cannot open %s: %s", path, std::strerror(errno));
    return -1;
  }
  struct stat st {};
  if (fstat(fd, &st) != 0) {
    close(fd);
    fail(S3H_EINVAL, "file_parts: cannot stat %s", path);
    return -1;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i] > uint64_t(st.st_size) || lengths[i] > uint64_t(st.st_size) - offsets[i]) {
      close(fd);
      fail(S3H_EINVAL, "file_parts: part %llu [%llu, +%llu) is past the end of %s (%llu B)",
           (unsigned long long)i, (unsigned long long)offsets[i],
           (unsigned long long)lengths[i], path, (unsigned long long)st.st_size);
      return -1;
    }
  return fd;
}

static int file_parts(const int* algos, int nalgo, const char* path, const uint64_t* offsets,
                      const uint64_t* lengths, uint64_t n, uint32_t* const* digests,
                      int ndevices, uint64_t slice_bytes) {
  if (!path || !offsets || !lengths || n == 0)
    return fail(S3H_EINVAL, "file_parts: bad arguments");
  for (int a = 0; a < nalgo; ++a)
    if (!digests[a]) return fail(S3H_EINVAL, "file_parts: null digest array");
  const int fd = open_file_parts(path, offsets, lengths, n);
  if (fd < 0) return S3H_EINVAL;
  PartSource src;
  src.fd = fd;
  src.file_off = offsets;
  const int rc = batch_host(algos, nalgo, src, lengths, n, digests, ndevices, slice_bytes);
  close(fd);
  return rc;
}

int s3h_sha256_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                          uint64_t n, uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  static const int algo = S3H_ALGO_SHA256;
  uint32_t* const out[1] = {digests};
  return file_parts(&algo, 1, path, offsets, lengths, n, out, ndevices, slice_bytes);
}

int s3h_sha256_md5_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                              uint64_t n, uint32_t* sha256_digests, uint32_t* md5_digests,
                              int ndevices, uint64_t slice_bytes) {
  static const int algos[2] = {S3H_ALGO_SHA256, S3H_ALGO_MD5};
  uint32_t* const out[2] = {sha256_digests, md5_digests};
  return file_parts(algos, 2, path, offsets, lengths, n, out, ndevices, slice_bytes);
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
    hipLaunchKernelGGL(s3h::compare_digests_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s,
                       d_dig, d_expected, n, dw, d_mismatch, d_count);
    unsigned long long c = 0;
    hipError_t e = hipGetLastError();
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

int s3h_verify_batch_host(int algo, const uint8_t* const* parts, const uint64_t* lengths,
                          uint64_t n, const uint32_t* expected, uint8_t* mismatch,
                          uint64_t* mismatches, int ndevices) {
  if (!expected || !mismatch || !mismatches) return fail(S3H_EINVAL, "verify: null argument");
  if (algo != S3H_ALGO_SHA256 && algo != S3H_ALGO_MD5)
    return fail(S3H_EINVAL, "verify: unknown algorithm %d", algo);
  const uint32_t dw = digest_words(algo);
  std::vector<uint32_t> got(n * dw);
  if (int rc = batch_host(algo, parts, lengths, n, got.data(), ndevices, 0)) return rc;
  uint64_t c = 0;
  for (uint64_t i = 0; i < n; ++i) {
    mismatch[i] = std::memcmp(&got[dw * i], expected + dw * i, dw * 4) != 0;
    c += mismatch[i];
  }
  *mismatches = c;
  return S3H_OK;
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
  hipLaunchKernelGGL(s3h::generate_kernel, dim3(gx, uint32_t(n)), dim3(256), 0, s,
                     static_cast<uint8_t*>(d_base), d_g, seed);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipFreeAsync(d_g, s));
  // the host vector `g` must outlive the async copy
  HIP_TRY(hipStreamSynchronize(s));
  return S3H_OK;
}

int s3h_stream_create(int device, int algo, uint64_t n, int kernel, s3h_stream_t* out) {
  if (!out) return fail(S3H_EINVAL, "stream: null out-pointer");
  *out = nullptr;
  if (n == 0 || n > kMaxParts) return fail(S3H_EINVAL, "stream: need 0 < n <= 2^31");
  std::vector<uint64_t> zeros(n, 0);
  auto* S = new s3h_stream_s();
  S->device = device;
  S->algo = algo;
  S->n = n;
  S->total.assign(n, 0);
  S->carry.assign(n, 0);
  S->offs.assign(n, 0);
  S->lens.assign(n, 0);
  S->offs2.assign(n, 0);
  S->lens2.assign(n, 0);
  int rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->head);
  if (!rc) rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->body);
  if (!rc) rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->fin);
  if (rc) {
    stream_free(S);
    return rc;
  }
  DeviceGuard g(device);
  const char* what = "chaining state";
  hipError_t e = hipMalloc(&S->d_state, n * 32);
  if (e == hipSuccess) e = hipMalloc(&S->d_carry, n * 64), what = "carries";
  if (e == hipSuccess) e = hipMalloc(&S->d_head, n * 64), what = "head blocks";
  if (e == hipSuccess) e = hipMalloc(&S->d_jobs, n * sizeof(s3h::SpliceJob)), what = "splice jobs";
  if (e == hipSuccess) e = hipMalloc(&S->d_bits, n * 8), what = "bit lengths";
  // per message and set: a splice job, two slots, the bit length, two order entries (8-B
  // aligned in this order)
  const size_t per = sizeof(s3h::SpliceJob) + 2 * sizeof(s3h::Slot) + 8 + 2 * 4;
  if (e == hipSuccess) {
    e = pinned_alloc(reinterpret_cast<void**>(&S->h_pin), 2 * n * per, device_place(device).node);
    what = e == hipSuccess ? "events / stream" : "pinned update staging";
  }
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    uint8_t* pin = S->h_pin + b * n * per;
    S->h_jobs[b] = reinterpret_cast<s3h::SpliceJob*>(pin);
    S->h_slots[b][0] = reinterpret_cast<s3h::Slot*>(pin + n * sizeof(s3h::SpliceJob));
    S->h_slots[b][1] = S->h_slots[b][0] + n;
    S->h_bits[b] = reinterpret_cast<uint64_t*>(S->h_slots[b][1] + n);
    S->h_order[b][0] = reinterpret_cast<uint32_t*>(S->h_bits[b] + n);
    S->h_order[b][1] = S->h_order[b][0] + n;
    e = hipEventCreateWithFlags(&S->staged[b], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&S->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&S->own, hipStreamNonBlocking);
  if (e == hipSuccess) {
    rc = stream_reset(S, S->own);
    // every event recorded once, so the first calls' waits have something to wait for
    for (hipEvent_t ev : {S->staged[0], S->staged[1], S->done})
      if (!rc && hipEventRecord(ev, S->own) != hipSuccess) rc = fail(S3H_EHIP, "stream: event record failed");
    if (!rc && hipStreamSynchronize(S->own) != hipSuccess) rc = fail(S3H_EHIP, "stream: init failed");
  } else {
    (void)hipGetLastError();
    rc = fail(e == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "stream (%llu messages): %s: %s",
              (unsigned long long)n, what, hipGetErrorString(e));
  }
  if (rc) {
    stream_free(S);
    return rc;
  }
  *out = S;
  return S3H_OK;
}

int s3h_stream_update_device(s3h_stream_t S, const void* d_base, const uint64_t* offsets,
                             const uint64_t* lengths, void* stream) {
  if (!S || !lengths || (!offsets && S->n)) return fail(S3H_EINVAL, "stream update: null argument");
  bool any = false;
  for (uint64_t i = 0; i < S->n; ++i) any |= lengths[i] != 0;
  if (any && !d_base) return fail(S3H_EINVAL, "stream update: null d_base");
  DeviceGuard g(S->device);
  return stream_update(S, static_cast<const uint8_t*>(d_base), offsets, lengths,
                       static_cast<hipStream_t>(stream));
}

int s3h_stream_final_device(s3h_stream_t S, uint32_t* d_digests, void* stream) {
  if (!S || !d_digests) return fail(S3H_EINVAL, "stream final: null argument");
  DeviceGuard g(S->device);
  return stream_final(S, d_digests, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {

// The copy threads of host-form stream updates: one pool per device, shared by every stream
// object on it (their copy phases take turns; each pool is as wide as the CPUs the process may
// use, on the device's NUMA node), created on first use and kept for the process.
struct StreamPools {
  std::mutex m;
  std::map<int, std::pair<std::unique_ptr<CopyPool>, std::unique_ptr<std::mutex>>> by_device;
};
StreamPools& stream_pools() {
  static auto* p = new StreamPools();  // never destroyed: threads may outlive static teardown
  return *p;
}

// fn(i) for i in [0, n) on `device`'s stream copy pool (exclusive while it runs)
void stream_pool_run(int device, uint64_t n, const std::function<void(uint64_t)>& fn) {
  StreamPools& P = stream_pools();
  CopyPool* pool;
  std::mutex* run_mu;
  {
    std::lock_guard<std::mutex> l(P.m);
    auto& e = P.by_device[device];
    if (!e.first) {
      e.first.reset(new CopyPool(host_threads_per_device(1) - 1, device_place(device)));
      e.second.reset(new std::mutex());
    }
    pool = e.first.get();
    run_mu = e.second.get();
  }
  std::lock_guard<std::mutex> l(*run_mu);
  pool->run(n, fn);
}

// One host-form update of at most a few hundred MiB (s3h_stream_update_host splits larger
// ones): the chunks are packed at 64-B aligned offsets into device staging set b and hashed on
// `own` once the set's copy has landed; the copy of the next update overlaps this hash.
//   pinned chunks of equal length at a constant stride -> one 2-D DMA;
//   a few other pinned chunks                          -> one DMA each;
//   anything else (pageable, or many ragged pinned)    -> copy threads fill pinned pieces,
//                                                         one DMA per piece.
// Returns once the chunks may be released by the caller.
int stream_host_update_one(s3h_stream_s* S, const uint8_t* const* chunks, const uint64_t* lengths) {
  const uint64_t n = S->n;
  std::vector<uint64_t> offs(n);
  uint64_t sum = 0, L0 = 0;
  bool equal = true;
  for (uint64_t i = 0; i < n; ++i) {
    offs[i] = sum;
    sum += (lengths[i] + 63) & ~uint64_t(63);
    if (i == 0) L0 = lengths[0];
    equal = equal && lengths[i] == L0;
  }
  const unsigned b = S->hs_set;
  S->hs_set ^= 1u;
  if (sum > S->d_hs_cap[b]) {
    HIP_TRY(hipEventSynchronize(S->hs_hashed[b]));  // the set's last hash has read it
    (void)hipFree(S->d_hs[b]);
    S->d_hs[b] = nullptr;
    S->d_hs_cap[b] = 0;
    HIP_TRY(hipMalloc(&S->d_hs[b], sum));
    S->d_hs_cap[b] = sum;
  }
  bool wait_copy = false;  // the DMA reads the caller's memory: wait for it before returning
  if (sum) {
    // set b is rewritten only after the hash that read it (two updates ago) has run
    HIP_TRY(hipStreamWaitEvent(S->copy_s, S->hs_hashed[b], 0));
    std::vector<uint64_t> all(n);
    std::iota(all.begin(), all.end(), uint64_t(0));
    const bool pinned = all_pinned(chunks, lengths, all);
    // equal non-empty chunks at one positive stride (ranges of one buffer): one 2-D DMA
    bool strided = pinned && equal && L0 > 0 && n > 1;
    const uintptr_t c0 = reinterpret_cast<uintptr_t>(chunks[0]);
    const uint64_t stride = strided ? uint64_t(reinterpret_cast<uintptr_t>(chunks[1]) - c0) : 0;
    strided = strided && stride >= L0 && stride < (uint64_t(1) << 62);
    for (uint64_t i = 2; strided && i < n; ++i)
      strided = uint64_t(reinterpret_cast<uintptr_t>(chunks[i]) - c0) == i * stride;
    if (strided) {
      HIP_TRY(hipMemcpy2DAsync(S->d_hs[b], (L0 + 63) & ~uint64_t(63), chunks[0], stride, L0, n,
                               hipMemcpyHostToDevice, S->copy_s));
      wait_copy = true;
    } else if (pinned && n <= kStreamDmaChunks) {
      for (uint64_t i = 0; i < n; ++i)
        if (lengths[i])
          HIP_TRY(hipMemcpyAsync(S->d_hs[b] + offs[i], chunks[i], lengths[i], hipMemcpyHostToDevice, S->copy_s));
      wait_copy = true;
    } else {
      // copy threads fill pinned piece q while piece q^1's DMA runs
      const uint64_t P = std::min<uint64_t>(sum, kStreamPiece);
      if (P > S->h_piece_cap) {
        for (hipEvent_t e : {S->piece_copied[0], S->piece_copied[1]}) HIP_TRY(hipEventSynchronize(e));
        pinned_free(S->h_piece[0]);
        pinned_free(S->h_piece[1]);
        S->h_piece[0] = S->h_piece[1] = nullptr;
        S->h_piece_cap = 0;
        const int node = device_place(S->device).node;
        for (uint8_t*& h : S->h_piece)
          HIP_TRY(pinned_alloc(reinterpret_cast<void**>(&h), P, node));
        S->h_piece_cap = P;
      }
      for (uint64_t lo = 0; lo < sum; lo += P) {
        const unsigned q = S->piece_next;  // alternates across updates too
        S->piece_next ^= 1u;
        const uint64_t hi = std::min(sum, lo + P);
        HIP_TRY(hipEventSynchronize(S->piece_copied[q]));  // its previous DMA has read it
        // the chunks overlapping [lo, hi) of the packed layout (offs ascending)
        const uint64_t i0 = uint64_t(std::upper_bound(offs.begin(), offs.end(), lo) - offs.begin()) - 1;
        const uint64_t i1 = uint64_t(std::lower_bound(offs.begin(), offs.end(), hi) - offs.begin());
        uint8_t* const dst = S->h_piece[q];
        stream_pool_run(S->device, i1 - i0, [&](uint64_t k) {
          const uint64_t i = i0 + k, a = std::max(offs[i], lo), e = std::min(offs[i] + lengths[i], hi);
          if (e > a) std::memcpy(dst + (a - lo), chunks[i] + (a - offs[i]), e - a);
        });
        HIP_TRY(hipMemcpyAsync(S->d_hs[b] + lo, dst, hi - lo, hipMemcpyHostToDevice, S->copy_s));
        HIP_TRY(hipEventRecord(S->piece_copied[q], S->copy_s));
      }
    }
    HIP_TRY(hipEventRecord(S->hs_copied[b], S->copy_s));
    HIP_TRY(hipStreamWaitEvent(S->own, S->hs_copied[b], 0));
  }
  const int rc = stream_update(S, S->d_hs[b], offs.data(), lengths, S->own);
  HIP_TRY(hipEventRecord(S->hs_hashed[b], S->own));
  if (wait_copy) HIP_TRY(hipEventSynchronize(S->hs_copied[b]));
  return rc;
}

}  // namespace

extern "C" {

// A large update is appended as consecutive sub-updates of at most `sl` bytes of every chunk
// (64-B multiples: no carry between them), so the copy of one overlaps the hash of the one
// before -- appending a chunk in pieces is the same as appending it whole.
int s3h_stream_update_host(s3h_stream_t S, const uint8_t* const* chunks, const uint64_t* lengths) {
  if (!S || !chunks || !lengths) return fail(S3H_EINVAL, "stream update: null argument");
  if (!S->failed.empty())
    return fail(S3H_EINVAL, "stream object failed earlier (%s): destroy it", S->failed.c_str());
  const uint64_t n = S->n;
  uint64_t sum = 0, longest = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (lengths[i] && !chunks[i]) return fail(S3H_EINVAL, "stream update: chunk %llu is null", (unsigned long long)i);
    sum += (lengths[i] + 63) & ~uint64_t(63);
    longest = std::max(longest, lengths[i]);
  }
  DeviceGuard g(S->device);
  if (!S->copy_s) {
    {  // staging left by an earlier object on this device, if any
      std::lock_guard<std::mutex> l(staging_cache().m);
      auto& v = staging_cache().free[S->device];
      if (!v.empty()) {
        const StreamStaging st = v.back();
        v.pop_back();
        std::copy(st.d_hs, st.d_hs + 2, S->d_hs);
        std::copy(st.d_hs_cap, st.d_hs_cap + 2, S->d_hs_cap);
        std::copy(st.h_piece, st.h_piece + 2, S->h_piece);
        S->h_piece_cap = st.h_piece_cap;
      }
    }
    HIP_TRY(hipStreamCreateWithFlags(&S->copy_s, hipStreamNonBlocking));
    for (hipEvent_t* e : {&S->hs_copied[0], &S->hs_copied[1], &S->hs_hashed[0], &S->hs_hashed[1],
                          &S->piece_copied[0], &S->piece_copied[1]})
      HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  const uint64_t sl = std::max<uint64_t>(kStreamSubMin, (kStreamSubBytes / std::max<uint64_t>(n, 1)) & ~uint64_t(63));
  if (sum <= 2 * kStreamSubBytes || longest <= sl) return stream_host_update_one(S, chunks, lengths);
  std::vector<const uint8_t*> p(n);
  std::vector<uint64_t> l(n);
  for (uint64_t at = 0; at < longest; at += sl) {
    for (uint64_t i = 0; i < n; ++i) {
      l[i] = lengths[i] > at ? std::min(sl, lengths[i] - at) : 0;
      p[i] = l[i] ? chunks[i] + at : nullptr;
    }
    if (int rc = stream_host_update_one(S, p.data(), l.data())) return rc;
  }
  return S3H_OK;
}

int s3h_stream_final_host(s3h_stream_t S, uint32_t* digests) {
  if (!S || !digests) return fail(S3H_EINVAL, "stream final: null argument");
  DeviceGuard g(S->device);
  const uint64_t bytes = S->n * digest_words(S->algo) * 4;
  if (!S->d_dig) HIP_TRY(hipMalloc(&S->d_dig, S->n * 32));
  int rc = stream_final(S, S->d_dig, S->own);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(digests, S->d_dig, bytes, hipMemcpyDeviceToHost, S->own));
  HIP_TRY(hipStreamSynchronize(S->own));
  return stream_check(S, S->own);
}

int s3h_stream_status(s3h_stream_t S, void* stream) {
  if (!S) return fail(S3H_EINVAL, "stream status: null stream");
  DeviceGuard g(S->device);
  return stream_check(S, static_cast<hipStream_t>(stream));
}

int s3h_stream_stats(s3h_stream_t S, uint64_t* slot_reuses, uint64_t* slot_refills) {
  if (!S) return fail(S3H_EINVAL, "stream stats: null stream");
  if (slot_reuses) *slot_reuses = S->slot_reuses;
  if (slot_refills) *slot_refills = S->slot_refills;
  return S3H_OK;
}

int s3h_stream_total(s3h_stream_t S, uint64_t i, uint64_t* total) {
  if (!S || !total || i >= S->n) return fail(S3H_EINVAL, "stream total: bad argument");
  *total = S->total[i];
  return S3H_OK;
}

int s3h_stream_destroy(s3h_stream_t S) {
  if (S) stream_free(S);
  return S3H_OK;
}

}  // extern "C"

#include "route.hpp"
