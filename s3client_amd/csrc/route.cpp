// route.cpp -- size-aware routing of host-resident batches (include/s3hash.h "size-aware
// routing"): the measured model, its observed corrections and re-measurement, and the routed
// entry points for SHA-256, MD5 and both digests (Content-MD5 + x-amz-content-sha256).
//
// The model's rates are measured on this host and on each device a routed call uses, lazily
// (a digest set's CPU rates on its first routed call, a device's chain and H2D rates on the
// first call that shards onto it).  A measurement is a snapshot taken under whatever load the
// host and the GPUs carry at that moment, so the model is not trusted forever:
//   * every AUTO / SPLIT call times the route it ran -- both sides of a split separately --
//     and keeps, per side (GPU, CPU) and digest set, the ratio observed / predicted as an
//     EWMA (weight 1/2, each observation clamped to [1/4, 8]); decisions scale that side's
//     estimate by it, and the factor of a side a call did not use relaxes 10 % toward 1;
//   * when a call's time differs from its corrected prediction by more than 25 %, the model is
//     marked stale and re-measured (rates of every digest set and device again) at the next
//     routed call once the back-off allows (0.5 s after the previous measurement at first);
//     a side's factors are reset when its re-measured rates moved by more than 15 % from the
//     ones the decisions used (the load changed: the factor described the old one), and kept
//     when they did not (a bias the probes cannot see -- e.g. a co-tenant holding some of the
//     host CPUs only while batches run), the back-off then doubling (to 60 s)
//     so a steady bias does not re-measure on every call;
//   * every s3h_route_refresh_calls routed calls (default 64) it is re-measured anyway, so a
//     route that looked slow when measured -- and was therefore never taken again, leaving
//     nothing to observe -- is re-priced within a bounded number of calls.
// AUTO needs a visible GPU (S3H_ENODEV otherwise): it chooses between paths with identical
// digests and is never a fallback for a missing device.  S3H_ROUTE_GPU (the default
// everywhere, and the only route the bench metric uses) is the batched host path unchanged.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "internal.hpp"
#include "route_plan.hpp"

namespace s3h::host {
// host_path.cpp: the GPU host path for any algorithm list (memory parts or file ranges)
int host_batch_algos(const int* algos, int nalgo, const uint8_t* const* parts, const char* path,
                     const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                     uint32_t* const* digests, int ndevices);
}  // namespace s3h::host

using namespace s3h::host;

namespace {

constexpr double kDiverge = 0.25;         // |observed / predicted - 1| that marks the model stale
constexpr double kRemeasureMinS = 0.5;    // divergence-triggered re-measurement back-off: first
constexpr double kRemeasureMaxS = 60.0;   // ... and longest (doubling while the rates hold)
constexpr double kMoved = 0.15;           // re-measured rates this far from the used ones: reset
constexpr double kRelax = 0.9;            // an unused side's factor: f <- 1 + (f - 1) x 0.9
constexpr int kRefreshCallsDefault = 64;  // re-measure after this many routed calls

struct DevRates {
  bool have_h2d = false;
  double h2d = 0;
  bool have_chain[3] = {false, false, false};
  double chain[3] = {0, 0, 0};
};

struct RouteState {
  std::mutex mu;
  bool have_cpu[3] = {false, false, false};
  double cpu1[3] = {0, 0, 0}, cpu_all[3] = {0, 0, 0};
  bool have_staged = false, have_call = false;
  double staged = 0, staged_file = 0, call_s = 0;
  int cpu_threads = 0;
  std::vector<DevRates> dev;
  double f_gpu[3] = {1, 1, 1}, f_cpu[3] = {1, 1, 1};  // observed / predicted, per digest set
  double scale[4] = {1, 1, 1, 1};  // s3h_route_scale: chain, h2d, cpu, staged
  double t_measured = -1e9;
  double backoff = kRemeasureMinS;
  // the effective rates (scale applied) decisions used before the last invalidation, and
  // whether a re-measurement moved them (per side): compared in ensure()
  bool have_prev = false;
  double prev_cpu1[3] = {0, 0, 0}, prev_chain[3] = {0, 0, 0}, prev_h2d = 0;
  bool moved_gpu = false, moved_cpu = false;
  uint64_t measurements = 0, calls = 0, divergences = 0, calls_since = 0;
  bool stale = false;
  int refresh_calls = [] {
    const char* e = std::getenv("S3H_ROUTE_REFRESH_CALLS");
    return e && *e ? std::max(0, std::atoi(e)) : kRefreshCallsDefault;
  }();
};

RouteState& route_state() {
  static auto* s = new RouteState();  // never destroyed: routed calls may outlive static teardown
  return *s;
}

bool trace_route() {
  static const bool on = std::getenv("S3H_TRACE_ROUTE") != nullptr;
  return on;
}

void invalidate(RouteState& S) {
  // remember what the decisions used (device 0's GPU rates, every digest set's CPU rate)
  S.have_prev = true;
  for (int a = 0; a < 3; ++a) {
    S.prev_cpu1[a] = S.have_cpu[a] ? S.cpu1[a] * S.scale[2] : 0;
    S.prev_chain[a] = !S.dev.empty() && S.dev[0].have_chain[a] ? S.dev[0].chain[a] * S.scale[0] : 0;
  }
  S.prev_h2d = !S.dev.empty() && S.dev[0].have_h2d ? S.dev[0].h2d * S.scale[1] : 0;
  for (bool& h : S.have_cpu) h = false;
  S.have_staged = S.have_call = false;
  for (DevRates& d : S.dev) d = DevRates{};
  for (double& x : S.scale) x = 1;
  S.stale = false;
  S.calls_since = 0;
  S.moved_gpu = S.moved_cpu = false;
}

bool moved(double before, double now) {
  return before > 0 && now > 0 && std::fabs(now / before - 1.0) > kMoved;
}

// One device's lone-chain rate of digest set `dig` and/or its pinned H2D rate.
int measure_device(int device, unsigned dig, bool chain, bool h2d, DevRates* out) {
  DeviceGuard g(device);
  constexpr uint64_t kChain = 1ull << 20, kCopy = 32ull << 20;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  uint8_t *d = nullptr, *hp = nullptr;
  uint32_t* dd = nullptr;
  s3h_plan_s* P[2] = {nullptr, nullptr};
  auto cleanup = [&] {
    if (s) (void)hipStreamSynchronize(s);
    for (s3h_plan_s* p : P) s3h_plan_destroy(p);
    if (hp) pinned_free(hp);
    (void)hipFree(d);
    (void)hipFree(dd);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipGetLastError();
  };
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMalloc(&d, h2d ? kCopy : kChain);
  if (e == hipSuccess) e = hipMalloc(&dd, 64);
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, h2d ? kCopy : kChain, s);
  float ms = 0;
  int rc = S3H_OK;
  auto timed = [&](auto launch, double* best) {  // best of launches 2-3 (the first ramps the clock)
    *best = 1e30;
    for (int r = 0; r < 3 && e == hipSuccess && rc == S3H_OK; ++r) {
      e = hipEventRecord(e0, s);
      if (e == hipSuccess) rc = launch();
      if (e == hipSuccess && rc == S3H_OK) e = hipEventRecord(e1, s);
      if (e == hipSuccess && rc == S3H_OK) e = hipEventSynchronize(e1);
      if (e == hipSuccess && rc == S3H_OK) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && rc == S3H_OK && r > 0) *best = std::min(*best, double(ms) * 1e-3);
    }
  };
  const int a = dig_index(dig);
  if (chain && e == hipSuccess) {
    const uint64_t off = 0, len = kChain;
    if (dig & S3H_DIGESTS_SHA256) rc = plan_build(device, S3H_ALGO_SHA256, &off, &len, 1, S3H_KERNEL_AUTO, &P[0]);
    if (rc == S3H_OK && (dig & S3H_DIGESTS_MD5))
      rc = plan_build(device, S3H_ALGO_MD5, &off, &len, 1, S3H_KERNEL_AUTO, &P[1]);
    double best = 0;
    if (rc == S3H_OK && dig == S3H_DIGESTS_BOTH)  // both digests from one grid, as the host path runs them
      timed([&] { return dual_launch(P[0], P[1], d, dd, dd + 8, 0, P[0]->max_blocks, 0, false, s); }, &best);
    else if (rc == S3H_OK)
      timed([&] {
        s3h_plan_s* Q = P[0] ? P[0] : P[1];
        return plan_launch(Q, d, dd, 0, Q->max_blocks, 0, s, false);
      }, &best);
    for (s3h_plan_s* p : P)
      if (rc == S3H_OK && e == hipSuccess && p) rc = plan_check(p, s);
    if (rc == S3H_OK && e == hipSuccess) {
      out->chain[a] = double(kChain) / best;
      out->have_chain[a] = true;
    }
  }
  if (h2d && e == hipSuccess && rc == S3H_OK) {
    e = pinned_alloc(reinterpret_cast<void**>(&hp), kCopy, device_place(device).node);
    if (e == hipSuccess) std::memset(hp, 0x5a, kCopy);
    double best = 1e30;
    for (int r = 0; r < 4 && e == hipSuccess; ++r) {
      e = hipEventRecord(e0, s);
      if (e == hipSuccess) e = hipMemcpyAsync(d, hp, kCopy, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(e1, s);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && r > 0) best = std::min(best, double(ms) * 1e-3);
    }
    if (e == hipSuccess) {
      out->h2d = double(kCopy) / best;
      out->have_h2d = true;
    }
  }
  const hipError_t err = e;
  cleanup();
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(err == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "route model, device %d: %s", device,
                hipGetErrorString(err));
  return S3H_OK;
}

// The rates a call of digest set `dig` over devices [0, devs) needs, measuring what is missing
// (and everything again when the model is stale or due for its refresh); S.mu held.
int ensure(RouteState& S, unsigned dig, int devs) {
  const double now = wall_s();
  const bool remeasure = (S.stale && now - S.t_measured >= S.backoff) ||
                         (S.refresh_calls > 0 && S.calls_since >= uint64_t(S.refresh_calls));
  if (remeasure) invalidate(S);
  const int a = dig_index(dig);
  bool measured = false;
  if (!S.cpu_threads) S.cpu_threads = int(host_cpus());
  if (!S.have_cpu[a]) {
    S.cpu1[a] = one_thread_rate(dig);
    S.cpu_all[a] = team_rate(unsigned(S.cpu_threads), dig);
    S.have_cpu[a] = measured = true;
    S.moved_cpu = S.moved_cpu || moved(S.prev_cpu1[a], S.cpu1[a]);
  }
  if (!S.have_staged) {
    S.staged = team_rate(unsigned(S.cpu_threads), 0);
    S.staged_file = pread_team_rate(unsigned(S.cpu_threads));
    S.have_staged = measured = true;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    (void)hipGetLastError();
    if (measured) S.t_measured = now;
    return fail(S3H_ENODEV, "no HIP device visible (S3H_ROUTE_AUTO chooses between the GPU and the "
                            "CPU drop-in; it is not a fallback)");
  }
  if (S.dev.size() < size_t(count)) S.dev.resize(size_t(count));
  devs = std::max(1, std::min(devs, count));
  for (int d = 0; d < devs; ++d) {
    DevRates& D = S.dev[size_t(d)];
    if (D.have_chain[a] && D.have_h2d) continue;
    if (int rc = measure_device(d, dig, !D.have_chain[a], !D.have_h2d, &D)) return rc;
    measured = true;
    if (d == 0) S.moved_gpu = S.moved_gpu || moved(S.prev_chain[a], D.chain[a]) || moved(S.prev_h2d, D.h2d);
  }
  if (!S.have_call) {
    // fixed cost of one host-path call: a one-block part, timed on its second call (the first
    // builds the device's cached host context)
    static const uint8_t tiny[64] = {};
    const uint8_t* tp = tiny;
    const uint64_t tl = sizeof tiny;
    uint32_t th[8];
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
      const double t0 = wall_s();
      if (int rc = s3h_sha256_batch_host(&tp, &tl, 1, th, 1, 0)) return rc;
      if (r > 0) best = std::min(best, wall_s() - t0);
    }
    S.call_s = best;
    S.have_call = measured = true;
  }
  if (measured) {
    S.t_measured = now;
    ++S.measurements;
  }
  if (remeasure && S.have_prev) {
    // the rates moved: the factors described the old conditions; else keep them and back off
    if (S.moved_gpu) for (double& f : S.f_gpu) f = 1;
    if (S.moved_cpu) for (double& f : S.f_cpu) f = 1;
    S.backoff = S.moved_gpu || S.moved_cpu ? kRemeasureMinS : std::min(kRemeasureMaxS, 2 * S.backoff);
  }
  return S3H_OK;
}

// The decision inputs for devices [0, devs): the slowest device's chain and H2D rates.
Rates snapshot(const RouteState& S, int devs, unsigned dig) {
  Rates R;
  R.cpu_threads = std::max(1, S.cpu_threads);
  R.devices = std::max(1, int(S.dev.size()));
  devs = std::min(devs, int(S.dev.size()));  // 0 without a device: no GPU rates
  for (int a = 0; a < 3; ++a) {
    R.cpu1[a] = S.cpu1[a] * S.scale[2];
    R.cpu_all[a] = S.cpu_all[a] * S.scale[2];
    double c = 0;
    for (int d = 0; d < devs; ++d)
      if (S.dev[size_t(d)].have_chain[a]) c = c > 0 ? std::min(c, S.dev[size_t(d)].chain[a]) : S.dev[size_t(d)].chain[a];
    R.chain[a] = c * S.scale[0];
  }
  double h = 0;
  for (int d = 0; d < devs; ++d)
    if (S.dev[size_t(d)].have_h2d) h = h > 0 ? std::min(h, S.dev[size_t(d)].h2d) : S.dev[size_t(d)].h2d;
  R.h2d = h * S.scale[1];
  R.staged = S.staged * S.scale[3];
  R.staged_file = S.staged_file * S.scale[3];
  R.call_s = S.call_s;
  R.f_gpu = S.f_gpu[dig_index(dig)];
  R.f_cpu = S.f_cpu[dig_index(dig)];
  return R;
}

int devices_for(int ndevices, int count) {
  return ndevices > 0 ? std::min(ndevices, count) : count;
}

// One observation of a side (0 GPU, 1 CPU) for digest set index a: raw prediction `raw`
// seconds, observed `t`.
void observe_side(RouteState& S, int side, int a, double raw, double t) {
  if (!(raw > 0) || !(t > 0)) return;
  double& f = side == 0 ? S.f_gpu[a] : S.f_cpu[a];
  const double ratio = std::min(8.0, std::max(0.25, t / raw));
  if (std::fabs(t / (raw * f) - 1.0) > kDiverge) {
    ++S.divergences;
    S.stale = true;
  }
  f = 0.5 * f + 0.5 * ratio;
}

void observe(const Decision& D, unsigned dig, double t, double t_gpu, double t_cpu) {
  RouteState& S = route_state();
  std::lock_guard<std::mutex> l(S.mu);
  const int a = dig_index(dig);
  ++S.calls;
  ++S.calls_since;
  if (D.route == S3H_ROUTE_GPU) {
    observe_side(S, 0, a, D.g, t);
    S.f_cpu[a] = 1 + (S.f_cpu[a] - 1) * kRelax;
  } else if (D.route == S3H_ROUTE_CPU) {
    observe_side(S, 1, a, D.c, t);
    S.f_gpu[a] = 1 + (S.f_gpu[a] - 1) * kRelax;
  } else {
    observe_side(S, 0, a, D.sp.g, t_gpu);
    observe_side(S, 1, a, D.sp.c, t_cpu);
  }
}

// The GPU host path for digest set `dig` (parts or file ranges).
int gpu_run(unsigned dig, const uint8_t* const* parts, const char* path, const uint64_t* offsets,
            const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5v, int ndevices) {
  int algos[2];
  uint32_t* out[2];
  int k = 0;
  if (dig & S3H_DIGESTS_SHA256) algos[k] = S3H_ALGO_SHA256, out[k++] = sha;
  if (dig & S3H_DIGESTS_MD5) algos[k] = S3H_ALGO_MD5, out[k++] = md5v;
  return host_batch_algos(algos, k, parts, path, offsets, lengths, n, out, ndevices);
}

struct GpuSideCtx {
  unsigned dig;
  const char* path;
  int ndevices;
};

int gpu_side(void* ctx, const uint8_t* const* parts, const uint64_t* offsets, const uint64_t* lengths,
             uint64_t n, uint32_t* sha, uint32_t* md5v) {
  const GpuSideCtx& c = *static_cast<GpuSideCtx*>(ctx);
  try {
    return gpu_run(c.dig, parts, c.path, offsets, lengths, n, sha, md5v, c.ndevices);
  } catch (const std::exception&) {  // nothing escapes into the split driver
    return fail(S3H_ENOMEM, "split route, gpu side: out of host resources");
  }
}

int cpu_run(unsigned dig, const uint8_t* const* parts, const char* path, const uint64_t* offsets,
            const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5v) {
  FdGuard fd;
  if (path)
    if (int rc = open_ranges(path, offsets, lengths, n, &fd.fd)) return rc;
  return cpu_batch(dig, parts, fd.fd, offsets, lengths, n, sha, md5v, host_cpus());
}

// The routed entry points: parts (path == null) or file ranges.
int routed(unsigned dig, const uint8_t* const* parts, const char* path, const uint64_t* offsets,
           const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5v, int ndevices,
           int route, int* taken) {
  if (taken) *taken = -1;
  if (!lengths || n == 0 || (!path && !parts) || (path && !offsets))
    return fail(S3H_EINVAL, "routed batch: null argument or n == 0");
  if (((dig & S3H_DIGESTS_SHA256) && !sha) || ((dig & S3H_DIGESTS_MD5) && !md5v))
    return fail(S3H_EINVAL, "routed batch: null digest array");
  if (route != S3H_ROUTE_GPU && route != S3H_ROUTE_CPU && route != S3H_ROUTE_AUTO && route != S3H_ROUTE_SPLIT)
    return fail(S3H_EINVAL, "routed batch: unknown route %d", route);
  if (parts && route != S3H_ROUTE_GPU)
    for (uint64_t i = 0; i < n; ++i)
      if (!parts[i] && lengths[i]) return fail(S3H_EINVAL, "cpu route: part %llu is null", (unsigned long long)i);
  int rc;
  if (route == S3H_ROUTE_GPU) {
    rc = gpu_run(dig, parts, path, offsets, lengths, n, sha, md5v, ndevices);
  } else if (route == S3H_ROUTE_CPU) {
    rc = cpu_run(dig, parts, path, offsets, lengths, n, sha, md5v);
  } else {
    RouteState& S = route_state();
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
      (void)hipGetLastError();
      return fail(S3H_ENODEV, "no HIP device visible (S3H_ROUTE_AUTO chooses between the GPU and "
                              "the CPU drop-in; it is not a fallback)");
    }
    const int devs = int(std::min<uint64_t>(n, uint64_t(devices_for(ndevices, count))));
    Rates R;
    {
      std::lock_guard<std::mutex> l(S.mu);
      if (int e = ensure(S, dig, devs)) return e;
      R = snapshot(S, devs, dig);
    }
    const int source = path ? S3H_SOURCE_FILE
                       : all_pinned(parts, lengths, nullptr, n) ? S3H_SOURCE_PINNED : S3H_SOURCE_PAGEABLE;
    const Decision D = decide(R, dig, lengths, n, ndevices, source, route);
    if (trace_route())
      std::fprintf(stderr, "[s3h route] %llu parts (%s, digests %u): gpu %.4f s, cpu %.4f s (%d threads), "
                   "split %.4f s (%llu longest on the cpu, %u staging threads per gpu), factors gpu %.3f "
                   "cpu %.3f -> %s\n", (unsigned long long)n,
                   source == S3H_SOURCE_FILE ? "file" : source ? "pageable" : "pinned", dig,
                   D.g * R.f_gpu, D.c * R.f_cpu, R.cpu_threads, D.sp.m ? D.sp.s : 0.0,
                   (unsigned long long)D.sp.m, D.sp.tg, R.f_gpu, R.f_cpu,
                   D.route == S3H_ROUTE_SPLIT ? "split" : D.route == S3H_ROUTE_CPU ? "cpu" : "gpu");
    const double t0 = wall_s();
    double tg = 0, tc = 0;
    if (D.route == S3H_ROUTE_SPLIT) {
      GpuSideCtx ctx{dig, path, ndevices};
      rc = split_run_impl(dig, parts, path, offsets, lengths, n, sha, md5v, ndevices, count, D.order,
                          D.sp, gpu_side, &ctx, &tg, &tc);
    } else if (D.route == S3H_ROUTE_GPU) {
      rc = gpu_run(dig, parts, path, offsets, lengths, n, sha, md5v, ndevices);
    } else {
      rc = cpu_run(dig, parts, path, offsets, lengths, n, sha, md5v);
    }
    const double t = wall_s() - t0;
    if (rc == S3H_OK) observe(D, dig, t, tg, tc);
    if (rc == S3H_OK && trace_route())
      std::fprintf(stderr, "[s3h route]   observed %.4f s (gpu side %.4f s vs %.4f raw, cpu side %.4f s vs "
                   "%.4f raw)\n", t, D.route == S3H_ROUTE_SPLIT ? tg : D.route == S3H_ROUTE_GPU ? t : 0.0,
                   D.route == S3H_ROUTE_SPLIT ? D.sp.g : D.g, D.route == S3H_ROUTE_SPLIT ? tc : D.route == S3H_ROUTE_CPU ? t : 0.0,
                   D.route == S3H_ROUTE_SPLIT ? D.sp.c : D.c);
    if (rc == S3H_OK && taken) *taken = D.route;
    return rc;
  }
  if (rc == S3H_OK && taken) *taken = route;
  return rc;
}

template <class F>
int guarded(const char* what, F f) {
  try {
    return f();
  } catch (const std::exception&) {  // nothing escapes the C-ABI
    return fail(S3H_ENOMEM, "%s: out of host resources", what);
  }
}

}  // namespace

extern "C" {

int s3h_route_model(s3h_route_model_t* m) {
  if (!m) return fail(S3H_EINVAL, "route model: null argument");
  return guarded("route model", [&]() -> int {
    RouteState& S = route_state();
    std::lock_guard<std::mutex> l(S.mu);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    const int rc = ensure(S, S3H_DIGESTS_SHA256, std::max(1, count));
    const Rates R = snapshot(S, std::max(1, count), S3H_DIGESTS_SHA256);
    *m = s3h_route_model_t{};
    m->cpu_bytes_per_s = R.cpu1[0];
    m->cpu_all_bytes_per_s = R.cpu_all[0];
    m->staged_bytes_per_s = R.staged;
    m->cpu_threads = R.cpu_threads;
    if (rc) return rc;  // S3H_ENODEV: the CPU fields are set
    m->chain_bytes_per_s = R.chain[0];
    m->h2d_bytes_per_s = R.h2d;
    m->call_s = R.call_s;
    m->devices = count;
    return S3H_OK;
  });
}

int s3h_route_rates(s3h_route_rates_t* r) {
  if (!r || r->size < offsetof(s3h_route_rates_t, staged_bytes_per_s))
    return fail(S3H_EINVAL, "route rates: null or too small (set size = sizeof(s3h_route_rates_t))");
  return guarded("route rates", [&]() -> int {
    RouteState& S = route_state();
    std::lock_guard<std::mutex> l(S.mu);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    int rc = S3H_OK;
    for (unsigned dig = 1; dig <= 3 && rc == S3H_OK; ++dig) rc = ensure(S, dig, std::max(1, count));
    const Rates R = snapshot(S, std::max(1, count), S3H_DIGESTS_SHA256);
    s3h_route_rates_t full{};
    full.size = uint32_t(std::min<size_t>(r->size, sizeof full));
    full.version = S3H_API_VERSION;
    full.cpu_threads = R.cpu_threads;
    full.devices = count;
    for (int a = 0; a < 3; ++a) {
      full.cpu_bytes_per_s[a] = R.cpu1[a];
      full.cpu_all_bytes_per_s[a] = R.cpu_all[a];
      full.chain_bytes_per_s[a] = R.chain[a];
    }
    full.h2d_bytes_per_s = R.h2d;
    full.staged_bytes_per_s = R.staged;
    full.call_s = R.call_s;
    for (int a = 0; a < 3; ++a) {
      full.gpu_factor[a] = S.f_gpu[a];
      full.cpu_factor[a] = S.f_cpu[a];
    }
    full.measurements = S.measurements;
    full.routed_calls = S.calls;
    full.divergences = S.divergences;
    full.age_s = wall_s() - S.t_measured;
    full.staged_file_bytes_per_s = R.staged_file;
    std::memcpy(r, &full, full.size);
    return rc;
  });
}

int s3h_route_device_rates(int device, int digests, double* chain_bytes_per_s, double* h2d_bytes_per_s) {
  if (!valid_digests(digests)) return fail(S3H_EINVAL, "route device rates: unknown digest set %d", digests);
  if (int rc = check_device(device)) return rc;
  return guarded("route device rates", [&]() -> int {
    RouteState& S = route_state();
    std::lock_guard<std::mutex> l(S.mu);
    if (int rc = ensure(S, unsigned(digests), device + 1)) return rc;
    const DevRates& D = S.dev[size_t(device)];
    if (chain_bytes_per_s) *chain_bytes_per_s = D.chain[dig_index(unsigned(digests))] * S.scale[0];
    if (h2d_bytes_per_s) *h2d_bytes_per_s = D.h2d * S.scale[1];
    return S3H_OK;
  });
}

int s3h_route_scale(int which, double factor) {
  if (which < S3H_RATE_CHAIN || which > S3H_RATE_STAGED || !(factor > 0) || !std::isfinite(factor))
    return fail(S3H_EINVAL, "route scale: rate %d, factor %g", which, factor);
  RouteState& S = route_state();
  std::lock_guard<std::mutex> l(S.mu);
  S.scale[which] = factor;
  return S3H_OK;
}

int s3h_route_refresh_calls(int calls, int* previous) {
  if (calls < 0) return fail(S3H_EINVAL, "route refresh: %d calls", calls);
  RouteState& S = route_state();
  std::lock_guard<std::mutex> l(S.mu);
  if (previous) *previous = S.refresh_calls;
  S.refresh_calls = calls;
  return S3H_OK;
}

int s3h_sha256_batch_routed(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                            uint32_t* digests, int ndevices, int route, int* taken) {
  return guarded("routed batch", [&]() -> int {
    return routed(S3H_DIGESTS_SHA256, parts, nullptr, nullptr, lengths, n, digests, nullptr, ndevices, route, taken);
  });
}

int s3h_md5_batch_routed(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                         uint32_t* digests, int ndevices, int route, int* taken) {
  return guarded("routed md5 batch", [&]() -> int {
    return routed(S3H_DIGESTS_MD5, parts, nullptr, nullptr, lengths, n, nullptr, digests, ndevices, route, taken);
  });
}

int s3h_sha256_md5_batch_routed(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                                uint32_t* sha256_digests, uint32_t* md5_digests, int ndevices,
                                int route, int* taken) {
  return guarded("routed dual batch", [&]() -> int {
    return routed(S3H_DIGESTS_BOTH, parts, nullptr, nullptr, lengths, n, sha256_digests, md5_digests,
                  ndevices, route, taken);
  });
}

int s3h_sha256_file_parts_routed(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                                 uint64_t n, uint32_t* digests, int ndevices, int route, int* taken) {
  if (!path) return fail(S3H_EINVAL, "routed file parts: null path");
  return guarded("routed file parts", [&]() -> int {
    return routed(S3H_DIGESTS_SHA256, nullptr, path, offsets, lengths, n, digests, nullptr, ndevices, route, taken);
  });
}

int s3h_sha256_md5_file_parts_routed(const char* path, const uint64_t* offsets,
                                     const uint64_t* lengths, uint64_t n, uint32_t* sha256_digests,
                                     uint32_t* md5_digests, int ndevices, int route, int* taken) {
  if (!path) return fail(S3H_EINVAL, "routed dual file parts: null path");
  return guarded("routed dual file parts", [&]() -> int {
    return routed(S3H_DIGESTS_BOTH, nullptr, path, offsets, lengths, n, sha256_digests, md5_digests,
                  ndevices, route, taken);
  });
}

int s3h_verify_batch_routed(int algo, const uint8_t* const* parts, const uint64_t* lengths,
                            uint64_t n, const uint32_t* expected, uint8_t* mismatch,
                            uint64_t* mismatches, int ndevices, int route, int* taken) {
  if (taken) *taken = -1;
  if (!expected || !mismatch || !mismatches) return fail(S3H_EINVAL, "verify routed: null argument");
  if (algo != S3H_ALGO_SHA256 && algo != S3H_ALGO_MD5)
    return fail(S3H_EINVAL, "verify routed: unknown algorithm %d", algo);
  return guarded("verify routed", [&]() -> int {
    const uint32_t dw = digest_words(algo);
    std::vector<uint32_t> got(uint64_t(dw) * n);
    const unsigned dig = algo == S3H_ALGO_MD5 ? S3H_DIGESTS_MD5 : S3H_DIGESTS_SHA256;
    if (int rc = routed(dig, parts, nullptr, nullptr, lengths, n, dig == S3H_DIGESTS_SHA256 ? got.data() : nullptr,
                        dig == S3H_DIGESTS_MD5 ? got.data() : nullptr, ndevices, route, taken))
      return rc;
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; ++i) {
      mismatch[i] = std::memcmp(&got[dw * i], expected + dw * i, dw * 4) != 0;
      c += mismatch[i];
    }
    *mismatches = c;
    return S3H_OK;
  });
}

}  // extern "C"
