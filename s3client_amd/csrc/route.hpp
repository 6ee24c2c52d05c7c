// route.hpp -- size-aware routing of host-resident batches, and the multipart-ETag helper
// (host-side C-ABI entry points that need no kernel; included at the end of capi.hip).
//
// One part's SHA-256 is one sequential chain: on the GPU it runs at ~69 MB/s (the skew
// kernel's per-wave issue bound), on one EPYC core with SHA-NI at ~1.5 GB/s.
// The GPU wins only when a batch has enough parts to fill its lanes -- and the reference's
// callers are per-job batches of a few parts (lib/src/upload.cpp:89-110, 136-140), exactly the
// shape where it loses (128 x 8 MiB took 0.123 s on the GPU against 0.045 s on 16
// SHA-NI threads).  S3H_ROUTE_AUTO sends each batch where a measured model says it finishes
// first:
//   gpu_s = call_s + max(longest part / chain rate, bytes per device / feed rate)
//           feed = pinned H2D rate, or min(H2D, staging memcpy rate) for pageable parts / files
//   cpu_s = longest-first makespan of the parts on k = min(n, threads) threads
//           / (rate(k) / k),  rate(k) = min(k x one-thread rate, all-threads rate)
// Round 5 replaced a linear "threads x one-thread rate" CPU estimate with the measured
// all-threads rate: SMT siblings, memory bandwidth and the cgroup quota bend it.
// The rates are measured ONCE per process (route_model, ~0.1 s on the first AUTO call) on
// this host and device, and s3h_route_model reports them.  AUTO needs a visible GPU
// (S3H_ENODEV otherwise): it is a routing choice between two equal-result paths, never a
// fallback for a missing device.  S3H_ROUTE_GPU (the default everywhere, and the only route
// the bench metric uses) is s3h_sha256_batch_host / s3h_sha256_file_parts unchanged.

#include "../../include/md5.h"
#include "../../include/sha256.h"

namespace {

// CPU route: the lib/hash drop-in (sha256::sha256, SHA-NI when CPUID has it) on host threads,
// parts handed out longest first.  File ranges are pread in 4 MiB chunks and streamed through
// sha256_stream, the last chunk padded with the part's total length (sha256_next's contract).
int cpu_batch(const uint8_t* const* parts, int fd, const uint64_t* offsets,
              const uint64_t* lengths, uint64_t n, uint32_t* digests, unsigned threads) {
  std::vector<uint64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint64_t a, uint64_t b) { return lengths[a] > lengths[b]; });
  std::atomic<uint64_t> next{0};
  std::atomic<int> io_error{0};
  auto work = [&] {
    constexpr uint64_t kChunk = 4ull << 20;
    std::vector<uint8_t> buf(fd >= 0 ? kChunk : 0);
    for (uint64_t k; (k = next.fetch_add(1)) < n && !io_error.load();) {
      const uint64_t i = order[k];
      uint32_t* h = digests + 8 * i;
      if (fd < 0 || lengths[i] == 0) {  // (sha256_next pads only when total_length > 0)
        static const uint8_t kEmpty[1] = {0};
        sha256::sha256(lengths[i] == 0 ? kEmpty : fd < 0 ? parts[i] : buf.data(), lengths[i], h);
        continue;
      }
      sha256::init_hash(h);
      uint64_t done = 0;
      do {
        const uint64_t want = std::min(kChunk, lengths[i] - done);
        for (uint64_t got = 0; got < want;) {
          const ssize_t r = pread(fd, buf.data() + got, want - got, off_t(offsets[i] + done + got));
          if (r <= 0) {
            io_error = 1;
            return;
          }
          got += uint64_t(r);
        }
        if (done + want < lengths[i]) sha256::sha256_stream(h, buf.data(), want);
        else sha256::sha256_next(buf.data(), uint32_t(want), h, lengths[i], nullptr);
        done += want;
      } while (done < lengths[i]);
      sha256::to_little(h);
    }
  };
  const unsigned t = unsigned(std::min<uint64_t>(std::max(1u, threads), n));
  std::vector<std::thread> pool;
  for (unsigned k = 1; k < t; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  if (io_error) return fail(S3H_EINVAL, "cpu route: reading a file range failed");
  return S3H_OK;
}

struct RouteModel {
  s3h_route_model_t m{};
  int rc = S3H_OK;
  std::string err;
};

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// `threads` threads at once, each hashing its own 2 MiB buffer three times (memcpy: copying
// it into a second buffer, the staging fill): aggregate bytes per second, best of 2 rounds.
// Not 1 thread x threads: SMT siblings, memory bandwidth and the cgroup quota bend the curve.
double team_rate(unsigned threads, bool copy) {
  constexpr uint64_t kBuf = 2ull << 20;
  constexpr int kReps = 3;
  std::vector<std::vector<uint8_t>> src(threads, std::vector<uint8_t>(kBuf, 0x5a));
  std::vector<std::vector<uint8_t>> dst(copy ? threads : 0, std::vector<uint8_t>(kBuf, 0));
  double best = 1e30;
  for (int round = 0; round < 2; ++round) {
    std::atomic<unsigned> ready{0};
    std::atomic<bool> go{false};
    auto work = [&](unsigned t) {
      uint32_t h[8];
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (int r = 0; r < kReps; ++r) {
        if (copy) std::memcpy(dst[t].data(), src[t].data(), kBuf);
        else sha256::sha256(src[t].data(), kBuf, h);
      }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < threads; ++t) pool.emplace_back(work, t);
    while (ready.load() + 1 < threads) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    work(0);
    for (auto& th : pool) th.join();
    best = std::min(best, seconds_since(t0));
  }
  return double(threads) * kBuf * kReps / best;
}

// Measures the model's rates on this host and device 0 (once per process).
RouteModel measure_route_model() {
  RouteModel R;
  s3h_route_model_t& m = R.m;
  m.cpu_threads = int(host_cpus());
  {  // one host thread on the drop-in: best of 3 over 4 MiB
    std::vector<uint8_t> buf(4u << 20, 0x5a);
    uint32_t h[8];
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      sha256::sha256(buf.data(), buf.size(), h);
      best = std::min(best, seconds_since(t0));
    }
    m.cpu_bytes_per_s = double(buf.size()) / best;
  }
  m.cpu_all_bytes_per_s = team_rate(unsigned(m.cpu_threads), false);
  m.staged_bytes_per_s = team_rate(unsigned(m.cpu_threads), true);
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    R.rc = S3H_ENODEV;
    R.err = "no HIP device visible (S3H_ROUTE_AUTO chooses between the GPU and the CPU drop-in; "
            "it is not a fallback)";
    return R;
  }
  m.devices = count;
  DeviceGuard g(0);
  auto hip_fail = [&](const char* what, hipError_t e) {
    R.rc = S3H_EHIP;
    R.err = std::string("route model: ") + what + ": " + hipGetErrorString(e);
    return R;
  };
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  uint8_t *d = nullptr, *hp = nullptr;
  uint32_t* dd = nullptr;
  constexpr uint64_t kChain = 1ull << 20, kCopy = 32ull << 20;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMalloc(&d, kCopy);
  if (e == hipSuccess) e = hipMalloc(&dd, 32);
  if (e == hipSuccess) e = hipHostMalloc(&hp, kCopy, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, kCopy, s);
  if (e == hipSuccess) std::memset(hp, 0x5a, kCopy);
  float ms = 0;
  // one lone chain (the skew kernel, 1 MiB = 16K blocks, ~15 ms): chain rate
  s3h_plan_s* P = nullptr;
  const uint64_t off = 0, len = kChain;
  if (e == hipSuccess) {
    if (int rc = plan_build(0, S3H_ALGO_SHA256, &off, &len, 1, S3H_KERNEL_AUTO, &P)) {
      R.rc = rc;
      R.err = g_err;
    }
  }
  if (e == hipSuccess && P) {  // best of launches 2-3 (the first ramps the clock up)
    double best = 1e30;
    for (int r = 0; r < 3 && e == hipSuccess; ++r) {
      e = hipEventRecord(e0, s);
      if (e == hipSuccess && s3h_plan_launch(P, d, dd, s) != S3H_OK) e = hipErrorLaunchFailure;
      if (e == hipSuccess) e = hipEventRecord(e1, s);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && r > 0) best = std::min(best, double(ms) * 1e-3);
    }
    if (e == hipSuccess) m.chain_bytes_per_s = double(kChain) / best;
    if (e == hipSuccess && s3h_plan_status(P, s) != S3H_OK) e = hipErrorLaunchFailure;
  }
  // pinned host -> device copy: best of 3 over 32 MiB
  if (e == hipSuccess) {
    double best = 1e30;
    for (int r = 0; r < 4 && e == hipSuccess; ++r) {
      e = hipEventRecord(e0, s);
      if (e == hipSuccess) e = hipMemcpyAsync(d, hp, kCopy, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(e1, s);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      if (e == hipSuccess && r > 0) best = std::min(best, double(ms) * 1e-3);
    }
    if (e == hipSuccess) m.h2d_bytes_per_s = double(kCopy) / best;
  }
  if (P) s3h_plan_destroy(P);
  (void)hipHostFree(hp);
  (void)hipFree(d);
  (void)hipFree(dd);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) (void)hipStreamDestroy(s);
  if (R.rc) return R;
  if (e != hipSuccess) return hip_fail("rate probe", e);
  // fixed cost of one host-path call: a one-block part, timed on its second call (the first
  // builds the device's cached host context)
  static const uint8_t tiny[64] = {};
  const uint8_t* tp = tiny;
  const uint64_t tl = sizeof tiny;
  uint32_t th[8];
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    if (int rc = s3h_sha256_batch_host(&tp, &tl, 1, th, 1, 0)) {
      R.rc = rc;
      R.err = g_err;
      return R;
    }
    if (r > 0) best = std::min(best, seconds_since(t0));
  }
  m.call_s = best;
  return R;
}

// The measured model, kept once it measured successfully; a failed measurement (no device, a
// transient HIP error) is returned to its caller and tried again on the next call.
RouteModel route_model() {
  static std::mutex mu;
  static bool have = false;
  static RouteModel cached;
  std::lock_guard<std::mutex> lk(mu);
  if (have) return cached;
  RouteModel R = measure_route_model();
  if (R.rc == S3H_OK) {
    cached = R;
    have = true;
  }
  return R;
}

// CPU route on k threads: aggregate rate min(k x one-thread rate, all-threads rate); a model
// without the all-threads rate (recorded before round 5) scales linearly.
double cpu_rate(const s3h_route_model_t& m, double k) {
  const double lin = k * m.cpu_bytes_per_s;
  return m.cpu_all_bytes_per_s > 0 ? std::min(lin, m.cpu_all_bytes_per_s) : lin;
}

// Makespan, in bytes of one thread, of the parts hashed longest first on k threads (each takes
// the next part when it frees): exact for up to 4,096 parts, the fluid bound beyond.
double cpu_makespan_bytes(const uint64_t* lengths, uint64_t n, uint64_t k, uint64_t total,
                          uint64_t longest) {
  if (n > 4096 || k >= n) return std::max(double(total) / double(k), double(longest));
  std::vector<uint64_t> L(lengths, lengths + n);
  std::sort(L.begin(), L.end(), std::greater<uint64_t>());
  std::vector<double> load(k, 0.0);  // min-heap of thread loads
  for (uint64_t x : L) {
    std::pop_heap(load.begin(), load.end(), std::greater<double>());
    load.back() += double(x);
    std::push_heap(load.begin(), load.end(), std::greater<double>());
  }
  return *std::max_element(load.begin(), load.end());
}

// AUTO's decision for a batch (S3H_ROUTE_GPU or S3H_ROUTE_CPU) and both estimates.
int route_choose(const s3h_route_model_t& m, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, double* gpu_s, double* cpu_s) {
  uint64_t total = 0, longest = 0;
  for (uint64_t i = 0; i < n; ++i) {
    total += lengths[i];
    longest = std::max(longest, lengths[i]);
  }
  const int devs = std::max(1, int(std::min<uint64_t>(n, uint64_t(ndevices > 0 ? std::min(ndevices, m.devices) : m.devices))));
  const double feed = source == S3H_SOURCE_PINNED || !(m.staged_bytes_per_s > 0)
                          ? m.h2d_bytes_per_s : std::min(m.h2d_bytes_per_s, m.staged_bytes_per_s);
  const double g = m.call_s + std::max(double(longest) / m.chain_bytes_per_s,
                                       double(total) / devs / feed);
  const uint64_t k = std::min<uint64_t>(n, uint64_t(std::max(1, m.cpu_threads)));
  const double per_thread = cpu_rate(m, double(k)) / double(k);
  const double c = cpu_makespan_bytes(lengths, n, k, total, longest) / per_thread;
  if (gpu_s) *gpu_s = g;
  if (cpu_s) *cpu_s = c;
  return c < g ? S3H_ROUTE_CPU : S3H_ROUTE_GPU;
}

// S3H_ROUTE_SPLIT: the CPU drop-in hashes the m LONGEST parts on its threads while the GPU
// host path hashes the rest, both at once (the calling thread drives the GPU side).  A part's
// GPU chain runs ~30x slower than one SHA-NI core, so the long parts go to the CPU and the
// GPU keeps the many shorter ones it needs to fill its lanes; for C2 from pinned memory the
// GPU alone is fed at the PCIe rate and the CPU alone at its threads' rate, together faster
// than either until the GPU side reaches its chain time:
//   split_s(m) = max(gpu_s(the n - m shorter parts), cpu_s(the m longest))   m = 1 .. n-1
// with gpu_s / cpu_s the estimates above on each side's parts; among the m within 0.5 % of the
// minimum, the one with the smallest max(GPU side's bytes / feed, cpu_s).  Parts are ordered by length,
// descending (ties: lower index first); the CPU side's longest-first schedule is built
// incrementally as m grows (exact LPT; the fluid bound beyond 4,096 parts).
constexpr double kSplitTie = 0.005;  // estimates within 0.5 % of the minimum tie

struct Split {
  uint64_t m = 0;   // parts on the CPU: order[0, m) (0: no split, e.g. a single part)
  unsigned tg = 0;  // staging threads of each GPU shard (0: pinned parts, no staging)
  double s = 0, g = 0, c = 0;
};

std::vector<uint64_t> longest_first(const uint64_t* lengths, uint64_t n) {
  std::vector<uint64_t> order(n);
  uint64_t longest = 0;
  bool equal = true;
  for (uint64_t i = 0; i < n; ++i) {
    longest = std::max(longest, lengths[i]);
    equal = equal && lengths[i] == lengths[0];
  }
  constexpr int kIdxBits = 24, kLenBits = 40;
  if (!equal && n < (1ull << kIdxBits) && longest < (1ull << kLenBits)) {
    // one key per part, (complemented length, index): a plain sort of integers
    for (uint64_t i = 0; i < n; ++i) order[i] = (((1ull << kLenBits) - 1 - lengths[i]) << kIdxBits) | i;
    std::sort(order.begin(), order.end());
    for (uint64_t& x : order) x &= (1ull << kIdxBits) - 1;
    return order;
  }
  std::iota(order.begin(), order.end(), 0);
  if (!equal)
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return lengths[a] > lengths[b]; });
  return order;
}

// The best m for a given split of the host threads: pinned parts (tg = 0) leave all T threads
// to the CPU side; staged parts give tg threads to each of the GPU side's device shards, which
// feed it at min(H2D, staged rate x tg / T), and the rest to the CPU side, whose threads then
// run at the all-threads rate per thread (every CPU busy).
Split split_choose(const s3h_route_model_t& M, const uint64_t* sorted, uint64_t n, int ndevices,
                   int source, unsigned tg, std::vector<double> (&ws)[3]) {
  Split best;
  if (n < 2) return best;
  const unsigned T = unsigned(std::max(1, M.cpu_threads));
  const int dev_cap = std::max(1, ndevices > 0 ? std::min(ndevices, M.devices) : M.devices);
  const bool staged = source != S3H_SOURCE_PINNED;
  if (!staged) tg = 0;
  else if (tg == 0 || uint64_t(tg) * unsigned(dev_cap) >= T) return best;
  const unsigned tc = staged ? T - tg * unsigned(dev_cap) : T;  // CPU side's threads
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += sorted[i];
  const double feed = !staged || !(M.staged_bytes_per_s > 0)
                          ? M.h2d_bytes_per_s : std::min(M.h2d_bytes_per_s, M.staged_bytes_per_s * tg / T);
  const uint64_t kmax = std::min<uint64_t>(n, tc);
  // exact longest-first schedule up to 4,096 parts, the fluid bound beyond (as route_choose)
  const bool exact = n <= 4096;
  std::vector<double> load(exact ? kmax : 0, 0.0);  // min-heap of the CPU threads' loads (bytes)
  std::vector<double>& G = ws[0]; std::vector<double>& C = ws[1]; std::vector<double>& F = ws[2];
  for (auto& v : ws) v.resize(n);  // per m: gpu_s, cpu_s, the GPU side's feed time
  double makespan = 0, smin = 1e300;
  uint64_t cpu_bytes = 0;
  for (uint64_t m = 1; m < n; ++m) {
    const uint64_t x = sorted[m - 1];
    cpu_bytes += x;
    const uint64_t k = std::min(m, kmax);
    if (exact) {
      std::pop_heap(load.begin(), load.end(), std::greater<double>());
      load.back() += double(x);
      makespan = std::max(makespan, load.back());
      std::push_heap(load.begin(), load.end(), std::greater<double>());
    } else {
      makespan = std::max(double(cpu_bytes) / double(k), double(sorted[0]));
    }
    const double per_thread = staged ? cpu_rate(M, double(T)) / double(T) : cpu_rate(M, double(k)) / double(k);
    const double c = makespan / per_thread;
    const int devs = std::max(1, int(std::min<uint64_t>(n - m, uint64_t(dev_cap))));
    F[m] = double(total - cpu_bytes) / devs / feed;
    G[m] = M.call_s + std::max(double(sorted[m]) / M.chain_bytes_per_s, F[m]);
    C[m] = c;
    smin = std::min(smin, std::max(G[m], C[m]));
  }
  // Where the GPU side's longest chain sets its time, a range of m ties: take the one that
  // balances the GPU side's feed against the CPU side, leaving both slack.
  double key = 1e300;
  for (uint64_t m = 1; m < n; ++m) {
    if (std::max(G[m], C[m]) > smin * (1 + kSplitTie)) continue;
    const double k2 = std::max(F[m], C[m]);
    if (k2 < key) {
      key = k2;
      best = Split{m, tg, std::max(G[m], C[m]), G[m], C[m]};
    }
  }
  return best;
}

// The split plan: pinned parts need no staging threads; staged parts (pageable, file ranges)
// try tg = T/12, T/3, T/2, 2T/3, 3T/4 staging threads per GPU shard and keep the fastest
// estimate (S3H_SPLIT_STAGE_THREADS fixes tg, for measurements).
Split split_plan(const s3h_route_model_t& M, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, const std::vector<uint64_t>& order) {
  std::vector<double> ws[3];
  std::vector<uint64_t> sorted(n);  // the lengths in `order`
  for (uint64_t k = 0; k < n; ++k) sorted[k] = lengths[order[k]];
  // Many small pinned parts go through the group pipeline (capi.hip run_host_groups), which
  // packs them with the copy threads once the CPU side has taken parts out of their range:
  // plan them as staged parts.
  // So are more than kPinnedStageMin (256) ragged pinned parts (the slice pipeline stages them).
  const bool packed = source == S3H_SOURCE_PINNED && n > 64 &&
                      (sorted[0] <= kGroupMaxPart || (n > kPinnedStageMin && sorted[0] != sorted[n - 1]));
  if (packed) source = S3H_SOURCE_PAGEABLE;
  if (source == S3H_SOURCE_PINNED) return split_choose(M, sorted.data(), n, ndevices, source, 0, ws);
  const unsigned T = unsigned(std::max(1, M.cpu_threads));
  std::vector<unsigned> cand;
  if (const char* e = std::getenv("S3H_SPLIT_STAGE_THREADS")) cand.push_back(unsigned(std::max(1, std::atoi(e))));
  else
    for (unsigned num : {1u, 4u, 6u, 8u, 9u}) {  // x T / 12: T/12 ... 3T/4
      const unsigned t = std::max(1u, T * num / 12);
      if (std::find(cand.begin(), cand.end(), t) == cand.end()) cand.push_back(t);
    }
  Split best;
  for (unsigned t : cand) {
    const Split sp = split_choose(M, sorted.data(), n, ndevices, source, t, ws);
    if (sp.m && (!best.m || sp.s < best.s)) best = sp;
  }
  return best;
}

// AUTO splits only when the split is estimated at least this much faster than the better
// single route.
constexpr double kSplitGain = 0.95;

// every non-empty part in page-locked host memory (hipPointerGetAttributes): the GPU route
// DMAs them directly instead of staging
bool all_pinned_parts(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n) {
  std::vector<uint64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  return parts && all_pinned(parts, lengths, idx);
}

bool trace_route() {
  static const bool on = std::getenv("S3H_TRACE_ROUTE") != nullptr;
  return on;
}

// Opens `path` for the CPU route and checks every range lies inside it.
int open_ranges(const char* path, const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int* fd_out) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(S3H_EINVAL, "cpu route: cannot open %s", path);
  struct stat st {};
  int rc = fstat(fd, &st) == 0 ? S3H_OK : fail(S3H_EINVAL, "cpu route: cannot stat %s", path);
  for (uint64_t i = 0; rc == S3H_OK && i < n; ++i)
    if (lengths[i] > uint64_t(st.st_size) || offsets[i] > uint64_t(st.st_size) - lengths[i])
      rc = fail(S3H_EINVAL, "cpu route: part %llu ends past the end of %s", (unsigned long long)i, path);
  if (rc) close(fd);
  else *fd_out = fd;
  return rc;
}

// The split route: order[0, m) on the CPU drop-in (a thread of its own starting the CPU
// route's threads), order[m, n) on the GPU host path from this thread; digests scattered back.
int split_run(const uint8_t* const* parts, const char* path, const uint64_t* offsets,
              const uint64_t* lengths, uint64_t n, uint32_t* digests, int ndevices,
              const std::vector<uint64_t>& order, const Split& sp) {
  const uint64_t m = sp.m, ng = n - m;
  std::vector<const uint8_t*> cp(parts ? m : 0), gp(parts ? ng : 0);
  std::vector<uint64_t> co(path ? m : 0), go(path ? ng : 0), cl(m), gl(ng);
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t i = order[k];
    const bool cpu = k < m;
    const uint64_t j = cpu ? k : k - m;
    (cpu ? cl : gl)[j] = lengths[i];
    if (parts) (cpu ? cp : gp)[j] = parts[i];
    else (cpu ? co : go)[j] = offsets[i];
  }
  int fd = -1;
  if (path)
    if (int rc = open_ranges(path, co.data(), cl.data(), m, &fd)) return rc;
  std::vector<uint32_t> cd(8 * m), gd(8 * ng);
  int crc = S3H_OK;
  std::string cerr;
  int count = 1;
  (void)hipGetDeviceCount(&count);
  const unsigned T = host_cpus();
  const unsigned devs = unsigned(std::max(1, ndevices > 0 ? std::min(ndevices, count) : count));
  const unsigned tc = sp.tg && uint64_t(sp.tg) * devs < T ? T - sp.tg * devs : T;
  std::thread cpu([&] {
    try {
      crc = cpu_batch(parts ? cp.data() : nullptr, fd, co.data(), cl.data(), m, cd.data(), tc);
    } catch (const std::exception&) {  // thread or buffer allocation
      crc = fail(S3H_ENOMEM, "out of host resources");
    }
    if (crc) cerr = g_err;
  });
  g_stage_threads_cap = sp.tg;  // the GPU side's staging threads (0: uncapped)
  const int grc = path ? s3h_sha256_file_parts(path, go.data(), gl.data(), ng, gd.data(), ndevices, 0)
                       : s3h_sha256_batch_host(gp.data(), gl.data(), ng, gd.data(), ndevices, 0);
  g_stage_threads_cap = 0;
  cpu.join();
  if (fd >= 0) close(fd);
  if (grc) return grc;  // this thread's last error already names it
  if (crc) return fail(crc, "split route, cpu side: %s", cerr.c_str());
  for (uint64_t k = 0; k < n; ++k)
    std::memcpy(digests + 8 * order[k], (k < m ? cd.data() + 8 * k : gd.data() + 8 * (k - m)), 32);
  return S3H_OK;
}

// The routed entry points: parts (fd < 0) or file ranges (fd >= 0, `path` for the GPU form).
int routed(const uint8_t* const* parts, const char* path, const uint64_t* offsets,
           const uint64_t* lengths, uint64_t n, uint32_t* digests, int ndevices, int route,
           int* taken) {
  if (taken) *taken = -1;
  if (!lengths || !digests || n == 0 || (!path && !parts) || (path && !offsets))
    return fail(S3H_EINVAL, "routed batch: null argument or n == 0");
  if (route != S3H_ROUTE_GPU && route != S3H_ROUTE_CPU && route != S3H_ROUTE_AUTO && route != S3H_ROUTE_SPLIT)
    return fail(S3H_EINVAL, "routed batch: unknown route %d", route);
  if (parts && route != S3H_ROUTE_GPU)
    for (uint64_t i = 0; i < n; ++i)
      if (!parts[i] && lengths[i]) return fail(S3H_EINVAL, "cpu route: part %llu is null", (unsigned long long)i);
  int use = route;
  std::vector<uint64_t> order;
  Split sp;
  if (route == S3H_ROUTE_AUTO || route == S3H_ROUTE_SPLIT) {
    const RouteModel& R = route_model();
    if (R.rc) return fail(R.rc, "%s", R.err.c_str());
    double g = 0, c = 0;
    const int source = path ? S3H_SOURCE_FILE : all_pinned_parts(parts, lengths, n) ? S3H_SOURCE_PINNED
                                                                                : S3H_SOURCE_PAGEABLE;
    const int pick = route_choose(R.m, lengths, n, ndevices, source, &g, &c);
    // AUTO skips the plan when even a perfect split -- the GPU side fed at the H2D rate on every
    // device, the CPU side at its all-threads rate -- could not beat the better route by 5 %
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += lengths[i];
    const int dev_cap = std::max(1, ndevices > 0 ? std::min(ndevices, R.m.devices) : R.m.devices);
    const double bound = double(total) / (dev_cap * R.m.h2d_bytes_per_s + cpu_rate(R.m, R.m.cpu_threads));
    if (route == S3H_ROUTE_SPLIT || bound < kSplitGain * std::min(g, c)) {
      order = longest_first(lengths, n);
      sp = split_plan(R.m, lengths, n, ndevices, source, order);
    }
    if (route == S3H_ROUTE_SPLIT) use = sp.m ? S3H_ROUTE_SPLIT : S3H_ROUTE_GPU;  // one part: the GPU
    else use = sp.m && sp.s < kSplitGain * std::min(g, c) ? S3H_ROUTE_SPLIT : pick;
    if (trace_route())
      std::fprintf(stderr, "[s3h route] %llu parts (%s): gpu %.4f s, cpu %.4f s (%d threads), split %.4f s "
                   "(%llu longest on the cpu, %u staging threads per gpu) -> %s\n",
                   (unsigned long long)n, source == S3H_SOURCE_FILE ? "file" : source ? "pageable" : "pinned",
                   g, c, R.m.cpu_threads, sp.m ? sp.s : 0.0, (unsigned long long)sp.m, sp.tg,
                   use == S3H_ROUTE_SPLIT ? "split" : use == S3H_ROUTE_CPU ? "cpu" : "gpu");
  }
  int rc;
  if (use == S3H_ROUTE_SPLIT) {
    rc = split_run(parts, path, offsets, lengths, n, digests, ndevices, order, sp);
  } else if (use == S3H_ROUTE_GPU) {
    rc = path ? s3h_sha256_file_parts(path, offsets, lengths, n, digests, ndevices, 0)
              : s3h_sha256_batch_host(parts, lengths, n, digests, ndevices, 0);
  } else if (path) {
    int fd = -1;
    rc = open_ranges(path, offsets, lengths, n, &fd);
    if (rc == S3H_OK) {
      rc = cpu_batch(nullptr, fd, offsets, lengths, n, digests, host_cpus());
      close(fd);
    }
  } else {
    rc = cpu_batch(parts, -1, nullptr, lengths, n, digests, host_cpus());
  }
  if (rc == S3H_OK && taken) *taken = use;
  return rc;
}

}  // namespace

extern "C" {

int s3h_route_model(s3h_route_model_t* m) {
  if (!m) return fail(S3H_EINVAL, "route model: null argument");
  const RouteModel& R = route_model();
  *m = R.m;
  return R.rc ? fail(R.rc, "%s", R.err.c_str()) : S3H_OK;
}

int s3h_route_estimate(const s3h_route_model_t* m, const uint64_t* lengths, uint64_t n,
                       int ndevices, double* gpu_s, double* cpu_s) {
  if (!m || !lengths || n == 0) return fail(S3H_EINVAL, "route estimate: bad argument");
  if (!(m->cpu_bytes_per_s > 0 && m->chain_bytes_per_s > 0 && m->h2d_bytes_per_s > 0))
    return fail(S3H_EINVAL, "route estimate: the model's rates must be positive");
  return route_choose(*m, lengths, n, ndevices, S3H_SOURCE_PINNED, gpu_s, cpu_s);
}

int s3h_route_estimate_ex(const s3h_route_model_t* m, const uint64_t* lengths, uint64_t n,
                          int ndevices, int source, double* gpu_s, double* cpu_s) {
  if (source < S3H_SOURCE_PINNED || source > S3H_SOURCE_FILE)
    return fail(S3H_EINVAL, "route estimate: unknown source %d", source);
  if (!m || !lengths || n == 0) return fail(S3H_EINVAL, "route estimate: bad argument");
  if (!(m->cpu_bytes_per_s > 0 && m->chain_bytes_per_s > 0 && m->h2d_bytes_per_s > 0))
    return fail(S3H_EINVAL, "route estimate: the model's rates must be positive");
  return route_choose(*m, lengths, n, ndevices, source, gpu_s, cpu_s);
}

int s3h_route_split_estimate(const s3h_route_model_t* m, const uint64_t* lengths, uint64_t n,
                             int ndevices, int source, uint64_t* cpu_parts, int* stage_threads,
                             double* split_s) {
  if (cpu_parts) *cpu_parts = 0;
  if (stage_threads) *stage_threads = 0;
  if (split_s) *split_s = 0;
  if (source < S3H_SOURCE_PINNED || source > S3H_SOURCE_FILE)
    return fail(S3H_EINVAL, "route split estimate: unknown source %d", source);
  if (!m || !lengths || n == 0) return fail(S3H_EINVAL, "route split estimate: bad argument");
  if (!(m->cpu_bytes_per_s > 0 && m->chain_bytes_per_s > 0 && m->h2d_bytes_per_s > 0))
    return fail(S3H_EINVAL, "route split estimate: the model's rates must be positive");
  Split sp;
  try {
    sp = split_plan(*m, lengths, n, ndevices, source, longest_first(lengths, n));
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "route split estimate: out of host memory");
  }
  if (cpu_parts) *cpu_parts = sp.m;
  if (stage_threads) *stage_threads = int(sp.tg);
  if (split_s) *split_s = sp.s;
  return S3H_OK;
}

int s3h_sha256_batch_routed(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                            uint32_t* digests, int ndevices, int route, int* taken) {
  try {
    return routed(parts, nullptr, nullptr, lengths, n, digests, ndevices, route, taken);
  } catch (const std::exception&) {  // nothing escapes the C-ABI
    return fail(S3H_ENOMEM, "routed batch: out of host resources");
  }
}

// S3 multipart ETag (what CompleteMultipartUpload returns, multipart_upload.cpp:162-183):
// hex(MD5(binary part MD5s concatenated in part order)) + "-" + part count.  The outer MD5
// covers 16 B per part, so it runs on the lib/hash MD5 drop-in.
int s3h_multipart_etag(const uint32_t* md5_digests, uint64_t n, char* out, uint64_t out_len) {
  if (out && out_len) out[0] = '\0';
  if (!out || out_len < S3H_ETAG_MAX) return fail(S3H_EINVAL, "multipart etag: need %d output bytes", S3H_ETAG_MAX);
  if (n == 0 || !md5_digests) return fail(S3H_EINVAL, "multipart etag: no part digests");
  uint32_t h[4];
  md5::md5(reinterpret_cast<const uint8_t*>(md5_digests), size_t(16 * n), h);
  md5::hash_to_text(h, out);
  std::snprintf(out + 32, size_t(out_len - 32), "-%llu", static_cast<unsigned long long>(n));
  return S3H_OK;
}

int s3h_verify_batch_routed(int algo, const uint8_t* const* parts, const uint64_t* lengths,
                            uint64_t n, const uint32_t* expected, uint8_t* mismatch,
                            uint64_t* mismatches, int ndevices, int route, int* taken) {
  if (taken) *taken = -1;
  if (!expected || !mismatch || !mismatches) return fail(S3H_EINVAL, "verify routed: null argument");
  if (algo != S3H_ALGO_SHA256 && algo != S3H_ALGO_MD5)
    return fail(S3H_EINVAL, "verify routed: unknown algorithm %d", algo);
  if (route == S3H_ROUTE_GPU) {
    const int rc = s3h_verify_batch_host(algo, parts, lengths, n, expected, mismatch, mismatches, ndevices);
    if (rc == S3H_OK && taken) *taken = S3H_ROUTE_GPU;
    return rc;
  }
  if (algo != S3H_ALGO_SHA256)
    return fail(S3H_EINVAL, "verify routed: route %d is SHA-256 only (MD5 verifies on the GPU route)", route);
  try {
    std::vector<uint32_t> got(8 * n);
    if (int rc = routed(parts, nullptr, nullptr, lengths, n, got.data(), ndevices, route, taken)) return rc;
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; ++i) {
      mismatch[i] = std::memcmp(&got[8 * i], expected + 8 * i, 32) != 0;
      c += mismatch[i];
    }
    *mismatches = c;
    return S3H_OK;
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "verify routed: out of host resources");
  }
}

int s3h_sha256_file_parts_routed(const char* path, const uint64_t* offsets,
                                 const uint64_t* lengths, uint64_t n, uint32_t* digests,
                                 int ndevices, int route, int* taken) {
  if (!path) return fail(S3H_EINVAL, "routed file parts: null path");
  try {
    return routed(nullptr, path, offsets, lengths, n, digests, ndevices, route, taken);
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "routed file parts: out of host resources");
  }
}

}  // extern "C"
