// route_plan.cpp -- routing arithmetic, the CPU route and the split route's driver
// (route_plan.hpp), plus the pure C-ABI estimates (s3h_route_estimate*, s3h_route_choose).
// HIP-free: the host-concurrency sanitizer build runs the CPU and split routes from here.
#include "route_plan.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <numeric>

#include "../../include/md5.h"
#include "../../include/sha256.h"
#include "cpu/cpu_hash.hpp"
#include "host_limits.hpp"
#include "host_queue.hpp"

namespace s3h::host {

Rates rates_from_model(const s3h_route_model_t& m) {
  Rates R;
  R.cpu_threads = std::max(1, m.cpu_threads);
  R.devices = std::max(1, m.devices);
  R.cpu1[0] = m.cpu_bytes_per_s;
  R.cpu_all[0] = m.cpu_all_bytes_per_s;
  R.chain[0] = m.chain_bytes_per_s;
  R.h2d = m.h2d_bytes_per_s;
  R.staged = m.staged_bytes_per_s;
  R.call_s = m.call_s;
  return R;
}

std::string rates_check(const Rates& R, unsigned dig) {
  const int a = dig_index(dig);
  if (a < 0 || a > 2) return "unknown digest set";
  if (!(R.cpu1[a] > 0 && R.chain[a] > 0 && R.h2d > 0)) return "the model's rates must be positive";
  if (!(R.f_gpu > 0 && R.f_cpu > 0)) return "the model's observed factors must be positive";
  return std::string();
}

// CPU route on k threads: aggregate rate min(k x one-thread rate, all-threads rate); a model
// without the all-threads rate (recorded before round 5) scales linearly.
double cpu_rate(const Rates& R, unsigned dig, double k) {
  const int a = dig_index(dig);
  const double lin = k * R.cpu1[a];
  return R.cpu_all[a] > 0 ? std::min(lin, R.cpu_all[a]) : lin;
}

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

namespace {

int dev_cap(const Rates& R, int ndevices) {
  return std::max(1, ndevices > 0 ? std::min(ndevices, R.devices) : R.devices);
}

double feed_rate(const Rates& R, bool staged) {
  return !staged || !(R.staged > 0) ? R.h2d : std::min(R.h2d, R.staged);
}

// The best m for a given split of the host threads: pinned parts (tg = 0) leave all T threads
// to the CPU side; staged parts give tg threads to each of the GPU side's device shards, which
// feed it at min(H2D, staged rate x tg / T), and the rest to the CPU side, whose threads then
// run at the all-threads rate per thread (every CPU busy).  Parts are ordered by length,
// descending (ties: lower index first); the CPU side's longest-first schedule is built
// incrementally as m grows (exact LPT; the fluid bound beyond 4,096 parts).
Split split_choose(const Rates& R, unsigned dig, const uint64_t* sorted, uint64_t n, int ndevices,
                   bool staged, unsigned tg, std::vector<double> (&ws)[4]) {
  Split best;
  if (n < 2) return best;
  const int a = dig_index(dig);
  const unsigned T = unsigned(std::max(1, R.cpu_threads));
  const int devs_cap = dev_cap(R, ndevices);
  if (!staged) tg = 0;
  else if (tg == 0 || uint64_t(tg) * unsigned(devs_cap) >= T) return best;
  const unsigned tc = staged ? T - tg * unsigned(devs_cap) : T;  // CPU side's threads
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += sorted[i];
  const double feed = !staged || !(R.staged > 0) ? R.h2d : std::min(R.h2d, R.staged * tg / T);
  const uint64_t kmax = std::min<uint64_t>(n, tc);
  const bool exact = n <= 4096;
  std::vector<double> load(exact ? kmax : 0, 0.0);  // min-heap of the CPU threads' loads (bytes)
  std::vector<double>& G = ws[0];
  std::vector<double>& C = ws[1];
  std::vector<double>& F = ws[2];
  std::vector<double>& S = ws[3];
  for (auto& v : ws) v.assign(n, 0.0);  // per m: raw gpu_s, raw cpu_s, feed time, split_s
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
    const double per_thread = staged ? cpu_rate(R, dig, double(T)) / double(T)
                                     : cpu_rate(R, dig, double(k)) / double(k);
    const int devs = std::max(1, int(std::min<uint64_t>(n - m, uint64_t(devs_cap))));
    F[m] = double(total - cpu_bytes) / devs / feed;
    G[m] = R.call_s + std::max(double(sorted[m]) / R.chain[a], F[m]);
    C[m] = makespan / per_thread;
    S[m] = std::max(G[m] * R.f_gpu, C[m] * R.f_cpu);
    smin = std::min(smin, S[m]);
  }
  // Where the GPU side's longest chain sets its time, a range of m ties: take the one that
  // balances the GPU side's feed against the CPU side, leaving both slack.
  double key = 1e300;
  for (uint64_t m = 1; m < n; ++m) {
    if (S[m] > smin * (1 + kSplitTie)) continue;
    const double k2 = std::max(F[m] * R.f_gpu, C[m] * R.f_cpu);
    if (k2 < key) {
      key = k2;
      best = Split{m, tg, S[m], G[m], C[m]};
    }
  }
  return best;
}

}  // namespace

void route_times(const Rates& R0, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, double* gpu_s, double* cpu_s) {
  const Rates R = for_source(R0, source);
  const int a = dig_index(dig);
  uint64_t total = 0, longest = 0;
  for (uint64_t i = 0; i < n; ++i) {
    total += lengths[i];
    longest = std::max(longest, lengths[i]);
  }
  const int devs = std::max(1, int(std::min<uint64_t>(n, uint64_t(dev_cap(R, ndevices)))));
  const double feed = feed_rate(R, source != S3H_SOURCE_PINNED);
  *gpu_s = R.call_s + std::max(double(longest) / R.chain[a], double(total) / devs / feed);
  const uint64_t k = std::min<uint64_t>(n, uint64_t(std::max(1, R.cpu_threads)));
  const double per_thread = cpu_rate(R, dig, double(k)) / double(k);
  *cpu_s = cpu_makespan_bytes(lengths, n, k, total, longest) / per_thread;
}

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
    std::stable_sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return lengths[x] > lengths[y]; });
  return order;
}

// The split plan: pinned parts need no staging threads; staged parts (pageable, file ranges)
// try each device's share of the host threads times 1, 4, 6, 8, 9 twelfths as staging threads
// per GPU shard (topology.cpp split_stage_candidates; S3H_SPLIT_STAGE_THREADS fixes it, for
// measurements) and keep the fastest estimate.
Split split_plan(const Rates& R0, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, const std::vector<uint64_t>& order) {
  const Rates R = for_source(R0, source);
  std::vector<double> ws[4];
  std::vector<uint64_t> sorted(n);  // the lengths in `order`
  for (uint64_t k = 0; k < n; ++k) sorted[k] = lengths[order[k]];
  // Many small pinned parts go through the group pipeline (host_path.cpp run_host_groups),
  // which packs them with the copy threads once the CPU side has taken parts out of their
  // range, and so are more than kPinnedStageMin ragged pinned parts (the slice pipeline stages
  // them): plan them as staged parts.
  const bool packed = source == S3H_SOURCE_PINNED && n > 64 &&
                      (sorted[0] <= kGroupMaxPart || (n > kPinnedStageMin && sorted[0] != sorted[n - 1]));
  const bool staged = source != S3H_SOURCE_PINNED || packed;
  if (!staged) return split_choose(R, dig, sorted.data(), n, ndevices, false, 0, ws);
  std::vector<unsigned> cand;
  if (const char* e = std::getenv("S3H_SPLIT_STAGE_THREADS")) cand.push_back(unsigned(std::max(1, std::atoi(e))));
  else cand = split_stage_candidates(unsigned(std::max(1, R.cpu_threads)), dev_cap(R, ndevices));
  Split best;
  for (unsigned t : cand) {
    const Split sp = split_choose(R, dig, sorted.data(), n, ndevices, true, t, ws);
    if (sp.m && (!best.m || sp.s < best.s)) best = sp;
  }
  return best;
}

Decision decide(const Rates& R, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                int source, int route) {
  Decision D;
  route_times(R, dig, lengths, n, ndevices, source, &D.g, &D.c);
  const double g = D.g * R.f_gpu, c = D.c * R.f_cpu;
  const int pick = c < g ? S3H_ROUTE_CPU : S3H_ROUTE_GPU;
  // AUTO skips the split plan when even a perfect split -- the GPU side fed at the H2D rate on
  // every device, the CPU side at its all-threads rate -- could not beat the better route by 5 %
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += lengths[i];
  const double bound = double(total) / (dev_cap(R, ndevices) * R.h2d / R.f_gpu +
                                        cpu_rate(R, dig, R.cpu_threads) / R.f_cpu);
  if (route == S3H_ROUTE_SPLIT || bound < kSplitGain * std::min(g, c)) {
    D.order = longest_first(lengths, n);
    D.sp = split_plan(R, dig, lengths, n, ndevices, source, D.order);
  }
  if (route == S3H_ROUTE_SPLIT) D.route = D.sp.m ? S3H_ROUTE_SPLIT : S3H_ROUTE_GPU;  // one part: the GPU
  else D.route = D.sp.m && D.sp.s < kSplitGain * std::min(g, c) ? S3H_ROUTE_SPLIT : pick;
  return D;
}

// ------------------------------------------------------------------ the CPU route
namespace {

constexpr uint64_t kFileChunk = 4ull << 20;
constexpr uint64_t kCacheChunk = 64ull << 10;

// Digests of one file range [off, off + len) read in 4 MiB chunks (false: a read failed).
bool file_digests(unsigned dig, int fd, uint64_t off, uint64_t len, uint8_t* buf, uint32_t* sha,
                  uint32_t* md5v) {
  if (dig & S3H_DIGESTS_SHA256) sha256::init_hash(sha);
  if (dig & S3H_DIGESTS_MD5) md5::init_hash(md5v);
  uint64_t done = 0;
  do {
    const uint64_t want = std::min(kFileChunk, len - done);
    for (uint64_t got = 0; got < want;) {
      const ssize_t r = pread(fd, buf + got, want - got, off_t(off + done + got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return false;
      got += uint64_t(r);
    }
    const bool last = done + want == len;
    const uint64_t whole = last ? want / 64 * 64 : want;  // chunks are 64-B multiples
    for (uint64_t at = 0; at < whole; at += kCacheChunk) {
      const uint64_t nb = std::min(kCacheChunk, whole - at) / 64;
      if (dig & S3H_DIGESTS_SHA256) s3h::cpu::sha256_blocks(sha, buf + at, nb);
      if (dig & S3H_DIGESTS_MD5) s3h::cpu::md5_blocks(md5v, buf + at, nb);
    }
    if (last) {
      if (dig & S3H_DIGESTS_SHA256) s3h::cpu::sha256_final(sha, buf + whole, want - whole, len);
      if (dig & S3H_DIGESTS_MD5) s3h::cpu::md5_final(md5v, buf + whole, want - whole, len);
    }
    done += want;
  } while (done < len);
  if (dig & S3H_DIGESTS_SHA256) sha256::to_little(sha);
  return true;
}

void mem_digests(unsigned dig, const uint8_t* p, uint64_t len, uint32_t* sha, uint32_t* md5v) {
  static const uint8_t kEmpty[1] = {0};
  if (len == 0) p = kEmpty;
  if (dig == S3H_DIGESTS_BOTH) s3h::cpu::sha256_md5(p, len, sha, md5v);
  else if (dig == S3H_DIGESTS_SHA256) sha256::sha256(p, len, sha);
  else md5::md5(p, len, md5v);
}

}  // namespace

int cpu_batch(unsigned dig, const uint8_t* const* parts, int fd, const uint64_t* offsets,
              const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5v, unsigned threads) {
  std::vector<uint64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint64_t a, uint64_t b) { return lengths[a] > lengths[b]; });
  std::atomic<uint64_t> next{0};
  std::atomic<int> io_error{0};
  auto work = [&] {
    std::vector<uint8_t> buf(fd >= 0 ? kFileChunk : 0);
    for (uint64_t k; (k = next.fetch_add(1)) < n && !io_error.load();) {
      const uint64_t i = order[k];
      uint32_t* hs = sha ? sha + 8 * i : nullptr;
      uint32_t* hm = md5v ? md5v + 4 * i : nullptr;
      if (fd < 0 || lengths[i] == 0) {
        mem_digests(dig, fd < 0 ? parts[i] : nullptr, lengths[i], hs, hm);
      } else if (!file_digests(dig, fd, offsets[i], lengths[i], buf.data(), hs, hm)) {
        io_error = 1;
        return;
      }
    }
  };
  const unsigned t = unsigned(std::min<uint64_t>(std::max(1u, threads), n));
  std::vector<std::thread> pool;
  try {
    for (unsigned k = 1; k < t; ++k) pool.emplace_back(work);
  } catch (const std::exception&) {  // fewer threads: the ones started and this one finish
  }
  work();
  for (auto& th : pool) th.join();
  if (io_error) return fail(S3H_EINVAL, "cpu route: reading a file range failed");
  return S3H_OK;
}

double one_thread_rate(unsigned dig) {
  std::vector<uint8_t> buf(4u << 20, 0x5a);
  uint32_t h[8], m[4];
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    mem_digests(dig, buf.data(), buf.size(), h, m);
    best = std::min(best, seconds_since(t0));
  }
  return double(buf.size()) / best;
}

double team_rate(unsigned threads, unsigned dig) {
  constexpr uint64_t kBuf = 2ull << 20;
  constexpr int kReps = 3;
  threads = std::max(1u, threads);
  std::vector<std::vector<uint8_t>> src(threads, std::vector<uint8_t>(kBuf, 0x5a));
  std::vector<std::vector<uint8_t>> dst(dig == 0 ? threads : 0, std::vector<uint8_t>(kBuf, 0));
  double best = 1e30;
  for (int round = 0; round < 2; ++round) {
    std::atomic<unsigned> ready{0};
    std::atomic<bool> go{false};
    auto work = [&](unsigned t) {
      uint32_t h[8], m[4];
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (int r = 0; r < kReps; ++r) {
        if (dig == 0) std::memcpy(dst[t].data(), src[t].data(), kBuf);
        else mem_digests(dig, src[t].data(), kBuf, h, m);
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

double pread_team_rate(unsigned threads) {
  constexpr uint64_t kBuf = 2ull << 20;
  constexpr int kReps = 3;
  threads = std::max(1u, threads);
  FdGuard fd{int(syscall(SYS_memfd_create, "s3h_pread_probe", 0u))};
  if (fd.fd < 0) return 0;
  std::vector<uint8_t> fill(kBuf, 0x5a);
  for (unsigned t = 0; t < threads; ++t)
    if (pwrite(fd.fd, fill.data(), kBuf, off_t(uint64_t(t) * kBuf)) != ssize_t(kBuf)) return 0;
  std::vector<std::vector<uint8_t>> dst(threads, std::vector<uint8_t>(kBuf, 0));
  std::atomic<bool> bad{false};
  double best = 1e30;
  for (int round = 0; round < 2; ++round) {
    std::atomic<unsigned> ready{0};
    std::atomic<bool> go{false};
    auto work = [&](unsigned t) {
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (int r = 0; r < kReps; ++r)
        if (pread(fd.fd, dst[t].data(), kBuf, off_t(uint64_t(t) * kBuf)) != ssize_t(kBuf)) bad = true;
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
  return bad ? 0.0 : double(threads) * kBuf * kReps / best;
}

Rates for_source(const Rates& R, int source) {
  Rates r = R;
  if (source == S3H_SOURCE_FILE && R.staged_file > 0) r.staged = R.staged_file;
  return r;
}

void FdGuard::close_now() {
  if (fd >= 0) ::close(fd);
  fd = -1;
}

int open_ranges(const char* path, const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int* fd_out) {
  FdGuard g{open(path, O_RDONLY | O_CLOEXEC)};
  if (g.fd < 0) return fail(S3H_EINVAL, "cpu route: cannot open %s", path);
  struct stat st {};
  if (fstat(g.fd, &st) != 0) return fail(S3H_EINVAL, "cpu route: cannot stat %s", path);
  for (uint64_t i = 0; i < n; ++i)
    if (lengths[i] > uint64_t(st.st_size) || offsets[i] > uint64_t(st.st_size) - lengths[i])
      return fail(S3H_EINVAL, "cpu route: part %llu ends past the end of %s", (unsigned long long)i, path);
  *fd_out = g.fd;
  g.fd = -1;
  return S3H_OK;
}

int split_run_impl(unsigned dig, const uint8_t* const* parts, const char* path,
                   const uint64_t* offsets, const uint64_t* lengths, uint64_t n, uint32_t* sha,
                   uint32_t* md5v, int ndevices, int devices_visible, const std::vector<uint64_t>& order,
                   const Split& sp,
                   int (*gpu_side)(void*, const uint8_t* const*, const uint64_t*, const uint64_t*,
                                   uint64_t, uint32_t*, uint32_t*),
                   void* ctx, double* t_gpu, double* t_cpu) {
  const uint64_t m = sp.m, ng = n - m;
  const bool want_sha = dig & S3H_DIGESTS_SHA256, want_md5 = dig & S3H_DIGESTS_MD5;
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
  FdGuard fd;  // closed on every return (advisor r5: an exception could leak it)
  if (path)
    if (int rc = open_ranges(path, co.data(), cl.data(), m, &fd.fd)) return rc;
  std::vector<uint32_t> cs(want_sha ? 8 * m : 0), cm(want_md5 ? 4 * m : 0);
  std::vector<uint32_t> gs(want_sha ? 8 * ng : 0), gm(want_md5 ? 4 * ng : 0);
  const unsigned T = host_cpus();
  const unsigned devs = unsigned(std::max(1, ndevices > 0 ? std::min(ndevices, devices_visible) : devices_visible));
  const unsigned tc = sp.tg && uint64_t(sp.tg) * devs < T ? T - sp.tg * devs : T;
  int crc = S3H_OK;
  std::string cerr;
  double tc_s = 0;
  auto cpu_side = [&] {
    const auto t0 = std::chrono::steady_clock::now();
    try {
      crc = cpu_batch(dig, parts ? cp.data() : nullptr, fd.fd, co.data(), cl.data(), m,
                      want_sha ? cs.data() : nullptr, want_md5 ? cm.data() : nullptr, tc);
    } catch (const std::exception&) {  // buffer allocation
      crc = fail(S3H_ENOMEM, "out of host resources");
    }
    if (crc) cerr = g_err;
    tc_s = seconds_since(t0);
  };
  std::thread cpu;
  try {
    cpu = std::thread(cpu_side);
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "split route: cannot start the cpu side's thread");
  }
  const auto t0 = std::chrono::steady_clock::now();
  g_stage_threads_cap = sp.tg;  // the GPU side's staging threads (0: uncapped)
  const int grc = gpu_side(ctx, parts ? gp.data() : nullptr, path ? go.data() : nullptr, gl.data(), ng,
                           want_sha ? gs.data() : nullptr, want_md5 ? gm.data() : nullptr);
  g_stage_threads_cap = 0;
  const double tg_s = seconds_since(t0);
  cpu.join();
  if (t_gpu) *t_gpu = tg_s;
  if (t_cpu) *t_cpu = tc_s;
  if (grc) return grc;  // this thread's last error already names it
  if (crc) return fail(crc, "split route, cpu side: %s", cerr.c_str());
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t i = order[k];
    if (want_sha) std::memcpy(sha + 8 * i, k < m ? &cs[8 * k] : &gs[8 * (k - m)], 32);
    if (want_md5) std::memcpy(md5v + 4 * i, k < m ? &cm[4 * k] : &gm[4 * (k - m)], 16);
  }
  return S3H_OK;
}

}  // namespace s3h::host

using namespace s3h::host;

extern "C" {

int s3h_route_estimate_ex(const s3h_route_model_t* m, const uint64_t* lengths, uint64_t n,
                          int ndevices, int source, double* gpu_s, double* cpu_s) {
  if (source < S3H_SOURCE_PINNED || source > S3H_SOURCE_FILE)
    return fail(S3H_EINVAL, "route estimate: unknown source %d", source);
  if (!m || !lengths || n == 0) return fail(S3H_EINVAL, "route estimate: bad argument");
  const Rates R = rates_from_model(*m);
  const std::string bad = rates_check(R, S3H_DIGESTS_SHA256);
  if (!bad.empty()) return fail(S3H_EINVAL, "route estimate: %s", bad.c_str());
  double g = 0, c = 0;
  route_times(R, S3H_DIGESTS_SHA256, lengths, n, ndevices, source, &g, &c);
  if (gpu_s) *gpu_s = g;
  if (cpu_s) *cpu_s = c;
  return c < g ? S3H_ROUTE_CPU : S3H_ROUTE_GPU;
}

int s3h_route_estimate(const s3h_route_model_t* m, const uint64_t* lengths, uint64_t n,
                       int ndevices, double* gpu_s, double* cpu_s) {
  return s3h_route_estimate_ex(m, lengths, n, ndevices, S3H_SOURCE_PINNED, gpu_s, cpu_s);
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
  const Rates R = rates_from_model(*m);
  const std::string bad = rates_check(R, S3H_DIGESTS_SHA256);
  if (!bad.empty()) return fail(S3H_EINVAL, "route split estimate: %s", bad.c_str());
  Split sp;
  try {
    sp = split_plan(R, S3H_DIGESTS_SHA256, lengths, n, ndevices, source, longest_first(lengths, n));
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "route split estimate: out of host memory");
  }
  if (cpu_parts) *cpu_parts = sp.m;
  if (stage_threads) *stage_threads = int(sp.tg);
  if (split_s) *split_s = sp.s;
  return S3H_OK;
}

int s3h_route_choose(const s3h_route_rates_t* rates, int digests, const uint64_t* lengths,
                     uint64_t n, int ndevices, int source, s3h_route_choice_t* out) {
  if (!out) return fail(S3H_EINVAL, "route choose: null output");
  *out = s3h_route_choice_t{};
  out->route = -1;
  if (!rates || !lengths || n == 0) return fail(S3H_EINVAL, "route choose: bad argument");
  if (!valid_digests(digests)) return fail(S3H_EINVAL, "route choose: unknown digest set %d", digests);
  if (source < S3H_SOURCE_PINNED || source > S3H_SOURCE_FILE)
    return fail(S3H_EINVAL, "route choose: unknown source %d", source);
  // size-aware read: a caller compiled against an older (shorter) struct leaves the rest zero
  s3h_route_rates_t r{};
  const size_t have = std::min<size_t>(rates->size, sizeof r);
  if (have < offsetof(s3h_route_rates_t, staged_bytes_per_s))
    return fail(S3H_EINVAL, "route choose: rates struct of %u bytes is too small", rates->size);
  std::memcpy(&r, rates, have);
  Rates R;
  R.cpu_threads = std::max(1, r.cpu_threads);
  R.devices = std::max(1, r.devices);
  for (int a = 0; a < 3; ++a) {
    R.cpu1[a] = r.cpu_bytes_per_s[a];
    R.cpu_all[a] = r.cpu_all_bytes_per_s[a];
    R.chain[a] = r.chain_bytes_per_s[a];
  }
  R.h2d = r.h2d_bytes_per_s;
  R.staged = r.staged_bytes_per_s;
  R.staged_file = r.staged_file_bytes_per_s;  // 0 when the caller's struct predates it
  R.call_s = r.call_s;
  const int a = dig_index(unsigned(digests));
  R.f_gpu = r.gpu_factor[a] > 0 ? r.gpu_factor[a] : 1;
  R.f_cpu = r.cpu_factor[a] > 0 ? r.cpu_factor[a] : 1;
  const std::string bad = rates_check(R, unsigned(digests));
  if (!bad.empty()) return fail(S3H_EINVAL, "route choose: %s", bad.c_str());
  try {
    const Decision D = decide(R, unsigned(digests), lengths, n, ndevices, source, S3H_ROUTE_AUTO);
    out->route = D.route;
    out->gpu_s = D.g * R.f_gpu;
    out->cpu_s = D.c * R.f_cpu;
    out->split_s = D.sp.m ? D.sp.s : 0;
    out->cpu_parts = D.sp.m;
    out->stage_threads = int(D.sp.tg);
  } catch (const std::exception&) {
    return fail(S3H_ENOMEM, "route choose: out of host memory");
  }
  return S3H_OK;
}

}  // extern "C"
