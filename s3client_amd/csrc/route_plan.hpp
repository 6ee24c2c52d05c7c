// route_plan.hpp -- size-aware routing arithmetic and the CPU route (HIP-free).
//
// One part's SHA-256 is one sequential chain: on the GPU it runs at ~69 MB/s (the skew
// kernel's per-wave issue bound), on one EPYC core with SHA-NI at ~2.5 GB/s.  The
// GPU wins only when a batch has enough parts to fill its lanes -- and the reference's callers
// are per-job batches of a few parts (lib/src/upload.cpp:89-110, 136-140), exactly the shape
// where it loses.  A routed call (route.cpp) prices each route from measured rates:
//   gpu_s = call_s + max(longest part / chain rate, bytes per device / feed rate)
//           feed = pinned H2D rate, or min(H2D, staging rate) for pageable parts (the threads'
//           memcpy) and file ranges (their pread from the page cache)
//   cpu_s = longest-first makespan of the parts on k = min(n, threads) threads
//           / (rate(k) / k),  rate(k) = min(k x one-thread rate, all-threads rate)
//   split_s(m) = max(gpu_s(the n - m shorter parts), cpu_s(the m longest))
// for the digest set the call asks for -- SHA-256, MD5, or both from one pass (Content-MD5 +
// x-amz-content-sha256) -- each with its own CPU and GPU-chain rates, and scales gpu_s / cpu_s
// by the observed / predicted ratio of earlier routed calls (route.cpp).  The CPU route is the
// product's own lib/hash drop-in (sha256::sha256, md5::md5; SHA-NI when CPUID has it).
#pragma once
#include <sys/types.h>

#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "../../include/s3hash.h"
#include "status.hpp"
#include "topology.hpp"

namespace s3h::host {

// Digest sets of a routed call (S3H_DIGESTS_*): bit 0 SHA-256, bit 1 MD5; rate arrays are
// indexed by dig_index.
inline int dig_index(unsigned dig) { return int(dig) - 1; }
inline bool valid_digests(int d) { return d >= S3H_DIGESTS_SHA256 && d <= S3H_DIGESTS_BOTH; }

// Everything one routing decision reads.
struct Rates {
  int cpu_threads = 1, devices = 1;
  double cpu1[3] = {0, 0, 0};     // one host thread, per digest set (bytes/s)
  double cpu_all[3] = {0, 0, 0};  // all cpu_threads at once, aggregate (0: linear in threads)
  double chain[3] = {0, 0, 0};    // one GPU chain (the slowest device in use)
  double h2d = 0;                 // pinned host -> device, the slowest device in use
  double staged = 0;              // pageable sources: the threads' memcpy into pinned staging
  double staged_file = 0;         // file ranges: the threads' pread from the page cache (0: staged)
  double call_s = 0;              // fixed cost of one host-path GPU call
  double f_gpu = 1, f_cpu = 1;    // observed / predicted wall time of earlier routed calls
};
// The frozen round-5 struct (SHA-256 rates only).
Rates rates_from_model(const s3h_route_model_t& m);
// Missing / zero rates of digest set `dig`: an error message, or "" when usable.
std::string rates_check(const Rates& R, unsigned dig);

double cpu_rate(const Rates& R, unsigned dig, double k);
// Makespan, in bytes of one thread, of the parts hashed longest first on k threads: exact for
// up to 4,096 parts, the fluid bound beyond.
double cpu_makespan_bytes(const uint64_t* lengths, uint64_t n, uint64_t k, uint64_t total, uint64_t longest);
// Raw estimates (no observed factors) of the GPU and the CPU route.
void route_times(const Rates& R, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, double* gpu_s, double* cpu_s);

// The split route's plan: order[0, m) (longest first) on the CPU, the rest on the GPU; tg
// staging threads per GPU shard for staged sources (0: pinned).  g / c: that split's raw side
// estimates, s = max(g x f_gpu, c x f_cpu).
struct Split {
  uint64_t m = 0;
  unsigned tg = 0;
  double s = 0, g = 0, c = 0;
};
constexpr double kSplitTie = 0.005;  // split estimates within 0.5 % of the minimum tie
constexpr double kSplitGain = 0.95;  // AUTO splits only when >= 5 % faster than the better route
std::vector<uint64_t> longest_first(const uint64_t* lengths, uint64_t n);
Split split_plan(const Rates& R, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                 int source, const std::vector<uint64_t>& order);

// AUTO's (or SPLIT's) whole decision for a batch.
struct Decision {
  int route = S3H_ROUTE_GPU;  // what runs: GPU, CPU or SPLIT
  double g = 0, c = 0;        // raw estimates of the GPU and the CPU route
  Split sp;                   // the split plan, if one was made (sp.m > 0)
  std::vector<uint64_t> order;
};
Decision decide(const Rates& R, unsigned dig, const uint64_t* lengths, uint64_t n, int ndevices,
                int source, int route);

// ------------------------------------------------------------------ the CPU route
// The drop-in on `threads` host threads, parts handed out longest first: memory parts
// (fd < 0) or file ranges (pread in 4 MiB chunks).  sha (n x 8) / md5 (n x 4) as `dig` asks.
int cpu_batch(unsigned dig, const uint8_t* const* parts, int fd, const uint64_t* offsets,
              const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5, unsigned threads);
// One thread's rate (best of 3 over 4 MiB) and `threads` threads' aggregate rate (each its own
// 2 MiB buffer, 3 passes, best of 2) of digest set `dig`; dig == 0: memcpy (staging fill).
double one_thread_rate(unsigned dig);
double team_rate(unsigned threads, unsigned dig);
// `threads` threads' aggregate pread rate from the page cache (each its own 2 MiB of a memfd,
// read in 2 MiB calls, 3 passes, best of 2): how fast the host path stages file ranges, ~0.6x
// the memcpy rate on the GPU box (profiles/r06_route_gpu_side_probe.json).  0 if unavailable.
double pread_team_rate(unsigned threads);
// The rates a decision over `source` uses: file ranges stage at the pread rate.
Rates for_source(const Rates& R, int source);
// Opens `path` and checks that every range lies inside it (CPU route); the descriptor in *fd.
int open_ranges(const char* path, const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int* fd);

// Closes a descriptor on every path out of a scope.
struct FdGuard {
  int fd = -1;
  ~FdGuard() { close_now(); }
  void close_now();
};

// The split route: order[0, sp.m) on the CPU drop-in (a thread of its own starting the CPU
// route's threads), order[m, n) through `gpu_side` from this thread, digests scattered back.
//   gpu_side(parts | nullptr, offsets | nullptr, lengths, n, sha | nullptr, md5 | nullptr) -> rc
// runs with g_stage_threads_cap = sp.tg.  *t_gpu / *t_cpu receive each side's wall time.
int split_run_impl(unsigned dig, const uint8_t* const* parts, const char* path,
                   const uint64_t* offsets, const uint64_t* lengths, uint64_t n, uint32_t* sha,
                   uint32_t* md5, int ndevices, int devices_visible, const std::vector<uint64_t>& order,
                   const Split& sp,
                   int (*gpu_side)(void* ctx, const uint8_t* const*, const uint64_t*, const uint64_t*,
                                   uint64_t, uint32_t*, uint32_t*),
                   void* ctx, double* t_gpu, double* t_cpu);

}  // namespace s3h::host
