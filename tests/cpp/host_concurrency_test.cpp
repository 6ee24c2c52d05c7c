// host_concurrency_test.cpp -- the host path's concurrent machinery under ThreadSanitizer and
// AddressSanitizer (tests/test_host_sanitizers.py builds it twice: -fsanitize=thread and
// -fsanitize=address,undefined).  No GPU: the HIP-free units are linked as they ship --
// host_queue.hpp (the per-device merge queue), copy_pool.hpp, route_plan.cpp (the CPU route
// and the split driver), topology.cpp, status.cpp and the CPU drop-in -- and the executor that
// would run a shard on a device is a fake that stages every part through a CopyPool, hashes it
// with the drop-in, sleeps, fails or throws.
//
// Concurrent callers, as lib/src/upload.cpp:136-140 makes them (std::async jobs):
//   1. 32 callers x rounds submit requests to 4 device queues, mixing algorithm sets (SHA-256,
//      MD5, both), slice sizes, memory parts and file ranges, and injected faults (a part that
//      makes the executor return an error naming its caller, throw std::bad_alloc, or throw
//      something else).  Each caller must get exactly its own status and message, and when it
//      succeeds its own digests -- also when its request was merged with failing ones.
//   2. 8 callers run the split route's driver (route_plan.cpp split_run_impl) at once with a
//      fake GPU side that hashes on the CPU, sleeps and sometimes fails; memory parts and file
//      ranges.  Every file descriptor it opens is closed again (advisor r5).
//   3. 16 callers run the CPU route (cpu_batch) at once on overlapping thread counts.
// Exit status 0 and "host concurrency ok" on success.
#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/md5.h"
#include "../../include/sha256.h"
#include "../../s3client_amd/csrc/copy_pool.hpp"
#include "../../s3client_amd/csrc/host_queue.hpp"
#include "../../s3client_amd/csrc/route_plan.hpp"

namespace s3h::host {
thread_local unsigned g_stage_threads_cap = 0;  // host_path.cpp's definition in the product
}

using namespace s3h::host;

namespace {

std::atomic<int> g_failures{0};

void check(bool ok, const std::string& what) {
  if (!ok) {
    if (g_failures.fetch_add(1) < 20) std::fprintf(stderr, "FAIL: %s\n", what.c_str());
  }
}

// A part's first bytes: caller id (4 B), then a fault kind: 0 none, 1 error, 2 bad_alloc,
// 3 another exception.
enum Fault : uint8_t { kNone = 0, kError = 1, kBadAlloc = 2, kThrow = 3 };

void reference_digests(const uint8_t* p, uint64_t len, const int* algos, int nalgo, uint32_t* out8,
                       uint32_t* out4) {
  static const uint8_t z[1] = {0};
  for (int a = 0; a < nalgo; ++a) {
    if (algos[a] == S3H_ALGO_SHA256) sha256::sha256(len ? p : z, len, out8);
    else md5::md5(len ? p : z, len, out4);
  }
}

// The fake device executor: per device one cached CopyPool (a private one when it is busy,
// like the product's HostCtxCache); each part staged through the pool into a buffer, hashed by
// the drop-in; faults injected by the parts' contents.
struct FakeExec {
  struct Dev {
    std::mutex m;
    std::unique_ptr<CopyPool> pool;
  };
  Dev dev[4];
  std::atomic<uint64_t> batches{0}, merged_parts{0}, private_pools{0};

  int operator()(const HostShard& sh, const int* algos, int nalgo, const PartSource& src,
                 const uint64_t* lengths, uint32_t* const* digests, uint64_t slice) {
    batches.fetch_add(1);
    merged_parts.fetch_add(sh.parts.size());
    Dev& D = dev[sh.device];
    std::unique_lock<std::mutex> l(D.m, std::try_to_lock);
    std::unique_ptr<CopyPool> priv;
    CopyPool* pool;
    if (l.owns_lock()) {
      if (!D.pool) D.pool.reset(new CopyPool(2, Place()));
      pool = D.pool.get();
    } else {
      private_pools.fetch_add(1);
      priv.reset(new CopyPool(1, Place()));
      pool = priv.get();
    }
    const uint64_t n = sh.parts.size();
    std::vector<std::vector<uint8_t>> staged(n);
    std::atomic<int> fault{0}, fault_caller{-1}, read_bad{0};
    pool->run(n, [&](uint64_t j) {
      const uint64_t i = sh.parts[j];
      std::vector<uint8_t>& b = staged[j];
      b.resize(lengths[i]);
      // staged in pieces of `slice` bytes (0: whole), as the slice pipeline does
      const uint64_t step = slice ? slice : std::max<uint64_t>(1, lengths[i]);
      for (uint64_t at = 0; at < lengths[i]; at += step)
        if (!src.fill(i, at, std::min(step, lengths[i] - at), b.data() + at)) read_bad.store(1);
      if (lengths[i] >= 5 && b[4] != kNone) {
        int expect = 0;
        fault.compare_exchange_strong(expect, b[4]);
        int id;
        std::memcpy(&id, b.data(), 4);
        fault_caller.store(id);
      }
    });
    std::this_thread::sleep_for(std::chrono::microseconds(50 * (n % 7)));
    if (read_bad.load()) return fail(S3H_EINVAL, "fake exec: reading a part failed");
    switch (fault.load()) {
      case kError: return fail(S3H_EHIP, "fake exec: poison part of caller %d", fault_caller.load());
      case kBadAlloc: throw std::bad_alloc();
      case kThrow: throw std::runtime_error("fake exec");
      default: break;
    }
    for (uint64_t j = 0; j < n; ++j) {
      const uint64_t i = sh.parts[j];
      uint32_t s8[8], m4[4];
      reference_digests(staged[j].data(), lengths[i], algos, nalgo, s8, m4);
      for (int a = 0; a < nalgo; ++a) {
        if (algos[a] == S3H_ALGO_SHA256) std::memcpy(digests[a] + 8 * i, s8, 32);
        else std::memcpy(digests[a] + 4 * i, m4, 16);
      }
    }
    return S3H_OK;
  }
};

int open_fds() {
  int n = 0;
  if (DIR* d = opendir("/proc/self/fd")) {
    while (readdir(d)) ++n;
    closedir(d);
  }
  return n;
}

// ------------------------------------------------------------------ 1. the merge queue
void queue_callers(const std::string& file_path, const std::vector<uint8_t>& file_bytes) {
  FakeExec exec;
  constexpr int kCallers = 32, kRounds = 6;
  const int file_fd = open(file_path.c_str(), O_RDONLY);
  check(file_fd >= 0, "open the test file");
  std::atomic<int> ok_calls{0}, failed_calls{0};
  std::atomic<int> arrived[kRounds] = {};
  auto caller = [&](int id) {
    std::mt19937_64 rng(1000 + id);
    for (int round = 0; round < kRounds; ++round) {
      // even rounds start together (bursts the queue merges), odd ones as the callers come
      if (round % 2 == 0) {
        arrived[round].fetch_add(1);
        while (arrived[round].load() < kCallers) std::this_thread::yield();
      }
      const int device = int(rng() % 4);
      const int kind = int(rng() % 3);  // algorithm set
      static const int kAlgos[3][2] = {{S3H_ALGO_SHA256, 0}, {S3H_ALGO_MD5, 0}, {S3H_ALGO_SHA256, S3H_ALGO_MD5}};
      const int nalgo = kind == 2 ? 2 : 1;
      const int* algos = kAlgos[kind];
      const uint64_t slice = (rng() % 2) ? 0 : 4096;
      const bool from_file = rng() % 4 == 0;
      const uint8_t fault = (rng() % 8 == 0) ? uint8_t(1 + rng() % 3) : uint8_t(kNone);
      const uint64_t n = 1 + rng() % 12;
      std::vector<std::vector<uint8_t>> bufs(n);
      std::vector<const uint8_t*> ptrs(n);
      std::vector<uint64_t> lens(n), offs(n);
      for (uint64_t i = 0; i < n; ++i) {
        lens[i] = rng() % 3 == 0 ? rng() % 70 : rng() % 200000;
        if (from_file) {
          offs[i] = rng() % (file_bytes.size() - lens[i]);
          continue;
        }
        bufs[i].resize(lens[i]);
        for (auto& b : bufs[i]) b = uint8_t(rng());
        if (lens[i] >= 5) {
          std::memcpy(bufs[i].data(), &id, 4);
          bufs[i][4] = kNone;
        }
        ptrs[i] = bufs[i].data();
      }
      uint64_t poison = n;
      if (fault != kNone && !from_file) {  // one part of this request carries the fault
        for (uint64_t i = 0; i < n && poison == n; ++i)
          if (lens[i] >= 5) poison = i;
        if (poison < n) bufs[poison][4] = fault;
      }
      // file ranges never carry a fault byte the fake reads: pick ranges whose 5th byte is 0
      if (from_file)
        for (uint64_t i = 0; i < n; ++i)
          if (lens[i] >= 5 && file_bytes[offs[i] + 4] != 0) lens[i] = 4;
      std::vector<uint32_t> sha(8 * n, 0xdeadbeef), m5(4 * n, 0xdeadbeef);
      uint32_t* outs[2];
      for (int a = 0; a < nalgo; ++a) outs[a] = algos[a] == S3H_ALGO_SHA256 ? sha.data() : m5.data();
      PartSource src;
      if (from_file) {
        src.fd = file_fd;
        src.file_off = offs.data();
      } else {
        src.parts = ptrs.data();
      }
      HostShard sh{device, 1, {}, 0};
      for (uint64_t i = 0; i < n; ++i) sh.parts.push_back(i);
      HostReq r{algos, nalgo, &src, lens.data(), outs, &sh, slice, S3H_OK, {}, false};
      submit(exec, r);
      const bool poisoned = poison < n;
      const std::string tag = "caller " + std::to_string(id) + " round " + std::to_string(round);
      if (!poisoned) {
        check(r.rc == S3H_OK, tag + ": expected success, got " + std::to_string(r.rc) + " " + r.err);
        for (uint64_t i = 0; i < n && r.rc == S3H_OK; ++i) {
          const uint8_t* p = from_file ? file_bytes.data() + offs[i] : ptrs[i];
          uint32_t s8[8], m4[4];
          reference_digests(p, lens[i], algos, nalgo, s8, m4);
          for (int a = 0; a < nalgo; ++a) {
            const bool is_sha = algos[a] == S3H_ALGO_SHA256;
            check(std::memcmp(is_sha ? &sha[8 * i] : &m5[4 * i], is_sha ? (void*)s8 : (void*)m4, is_sha ? 32 : 16) == 0,
                  tag + ": digest of part " + std::to_string(i));
          }
        }
        ok_calls.fetch_add(1);
      } else {
        const int want = fault == kError ? S3H_EHIP : fault == kBadAlloc ? S3H_ENOMEM : S3H_EHIP;
        check(r.rc == want, tag + ": fault " + std::to_string(fault) + " -> rc " + std::to_string(r.rc));
        if (fault == kError)
          check(r.err == "fake exec: poison part of caller " + std::to_string(id), tag + ": own message, got '" + r.err + "'");
        else if (fault == kBadAlloc)
          check(r.err == "host batch: out of host memory", tag + ": bad_alloc message, got '" + r.err + "'");
        else
          check(r.err == "host batch: unexpected exception", tag + ": exception message, got '" + r.err + "'");
        failed_calls.fetch_add(1);
      }
    }
  };
  std::vector<std::thread> ts;
  for (int id = 0; id < kCallers; ++id) ts.emplace_back(caller, id);
  for (auto& t : ts) t.join();
  close(file_fd);
  std::printf("queue: %d ok, %d failed as injected, %llu batches over %llu parts, %llu private pools\n",
              ok_calls.load(), failed_calls.load(), (unsigned long long)exec.batches.load(),
              (unsigned long long)exec.merged_parts.load(), (unsigned long long)exec.private_pools.load());
  check(ok_calls.load() + failed_calls.load() == kCallers * kRounds, "every call returned");
  check(exec.merged_parts.load() > 0, "the executor ran");
}

// ------------------------------------------------------------------ 2. the split driver
struct FakeGpu {
  std::atomic<int> calls{0};
  bool fail_next = false;
};

int fake_gpu_side(void* ctx, const uint8_t* const* parts, const uint64_t* offsets,
                  const uint64_t* lengths, uint64_t n, uint32_t* sha, uint32_t* md5v) {
  auto* G = static_cast<std::pair<FakeGpu*, const std::vector<uint8_t>*>*>(ctx);
  const int k = G->first->calls.fetch_add(1);
  std::this_thread::sleep_for(std::chrono::microseconds(200 + 37 * (k % 5)));
  if (k % 7 == 3) return fail(S3H_EHIP, "fake gpu side: injected failure %d", k);
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* p = parts ? parts[i] : G->second->data() + offsets[i];
    static const uint8_t z[1] = {0};
    if (sha) sha256::sha256(lengths[i] ? p : z, lengths[i], sha + 8 * i);
    if (md5v) md5::md5(lengths[i] ? p : z, lengths[i], md5v + 4 * i);
  }
  return S3H_OK;
}

void split_callers(const std::string& file_path, const std::vector<uint8_t>& file_bytes) {
  FakeGpu gpu;
  const int fds_before = open_fds();
  std::atomic<int> injected{0}, ok{0};
  auto caller = [&](int id) {
    std::mt19937_64 rng(2000 + id);
    for (int round = 0; round < 5; ++round) {
      const unsigned dig = unsigned(1 + rng() % 3);
      const bool from_file = rng() % 2 == 0;
      const uint64_t n = 2 + rng() % 30;
      std::vector<std::vector<uint8_t>> bufs(n);
      std::vector<const uint8_t*> ptrs(n);
      std::vector<uint64_t> lens(n), offs(n);
      for (uint64_t i = 0; i < n; ++i) {
        lens[i] = rng() % 300000;
        if (from_file) {
          offs[i] = rng() % (file_bytes.size() - lens[i]);
        } else {
          bufs[i].resize(lens[i]);
          for (auto& b : bufs[i]) b = uint8_t(rng());
          ptrs[i] = bufs[i].data();
        }
      }
      const std::vector<uint64_t> order = longest_first(lens.data(), n);
      Split sp;
      sp.m = 1 + rng() % (n - 1);
      sp.tg = unsigned(rng() % 3);
      std::vector<uint32_t> sha(8 * n), m5(4 * n);
      std::pair<FakeGpu*, const std::vector<uint8_t>*> ctx{&gpu, &file_bytes};
      double tg = 0, tc = 0;
      const int rc = split_run_impl(dig, from_file ? nullptr : ptrs.data(), from_file ? file_path.c_str() : nullptr,
                                    from_file ? offs.data() : nullptr, lens.data(), n,
                                    (dig & S3H_DIGESTS_SHA256) ? sha.data() : nullptr,
                                    (dig & S3H_DIGESTS_MD5) ? m5.data() : nullptr, 2, 2, order, sp,
                                    fake_gpu_side, &ctx, &tg, &tc);
      const std::string tag = "split caller " + std::to_string(id) + " round " + std::to_string(round);
      if (rc != S3H_OK) {
        check(rc == S3H_EHIP && g_err.rfind("fake gpu side: injected failure", 0) == 0, tag + ": " + g_err);
        injected.fetch_add(1);
        continue;
      }
      check(tg > 0 && tc > 0, tag + ": side times");
      for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* p = from_file ? file_bytes.data() + offs[i] : ptrs[i];
        static const uint8_t z[1] = {0};
        uint32_t s8[8], m4[4];
        sha256::sha256(lens[i] ? p : z, lens[i], s8);
        md5::md5(lens[i] ? p : z, lens[i], m4);
        if (dig & S3H_DIGESTS_SHA256) check(std::memcmp(&sha[8 * i], s8, 32) == 0, tag + ": sha part " + std::to_string(i));
        if (dig & S3H_DIGESTS_MD5) check(std::memcmp(&m5[4 * i], m4, 16) == 0, tag + ": md5 part " + std::to_string(i));
      }
      ok.fetch_add(1);
    }
  };
  std::vector<std::thread> ts;
  for (int id = 0; id < 8; ++id) ts.emplace_back(caller, id);
  for (auto& t : ts) t.join();
  // a range past the end fails before any thread starts, and closes the file again
  {
    std::vector<uint64_t> lens{10, file_bytes.size()}, offs{0, 1};
    const std::vector<uint64_t> order = longest_first(lens.data(), 2);
    Split sp;
    sp.m = 1;
    std::vector<uint32_t> sha(16);
    std::pair<FakeGpu*, const std::vector<uint8_t>*> ctx{&gpu, &file_bytes};
    const int rc = split_run_impl(S3H_DIGESTS_SHA256, nullptr, file_path.c_str(), offs.data(), lens.data(), 2,
                                  sha.data(), nullptr, 1, 1, order, sp, fake_gpu_side, &ctx, nullptr, nullptr);
    check(rc == S3H_EINVAL, "split: a range past the end of the file is rejected");
  }
  const int fds_after = open_fds();
  std::printf("split: %d ok, %d failed as injected, fds %d -> %d\n", ok.load(), injected.load(), fds_before, fds_after);
  check(fds_after == fds_before, "split route leaked a file descriptor");
  check(ok.load() > 0 && injected.load() > 0, "split: both outcomes exercised");
}

// ------------------------------------------------------------------ 3. the CPU route
void cpu_callers() {
  std::atomic<int> done{0};
  auto caller = [&](int id) {
    std::mt19937_64 rng(3000 + id);
    const unsigned dig = unsigned(1 + id % 3);
    const uint64_t n = 1 + rng() % 40;
    std::vector<std::vector<uint8_t>> bufs(n);
    std::vector<const uint8_t*> ptrs(n);
    std::vector<uint64_t> lens(n);
    for (uint64_t i = 0; i < n; ++i) {
      lens[i] = rng() % 3 == 0 ? rng() % 130 : rng() % 400000;
      bufs[i].resize(lens[i]);
      for (auto& b : bufs[i]) b = uint8_t(rng());
      ptrs[i] = bufs[i].data();
    }
    std::vector<uint32_t> sha(8 * n), m5(4 * n);
    const int rc = cpu_batch(dig, ptrs.data(), -1, nullptr, lens.data(), n,
                             (dig & S3H_DIGESTS_SHA256) ? sha.data() : nullptr,
                             (dig & S3H_DIGESTS_MD5) ? m5.data() : nullptr, 1 + unsigned(id % 6));
    check(rc == S3H_OK, "cpu_batch rc");
    for (uint64_t i = 0; i < n; ++i) {
      static const uint8_t z[1] = {0};
      uint32_t s8[8], m4[4];
      sha256::sha256(lens[i] ? ptrs[i] : z, lens[i], s8);
      md5::md5(lens[i] ? ptrs[i] : z, lens[i], m4);
      if (dig & S3H_DIGESTS_SHA256) check(std::memcmp(&sha[8 * i], s8, 32) == 0, "cpu route sha");
      if (dig & S3H_DIGESTS_MD5) check(std::memcmp(&m5[4 * i], m4, 16) == 0, "cpu route md5");
    }
    done.fetch_add(1);
  };
  std::vector<std::thread> ts;
  for (int id = 0; id < 16; ++id) ts.emplace_back(caller, id);
  for (auto& t : ts) t.join();
  std::printf("cpu route: %d callers\n", done.load());
}

}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string path = dir + "/host_concurrency_test.bin";
  std::vector<uint8_t> bytes(3u << 20);
  std::mt19937_64 rng(7);
  for (auto& b : bytes) b = uint8_t(rng());
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(bytes.data(), 1, bytes.size(), f) != bytes.size()) return 2;
    std::fclose(f);
  }
  queue_callers(path, bytes);
  split_callers(path, bytes);
  cpu_callers();
  std::remove(path.c_str());
  if (g_failures.load()) {
    std::fprintf(stderr, "%d failures\n", g_failures.load());
    return 1;
  }
  std::printf("host concurrency ok\n");
  return 0;
}
