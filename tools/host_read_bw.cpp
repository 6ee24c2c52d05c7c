// host_read_bw.cpp -- host DRAM read bandwidth of one NUMA node (the cap on the
// N-device host-resident rate, where four GPUs behind one socket DMA from that socket's DRAM).
//
// T threads bound to node K's CPUs each stream-read (and sum) their own buffer, first-touched
// on node K; best of R passes, aggregate GB/s.  CPU threads measure what the socket delivers to
// cores -- a LOWER bound on what its DRAM can feed four DMA engines -- under the process's CPU
// quota (16 on the GPU box).  Prints one JSON object.
//
//   g++ -O2 -march=x86-64-v3 -pthread -o tools/host_read_bw tools/host_read_bw.cpp
//   tools/host_read_bw NODE THREADS [MIB_PER_THREAD=1024] [PASSES=5]
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static bool node_cpus(int node, cpu_set_t* set) {
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string s;
  if (!std::getline(f, s)) return false;
  CPU_ZERO(set);
  const char* p = s.c_str();
  while (*p) {
    char* e;
    long a = std::strtol(p, &e, 10), b = a;
    p = e;
    if (*p == '-') b = std::strtol(p + 1, &e, 10), p = e;
    for (long c = a; c <= b; ++c) CPU_SET(int(c), set);
    if (*p == ',') ++p;
  }
  return true;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s NODE THREADS [MIB_PER_THREAD] [PASSES]\n", argv[0]);
    return 2;
  }
  const int node = std::atoi(argv[1]), threads = std::atoi(argv[2]);
  const size_t bytes = size_t(argc > 3 ? std::atoi(argv[3]) : 1024) << 20;
  const int passes = argc > 4 ? std::atoi(argv[4]) : 5;
  cpu_set_t want, mine, both;
  if (!node_cpus(node, &want) || sched_getaffinity(0, sizeof mine, &mine) != 0) return 2;
  CPU_AND(&both, &want, &mine);
  std::vector<uint64_t*> buf(threads);
  std::atomic<int> ready{0}, pass{-1}, done{0};
  std::vector<double> sums(threads);
  auto work = [&](int t) {
    (void)pthread_setaffinity_np(pthread_self(), sizeof both, &both);
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    unsigned long mask[16] = {};
    mask[node / 64] = 1ul << (node % 64);
    (void)syscall(SYS_mbind, p, bytes, 1 /*MPOL_PREFERRED*/, mask, 1025, 0);
    std::memset(p, 1, bytes);
    buf[t] = static_cast<uint64_t*>(p);
    ready.fetch_add(1);
    for (int k = 0; k < passes; ++k) {
      while (pass.load() < k) std::this_thread::yield();
      uint64_t s = 0;
      const uint64_t* q = buf[t];
      for (size_t i = 0; i < bytes / 8; i += 4) s += q[i] ^ q[i + 1] ^ q[i + 2] ^ q[i + 3];
      sums[t] += double(s);
      done.fetch_add(1);
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
  while (ready.load() < threads) std::this_thread::yield();
  double best = 1e30;
  for (int k = 0; k < passes; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    pass.store(k);
    while (done.load() < threads * (k + 1)) std::this_thread::yield();
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  for (auto& t : ts) t.join();
  double chk = 0;
  for (double s : sums) chk += s;
  std::printf("{\"node\": %d, \"threads\": %d, \"bound_cpus\": %d, \"bytes_per_thread\": %zu, "
              "\"passes\": %d, \"best_s\": %.5f, \"GBps\": %.1f, \"GiBps\": %.1f, \"checksum\": %.0f}\n",
              node, threads, CPU_COUNT(&both), bytes, passes, best,
              double(bytes) * threads / best / 1e9, double(bytes) * threads / best / 1073741824.0, chk);
  return 0;
}
