// cpu_dual_probe.cpp -- why the CPU route's SHA-256 + MD5 pass runs slower than its model
// (profiles/r06_route_sweep_dual.json: 250-300 MB/s per thread on 8 MiB parts against the
// model's 690 MB/s, measured on 2-4 MiB cache-resident buffers).  On the GPU box's host CPUs,
// over 8 MiB parts in a DRAM-resident buffer: the route (cpu_batch) for each digest set at 1,
// 8 and 16 threads, the model's probes (one_thread_rate, team_rate), and the fused pass with
// other chunk sizes (one thread).  Prints one JSON object.
//
//   g++ -O2 -std=c++17 -pthread -Iinclude -o tools/cpu_dual_probe tools/cpu_dual_probe.cpp \
//       s3client_amd/csrc/{route_plan,topology,status}.cpp s3client_amd/csrc/cpu/lib_{hash,md5}.cpp
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/md5.h"
#include "../include/sha256.h"
#include "../s3client_amd/csrc/cpu/cpu_hash.hpp"
#include "../s3client_amd/csrc/route_plan.hpp"

namespace s3h::host {
thread_local unsigned g_stage_threads_cap = 0;
}
using namespace s3h::host;

static double secs(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  constexpr uint64_t L = 8ull << 20, n = 64;
  std::vector<uint8_t> big(n * L);
  for (uint64_t i = 0; i < big.size(); i += 4096) big[i] = uint8_t(i >> 12);
  std::vector<const uint8_t*> parts(n);
  std::vector<uint64_t> lens(n, L);
  for (uint64_t i = 0; i < n; ++i) parts[i] = big.data() + i * L;
  std::vector<uint32_t> sha(8 * n), md5v(4 * n);
  std::string out = "{\"part_bytes\": 8388608, \"parts\": 64";
  const char* names[4] = {"memcpy", "sha256", "md5", "both"};
  for (unsigned dig = 1; dig <= 3; ++dig) {
    out += std::string(", \"") + names[dig] + "\": {\"model_one_thread_MBps\": " +
           std::to_string(int(one_thread_rate(dig) / 1e6)) +
           ", \"model_team16_MBps\": " + std::to_string(int(team_rate(16, dig) / 1e6));
    for (unsigned T : {1u, 8u, 16u}) {
      const uint64_t m = T == 1 ? 4 : n;
      double best = 1e30;
      for (int r = 0; r < 3; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        cpu_batch(dig, parts.data(), -1, nullptr, lens.data(), m, sha.data(), md5v.data(), T);
        best = std::min(best, secs(t0));
      }
      out += ", \"route_T" + std::to_string(T) + "_MBps\": " + std::to_string(int(m * L / best / 1e6));
    }
    out += "}";
  }
  // the fused pass with other chunk sizes, one thread, 4 parts from DRAM
  out += ", \"fused_chunk_one_thread_MBps\": {";
  bool first = true;
  for (uint64_t chunk : {4096ull, 16384ull, 32768ull, 65536ull, 262144ull, 8388608ull}) {
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int p = 0; p < 4; ++p) {
        uint32_t h[8], m4[4];
        sha256::init_hash(h);
        md5::init_hash(m4);
        const uint8_t* d = parts[8 + 4 * r + p];
        for (uint64_t at = 0; at < L; at += chunk) {
          s3h::cpu::sha256_blocks(h, d + at, chunk / 64);
          s3h::cpu::md5_blocks(m4, d + at, chunk / 64);
        }
      }
      best = std::min(best, secs(t0));
    }
    out += std::string(first ? "" : ", ") + "\"" + std::to_string(chunk) + "\": " + std::to_string(int(4 * L / best / 1e6));
    first = false;
  }
  out += "}}";
  std::printf("%s\n", out.c_str());
  return 0;
}
