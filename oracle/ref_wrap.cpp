// oracle/ref_wrap.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" shims over the REAL reference lib/hash (compiled from /root/reference by
// oracle/Makefile into oracle/_ref/libref_hash.so).  No reference source is copied: this
// file only calls the reference's own symbols.  Used (a) by tests/golden/gen_golden.py to
// produce the committed fixtures, (b) by tests/test_ref_differential.py and (c) by
// tools/calibrate_cpu_baseline.py to calibrate oracle/cpu_baseline.c against the real lib/hash
// (all in the build container: oracle/_ref never travels to the GPU box).
#include <cstdint>
#include <cstddef>
#include <thread>
#include <vector>

#include "md5.h"     // /root/reference/lib/hash/md5.h (via -I)
#include "sha256.h"  // /root/reference/lib/hash/sha256.h (via -I)

namespace md5 {
void md5_file(const char *fname, uint32_t hash[4]);  // md5.cpp:132 (no header declaration)
}

void hmac256(const uint8_t *data, size_t length, const uint8_t *key, size_t key_length,
             uint8_t hmac_hash[32]);  // declared ad hoc like lib/src/aws_sign.cpp:54-55

extern "C" {

void ref_sha256(const uint8_t *data, uint64_t len, uint32_t out[8]) {
  sha256::sha256(data, (size_t)len, out);
}

void ref_sha256_stream(uint32_t h[8], const uint8_t *data, uint64_t len) {
  sha256::sha256_stream(h, data, len);
}

void ref_hmac256(const uint8_t *data, uint64_t len, const uint8_t *key, uint64_t klen,
                 uint8_t out[32]) {
  hmac256(data, (size_t)len, key, (size_t)klen, out);
}

void ref_md5_stream(uint32_t h[4], const uint8_t *data, uint64_t len) {
  md5::md5_stream(h, data, len);
}

// md5_file is the reference's only correctly padded MD5 entry point (md5.cpp:132-180).
void ref_md5_file(const char *path, uint32_t out[4]) { md5::md5_file(path, out); }

// lib/hash's sha256() over n parts with `threads` std::threads, parts round-robin
// (BASELINE.md "CPU baseline plan").
void ref_sha256_batch(const uint8_t *base, const uint64_t *offsets, const uint64_t *lengths,
                      uint64_t n, uint32_t *out, int threads) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([=] {
      for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)threads)
        sha256::sha256(base + offsets[i], (size_t)lengths[i], out + 8 * i);
    });
  for (auto &th : pool) th.join();
}
}
