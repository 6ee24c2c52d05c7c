// lib_md5.cpp -- CPU side of the MD5 drop-in (include/md5.h).  RFC 1321 MD5 with the state
// and output layout of /root/reference/lib/hash/md5.cpp (digest bytes = state words in
// little-endian memory order), and the S3 multipart ETag built on it.
//
// The 64 steps are expanded at compile time (step index, round function, message word and
// shift are template constants), so each step is a handful of register operations with no
// table lookups or branches: the routed CPU path prices a dual-digest part by this loop.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "../../../include/md5.h"
#include "../../../include/s3hash.h"
#include "../status.hpp"
#include "cpu_hash.hpp"

namespace {

constexpr uint32_t kT[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u,
    0xfd469501u, 0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u,
    0xa679438eu, 0x49b40821u, 0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du,
    0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u, 0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu,
    0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au, 0xfffa3942u, 0x8771f681u, 0x6d9d6122u,
    0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u, 0x289b7ec6u, 0xeaa127fau,
    0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u, 0xf4292244u,
    0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu,
    0xeb86d391u};

// per round (16 steps): the left-rotation of step i & 3, and message word of step i
constexpr int shift_of(int i) {
  constexpr int s[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
  return s[i / 16][i % 4];
}
constexpr int word_of(int i) {
  return i < 16 ? i : i < 32 ? (5 * i + 1) % 16 : i < 48 ? (3 * i + 5) % 16 : (7 * i) % 16;
}

inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// Step I updates `a` from b, c, d (the caller rotates the names).  Round functions in their
// select forms: F = d ^ (b & (c ^ d)), G = c ^ (d & (b ^ c)), H = b ^ c ^ d, I = c ^ (b | ~d).
template <int I>
inline void step(uint32_t& a, uint32_t b, uint32_t c, uint32_t d, const uint32_t* m) {
  uint32_t f;
  if constexpr (I < 16) f = d ^ (b & (c ^ d));
  else if constexpr (I < 32) f = c ^ (d & (b ^ c));
  else if constexpr (I < 48) f = b ^ c ^ d;
  else f = c ^ (b | ~d);
  a = b + rotl(a + f + kT[I] + m[word_of(I)], shift_of(I));
}

template <int G>
inline void group(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* m) {
  step<4 * G + 0>(a, b, c, d, m);
  step<4 * G + 1>(d, a, b, c, m);
  step<4 * G + 2>(c, d, a, b, m);
  step<4 * G + 3>(b, c, d, a, m);
}

template <int... G>
inline void all_groups(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* m,
                       std::integer_sequence<int, G...>) {
  (group<G>(a, b, c, d, m), ...);
}

// The chaining state stays in locals for the whole run: `st` usually points into the caller's
// digest array, where neighbouring parts' states share a cache line, and a store per block
// (the compiler must assume `p` may alias `st`) made threads hashing adjacent parts fight over
// that line -- the CPU route ran at half its single-thread rate x threads.
void compress(uint32_t st[4], const uint8_t *p, uint64_t nblk) {
  uint32_t s0 = st[0], s1 = st[1], s2 = st[2], s3 = st[3];
  for (; nblk; --nblk, p += 64) {
    uint32_t m[16];
    std::memcpy(m, p, 64);  // little-endian words on x86
    uint32_t a = s0, b = s1, c = s2, d = s3;
    all_groups(a, b, c, d, m, std::make_integer_sequence<int, 16>());
    s0 += a; s1 += b; s2 += c; s3 += d;
  }
  st[0] = s0; st[1] = s1; st[2] = s2; st[3] = s3;
}

void finish(uint32_t st[4], const uint8_t *data, uint64_t len, uint64_t total) {
  const uint64_t whole = len / 64;
  compress(st, data, whole);
  uint8_t tail[128] = {0};
  const uint64_t rem = len - whole * 64;
  if (rem) std::memcpy(tail, data + whole * 64, rem);
  tail[rem] = 0x80;
  const uint64_t tb = rem < 56 ? 64 : 128;
  const uint64_t bits = 8 * total;
  std::memcpy(tail + tb - 8, &bits, 8);  // little-endian bit length (md5.cpp:168-170)
  compress(st, tail, tb / 64);
}

}  // namespace

namespace s3h::cpu {

void md5_blocks(uint32_t st[4], const uint8_t *p, uint64_t nblk) { compress(st, p, nblk); }
void md5_final(uint32_t st[4], const uint8_t *data, uint64_t len, uint64_t total) {
  finish(st, data, len, total);
}

}  // namespace s3h::cpu

namespace md5 {

void md5_stream(uint32_t hash[4], const uint8_t data[], uint64_t length) {
  compress(hash, data, length / 64);
}

void md5(const uint8_t data[], size_t length, uint32_t hash[4]) {
  init_hash(hash);
  finish(hash, data, length, length);
}

void print_hash(uint32_t hash[4]) {
  char t[33];
  hash_to_text(hash, t);
  std::printf("%s\n", t);
}

void md5_file(const char *fname, uint32_t hash[4]) {
  FILE *f = std::fopen(fname, "rb");
  if (!f) {  // reference convention (md5.cpp:134-137)
    std::fprintf(stderr, "Error opening file %s\n", fname);
    std::exit(EXIT_FAILURE);
  }
  const size_t kBuf = size_t(16) << 20;
  std::vector<uint8_t> buf(kBuf);
  init_hash(hash);
  uint64_t total = 0;
  size_t have = 0;
  for (;;) {
    const size_t got = std::fread(buf.data() + have, 1, kBuf - have, f);
    have += got;
    total += got;
    if (got == 0) break;
    const size_t whole = have / 64 * 64;
    compress(hash, buf.data(), whole / 64);
    std::memmove(buf.data(), buf.data() + whole, have - whole);
    have -= whole;
  }
  if (std::ferror(f)) {
    std::perror("Error reading from file");
    std::exit(EXIT_FAILURE);
  }
  std::fclose(f);
  finish(hash, buf.data(), have, total);
}

}  // namespace md5

extern "C" {

void s3h_cpu_md5(const uint8_t *data, uint64_t length, uint32_t hash[4]) {
  md5::md5(data, size_t(length), hash);
}

// S3 multipart ETag (what CompleteMultipartUpload returns, multipart_upload.cpp:162-183):
// hex(MD5(binary part MD5s concatenated in part order)) + "-" + part count.  The outer MD5
// covers 16 B per part, so it runs on the MD5 drop-in.
int s3h_multipart_etag(const uint32_t *md5_digests, uint64_t n, char *out, uint64_t out_len) {
  using s3h::host::fail;
  if (out && out_len) out[0] = '\0';
  if (!out || out_len < S3H_ETAG_MAX) return fail(S3H_EINVAL, "multipart etag: need %d output bytes", S3H_ETAG_MAX);
  if (n == 0 || !md5_digests) return fail(S3H_EINVAL, "multipart etag: no part digests");
  uint32_t h[4];
  md5::md5(reinterpret_cast<const uint8_t *>(md5_digests), size_t(16 * n), h);
  md5::hash_to_text(h, out);
  std::snprintf(out + 32, size_t(out_len - 32), "-%llu", static_cast<unsigned long long>(n));
  return S3H_OK;
}

}  // extern "C"
