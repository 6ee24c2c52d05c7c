// lib_hash.cpp -- CPU side of the lib/hash drop-in (include/sha256.h, include/utility.h).
//
// Single-message hashing stays on the host, exactly as the SigV4 signer uses it
// (lib/src/aws_sign.cpp:63-75: a ~200-byte canonical request plus five HMACs, ~25
// compressions).  A GPU round trip costs more than the whole message here, and one part on
// one GPU lane is ~10x slower than one CPU core, so the GPU is reached only
// through the batched C-ABI in capi.hip.
//
// Compression: x86 SHA extensions when CPUID reports them (runtime dispatch), otherwise a
// portable scalar loop.  S3H_CPU_SCALAR=1 in the environment forces the scalar loop.
#include <cpuid.h>
#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../../include/s3hash.h"
#include "../../../include/sha256.h"
#include "../../../include/md5.h"
#include "cpu_hash.hpp"

namespace {

alignas(64) const uint32_t kRoundK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u,
    0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u,
    0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u,
    0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
    0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u,
    0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au,
    0x5b9cca4fu, 0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
    0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

inline uint32_t rr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t load_be32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return __builtin_bswap32(v);
}

void compress_scalar(uint32_t st_out[8], const uint8_t *p, uint64_t nblk) {
  uint32_t st[8];  // local across blocks: st_out shares cache lines with other parts' digests
  std::memcpy(st, st_out, sizeof st);
  for (; nblk; --nblk, p += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(p + 4 * i);
    uint32_t v[8];
    std::memcpy(v, st, sizeof v);
    for (int t = 0; t < 64; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {  // 16-word ring: w[t&15] holds W[t-16] before the update
        const uint32_t x = w[(t + 1) & 15], y = w[(t + 14) & 15];
        wt = w[t & 15] += (rr(x, 7) ^ rr(x, 18) ^ (x >> 3)) + w[(t + 9) & 15] +
                          (rr(y, 17) ^ rr(y, 19) ^ (y >> 10));
      }
      const uint32_t e = v[4], a = v[0];
      const uint32_t t1 = v[7] + (rr(e, 6) ^ rr(e, 11) ^ rr(e, 25)) + ((e & v[5]) ^ (~e & v[6])) +
                          kRoundK[t] + wt;
      const uint32_t t2 = (rr(a, 2) ^ rr(a, 13) ^ rr(a, 22)) + ((a & v[1]) | (v[2] & (a | v[1])));
      v[7] = v[6]; v[6] = v[5]; v[5] = v[4]; v[4] = v[3] + t1;
      v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t1 + t2;
    }
    for (int i = 0; i < 8; ++i) st[i] += v[i];
  }
  std::memcpy(st_out, st, sizeof st);
}

__attribute__((target("sha,sse4.1,ssse3")))
void compress_shani(uint32_t st[8], const uint8_t *p, uint64_t nblk) {
  const __m128i bswap_mask = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  // state words a..h -> the (ABEF, CDGH) register pair the SHA instructions work on
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i *>(st)), 0xB1);
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i *>(st + 4)), 0x1B);
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);  // ABEF
  s1 = _mm_blend_epi16(s1, t, 0xF0);        // CDGH
  for (; nblk; --nblk, p += 64) {
    const __m128i save0 = s0, save1 = s1;
    __m128i m[4];
    for (int g = 0; g < 16; ++g) {  // 16 groups of four rounds
      __m128i cur;
      if (g < 4) {
        cur = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * g)), bswap_mask);
      } else {
        cur = _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]);                 // W[t-16] + s0(W[t-15])
        cur = _mm_add_epi32(cur, _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));  // + W[t-7]
        cur = _mm_sha256msg2_epu32(cur, m[(g + 3) & 3]);                     // + s1(W[t-2])
      }
      m[g & 3] = cur;
      __m128i wk = _mm_add_epi32(cur, _mm_load_si128(reinterpret_cast<const __m128i *>(kRoundK + 4 * g)));
      s1 = _mm_sha256rnds2_epu32(s1, s0, wk);
      wk = _mm_shuffle_epi32(wk, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, wk);
    }
    s0 = _mm_add_epi32(s0, save0);
    s1 = _mm_add_epi32(s1, save1);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);   // FEBA
  s1 = _mm_shuffle_epi32(s1, 0xB1);  // DCHG
  _mm_storeu_si128(reinterpret_cast<__m128i *>(st), _mm_blend_epi16(t, s1, 0xF0));     // DCBA
  _mm_storeu_si128(reinterpret_cast<__m128i *>(st + 4), _mm_alignr_epi8(s1, t, 8));    // HGFE
}

using CompressFn = void (*)(uint32_t *, const uint8_t *, uint64_t);

CompressFn pick_compress() {
  const char *force = std::getenv("S3H_CPU_SCALAR");
  if (force && force[0] == '1') return compress_scalar;
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return compress_scalar;
  const bool sse41 = c & (1u << 19), ssse3 = c & (1u << 9);
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return compress_scalar;
  const bool sha = b & (1u << 29);
  return (sha && sse41 && ssse3) ? compress_shani : compress_scalar;
}

const CompressFn g_compress = pick_compress();

// Digest of `len` bytes: whole blocks straight from the caller's buffer, then the one or two
// padded tail blocks built on the stack (no padded copy of the message, unlike
// sha256.cpp:151-158 which copies anything over 4087 bytes).
void digest_native(const uint8_t *data, uint64_t len, uint64_t bitlen, uint32_t st[8]) {
  const uint64_t whole = len / 64;
  g_compress(st, data, whole);
  uint8_t tail[128] = {0};
  const uint64_t rem = len - whole * 64;
  if (rem) std::memcpy(tail, data + whole * 64, rem);
  tail[rem] = 0x80;
  const uint64_t tb = rem < 56 ? 64 : 128;
  const uint64_t be = __builtin_bswap64(bitlen);
  std::memcpy(tail + tb - 8, &be, 8);
  g_compress(st, tail, tb / 64);
}

}  // namespace

// ------------------------------------------------------------------ lib/hash drop-in
uint8_t *alloc_padded(uint64_t size, uint64_t /*buffer_size*/, size_t *sz, uint8_t *tmpbuf) {
  const uint64_t n = next_div_by(size + 9, 64);
  *sz = n;
  uint8_t *buf = tmpbuf;
  if (buf) std::memset(buf, 0, n);
  else buf = static_cast<uint8_t *>(std::calloc(n, 1));
  if (!buf) return nullptr;
  buf[size] = 0x80;
  const uint64_t be = to_big_endian(8 * size);
  std::memcpy(buf + n - 8, &be, 8);
  return buf;
}

namespace sha256 {

void sha256_stream(uint32_t hash[8], const uint8_t data[], uint64_t length) {
  g_compress(hash, data, length / 64);
}

void sha256(const uint8_t data[], size_t length, uint32_t hash[8]) {
  init_hash(hash);
  digest_native(data, length, 8ull * length, hash);
  to_little(hash);
}

void sha256_next(const uint8_t data[], uint32_t length, uint32_t hash[8], size_t total_length,
                 uint8_t * /*tmpbuf*/) {
  if (total_length == 0) {
    g_compress(hash, data, length / 64);
    return;
  }
  digest_native(data, length, 8ull * total_length, hash);
}

void print_hash(uint32_t hash[8]) {
  char text[65];
  hash_to_text(hash, text);
  std::printf("%s\n", text);
}

void sha256_file(const char *fname, uint32_t hash[8]) {
  FILE *f = std::fopen(fname, "rb");
  if (!f) {  // same error convention as the reference (sha256.cpp:185-187)
    std::fprintf(stderr, "Error opening file %s\n", fname);
    std::exit(EXIT_FAILURE);
  }
  const size_t kBuf = size_t(16) << 20;
  std::vector<uint8_t> buf(kBuf);
  init_hash(hash);
  uint64_t total = 0;
  size_t have = 0;  // bytes buffered, always < 64 after each compress
  for (;;) {
    const size_t got = std::fread(buf.data() + have, 1, kBuf - have, f);
    have += got;
    total += got;
    if (got == 0) break;
    const size_t whole = have / 64 * 64;
    g_compress(hash, buf.data(), whole / 64);
    std::memmove(buf.data(), buf.data() + whole, have - whole);
    have -= whole;
  }
  if (std::ferror(f)) {
    std::perror("Error reading from file");
    std::exit(EXIT_FAILURE);
  }
  std::fclose(f);
  digest_native(buf.data(), have, 8ull * total, hash);
  to_little(hash);
}

}  // namespace sha256

// RFC 2104 HMAC with SHA-256 (reference: hmac256.cpp:60-95).  Keys longer than the 64-byte
// block are hashed over their own key_length bytes; the reference hashes `length` (message)
// bytes of the key there (hmac256.cpp:72).  Both agree whenever key_length <= 64, which holds
// for every SigV4 key ("AWS4"+secret is 40-44 bytes, derived keys 32 bytes).
void hmac256(const uint8_t *data, size_t length, const uint8_t *key, size_t key_length,
             uint8_t hmac_hash[32]) {
  uint8_t k[64] = {0};
  if (key_length <= 64) {
    if (key_length) std::memcpy(k, key, key_length);
  } else {
    sha256::sha256(key, key_length, reinterpret_cast<uint32_t *>(k));
  }
  uint8_t pad[64];
  uint32_t st[8];
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x36;
  sha256::init_hash(st);
  g_compress(st, pad, 1);
  digest_native(data, length, 8ull * (64 + length), st);
  uint8_t inner[32];
  for (int i = 0; i < 8; ++i) {
    const uint32_t be = __builtin_bswap32(st[i]);
    std::memcpy(inner + 4 * i, &be, 4);
  }
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x5c;
  sha256::init_hash(st);
  g_compress(st, pad, 1);
  digest_native(inner, 32, 8ull * 96, st);
  for (int i = 0; i < 8; ++i) {
    const uint32_t be = __builtin_bswap32(st[i]);
    std::memcpy(hmac_hash + 4 * i, &be, 4);
  }
}

// ------------------------------------------------------------------ block-level (cpu_hash.hpp)
namespace s3h::cpu {

void sha256_blocks(uint32_t st[8], const uint8_t *p, uint64_t nblk) { g_compress(st, p, nblk); }

void sha256_final(uint32_t st[8], const uint8_t *data, uint64_t len, uint64_t total) {
  digest_native(data, len, 8ull * total, st);
}

void sha256_md5(const uint8_t *data, uint64_t len, uint32_t sha[8], uint32_t md5[4]) {
  constexpr uint64_t kChunk = 64ull << 10;  // both passes over a chunk hit L1/L2
  sha256::init_hash(sha);
  md5::init_hash(md5);
  const uint64_t whole = len / 64 * 64;
  for (uint64_t at = 0; at < whole; at += kChunk) {
    const uint64_t nb = std::min(kChunk, whole - at) / 64;
    g_compress(sha, data + at, nb);
    md5_blocks(md5, data + at, nb);
  }
  sha256_final(sha, data + whole, len - whole, len);
  md5_final(md5, data + whole, len - whole, len);
  sha256::to_little(sha);
}

}  // namespace s3h::cpu

// ------------------------------------------------------------------ C view (s3hash.h)
extern "C" {
void s3h_cpu_sha256(const uint8_t *data, uint64_t length, uint32_t hash[8]) {
  sha256::sha256(data, size_t(length), hash);
}
void s3h_cpu_hmac256(const uint8_t *data, uint64_t length, const uint8_t *key,
                     uint64_t key_length, uint8_t mac[32]) {
  hmac256(data, size_t(length), key, size_t(key_length), mac);
}
void s3h_hash_to_text(const uint32_t hash[8], char text[65]) {
  sha256::hash_to_text(const_cast<uint32_t *>(hash), text);
}
const char *s3h_cpu_backend(void) { return g_compress == compress_shani ? "sha-ni" : "scalar"; }
}
