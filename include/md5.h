// include/md5.h -- drop-in for lib/hash/md5.h (uv-cpp/s3client @ 2024-10-08).
//
// Same namespace, names and parameter types as the reference (hence the same mangled symbols
// in libs3hash.so).  MD5 is what S3 uses for Content-MD5 and multipart ETags; batches of
// parts go to the GPU through include/s3hash.h (s3h_md5_*), single messages stay here.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "utility.h"

namespace md5 {

// MD5 initial state (reference: md5.h:51-56).
inline void init_hash(uint32_t h[4]) {
  h[0] = 0x67452301u;
  h[1] = 0xefcdab89u;
  h[2] = 0x98badcfeu;
  h[3] = 0x10325476u;
}

// Compress the whole 64-byte blocks of `length` bytes into `hash` (reference: md5.h:67).
// The reference loop also consumes a trailing partial block (md5.cpp:72), reading past
// `data`; this one ignores the tail, as sha256_stream does.
void md5_stream(uint32_t hash[4], const uint8_t data[], uint64_t length);

// Padded one-shot MD5 (reference: md5.cpp:119-122, which forgets to pad).
void md5(const uint8_t data[], size_t length, uint32_t hash[4]);

// Lowercase hex of the 16 digest bytes (reference: md5.h:72-77).
inline void hash_to_text(uint32_t hash[4], char *text) {
  static const char kHex[] = "0123456789abcdef";
  const unsigned char *b = reinterpret_cast<const unsigned char *>(hash);
  for (int i = 0; i < 16; ++i) {
    text[2 * i] = kHex[b[i] >> 4];
    text[2 * i + 1] = kHex[b[i] & 15];
  }
  text[32] = '\0';
}

void print_hash(uint32_t hash[4]);              // reference: md5.h:83
void md5_file(const char *fname, uint32_t hash[4]);  // reference: md5.cpp:132-180

}  // namespace md5
