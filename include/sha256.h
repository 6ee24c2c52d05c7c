// include/sha256.h -- drop-in for lib/hash/sha256.h (uv-cpp/s3client @ 2024-10-08).
//
// Keeps every declaration of the reference header (same namespace, names, parameter types,
// hence the same mangled symbols in libs3hash.so) and its inline helpers, so the SigV4
// signer (lib/src/aws_sign.cpp:63-75) and the upload/download tools link unchanged.
// Single-message calls run on the CPU (SHA-NI when the host has it, scalar otherwise);
// batches of upload parts go to the GPU through include/s3hash.h / s3hash_batch.hpp.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "utility.h"

namespace sha256 {

// SHA-256 initial hash value H(0) (reference: sha256.h:53-62).
inline void init_hash(uint32_t hash[8]) {
  static const uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                  0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  for (int i = 0; i < 8; ++i) hash[i] = kIV[i];
}

// One-shot digest of `length` bytes; hash[i] = bswap32(H_i) (reference: sha256.h:70).
void sha256(const uint8_t data[], size_t length, uint32_t hash[8]);

// Chunked form (reference: sha256.h:88-89).  total_length == 0: compress the whole 64-byte
// blocks of this chunk into `hash`.  Otherwise this is the final chunk: it is padded with
// the bit length of `total_length` and compressed.  The state stays in native word order
// (call to_little afterwards).  NOTE: this follows the documented contract; the reference
// body (sha256.cpp:162-174) pads with the chunk length and compresses the unpadded input.
void sha256_next(const uint8_t data[], uint32_t length, uint32_t hash[8], size_t total_length,
                 uint8_t *tmpbuf);

// Compress floor(length/64) whole blocks into `hash` (reference: sha256.h:97).
void sha256_stream(uint32_t hash[8], const uint8_t data[], uint64_t length);

// Native state words -> digest words (reference: sha256.h:103-106).
inline void to_little(uint32_t hash[8]) {
  for (int i = 0; i < 8; ++i) hash[i] = to_little_endian(hash[i]);
}

// Lowercase hex of the 32 digest bytes as laid out in memory (reference: sha256.h:113-119).
inline void hash_to_text(uint32_t hash[8], char *text) {
  static const char kHex[] = "0123456789abcdef";
  const unsigned char *b = reinterpret_cast<const unsigned char *>(hash);
  for (int i = 0; i < 32; ++i) {
    text[2 * i] = kHex[b[i] >> 4];
    text[2 * i + 1] = kHex[b[i] & 15];
  }
  text[64] = '\0';
}

// Print the digest as hex plus newline (reference: sha256.h:125).
void print_hash(uint32_t hash[8]);

// Digest of a whole file (reference: sha256.cpp:183-233, no header declaration there).
void sha256_file(const char *fname, uint32_t hash[8]);

}  // namespace sha256

// HMAC-SHA256 (reference: hmac256.cpp:60-95; declared ad hoc at aws_sign.cpp:54-55).
void hmac256(const uint8_t *data, size_t length, const uint8_t *key, size_t key_length,
             uint8_t hmac_hash[32]);
