// cpu_hash.hpp -- block-level entry points of the CPU drop-in (lib_hash.cpp, lib_md5.cpp) for
// the library's own CPU route: resumable SHA-256 / MD5 states and one pass that produces both
// digests of a buffer (x-amz-content-sha256 + Content-MD5 of an upload part) while each chunk
// is still in cache.  Not part of the lib/hash surface (include/sha256.h, include/md5.h).
#pragma once
#include <cstdint>

namespace s3h::cpu {

// SHA-256 (native-word state, sha256::init_hash): compress nblk whole blocks.
void sha256_blocks(uint32_t st[8], const uint8_t* p, uint64_t nblk);
// The final `len` bytes (any length) of a message of `total` bytes: whole blocks, then the
// padding with the bit length of `total` (lib/hash/utility.cpp:42-56).  Call sha256::to_little
// afterwards for lib/hash's digest words.
void sha256_final(uint32_t st[8], const uint8_t* data, uint64_t len, uint64_t total);
// MD5 (md5::init_hash): compress nblk whole blocks.
void md5_blocks(uint32_t st[4], const uint8_t* p, uint64_t nblk);
// The final `len` bytes of a message of `total` bytes, padded (little-endian bit length).
void md5_final(uint32_t st[4], const uint8_t* data, uint64_t len, uint64_t total);
// Both digests of one buffer in one pass over memory: 64 KiB chunks, each compressed by
// SHA-256 and then by MD5 while it sits in L1/L2.  sha: lib/hash digest words (to_little
// applied); md5: the 16 digest bytes as md5::md5 writes them.
void sha256_md5(const uint8_t* data, uint64_t len, uint32_t sha[8], uint32_t md5[4]);

}  // namespace s3h::cpu
