// include/utility.h -- drop-in for lib/hash/utility.h (uv-cpp/s3client @ 2024-10-08).
//
// Same names, signatures and results as the reference helpers, so code written against
// lib/hash (the SigV4 signer, lib/src/aws_sign.cpp, and the upload tools) compiles and links
// unchanged against libs3hash.so.  Bodies are this project's own.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

// 64-bit byte reversal (reference: utility.h:53-63).
inline uint64_t to_big_endian(uint64_t n) { return __builtin_bswap64(n); }

// 32-bit byte reversal (reference: utility.h:71-77).
inline uint32_t to_little_endian(uint32_t n) { return __builtin_bswap32(n); }

// Smallest multiple of d that is >= n (reference: utility.h:86-90, a linear search there).
inline uint64_t next_div_by(uint64_t n, uint64_t d) { return (n + d - 1) / d * d; }

// Rotations on 32-bit words (reference: utility.h:100-112).
inline uint32_t right_rotate(uint32_t x, uint32_t n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t left_rotate(uint32_t x, uint32_t n) { return (x << n) | (x >> (32 - n)); }

// Byte widened to 32 bits, then shifted (reference: utility.h:121-123).
inline uint32_t lshift(uint8_t n, uint8_t nshifts) { return uint32_t(n) << nshifts; }

// SHA-256 padding buffer (reference: utility.h:135-136, utility.cpp:42-56):
// *sz = ceil64(size + 9); the buffer is zeroed, buf[size] = 0x80 and its last 8 bytes hold
// the big-endian bit length 8*size.  Uses tmpbuf (which must hold *sz bytes) when non-null,
// otherwise calloc's a buffer the caller frees.  buffer_size is ignored, as in the reference.
uint8_t *alloc_padded(uint64_t size, uint64_t buffer_size, size_t *sz, uint8_t *tmpbuf);
