// sha256_device.hpp -- gfx950 (CDNA4) device primitives for the batched SHA-256 path.
//
// The arithmetic is FIPS 180-4 SHA-256 exactly as lib/hash computes it
// (/root/reference/lib/hash/sha256.cpp:50-143), re-expressed for the CDNA4 VALU:
//   * rotates are one v_alignbit_b32 each (utility.h:100-102 right_rotate),
//   * the three-way XORs of Sigma/sigma are one v_bitop3_b32 (truth table 0x96),
//   * Maj is one v_bitop3_b32 (0xE8), Ch one v_bfi_b32,
//   * the big-endian byte assembly of sha256.cpp:99-100 (and any sub-dword misalignment of
//     the part) is a single v_perm_b32 per word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exp_config.hpp"
#include "kernel_abi.hpp"

namespace s3h {

// Round constants as compile-time literals (folded into SGPR/literal operands).
#define S3H_K(i) ((uint32_t)(                                                            \
  (i)==0?0x428a2f98u:(i)==1?0x71374491u:(i)==2?0xb5c0fbcfu:(i)==3?0xe9b5dba5u:           \
  (i)==4?0x3956c25bu:(i)==5?0x59f111f1u:(i)==6?0x923f82a4u:(i)==7?0xab1c5ed5u:           \
  (i)==8?0xd807aa98u:(i)==9?0x12835b01u:(i)==10?0x243185beu:(i)==11?0x550c7dc3u:         \
  (i)==12?0x72be5d74u:(i)==13?0x80deb1feu:(i)==14?0x9bdc06a7u:(i)==15?0xc19bf174u:       \
  (i)==16?0xe49b69c1u:(i)==17?0xefbe4786u:(i)==18?0x0fc19dc6u:(i)==19?0x240ca1ccu:       \
  (i)==20?0x2de92c6fu:(i)==21?0x4a7484aau:(i)==22?0x5cb0a9dcu:(i)==23?0x76f988dau:       \
  (i)==24?0x983e5152u:(i)==25?0xa831c66du:(i)==26?0xb00327c8u:(i)==27?0xbf597fc7u:       \
  (i)==28?0xc6e00bf3u:(i)==29?0xd5a79147u:(i)==30?0x06ca6351u:(i)==31?0x14292967u:       \
  (i)==32?0x27b70a85u:(i)==33?0x2e1b2138u:(i)==34?0x4d2c6dfcu:(i)==35?0x53380d13u:       \
  (i)==36?0x650a7354u:(i)==37?0x766a0abbu:(i)==38?0x81c2c92eu:(i)==39?0x92722c85u:       \
  (i)==40?0xa2bfe8a1u:(i)==41?0xa81a664bu:(i)==42?0xc24b8b70u:(i)==43?0xc76c51a3u:       \
  (i)==44?0xd192e819u:(i)==45?0xd6990624u:(i)==46?0xf40e3585u:(i)==47?0x106aa070u:       \
  (i)==48?0x19a4c116u:(i)==49?0x1e376c08u:(i)==50?0x2748774cu:(i)==51?0x34b0bcb5u:       \
  (i)==52?0x391c0cb3u:(i)==53?0x4ed8aa4au:(i)==54?0x5b9cca4fu:(i)==55?0x682e6ff3u:       \
  (i)==56?0x748f82eeu:(i)==57?0x78a5636fu:(i)==58?0x84c87814u:(i)==59?0x8cc70208u:       \
  (i)==60?0x90befffau:(i)==61?0xa4506cebu:(i)==62?0xbef9a3f7u:0xc67178f2u))

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return (e & f) | (~e & g); }
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

__device__ __forceinline__ void init_state(uint32_t s[8]) {
  s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
  s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

// Slot, nblocks: kernel_abi.hpp (shared with the host).

// One round with the state held in rotating names: only d and h are written.
#define S3H_RND(a, b, c, d, e, f, g, h, wk)            \
  do {                                                 \
    const uint32_t t1_ = (h) + (wk) + bsig1(e) + ch(e, f, g); \
    (d) += t1_;                                        \
    (h) = t1_ + bsig0(a) + maj(a, b, c);               \
  } while (0)

// 64 rounds over precomputed W[t] + K[t].
__device__ __forceinline__ void rounds_wk(uint32_t st[8], const uint32_t wk[64]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t += 8) {
    S3H_RND(a, b, c, d, e, f, g, h, wk[t + 0]);
    S3H_RND(h, a, b, c, d, e, f, g, wk[t + 1]);
    S3H_RND(g, h, a, b, c, d, e, f, wk[t + 2]);
    S3H_RND(f, g, h, a, b, c, d, e, wk[t + 3]);
    S3H_RND(e, f, g, h, a, b, c, d, wk[t + 4]);
    S3H_RND(d, e, f, g, h, a, b, c, wk[t + 5]);
    S3H_RND(c, d, e, f, g, h, a, b, wk[t + 6]);
    S3H_RND(b, c, d, e, f, g, h, a, wk[t + 7]);
  }
  st[0] = a; st[1] = b; st[2] = c; st[3] = d; st[4] = e; st[5] = f; st[6] = g; st[7] = h;
}

// Message schedule: w[0..15] in, W[t] + K[t] for t = 0..63 out (sha256.cpp:116-123).
__device__ __forceinline__ void schedule_wk(const uint32_t w16[16], uint32_t wk[64]) {
  uint32_t w[64];
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = w16[t];
#pragma unroll
  for (int t = 16; t < 64; ++t) w[t] = w[t - 16] + ssig0(w[t - 15]) + w[t - 7] + ssig1(w[t - 2]);
#pragma unroll
  for (int t = 0; t < 64; ++t) wk[t] = w[t] + S3H_K(t);
}

// Length a producer lane decodes with.  A lane without a part (its slot is past n in the
// last, partial group) loads the zero page like any block outside a part; a length past every
// block keeps it on the full-block decode -- with its true length 0 it would take the
// padded-tail branch every block, and, the wave being SIMT, so would the whole wave
// (1,800 x 8 MiB SHA-256 + MD5: 2.9x slower; profiles/r02_exp_dual_partial_groups.jsonl).
__device__ __forceinline__ uint64_t decode_len(bool has_part, uint64_t len) {
  return has_part ? len : (1ull << 62);
}

// Raw fetch of one FULL 64-byte block whose first byte is at `p` (any alignment).
// Loads the 17 dwords covering it from the dword-aligned address below `p`; the 17th is
// only touched when p is not dword aligned, so no dword without a part byte is read.
struct RawBlock { uint32_t d[17]; };
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
// Explicit global (address space 1) pointers: a generic pointer would compile to flat_load,
// which completes out of order with LDS traffic, so the compiler must drain vmcnt(0) before
// every use -- defeating the producer's prefetch.  global_load keeps counted vmcnt waits.
typedef const __attribute__((address_space(1))) v4u32 gv4u32;
typedef const __attribute__((address_space(1))) uint32_t gu32;

// Branch-free: when `ok` is false (block outside the part or the launch's range) the same
// loads read the plan's 256-byte zero page instead, so every lane issues the same loads and
// the compiler can keep COUNTED vmcnt waits (a divergent branch around the loads makes it
// drain vmcnt(0) at every use, i.e. no prefetch).  The 17th dword is read from the block
// only when p is not dword aligned, so no dword without a part byte is ever touched.
// Cached loads (round 3): a lane's 64-byte block arrives as four 16-B loads; non-temporal ones
// reached L2 separately, and a producer whose 64 lanes read 64 different parts (md5_pc_kernel)
// paced the C4 shard at 1,390 cycles per block against its consumer's 1,236 alone; cached, L1
// merges them: MD5 C4 shard 836 -> 934 GiB/s, SHA-256 skews C4 503 -> 507, C2 / C3 unchanged
// (profiles/r03_exp_fetch_temporal*.jsonl, alternating on one box).
__device__ __forceinline__ void fetch_full(const uint8_t* p, bool ok, const uint8_t* zero,
                                           RawBlock& r) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(ok ? p : zero);
  gv4u32* q = reinterpret_cast<gv4u32*>(a & ~uintptr_t(3));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#ifdef S3H_EXP_NONTEMPORAL_FETCH  // experiment: round 1-3's non-temporal loads
    const v4u32 v = __builtin_nontemporal_load(q + i);
#else
    const v4u32 v = q[i];
#endif
    r.d[4 * i + 0] = v.x; r.d[4 * i + 1] = v.y; r.d[4 * i + 2] = v.z; r.d[4 * i + 3] = v.w;
  }
  gu32* x = reinterpret_cast<gu32*>((a & 3) ? reinterpret_cast<uintptr_t>(q + 4)
                                             : reinterpret_cast<uintptr_t>(zero));
#ifdef S3H_EXP_NONTEMPORAL_FETCH
  r.d[16] = __builtin_nontemporal_load(x);
#else
  r.d[16] = *x;
#endif
}

// v_perm selector turning {d[j+1]:d[j]} into the big-endian word at byte shift `sh`.
__device__ __forceinline__ uint32_t be_selector(uint32_t sh) {
  return ((sh) << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
}

// v_perm selector turning {d[j+1]:d[j]} into the little-endian word at byte shift `sh`.
__device__ __forceinline__ uint32_t le_selector(uint32_t sh) {
  return ((sh + 3) << 24) | ((sh + 2) << 16) | ((sh + 1) << 8) | sh;
}

__device__ __forceinline__ void decode_full(const RawBlock& r, uint32_t sel, uint32_t w[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(r.d[j + 1], r.d[j], sel);
}

// Tail block `blk` >= floor(len/64) of a part whose block-`blk` bytes start at `p`:
// the last data bytes, 0x80, zeros, and the big-endian bit length in the final block
// (lib/hash/utility.cpp:42-56 alloc_padded, synthesized in registers -- never in HBM).
// `bits` is the WHOLE message's bit length: 8*len for a one-shot part, larger for the final
// segment of a streamed message (len == total mod 64 then, so the block count agrees).
__device__ __forceinline__ void build_tail(const uint8_t* p, uint64_t len, uint64_t bits,
                                           uint64_t blk, uint32_t w[16]) {
  const uint64_t nfull = len >> 6;
  const int rem = (blk == nfull) ? int(len & 63) : -1;  // data bytes in this block
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = 4 * j + k;
      uint32_t byte = 0;
      if (i < rem) byte = p[i];
      else if (i == rem) byte = 0x80u;
      x |= byte << (24 - 8 * k);
    }
    w[j] = x;
  }
  if (blk == nblocks(len) - 1) {
    w[14] = uint32_t(bits >> 32);
    w[15] = uint32_t(bits);
  }
}

}  // namespace s3h
