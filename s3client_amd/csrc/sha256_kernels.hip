// sha256_kernels.hip -- batched many-message SHA-256 kernels for MI355X (gfx950).
//
// Why one part per LANE (not per workgroup): SHA-256 of one part is a strictly sequential
// Merkle-Damgard chain (lib/hash/sha256.cpp:88-143: block i needs the state of block i-1),
// so the only parallelism is across parts.  A wave64 VALU instruction costs the SIMD the
// same issue slot whether 1 or 64 lanes are active, so each lane carries its own part and
// the workgroup is the staging / scheduling unit.
//
// Two kernels:
//   sha256_pc_kernel   (producer/consumer) -- a 128-thread workgroup = 64 parts.  Wave 1
//       (producer) streams each lane's 64-byte blocks from HBM, decodes them (alignment +
//       big-endian in one v_perm per word), synthesises the padding, expands the message
//       schedule and writes W[t]+K[t] into an LDS double buffer.  Wave 0 (consumer) runs
//       only the 64-round chain (~14 VALU per round), reading W+K with ds_read_b128.  A
//       chain issues ~920 instead of ~1400 instructions per block, so each part hashes
//       ~1.5x faster.  This is the right kernel while parts are scarcer than SIMD lanes
//       (every BASELINE config: 1024-8192 parts per GPU vs 1024 SIMDs x 64 lanes).
//   sha256_lane_kernel (fused) -- one lane does schedule + rounds; no LDS, 8 waves/SIMD.
//       Used when parts are plentiful enough to saturate every SIMD (>= ~128K parts).
//
// Both kernels are resumable: a launch processes blocks [blk_begin, blk_end) of every part,
// loading/saving the 8-word chaining state in `state` (slot order) between launches.  The
// device-resident path is one launch over [0, max); the host path streams slices.
#include "sha256_device.hpp"

namespace s3h {

struct LaunchArgs {
  const uint8_t* base;       // part p's block b is at base + slots[p].off + 64*(b - blk_origin)
  const Slot* slots;         // sorted by nblocks descending
  const uint32_t* out_idx;   // slot -> output part index
  uint32_t* state;           // n*8 words (slot order); may be null for single-launch plans
  uint32_t* digests;         // n*8 words (part order), bswap32(H_i) like lib/hash to_little
  uint64_t blk_begin, blk_end, blk_origin;
  uint32_t n;
};

__device__ __forceinline__ void load_state(const LaunchArgs& A, uint32_t slot, uint32_t st[8]) {
  if (A.blk_begin == 0 || A.state == nullptr) {
    init_state(st);
  } else {
    const uint4* s = reinterpret_cast<const uint4*>(A.state + 8ull * slot);
    const uint4 x = s[0], y = s[1];
    st[0] = x.x; st[1] = x.y; st[2] = x.z; st[3] = x.w;
    st[4] = y.x; st[5] = y.y; st[6] = y.z; st[7] = y.w;
  }
}

__device__ __forceinline__ void store_result(const LaunchArgs& A, uint32_t slot, uint64_t nb,
                                             const uint32_t st[8]) {
  if (nb <= A.blk_end) {  // chain finished inside this launch: emit the digest
    uint4* o = reinterpret_cast<uint4*>(A.digests + 8ull * A.out_idx[slot]);
    o[0] = make_uint4(bswap(st[0]), bswap(st[1]), bswap(st[2]), bswap(st[3]));
    o[1] = make_uint4(bswap(st[4]), bswap(st[5]), bswap(st[6]), bswap(st[7]));
  } else if (A.state) {
    uint4* s = reinterpret_cast<uint4*>(A.state + 8ull * slot);
    s[0] = make_uint4(st[0], st[1], st[2], st[3]);
    s[1] = make_uint4(st[4], st[5], st[6], st[7]);
  }
}

// Decode block `blk` of the part whose bytes for that block start at `p`.
__device__ __forceinline__ void make_block(const RawBlock& r, uint32_t sel, const uint8_t* p,
                                           uint64_t len, uint64_t blk, uint32_t w[16]) {
  if (blk < (len >> 6)) decode_full(r, sel, w);
  else build_tail(p, len, blk, w);
}

// ------------------------------------------------------------------ fused lane kernel
__global__ __launch_bounds__(256) void sha256_lane_kernel(LaunchArgs A) {
  const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
  if (slot >= A.n) return;
  const Slot s = A.slots[slot];
  const uint64_t nb = nblocks(s.len);
  if (nb <= A.blk_begin) return;  // finished in an earlier launch
  const uint64_t end = nb < A.blk_end ? nb : A.blk_end;
  uint32_t st[8];
  load_state(A, slot, st);
  const uint8_t* p = A.base + s.off + 64ull * (A.blk_begin - A.blk_origin);
  const uint32_t sel = be_selector(uint32_t(reinterpret_cast<uintptr_t>(p) & 3));
  const uint64_t nfull = s.len >> 6;
  RawBlock cur;
  if (A.blk_begin < nfull) fetch_full(p, cur);
  for (uint64_t b = A.blk_begin; b < end; ++b) {
    RawBlock nxt;
    if (b + 1 < nfull) fetch_full(p + 64, nxt);  // prefetch one block ahead
    uint32_t w[16], wk[64];
    make_block(cur, sel, p, s.len, b, w);
    schedule_wk(w, wk);
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = st[i];
    rounds_wk(t, wk);
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] += t[i];
    cur = nxt;
    p += 64;
  }
  store_result(A, slot, nb, st);
}

// ------------------------------------------------------------- producer/consumer kernel
// Decode + pad + schedule one block and store W[t]+K[t] as 16 x 16 B rows of LDS.
__device__ __forceinline__ void produce_block(const RawBlock& r, uint32_t sel, const uint8_t* bp,
                                              uint64_t len, uint64_t blk, uint4 (*buf)[64],
                                              uint32_t lane) {
  uint32_t w[16], wk[64];
  make_block(r, sel, bp, len, blk, w);
  schedule_wk(w, wk);
#pragma unroll
  for (int q = 0; q < 16; ++q)
    buf[q][lane] = make_uint4(wk[4 * q], wk[4 * q + 1], wk[4 * q + 2], wk[4 * q + 3]);
}

constexpr int kPcThreads = 128;  // wave 0 consumer, wave 1 producer; 64 parts per workgroup

__global__ __launch_bounds__(kPcThreads) void sha256_pc_kernel(LaunchArgs A) {
  __shared__ uint4 lds_wk[2][16][64];  // [buffer][group of 4 rounds][lane]: 32 KiB

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot0 = blockIdx.x * 64u;
  const uint32_t slot = slot0 + lane;
  const bool valid = slot < A.n;
  Slot s = {0, 0};
  if (valid) s = A.slots[slot];
  const uint64_t nb = valid ? nblocks(s.len) : 0;
  // Slots are sorted by block count, so the workgroup's first slot bounds the loop; the
  // trip count is identical in both waves, so their s_barrier counts match.
  const uint64_t wg_nb = nblocks(A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  if (wg_end <= A.blk_begin) return;  // whole workgroup done in earlier launches
  const uint64_t iters = wg_end - A.blk_begin;

  if (wave == 1) {
    // ---------------------------------------------------------------- producer
    // Block (b0 + k) is produced into LDS buffer k&1 ahead of barrier k; its raw dwords were
    // fetched one block earlier, so each HBM load has a whole consumer block (~3.7k cycles)
    // to land.  Two named register blocks ping-pong (no struct copies -> no scratch).
    const uint64_t b0 = A.blk_begin;
    const uint8_t* p = A.base + s.off + 64ull * (b0 - A.blk_origin);
    const uint32_t sel = be_selector(uint32_t(reinterpret_cast<uintptr_t>(p) & 3));
    const uint64_t nfull = s.len >> 6;
    RawBlock ra, rb;
    if (b0 < nfull) fetch_full(p, ra);
    if (b0 + 1 < nfull) fetch_full(p + 64, rb);
    produce_block(ra, sel, p, s.len, b0, lds_wk[0], lane);
    __syncthreads();
    for (uint64_t k = 1; k <= iters; k += 2) {
      // odd step: block b0+k from rb into buffer 1; refill ra with block b0+k+1
      if (k < iters) {
        if (b0 + k + 1 < nfull) fetch_full(p + 64 * (k + 1), ra);
        produce_block(rb, sel, p + 64 * k, s.len, b0 + k, lds_wk[1], lane);
      }
      __syncthreads();
      if (k + 1 > iters) break;
      // even step: block b0+k+1 from ra into buffer 0; refill rb with block b0+k+2
      if (k + 1 < iters) {
        if (b0 + k + 2 < nfull) fetch_full(p + 64 * (k + 2), rb);
        produce_block(ra, sel, p + 64 * (k + 1), s.len, b0 + k + 1, lds_wk[0], lane);
      }
      __syncthreads();
    }
  } else {
    // ---------------------------------------------------------------- consumer
    __builtin_amdgcn_s_setprio(3);
    uint32_t st[8];
    if (valid) load_state(A, slot, st);
    else init_state(st);
    __syncthreads();
    for (uint64_t i = 0; i < iters; ++i) {
      const int buf = int(i & 1);
      uint32_t wk[64];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint4 v = lds_wk[buf][q][lane];
        wk[4 * q] = v.x; wk[4 * q + 1] = v.y; wk[4 * q + 2] = v.z; wk[4 * q + 3] = v.w;
      }
      uint32_t t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = st[k];
      rounds_wk(t, wk);
      const bool live = (A.blk_begin + i) < nb;
#pragma unroll
      for (int k = 0; k < 8; ++k) st[k] = live ? st[k] + t[k] : st[k];
      __syncthreads();
    }
    if (valid && nb > A.blk_begin) store_result(A, slot, nb, st);
  }
}

// ------------------------------------------------------------- synthetic input generator
// G(seed, p, L) of SURVEY.md 8(d): word j of part p is splitmix64(x0 + (j+1)*golden),
// x0 = seed ^ p*0xD1B54A32D192ED03, serialised little-endian.  Parts must start 8-B aligned.
struct GenPart { uint64_t off, len, id; };

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void generate_kernel(uint8_t* base, const GenPart* parts,
                                                       uint64_t seed) {
  const GenPart g = parts[blockIdx.y];
  const uint64_t x0 = seed ^ (g.id * 0xD1B54A32D192ED03ull);
  const uint64_t nw = (g.len + 7) >> 3;
  uint8_t* dst = base + g.off;
  for (uint64_t j = uint64_t(blockIdx.x) * 256u + threadIdx.x; j < nw;
       j += uint64_t(gridDim.x) * 256u) {
    const uint64_t v = mix64(x0 + (j + 1) * 0x9E3779B97F4A7C15ull);
    if (8 * j + 8 <= g.len) {
      reinterpret_cast<uint64_t*>(dst)[j] = v;
    } else {
      for (uint64_t k = 8 * j; k < g.len; ++k) dst[k] = uint8_t(v >> (8 * (k - 8 * j)));
    }
  }
}

}  // namespace s3h
