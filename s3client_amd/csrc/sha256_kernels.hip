// sha256_kernels.hip -- batched many-message SHA-256 (and MD5) kernels for MI355X (gfx950).
//
// Why one part per chain of lanes, never per workgroup: SHA-256 of one part is a strictly
// sequential Merkle-Damgard chain (lib/hash/sha256.cpp:88-143: block i needs the state of
// block i-1), so the only parallelism is across parts, and BASELINE's batches (C2: 1,024
// parts, C4: 8,192 per GPU) fill at most 1.6-12.5 % of the chip's 65,536 lanes.  What sets
// the time is how fast ONE chain runs: a wave issues at most one instruction per ~4 cycles
// whatever its type (4.05 measured on an aligned lone-wave stream,
// profiles/r01_ubench_alignment.txt), so every design choice below removes instructions from
// the chain's wave.
//
// Kernels and what AUTO (capi.hip resolve_kernel) picks, by part count n on 256 CUs:
//   sha256_skew_kernel<1>       n <= 2,048   the C2 metric kernel: each chain on 8 lanes (an
//       e-quad and an a-quad), the a-quad two rounds behind -> 8 VALU per round; one consumer
//       wave (8 chains) + one producer wave per workgroup.  543.9 instructions per block in
//       the shipped code object (kernel_isa_counts.json); measured 2,205 cycles per block =
//       4.06 cycles per instruction = 98.6 % of the issue floor.
//   sha256_skew_pairs_kernel    n <= 4,096   two flag-synchronised skew groups per
//       workgroup; the longest parts' groups run solo (capi.hip plan_solo).
//   sha256_skew_shared_kernel   n <= 32 x CUs (8,192)  "skews": four skew groups per
//       workgroup, each producer on its consumer's SIMD in simple-class instructions
//       (sha256_producer_simple.inc) -- the C4 shard kernel.
//   sha256_skew_kernel<1, PAIR> n <= 28,672  "skewp": the skewed schedule on lane pairs,
//       9 VALU per round, 32 chains per consumer wave.
//   sha256_pair_kernel          n <= 32,768  each chain on a lane pair.
//   sha256_pc_kernel            n <= 65,536  one lane per chain, producer/consumer.
//   sha256_lane_kernel          above        fused: one lane loads, schedules and compresses.
//   sha256_quad_kernel<NC>      explicit, and skew ranges of >= 2^31 blocks (64-bit counters).
//   md5_pc_kernel<4 | 1>        MD5 (Content-MD5 / ETag): 4-block producer steps
//       while the grid fits one workgroup per CU, 1-block steps (32 KiB LDS) beyond.
//   sha256_md5_*_kernel         both digests of every part from one grid (capi.hip dual).
// In the producer/consumer kernels the producer wave streams each part's 64-byte blocks from
// HBM (cached loads), aligns and byte-swaps them (one v_perm per word), synthesises the
// padding, expands the message schedule and writes W[t]+K[t] into an LDS double buffer; the
// consumer wave runs only the 64-round chain.
//
// All kernels are resumable: a launch processes blocks [blk_begin, blk_end) of every part,
// loading/saving the 8-word chaining state in `state` (message order) between launches.  The
// device-resident path is one launch over [0, max); the host path streams slices; the
// multi-object stream (s3h_stream_*) runs unpadded launches over appended whole blocks
// (kNoPad | kResume) and a final padded launch with each message's total bit length.
#include "sha256_device.hpp"

// Experiment switches and their product values: exp_config.hpp (included by sha256_device.hpp).
#if S3H_EXP_PRODUCER_ROLLED
#define S3H_PROD_UNROLL _Pragma("unroll 1")
#else
#define S3H_PROD_UNROLL _Pragma("unroll")
#endif

namespace s3h {

// LaunchArgs, its flags and the error-word bits: kernel_abi.hpp (shared with the host).

// Compressions the launch sequence runs for a slot of `len` bytes.
__device__ __forceinline__ uint64_t slot_blocks(const LaunchArgs& A, uint64_t len) {
  return (A.flags & kNoPad) ? (len >> 6) : nblocks(len);
}
__device__ __forceinline__ bool resumes(const LaunchArgs& A) {
  return A.state != nullptr && (A.blk_begin > 0 || (A.flags & kResume));
}
// The chain of a slot with `nb` blocks ends inside this launch and its digest is written.
__device__ __forceinline__ bool emits(const LaunchArgs& A, uint64_t nb) {
  return !(A.flags & kNoPad) && nb <= A.blk_end;
}
__device__ __forceinline__ uint64_t msg_bits(const LaunchArgs& A, uint32_t slot, uint64_t len) {
  return A.bits ? A.bits[A.out_idx[slot]] : len << 3;
}

__device__ __forceinline__ void load_state(const LaunchArgs& A, uint32_t slot, uint32_t st[8]) {
  if (!resumes(A)) {
    init_state(st);
  } else {
    const uint4* s = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot]);
    const uint4 x = s[0], y = s[1];
    st[0] = x.x; st[1] = x.y; st[2] = x.z; st[3] = x.w;
    st[4] = y.x; st[5] = y.y; st[6] = y.z; st[7] = y.w;
  }
}

__device__ __forceinline__ void store_result(const LaunchArgs& A, uint32_t slot, uint64_t nb,
                                             const uint32_t st[8]) {
  if (emits(A, nb)) {  // chain finished inside this launch: emit the digest
    uint4* o = reinterpret_cast<uint4*>(A.digests + 8ull * A.out_idx[slot]);
    o[0] = make_uint4(bswap(st[0]), bswap(st[1]), bswap(st[2]), bswap(st[3]));
    o[1] = make_uint4(bswap(st[4]), bswap(st[5]), bswap(st[6]), bswap(st[7]));
  } else if (A.state) {
    uint4* s = reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot]);
    s[0] = make_uint4(st[0], st[1], st[2], st[3]);
    s[1] = make_uint4(st[4], st[5], st[6], st[7]);
  }
}

// First block index that may NOT be loaded with fetch_full: the part's first partial block
// or the end of the launch's range, whichever comes first.
__device__ __forceinline__ uint64_t fetch_end(uint64_t len, uint64_t blk_end) {
  const uint64_t nfull = len >> 6;
  return nfull < blk_end ? nfull : blk_end;
}

// Decode block `blk` of the part whose bytes for that block start at `p`.
// Blocks at or past `limit` (the launch's blk_end) are never consumed; they are zero-filled
// without touching memory (the pair producer's odd lanes can step one block past the range).
__device__ __forceinline__ void make_block(const RawBlock& r, uint32_t sel, const uint8_t* p,
                                           uint64_t len, uint64_t bits, uint64_t blk,
                                           uint64_t limit, uint32_t w[16]) {
  if (blk >= limit) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = 0;
  } else if (blk < (len >> 6)) {
    decode_full(r, sel, w);
  } else {
    build_tail(p, len, bits, blk, w);
  }
}

// ------------------------------------------------------------------ fused lane kernel
__global__ __launch_bounds__(256) void sha256_lane_kernel(LaunchArgs A) {
  const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
  if (slot >= A.n) return;
  const Slot s = A.slots[slot];
  const uint64_t nb = slot_blocks(A, s.len);
  if (nb <= A.blk_begin) return;  // finished in an earlier launch
  const uint64_t bits = msg_bits(A, slot, s.len);
  const uint64_t end = nb < A.blk_end ? nb : A.blk_end;
  uint32_t st[8];
  load_state(A, slot, st);
  const uint8_t* p = A.base + s.off + 64ull * (A.blk_begin - A.blk_origin);
  const uint32_t sel = be_selector(uint32_t(reinterpret_cast<uintptr_t>(p) & 3));
  // Only whole blocks inside both the part and this launch's range are ever loaded: a ranged
  // launch's base may hold nothing beyond blk_end (host streaming ring).
  const uint64_t fend = fetch_end(s.len, A.blk_end);
  RawBlock cur;
  fetch_full(p, A.blk_begin < fend, A.zero, cur);
  for (uint64_t b = A.blk_begin; b < end; ++b) {
    RawBlock nxt;
    fetch_full(p + 64, b + 1 < fend, A.zero, nxt);  // prefetch one block ahead
    uint32_t w[16], wk[64];
    make_block(cur, sel, p, s.len, bits, b, A.blk_end, w);
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
template <int kRow>
__device__ __forceinline__ void produce_block(const RawBlock& r, uint32_t sel, const uint8_t* bp,
                                              uint64_t len, uint64_t bits, uint64_t blk,
                                              uint64_t limit, uint4 (*buf)[kRow], uint32_t lane) {
  uint32_t w[16], wk[64];
  make_block(r, sel, bp, len, bits, blk, limit, w);
  schedule_wk(w, wk);
#pragma unroll
  for (int q = 0; q < 16; ++q)
    buf[q][lane] = make_uint4(wk[4 * q], wk[4 * q + 1], wk[4 * q + 2], wk[4 * q + 3]);
}

__global__ __launch_bounds__(kPcThreads) void sha256_pc_kernel(LaunchArgs A) {
  __shared__ uint4 lds_wk[2][16][64];  // [buffer][group of 4 rounds][lane]: 32 KiB

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot0 = blockIdx.x * 64u;
  const uint32_t slot = slot0 + lane;
  const bool valid = slot < A.n;
  Slot s = {0, 0};
  if (valid) s = A.slots[slot];
  const uint64_t nb = valid ? slot_blocks(A, s.len) : 0;
  // Slots are sorted by block count, so the workgroup's first slot bounds the loop; the
  // trip count is identical in both waves, so their s_barrier counts match.
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
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
    const uint64_t fend = fetch_end(s.len, A.blk_end);
    const uint64_t bits = valid ? msg_bits(A, slot, s.len) : 0;
    const uint64_t dl = decode_len(valid, s.len);
    RawBlock ra, rb;
    fetch_full(p, b0 < fend, A.zero, ra);
    fetch_full(p + 64, b0 + 1 < fend, A.zero, rb);
    produce_block(ra, sel, p, dl, bits, b0, A.blk_end, lds_wk[0], lane);
    __syncthreads();
    for (uint64_t k = 1; k <= iters; k += 2) {
      // odd step: block b0+k from rb into buffer 1; refill ra with block b0+k+1
      if (k < iters) {
        fetch_full(p + 64 * (k + 1), b0 + k + 1 < fend, A.zero, ra);
        produce_block(rb, sel, p + 64 * k, dl, bits, b0 + k, A.blk_end, lds_wk[1], lane);
      }
      __syncthreads();
      if (k + 1 > iters) break;
      // even step: block b0+k+1 from ra into buffer 0; refill rb with block b0+k+2
      if (k + 1 < iters) {
        fetch_full(p + 64 * (k + 2), b0 + k + 2 < fend, A.zero, rb);
        produce_block(ra, sel, p + 64 * (k + 1), dl, bits, b0 + k + 1, A.blk_end, lds_wk[0], lane);
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

// ------------------------------------------------------------- lane-pair kernel
// Each part's 64-round chain is split over a PAIR of lanes: the "e-half" (lanes in DPP banks
// 0 and 2 of every 16-lane row) holds e,f,g,h and computes T1 = h + W+K + Sigma1(e) + Ch;
// the "a-half" (banks 1 and 3, partner = lane + 4) holds a,b,c,d and computes
// T2 = Sigma0(a) + Maj(a,b,c) with the SAME instruction stream (per-lane rotate amounts,
// Ch and Maj unified as one bfi over a per-lane selector).  Two bank-masked DPP adds finish
// the round: e' = d(partner) + T1 on the e-half, a' = T1(partner) + T2 on the a-half.
// A round is 10 VALU instead of 14, and since a lone wave issues ~1 VALU per 5 cycles
// whatever the op (profiles/r01_ubench_valu_issue.txt), each chain runs ~1.35x faster.
// Workgroup = 128 threads: wave 0 consumes 32 parts (64 lanes), wave 1 produces W+K for
// those 32 parts, two blocks per step (lanes 0-31 even blocks, 32-63 odd blocks).

__device__ __forceinline__ uint32_t pair_chain(uint32_t lane) {
  return (lane >> 4) * 8u + ((lane >> 3) & 1u) * 4u + (lane & 3u);
}
__device__ __forceinline__ bool pair_is_ahalf(uint32_t lane) { return (lane >> 2) & 1u; }

// One round on the pair, as asm text over named operands: the new value lands in d (in
// place), x is this round's h+W+K on the e-half (0 on the a-half) and xn receives the next
// round's (c + wn) on the e-half.  Hazards: the a-half DPP reads q3 two instructions after it
// is written (the two wait states a DPP read of a fresh VALU result needs); every other DPP
// source was written >= 2 rounds earlier.
#define S3H_PAIR_TXT(a, b, c, d, x, xn, wn)                                                   \
  "v_alignbit_b32 %[q1], %[" #a "], %[" #a "], %[h1]\n\t"                                     \
  "v_alignbit_b32 %[q2], %[" #a "], %[" #a "], %[h2]\n\t"                                     \
  "v_alignbit_b32 %[q3], %[" #a "], %[" #a "], %[h3]\n\t"                                     \
  "v_bitop3_b32 %[q4], %[" #a "], %[" #b "], %[m] bitop3:0xd2\n\t"                            \
  "v_bitop3_b32 %[q1], %[q1], %[q2], %[q3] bitop3:0x96\n\t"                                   \
  "v_bfi_b32 %[q2], %[q4], %[" #b "], %[" #c "]\n\t"                                          \
  "v_add3_u32 %[q3], %[" #x "], %[q1], %[q2]\n\t"                                             \
  "v_add_u32_dpp %[" #xn "], %[" #c "], %[" #wn "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t" \
  "v_add_u32_dpp %[" #d "], %[" #d "], %[q3] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"       \
  "v_add_u32_dpp %[" #d "], %[q3], %[q3] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

// Every round instruction is 8 bytes (VOP3 / DPP).  An 8-byte instruction at an address
// = 4 (mod 8) issues at ~5.05 instead of ~4.05 cycles (tools/ubench_cu_waves.hip,
// profiles/r01_ubench_alignment.txt), so each round statement starts 8-byte aligned: the
// assembler pads with one 4-byte s_nop when the preceding code leaves it misaligned.
#define S3H_ALIGN8 ".p2align 3\n\t"

// Sixteen rounds (four rotations of the state names) per asm statement (30 operands, the
// inline-asm maximum): the compiler pads with an s_nop between consecutive asm statements,
// so fewer, longer statements keep the stream at one VALU per issue slot.
#define S3H_PAIR_4TXT(wa, wb, wc, wd)                                                         \
  S3H_PAIR_TXT(s0, s1, s2, s3, xa, xb, wa) S3H_PAIR_TXT(s3, s0, s1, s2, xb, xa, wb)              \
  S3H_PAIR_TXT(s2, s3, s0, s1, xa, xb, wc) S3H_PAIR_TXT(s1, s2, s3, s0, xb, xa, wd)
#define S3H_PAIR_16RND(WK, T)                                                                   \
  asm volatile(S3H_ALIGN8 S3H_PAIR_4TXT(w1, w2, w3, w4) S3H_PAIR_4TXT(w5, w6, w7, w8)                       \
               S3H_PAIR_4TXT(w9, w10, w11, w12) S3H_PAIR_4TXT(w13, w14, w15, w16)               \
               : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),    \
                 [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)  \
               : [w1] "v"(WK[(T + 1) & 63]), [w2] "v"(WK[(T + 2) & 63]),                       \
                 [w3] "v"(WK[(T + 3) & 63]), [w4] "v"(WK[(T + 4) & 63]),                       \
                 [w5] "v"(WK[(T + 5) & 63]), [w6] "v"(WK[(T + 6) & 63]),                       \
                 [w7] "v"(WK[(T + 7) & 63]), [w8] "v"(WK[(T + 8) & 63]),                       \
                 [w9] "v"(WK[(T + 9) & 63]), [w10] "v"(WK[(T + 10) & 63]),                     \
                 [w11] "v"(WK[(T + 11) & 63]), [w12] "v"(WK[(T + 12) & 63]),                   \
                 [w13] "v"(WK[(T + 13) & 63]), [w14] "v"(WK[(T + 14) & 63]),                   \
                 [w15] "v"(WK[(T + 15) & 63]), [w16] "v"(WK[(T + 16) & 63]), [h1] "v"(sh1),    \
                 [h2] "v"(sh2), [h3] "v"(sh3), [m] "v"(msk))

__global__ __launch_bounds__(kPairThreads) void sha256_pair_kernel(LaunchArgs A) {
  __shared__ uint4 lds_wk[2][2][16][kPairParts];  // [buffer][block in step][round group][part]

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot0 = blockIdx.x * kPairParts;
  const uint64_t b0 = A.blk_begin;
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  if (wg_end <= b0) return;
  const uint64_t iters = wg_end - b0;          // blocks this launch, uniform in the workgroup
  const uint64_t steps = (iters + 1) >> 1;     // two blocks per producer step

  if (wave == 1) {
    // ---------------------------------------------------------------- producer
    const uint32_t part = lane & 31u, half = lane >> 5;
    const uint32_t slot = slot0 + part;
    Slot s = {0, 0};
    if (slot < A.n) s = A.slots[slot];
    const uint8_t* p = A.base + s.off + 64ull * (b0 + half - A.blk_origin);
    const uint32_t sel = be_selector(uint32_t(reinterpret_cast<uintptr_t>(A.base + s.off) & 3));
    const uint64_t fend = fetch_end(s.len, A.blk_end);
    const uint64_t bh = b0 + half;  // this lane's first block
    const uint64_t bits = slot < A.n ? msg_bits(A, slot, s.len) : 0;
    const uint64_t dl = decode_len(slot < A.n, s.len);
    RawBlock ra, rb;
    fetch_full(p, bh < fend, A.zero, ra);
    fetch_full(p + 128, bh + 2 < fend, A.zero, rb);
    produce_block(ra, sel, p, dl, bits, bh, A.blk_end, lds_wk[0][half], part);
    __syncthreads();
    for (uint64_t k = 1; k <= steps; k += 2) {
      if (k < steps) {
        fetch_full(p + 128 * (k + 1), bh + 2 * (k + 1) < fend, A.zero, ra);
        produce_block(rb, sel, p + 128 * k, dl, bits, bh + 2 * k, A.blk_end, lds_wk[1][half], part);
      }
      __syncthreads();
      if (k + 1 > steps) break;
      if (k + 1 < steps) {
        fetch_full(p + 128 * (k + 2), bh + 2 * (k + 2) < fend, A.zero, rb);
        produce_block(ra, sel, p + 128 * (k + 1), dl, bits, bh + 2 * (k + 1), A.blk_end, lds_wk[0][half], part);
      }
      __syncthreads();
    }
  } else {
    // ---------------------------------------------------------------- consumer
    __builtin_amdgcn_s_setprio(3);  // wins VALU arbitration if a producer shares the SIMD
    const uint32_t part = pair_chain(lane);
    const bool ahalf = pair_is_ahalf(lane);
    const uint32_t slot = slot0 + part;
    const bool valid = slot < A.n;
    const uint64_t nb = valid ? slot_blocks(A, A.slots[slot].len) : 0;
    const uint32_t sh1 = ahalf ? 2u : 6u, sh2 = ahalf ? 13u : 11u, sh3 = ahalf ? 22u : 25u;
    const uint32_t msk = ahalf ? 0xffffffffu : 0u;
    const uint32_t w0 = ahalf ? 0u : 4u;  // which half of the chaining state this lane holds
    uint32_t s0, s1, s2, s3;
    if (valid && resumes(A)) {
      const uint4 v = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot] + w0)[0];
      s0 = v.x; s1 = v.y; s2 = v.z; s3 = v.w;
    } else {
      s0 = ahalf ? 0x6a09e667u : 0x510e527fu;
      s1 = ahalf ? 0xbb67ae85u : 0x9b05688cu;
      s2 = ahalf ? 0x3c6ef372u : 0x1f83d9abu;
      s3 = ahalf ? 0xa54ff53au : 0x5be0cd19u;
    }
    uint32_t xa = 0, xb = 0;  // a-half lanes are never written: their X stays 0
    uint32_t q1, q2, q3, q4;
    // Slots are sorted by length: every lane is live for blocks below the last slot's count.
    const uint32_t last = (slot0 + kPairParts <= A.n ? slot0 + kPairParts : A.n) - 1;
    const uint64_t all_live_end = slot_blocks(A, A.slots[last].len);
    auto block = [&](const uint32_t wk[64], uint64_t i) {
      const uint32_t t0 = s0, t1 = s1, t2 = s2, t3 = s3;
      asm volatile(
          "s_nop 1\n\t" S3H_ALIGN8
          "v_add_u32_dpp %0, %1, %2 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5"
          : "+v"(xa) : "v"(s3), "v"(wk[0]));
      S3H_PAIR_16RND(wk, 0);
      S3H_PAIR_16RND(wk, 16);
      S3H_PAIR_16RND(wk, 32);
      S3H_PAIR_16RND(wk, 48);
      if (b0 + i < all_live_end) {  // uniform branch: no per-lane select
        s0 += t0; s1 += t1; s2 += t2; s3 += t3;
      } else {
        const bool live = (b0 + i) < nb;
        s0 = live ? s0 + t0 : t0;
        s1 = live ? s1 + t1 : t1;
        s2 = live ? s2 + t2 : t2;
        s3 = live ? s3 + t3 : t3;
      }
    };
    __syncthreads();
    for (uint64_t j = 0; j < steps; ++j) {
      // Both blocks' W+K rows are read up front and waited for ONCE (one exposed LDS latency
      // per step instead of a counted wait before every 4-round group).
      const bool second = 2 * j + 1 < iters;
      uint32_t wk0[64], wk1[64];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint4 v = lds_wk[j & 1][0][q][part];
        wk0[4 * q] = v.x; wk0[4 * q + 1] = v.y; wk0[4 * q + 2] = v.z; wk0[4 * q + 3] = v.w;
        const uint4 u = lds_wk[j & 1][1][q][part];
        wk1[4 * q] = u.x; wk1[4 * q + 1] = u.y; wk1[4 * q + 2] = u.z; wk1[4 * q + 3] = u.w;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      block(wk0, 2 * j);
      if (second) block(wk1, 2 * j + 1);
      __syncthreads();
    }
    if (valid && nb > b0) {
      if (emits(A, nb)) {
        uint4* o = reinterpret_cast<uint4*>(A.digests + 8ull * A.out_idx[slot] + w0);
        o[0] = make_uint4(bswap(s0), bswap(s1), bswap(s2), bswap(s3));
      } else if (A.state) {
        reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot] + w0)[0] = make_uint4(s0, s1, s2, s3);
      }
    }
  }
}

// ------------------------------------------------------------- lane-quad kernel
// Each half of a chain's state lives on a QUAD of lanes (one DPP bank): the e-quad (banks 0
// and 2) holds e,f,g,h in all four lanes, the a-quad (banks 1 and 3, partner = lane + 4) holds
// a,b,c,d.  Sigma needs one rotation per lane instead of three: lane k of a quad rotates by
// its own amount (e: 6, 11, 25, 6; a: 2, 13, 22, 2) and two quad_perm v_xor_b32_dpp fold the
// three rotations into every lane of the quad.  The rest of the round is the pair kernel's:
// Ch and Maj as one bfi over a per-lane selector, the e-half's h+W+K precomputed, two
// bank-masked adds exchanging T1 and d between the quads.  9 VALU per round instead of 10,
// at 8 chains per wave.  A workgroup is NC consumer waves (8 chains each) and one producer
// wave that feeds all of them (2 blocks x 8*NC chains per step), so the producer's issue cost
// per chain matches the pair kernel's once NC = 4.
// Hazards: the first xor_dpp reads the rotation 3 instructions after it is written (2 wait
// states needed); the a-quad's exchange reads T1 two instructions after the add3.

// One quad round.  W+K reaches the e-quad by DPP broadcast: lane L of every quad holds W+K
// rows L, L+4, L+8, L+12 (4 ds_read_b128 per block instead of 16), and the h+W+K precompute
// reads word `wreg` of lane L with quad_perm:[L,L,L,L] (an LDS-loaded source: no DPP hazard).
// `din`/`dout`: the d slot read / written (different only in the first four rounds of a block,
// which read the block-start state s0..s3 and write fresh n0..n3, so the state survives for
// the feed-forward without copies).
#define S3H_QR(a, b, c, din, dout, x, xn, wreg, L)                                            \
  "v_alignbit_b32 %[q1], %[" #a "], %[" #a "], %[h1]\n\t"                                     \
  "v_bitop3_b32 %[q4], %[" #a "], %[" #b "], %[m] bitop3:0xd2\n\t"                            \
  "v_bfi_b32 %[q2], %[q4], %[" #b "], %[" #c "]\n\t"                                          \
  "v_xor_b32_dpp %[q3], %[q1], %[q1] quad_perm:[1,2,0,1] row_mask:0xf bank_mask:0xf\n\t"     \
  "v_xor_b32_dpp %[q3], %[q1], %[q3] quad_perm:[2,0,1,2] row_mask:0xf bank_mask:0xf\n\t"     \
  "v_add3_u32 %[q3], %[" #x "], %[q3], %[q2]\n\t"                                             \
  "v_add_u32_dpp %[" #xn "], %[" #wreg "], %[" #c "] quad_perm:[" #L "," #L "," #L "," #L     \
  "] row_mask:0xf bank_mask:0x5\n\t"                                                          \
  "v_add_u32_dpp %[" #dout "], %[" #din "], %[q3] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"  \
  "v_add_u32_dpp %[" #dout "], %[q3], %[q3] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

// Four in-place rounds on n0..n3; rounds use words 1,2,3 of lane L, then word 0 of lane LN
// from register set WS (the next group's first word).
#define S3H_QG(S, L, WN, LN)                                                                   \
  S3H_QR(n0, n1, n2, n3, n3, xa, xb, S##1, L) S3H_QR(n3, n0, n1, n2, n2, xb, xa, S##2, L)        \
  S3H_QR(n2, n3, n0, n1, n1, xa, xb, S##3, L) S3H_QR(n1, n2, n3, n0, n0, xb, xa, WN, LN)
// The block's first four rounds: read s0..s3, write n3, n2, n1, n0.
#define S3H_QG_FIRST                                                                           \
  S3H_QR(s0, s1, s2, s3, n3, xa, xb, a1, 0) S3H_QR(n3, s0, s1, s2, n2, xb, xa, a2, 0)            \
  S3H_QR(n2, n3, s0, s1, n1, xa, xb, a3, 0) S3H_QR(n1, n2, n3, s0, n0, xb, xa, a0, 1)
// 16 rounds of register set S (rounds 16m..16m+15 use set m on lanes 0..3), ending with the
// next set's word 0 (NX).
#define S3H_Q16(S, NX) S3H_QG(S, 0, S##0, 1) S3H_QG(S, 1, S##0, 2) S3H_QG(S, 2, S##0, 3) S3H_QG(S, 3, NX, 0)
#define S3H_Q16_FIRST S3H_QG_FIRST S3H_QG(a, 1, a0, 2) S3H_QG(a, 2, a0, 3) S3H_QG(a, 3, b0, 0)

template <int NC>
__global__ __launch_bounds__(64 * (NC + 1)) void sha256_quad_kernel(LaunchArgs A) {
  constexpr uint32_t kParts = kQuadChainsPerWave * NC;
  constexpr uint32_t kProducer = NC;
  // Blocks per step: the producer's 64 lanes each make one (part, block) per step, so a step
  // covers 64 / kParts blocks (8 at NC = 1) for the same producer issue time, and the
  // consumers pass one barrier per step instead of one per 2 blocks.
  constexpr uint32_t kBps = 64 / kParts >= 2 ? 64 / kParts : 2;
  constexpr uint32_t kLanes = kParts * kBps;  // producer lanes with distinct work (<= 64)
  __shared__ uint4 lds_wk[2][kBps][16][kParts];  // [buffer][block in step][row][part]

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot0 = blockIdx.x * kParts;
  const uint64_t b0 = A.blk_begin;
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  if (wg_end <= b0) return;
  const uint64_t iters = wg_end - b0;
  const uint64_t steps = (iters + kBps - 1) / kBps;

  if (wave == kProducer) {
    // ---------------------------------------------------------------- producer
    // Lane = (part, block h of the step): consecutive lanes take consecutive blocks of one
    // part (coalesced 64*kBps-byte runs).  Lanes >= kLanes repeat lanes 0.. (same loads, same
    // LDS writes), which keeps every lane on one branch-free path at no extra issue cost.
    const uint32_t pl = lane % kLanes;
    const uint32_t part = pl / kBps, h = pl % kBps;
    const uint32_t slot = slot0 + part;
    Slot s = {0, 0};
    if (slot < A.n) s = A.slots[slot];
    const uint8_t* p = A.base + s.off + 64ull * (b0 + h - A.blk_origin);
    const uint32_t sel = be_selector(uint32_t(reinterpret_cast<uintptr_t>(A.base + s.off) & 3));
    const uint64_t fend = fetch_end(s.len, A.blk_end);
    const uint64_t bh = b0 + h;
    const uint64_t bits = slot < A.n ? msg_bits(A, slot, s.len) : 0;
    const uint64_t dl = decode_len(slot < A.n, s.len);
    constexpr uint64_t kStride = 64ull * kBps;
    RawBlock ra, rb;
    fetch_full(p, bh < fend, A.zero, ra);
    fetch_full(p + kStride, bh + kBps < fend, A.zero, rb);
    produce_block(ra, sel, p, dl, bits, bh, A.blk_end, lds_wk[0][h], part);
    __syncthreads();
    for (uint64_t k = 1; k <= steps; k += 2) {
      if (k < steps) {
        fetch_full(p + kStride * (k + 1), bh + kBps * (k + 1) < fend, A.zero, ra);
        produce_block(rb, sel, p + kStride * k, dl, bits, bh + kBps * k, A.blk_end, lds_wk[1][h], part);
      }
      __syncthreads();
      if (k + 1 > steps) break;
      if (k + 1 < steps) {
        fetch_full(p + kStride * (k + 2), bh + kBps * (k + 2) < fend, A.zero, rb);
        produce_block(ra, sel, p + kStride * (k + 1), dl, bits, bh + kBps * (k + 1), A.blk_end, lds_wk[0][h], part);
      }
      __syncthreads();
    }
  } else {
    // ---------------------------------------------------------------- consumer
    __builtin_amdgcn_s_setprio(3);
    const uint32_t part = kQuadChainsPerWave * wave + (lane >> 4) * 2u + ((lane >> 3) & 1u);
    const bool ahalf = (lane >> 2) & 1u;
    const uint32_t k4 = lane & 3u;
    const uint32_t slot = slot0 + part;
    const bool valid = slot < A.n;
    const uint64_t nb = valid ? slot_blocks(A, A.slots[slot].len) : 0;
    const uint32_t sh = ahalf ? (k4 == 1 ? 13u : k4 == 2 ? 22u : 2u)
                              : (k4 == 1 ? 11u : k4 == 2 ? 25u : 6u);
    const uint32_t msk = ahalf ? 0xffffffffu : 0u;
    const uint32_t w0 = ahalf ? 0u : 4u;
    uint32_t s0, s1, s2, s3;
    if (valid && resumes(A)) {
      const uint4 v = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot] + w0)[0];
      s0 = v.x; s1 = v.y; s2 = v.z; s3 = v.w;
    } else {
      s0 = ahalf ? 0x6a09e667u : 0x510e527fu;
      s1 = ahalf ? 0xbb67ae85u : 0x9b05688cu;
      s2 = ahalf ? 0x3c6ef372u : 0x1f83d9abu;
      s3 = ahalf ? 0xa54ff53au : 0x5be0cd19u;
    }
    uint32_t xa = 0, xb = 0;
    uint32_t q1, q2, q3, q4, n0, n1, n2, n3;
    const uint32_t last = (slot0 + kParts <= A.n ? slot0 + kParts : A.n) - 1;
    const uint64_t all_live_end = slot_blocks(A, A.slots[last].len);
    // W[j] = W+K row (k4 + 4j) of the block: word w of round 16j + 4r + w sits on lane r.
    auto block = [&](const uint4 W[4], uint64_t i) {
      asm volatile(
          "s_nop 1\n\t" S3H_ALIGN8
          "v_add_u32_dpp %0, %1, %2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0x5"
          : "+v"(xa) : "v"(W[0].x), "v"(s3));
      asm volatile(S3H_ALIGN8 S3H_Q16_FIRST S3H_Q16(b, c0)
                   : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3),
                     [xa] "+v"(xa), [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2),
                     [q3] "=&v"(q3), [q4] "=&v"(q4)
                   : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3),
                     [a0] "v"(W[0].x), [a1] "v"(W[0].y), [a2] "v"(W[0].z), [a3] "v"(W[0].w),
                     [b0] "v"(W[1].x), [b1] "v"(W[1].y), [b2] "v"(W[1].z), [b3] "v"(W[1].w),
                     [c0] "v"(W[2].x), [h1] "v"(sh), [m] "v"(msk));
      asm volatile(S3H_ALIGN8 S3H_Q16(c, d0) S3H_Q16(d, d0)
                   : [n0] "+v"(n0), [n1] "+v"(n1), [n2] "+v"(n2), [n3] "+v"(n3),
                     [xa] "+v"(xa), [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2),
                     [q3] "=&v"(q3), [q4] "=&v"(q4)
                   : [c0] "v"(W[2].x), [c1] "v"(W[2].y), [c2] "v"(W[2].z), [c3] "v"(W[2].w),
                     [d0] "v"(W[3].x), [d1] "v"(W[3].y), [d2] "v"(W[3].z), [d3] "v"(W[3].w),
                     [h1] "v"(sh), [m] "v"(msk));
      if (b0 + i < all_live_end) {
        s0 += n0; s1 += n1; s2 += n2; s3 += n3;
      } else {
        const bool live = (b0 + i) < nb;
        s0 = live ? s0 + n0 : s0;
        s1 = live ? s1 + n1 : s1;
        s2 = live ? s2 + n2 : s2;
        s3 = live ? s3 + n3 : s3;
      }
    };
    auto load = [&](uint4 W[4], uint32_t buf, uint32_t blk) {
#pragma unroll
      for (int q = 0; q < 4; ++q) W[q] = lds_wk[buf][blk][k4 + 4 * q][part];
    };
    __syncthreads();
    for (uint64_t j = 0; j < steps; ++j) {
      // The next block's W+K is read while the current block runs: only the step's first read
      // waits on LDS latency.
      const uint32_t buf = uint32_t(j & 1);
      const uint64_t base_i = kBps * j;
      uint4 wa[4], wb[4];
      load(wa, buf, 0);
#pragma unroll
      for (uint32_t i = 0; i < kBps; i += 2) {
        load(wb, buf, i + 1);
        if (base_i + i < iters) block(wa, base_i + i);
        if (i + 2 < kBps) load(wa, buf, i + 2);
        if (base_i + i + 1 < iters) block(wb, base_i + i + 1);
      }
      __syncthreads();
    }
    if (valid && nb > b0 && k4 == 0) {
      if (emits(A, nb)) {
        uint4* o = reinterpret_cast<uint4*>(A.digests + 8ull * A.out_idx[slot] + w0);
        o[0] = make_uint4(bswap(s0), bswap(s1), bswap(s2), bswap(s3));
      } else if (A.state) {
        reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot] + w0)[0] = make_uint4(s0, s1, s2, s3);
      }
    }
  }
}

// ------------------------------------------------------------- skewed lane-octet kernel
// The quad kernel's lane layout (each chain on 8 lanes: e-quad + a-quad) with the a-quad run
// two rounds BEHIND the e-quad (tools/gen_skew.py derives and simulates the schedule).  The
// skew turns both halves' updates into "own nonlinear part + one precomputed sum", and the
// sum for the next round is one row_half_mirror DPP add (cross term + W+K) plus one v_xad
// (own term, negated in the a-quad by a per-lane mask): 8 VALU per round instead of 9.  The
// pipeline runs across blocks (the a-quad finishes block k in block k+1's first two rounds);
// the feed-forward and three boundary corrections add 11 VALU per block: 523 per block in all,
// against the quad kernel's 592.  Each lane needs its own copy of every W+K word (the DPP
// operand slot carries the cross term), so the consumer reads all 16 rows per block; the
// a-quad lanes read a column of ones (their "W" restores the +1 of ~x = -x - 1).
#include "sha256_skew_rounds.inc"

#define S3H_SKEW_STATE                                                                        \
  [g0_0] "+v"(g00), [g0_1] "+v"(g01), [g1_0] "+v"(g10), [g1_1] "+v"(g11), [e0_0] "+v"(e00),    \
      [e0_1] "+v"(e01), [e0_2] "+v"(e02), [e0_3] "+v"(e03), [e1_0] "+v"(e10), [e1_1] "+v"(e11), \
      [e1_2] "+v"(e12), [e1_3] "+v"(e13), [n0] "+v"(n0), [n1] "+v"(n1), [n2] "+v"(n2),          \
      [n3] "+v"(n3), [x0] "+v"(x0), [x1] "+v"(x1), [q1] "=&v"(q1), [q3] "=&v"(q3),               \
      [sl] "=&v"(sl), [cm] "=&v"(cm), [t] "=&v"(tt), [q2] "=&v"(q2)
#define S3H_SKEW_W(W)                                                                           \
  [w1] "v"(W[1]), [w2] "v"(W[2]), [w3] "v"(W[3]), [w4] "v"(W[4]), [w5] "v"(W[5]), [w6] "v"(W[6]), \
      [w7] "v"(W[7]), [w8] "v"(W[8]), [w9] "v"(W[9]), [w10] "v"(W[10]), [w11] "v"(W[11]),         \
      [w12] "v"(W[12]), [w13] "v"(W[13]), [w14] "v"(W[14]), [w15] "v"(W[15]), [w16] "v"(W[16]),   \
      [w17] "v"(W[17]), [w18] "v"(W[18]), [w19] "v"(W[19]), [w20] "v"(W[20]), [w21] "v"(W[21]),   \
      [w22] "v"(W[22]), [w23] "v"(W[23]), [w24] "v"(W[24]), [w25] "v"(W[25]), [w26] "v"(W[26]),   \
      [w27] "v"(W[27]), [w28] "v"(W[28]), [w29] "v"(W[29]), [w30] "v"(W[30]), [w31] "v"(W[31]),   \
      [w32] "v"(W[32]), [w33] "v"(W[33]), [w34] "v"(W[34]), [w35] "v"(W[35]), [w36] "v"(W[36]),   \
      [w37] "v"(W[37]), [w38] "v"(W[38]), [w39] "v"(W[39]), [w40] "v"(W[40]), [w41] "v"(W[41]),   \
      [w42] "v"(W[42]), [w43] "v"(W[43]), [w44] "v"(W[44]), [w45] "v"(W[45]), [w46] "v"(W[46]),   \
      [w47] "v"(W[47]), [w48] "v"(W[48]), [w49] "v"(W[49]), [w50] "v"(W[50]), [w51] "v"(W[51]),   \
      [w52] "v"(W[52]), [w53] "v"(W[53]), [w54] "v"(W[54]), [w55] "v"(W[55]), [w56] "v"(W[56]),   \
      [w57] "v"(W[57]), [w58] "v"(W[58]), [w59] "v"(W[59]), [w60] "v"(W[60]), [w61] "v"(W[61]),   \
      [w62] "v"(W[62]), [w63] "v"(W[63]), [am] "v"(am), [mk] "v"(mk), [am2] "v"(am2), [am3] "v"(am3)

// The next block's rows as inputs of the statement that ends a block (skew_body kMergeNext):
// w0 is NEXT's operand, the rest only make the compiler wait for every row there.
#define S3H_SKEW_WNEXT(W) [w0] "v"(W[0]), [nw1] "v"(W[1]), [nw2] "v"(W[2]), [nw3] "v"(W[3]), [nw4] "v"(W[4]), [nw5] "v"(W[5]), [nw6] "v"(W[6]), [nw7] "v"(W[7]), [nw8] "v"(W[8]), [nw9] "v"(W[9]), [nw10] "v"(W[10]), [nw11] "v"(W[11]), [nw12] "v"(W[12]), [nw13] "v"(W[13]), [nw14] "v"(W[14]), [nw15] "v"(W[15]), [nw16] "v"(W[16]), [nw17] "v"(W[17]), [nw18] "v"(W[18]), [nw19] "v"(W[19]), [nw20] "v"(W[20]), [nw21] "v"(W[21]), [nw22] "v"(W[22]), [nw23] "v"(W[23]), [nw24] "v"(W[24]), [nw25] "v"(W[25]), [nw26] "v"(W[26]), [nw27] "v"(W[27]), [nw28] "v"(W[28]), [nw29] "v"(W[29]), [nw30] "v"(W[30]), [nw31] "v"(W[31]), [nw32] "v"(W[32]), [nw33] "v"(W[33]), [nw34] "v"(W[34]), [nw35] "v"(W[35]), [nw36] "v"(W[36]), [nw37] "v"(W[37]), [nw38] "v"(W[38]), [nw39] "v"(W[39]), [nw40] "v"(W[40]), [nw41] "v"(W[41]), [nw42] "v"(W[42]), [nw43] "v"(W[43]), [nw44] "v"(W[44]), [nw45] "v"(W[45]), [nw46] "v"(W[46]), [nw47] "v"(W[47]), [nw48] "v"(W[48]), [nw49] "v"(W[49]), [nw50] "v"(W[50]), [nw51] "v"(W[51]), [nw52] "v"(W[52]), [nw53] "v"(W[53]), [nw54] "v"(W[54]), [nw55] "v"(W[55]), [nw56] "v"(W[56]), [nw57] "v"(W[57]), [nw58] "v"(W[58]), [nw59] "v"(W[59]), [nw60] "v"(W[60]), [nw61] "v"(W[61]), [nw62] "v"(W[62]), [nw63] "v"(W[63])

// PAIR: the lane-pair layout of the same schedule (S3H_SKEWP_*, 9 VALU per round): a chain on
// e-lane k and a-lane 7-k of a half-row, 32 chains per consumer wave.
//
// A GROUP is NC consumer waves (kCpw chains each) fed by one producer wave through a W+K
// double buffer in LDS.  Two ways to synchronise a group:
//   FLAGS = false: s_barrier, one per producer step (the group is the whole workgroup);
//   FLAGS = true : two LDS step counters per group (produced / consumed, release-acquire at
//                  workgroup scope), so several independent groups -- or a SHA-256 group and
//                  an MD5 group -- share one workgroup without stalling on each other's
//                  barriers (NC = 1 in this mode).  Every wait is bounded (kFlagSpinLimit), so
//                  a wave can never hang on a counter, and a wait that times out sets the
//                  launch's error word, which fails the host call (flag_wait_ge).
// `group` numbers the group's parts (slots group*kParts...), `role` is the wave's job in it:
// consumer index 0..NC-1, or NC for the producer.
template <int NC, bool PAIR>
struct SkewGeom {
  static constexpr uint32_t kCpw = PAIR ? 32 : kQuadChainsPerWave;  // chains per consumer wave
  static constexpr uint32_t kParts = kCpw * NC;
  // Blocks per producer step: 8 when the producer's lanes make at most two (part, block)
  // items per step (one step of prefetch = ~8 blocks of chain time, one sync per 8 blocks);
  // fewer for wider groups, whose producer would spill.
  static constexpr uint32_t kBps = PAIR ? 4 : NC >= 4 ? 2 : NC == 2 ? S3H_EXP_SKEW_BPS_NC2 : 8;
  static constexpr uint32_t kCols = kParts + 1;  // column kParts holds ones (read by the a-quads)
  // uint4s of padding after each block's 16 rows (skew layout).  A block is 16 x 9 uint4 =
  // 576 dwords = 0 mod 64 banks, so the producer's lanes (8 parts x 8 blocks) write each W+K
  // word 8-way bank-conflicted; 8 uint4 (128 B) would halve that, but the C4 shard runs the same
  // 2,243.6 cycles/block either way (profiles/r02_exp_skews_lds.jsonl): kept at 0.
  static constexpr uint32_t kBlkPad = PAIR ? 0 : S3H_EXP_SKEW_BLK_PAD;
  static constexpr uint32_t kBlkStride = 16 * kCols + kBlkPad;  // uint4 between blocks
};
// wk[buffer][block of the step][row * kCols + part] (+ kBlkPad after each block)
template <int NC, bool PAIR>
struct SkewLds {
  uint4 wk[2][SkewGeom<NC, PAIR>::kBps][SkewGeom<NC, PAIR>::kBlkStride];
};

constexpr uint32_t kFlagSpinLimit = S3H_EXP_SPIN_LIMIT;  // x s_sleep 1 (64 clocks): ~0.45 s
__device__ __forceinline__ void flag_publish(uint32_t* f, uint32_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Wait for *f >= v.  A wait that times out ORs kErrSyncTimeout into the launch's device error
// word (a global vector atomic), and `alive` (wave-uniform) turns false so every later wait of
// the wave returns at once: the grid always drains -- one timeout per wave, never a hung GPU
// -- and the host entry point that reads the word fails the call (S3H_EHIP) instead of
// returning the launch's now meaningless digests.
__device__ __forceinline__ void flag_wait_ge(uint32_t* f, uint32_t v, bool& alive, uint32_t* err) {
  if (!alive) return;
  uint32_t spin = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) {
    if (++spin >= kFlagSpinLimit) {
      alive = false;
      __hip_atomic_fetch_or(err, kErrSyncTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The generated producer's v_mul_f32 left shifts need f32 denormals kept on input and output
// (the default: .amdhsa_float_denorm_mode_32 3, checked by tests/test_producer_schedule.py).
#if defined(__FAST_MATH__) || defined(__AMDGCN_FLUSH_DENORMALS__)
#error "sha256_producer_simple.inc needs f32 denormals: do not build with fast-math / FTZ"
#endif
#ifdef S3H_EXP_PRODUCER_INC  // tools/ experiment builds only: another generated producer
#include S3H_EXP_PRODUCER_INC
#else
#include "sha256_producer_simple.inc"
#endif
#if defined(S3H_PROD_ZYV) && !defined(S3H_EXPERIMENT_BUILD)
// gen_producer.py --zyv / --zyv-plain: byte swap from unaligned in-block loads -- measured
// slower on the C4 shard (2,246-2,250 vs 2,241 cycles per block at the same board power,
// profiles/r05_exp_producer_zyv.jsonl), so an experiment only
#error "the --zyv producer is an experiment (make exp)"
#endif

// The same for a producer that shares its consumer's SIMD (sha256_skew_shared_kernel): that
// SIMD issues a second wave's v_add_u32, v_xor/or/and_b32, v_lshrrev_b32 and f32 add/mul
// beside the round stream at the lone-wave rate, but not its left shifts, alignbit, perm or
// add3 (tools/ubench_coissue2.hip, profiles/r02_ubench_coissue_*.txt).  The block's byte swap
// and schedule are therefore one generated asm statement in those classes
// (tools/gen_producer.py: each left shift is one v_mul_f32 by 2^k on a denormal bit pattern --
// exact because f32 denormals are preserved, see below -- plus doublings), fed the block's 16
// words as little-endian dwords: the raw loads
// when every lane of the wave reads dword-aligned parts (`aligned`), one v_perm per word
// otherwise, and the padded tail block (once per part) byte-swapped back with v_perm.
#ifdef S3H_PROD_ZYV
// The block's bytes loaded again at byte offsets 4k+1 (z[k], k = 0..14) and 4j-1 (y[j-1],
// j = 1..15): unaligned global loads that stay inside the block (bytes 1..60 and 3..62), so each
// word's four bytes arrive in the lanes its big-endian form needs and the producer assembles
// them with three v_bitop3 selects instead of doublings (tools/gen_producer.py bswap_zyv).
// The loads go to the memory pipeline, not the VALU the consumer's round stream shares.
struct ZYBlock { uint32_t z[15], y[15]; };
typedef uint32_t v4u32a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t v3u32a1 __attribute__((ext_vector_type(3), aligned(1)));
typedef const __attribute__((address_space(1))) v4u32a1 gv4u32a1;
typedef const __attribute__((address_space(1))) v3u32a1 gv3u32a1;

__device__ __forceinline__ void fetch_zy(const uint8_t* p, bool ok, const uint8_t* zero, ZYBlock& r) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(ok ? p : zero);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const v4u32a1 z = *reinterpret_cast<gv4u32a1*>(a + 1 + 16 * i);
    const v4u32a1 y = *reinterpret_cast<gv4u32a1*>(a + 3 + 16 * i);
    r.z[4 * i] = z.x; r.z[4 * i + 1] = z.y; r.z[4 * i + 2] = z.z; r.z[4 * i + 3] = z.w;
    r.y[4 * i] = y.x; r.y[4 * i + 1] = y.y; r.y[4 * i + 2] = y.z; r.y[4 * i + 3] = y.w;
  }
  const v3u32a1 z = *reinterpret_cast<gv3u32a1*>(a + 49);
  const v3u32a1 y = *reinterpret_cast<gv3u32a1*>(a + 51);
  r.z[12] = z.x; r.z[13] = z.y; r.z[14] = z.z;
  r.y[12] = y.x; r.y[13] = y.y; r.y[14] = y.z;
}

// The same values formed from the block's 16 little-endian words (blocks that were not loaded
// in place: unaligned parts, the padded tail, blocks past the launch).
__device__ __forceinline__ void zy_from_words(const uint32_t w[16], ZYBlock& r) {
#pragma unroll
  for (int k = 0; k < 15; ++k) r.z[k] = (w[k] >> 8) | (w[k + 1] << 24);
#pragma unroll
  for (int j = 1; j < 16; ++j) r.y[j - 1] = (w[j - 1] >> 24) | (w[j] << 8);
}
#endif

template <int kRow>
__device__ __forceinline__ void produce_block_simple(const RawBlock& r,
#ifdef S3H_PROD_ZYV
                                                     const ZYBlock& zy_loaded,
#endif
                                                     uint32_t sel,
                                                     const uint8_t* bp, uint64_t len, uint64_t bits,
                                                     uint64_t blk, uint64_t limit, bool aligned,
                                                     uint4 (*buf)[kRow], uint32_t lane) {
  static_assert(kRow * 16 == 144, "tools/gen_producer.py ROW");
  uint32_t w[16];
#ifdef S3H_PROD_ZYV
  ZYBlock zy;
  const bool in_place = aligned && blk < limit && blk < (len >> 6);
  if (in_place) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = r.d[j];
    zy = zy_loaded;
  } else {
#endif
  if (blk >= limit) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = 0;
  } else if (blk < (len >> 6)) {
    if (aligned) {
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = r.d[j];
    } else {
      const uint32_t le = le_selector(sel >> 24);
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(r.d[j + 1], r.d[j], le);
    }
  } else {
    build_tail(bp, len, bits, blk, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
  }
#ifdef S3H_PROD_ZYV
    zy_from_words(w, zy);
  }
  uint32_t z0 = zy.z[0], z1 = zy.z[1], z2 = zy.z[2], z3 = zy.z[3], z4 = zy.z[4], z5 = zy.z[5],
           z6 = zy.z[6], z7 = zy.z[7], z8 = zy.z[8], z9 = zy.z[9], z10 = zy.z[10], z11 = zy.z[11],
           z12 = zy.z[12], z13 = zy.z[13], z14 = zy.z[14];
  uint32_t y1 = zy.y[0], y2 = zy.y[1], y3 = zy.y[2], y4 = zy.y[3], y5 = zy.y[4], y6 = zy.y[5],
           y7 = zy.y[6], y8 = zy.y[7], y9 = zy.y[8], y10 = zy.y[9], y11 = zy.y[10], y12 = zy.y[11],
           y13 = zy.y[12], y14 = zy.y[13], y15 = zy.y[14];
  const uint32_t mhi = 0xFF000000u, mlo = 0xFFFFFF00u, mmid = 0xFFFF0000u;
#endif
  typedef __attribute__((address_space(3))) uint4 lds_uint4;
  const uint32_t la = uint32_t(reinterpret_cast<uintptr_t>((lds_uint4*)(&buf[0][lane])));
  uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5], w6 = w[6], w7 = w[7],
           w8 = w[8], w9 = w[9], w10 = w[10], w11 = w[11], w12 = w[12], w13 = w[13], w14 = w[14],
           w15 = w[15];
#ifdef S3H_EXP_PROD_ROWS  // experiment: one asm statement and one ds_write_b128 per W+K row
  uint32_t l0_0 = 0, l0_1 = 0, l0_2 = 0, l0_3 = 0, l0_4 = 0, l0_5 = 0, l0_6 = 0, l0_7 = 0, l0_8 = 0,
           l0_9 = 0, l0_10 = 0, l0_11 = 0, l0_12 = 0, l0_13 = 0, l0_14 = 0, l0_15 = 0, l1_0 = 0,
           l1_1 = 0, l1_2 = 0, l1_3 = 0, c0, c1, c2, c3, c4, c5, s0, s1, s2, s3, rk0, rk1, rk2, rk3;
  (void)la;
#define S3H_ROW(q)                                                                        \
  asm volatile(S3H_ALIGN8 S3H_PROD_ROW_##q : S3H_PROD_ROW_OUTS);                         \
  buf[q][lane] = make_uint4(rk0, rk1, rk2, rk3);
  S3H_ROW(0) S3H_ROW(1) S3H_ROW(2) S3H_ROW(3) S3H_ROW(4) S3H_ROW(5) S3H_ROW(6) S3H_ROW(7)
  S3H_ROW(8) S3H_ROW(9) S3H_ROW(10) S3H_ROW(11) S3H_ROW(12) S3H_ROW(13) S3H_ROW(14) S3H_ROW(15)
#undef S3H_ROW
#else
  S3H_PROD_SIMPLE_TEMPS
  const uint32_t bsel = 0x00010203u;  // v_perm byte swap (tools/gen_producer.py --perm-bswap only)
#ifdef S3H_PROD_ZYV
  asm volatile(S3H_ALIGN8 S3H_PROD_SIMPLE_ASM : S3H_PROD_SIMPLE_OUTS
               : [la] "v"(la), [bsel] "v"(bsel), S3H_PROD_SIMPLE_INS : "memory");
#else
  asm volatile(S3H_ALIGN8 S3H_PROD_SIMPLE_ASM : S3H_PROD_SIMPLE_OUTS : [la] "v"(la), [bsel] "v"(bsel)
               : "memory");
#endif
#endif
}

// SIMPLE: the producer is written in the co-issuable instruction classes (it shares its
// consumer's SIMD: sha256_skew_shared_kernel).  GPROG: the producer also stores each published
// step count, tagged (epoch << 32 | steps), to `gprog` when it is non-null -- the pacing hint
// of MD5 waves on other workgroups of the same XCD (ShaPacer): a plain store, which stays in
// this XCD's L2 where those waves' L2-served polls read it (an agent-scope store would write
// through to memory and drop the line, and every poll would then cross the fabric); one 8-byte
// store per step, never read back by this group.
template <int NC, bool PAIR, bool FLAGS, bool SIMPLE = false, bool GPROG = false>
__device__ __forceinline__ void skew_body(const LaunchArgs& A, const uint32_t group,
                                          const uint32_t role, SkewLds<NC, PAIR>& L,
                                          uint32_t* flags, uint64_t* gprog = nullptr,
                                          uint32_t epoch = 0) {
  static_assert(!FLAGS || NC == 1, "flag-synchronised groups have one consumer wave");
  using G = SkewGeom<NC, PAIR>;
  constexpr uint32_t kCpw = G::kCpw, kParts = G::kParts, kBps = G::kBps, kCols = G::kCols;
  constexpr uint32_t kLanes = kParts * kBps;
  constexpr uint32_t kItems = kLanes / 64;  // == NC
  auto& lds_wk = L.wk;
  // the 16 x kCols rows of block h of buffer b
  auto rows = [&](uint32_t b, uint32_t h) { return reinterpret_cast<uint4 (*)[kCols]>(lds_wk[b][h]); };
  bool alive = true;  // FLAGS: false after a timed-out wait (flag_wait_ge)
  // FLAGS: flags[0] = producer steps published, flags[1] = consumer steps released
#define S3H_SYNC_PRODUCED(m)                                                  \
  do {                                                                        \
    if constexpr (FLAGS) {                                                    \
      if (!S3H_EXP_STALL_PRODUCER || (m) <= 1u) flag_publish(&flags[0], (m)); \
    } else {                                                                  \
      __syncthreads();                                                        \
    }                                                                         \
    if constexpr (GPROG && !S3H_EXP_GPROG_OFF) {                              \
      if (gprog)                                                              \
        __hip_atomic_store(gprog, (uint64_t(epoch) << 32) | uint64_t(m),      \
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   \
    }                                                                         \
  } while (0)

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t slot0 = group * kParts;
  if (slot0 >= A.n) return;
  const uint64_t b0 = A.blk_begin;
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  if (wg_end <= b0) return;
  const uint64_t iters = wg_end - b0;
  const uint64_t steps = (iters + kBps - 1) / kBps;

  if (role == NC) {
    // ---------------------------------------------------------------- producer
    for (uint32_t i = lane; i < 2 * kBps * 16; i += 64)
      lds_wk[i / (kBps * 16)][(i / 16) % kBps][(i % 16) * kCols + kParts] = make_uint4(1u, 1u, 1u, 1u);
    // Item r of this lane = (part, block h of the step); consecutive lanes take consecutive
    // blocks of one part (coalesced 512-byte runs).
    const uint8_t* p[kItems];
    uint32_t sel[kItems], part[kItems], h[kItems];
    uint64_t len[kItems], fend[kItems], bh[kItems], bits[kItems];
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
      const uint32_t it = lane + 64u * r;
      part[r] = it / kBps;
      h[r] = it % kBps;
      const uint32_t slot = slot0 + part[r];
      Slot s = {0, 0};
      if (slot < A.n) s = A.slots[slot];
      p[r] = A.base + s.off + 64ull * (b0 + h[r] - A.blk_origin);
      sel[r] = be_selector(uint32_t(reinterpret_cast<uintptr_t>(A.base + s.off) & 3));
      len[r] = decode_len(slot < A.n, s.len);
      fend[r] = fetch_end(s.len, A.blk_end);
      bh[r] = b0 + h[r];
      bits[r] = slot < A.n ? msg_bits(A, slot, s.len) : 0;
    }
    // SIMPLE: every lane's part starts dword-aligned (wave-uniform: the s_bswap decode)
    const bool aligned = SIMPLE && __all(sel[0] == 0x00010203u);
#ifdef S3H_PROD_ZYV  // the SIMPLE producer's in-place unaligned loads, double-buffered like RAW
#define S3H_ZY(ZY) ZY,
#define S3H_FETCH_ZY(PTR, OK, ZY)                             \
  do {                                                        \
    if constexpr (SIMPLE) fetch_zy(PTR, OK, A.zero, ZY);      \
  } while (0)
#else
#define S3H_ZY(ZY)
#define S3H_FETCH_ZY(PTR, OK, ZY) do {} while (0)
#endif
#define S3H_PRODUCE(RAW, ZY, R, BP, BLK, BUF)                                                  \
  do {                                                                                         \
    if constexpr (SIMPLE)                                                                      \
      produce_block_simple(RAW, S3H_ZY(ZY) sel[R], BP, len[R], bits[R], BLK, A.blk_end, aligned, BUF, part[R]); \
    else                                                                                       \
      produce_block(RAW, sel[R], BP, len[R], bits[R], BLK, A.blk_end, BUF, part[R]);           \
  } while (0)
    constexpr uint64_t kStride = 64ull * kBps;
    RawBlock ra[kItems], rb[kItems];
#ifdef S3H_PROD_ZYV
    ZYBlock za[kItems], zb[kItems];
#endif
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
      fetch_full(p[r], bh[r] < fend[r], A.zero, ra[r]);
      S3H_FETCH_ZY(p[r], bh[r] < fend[r], za[r]);
      fetch_full(p[r] + kStride, bh[r] + kBps < fend[r], A.zero, rb[r]);
      S3H_FETCH_ZY(p[r] + kStride, bh[r] + kBps < fend[r], zb[r]);
    }
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) S3H_PRODUCE(ra[r], za[r], r, p[r], bh[r], rows(0, h[r]));
    S3H_SYNC_PRODUCED(1u);
#ifdef S3H_EXP_PRODUCER_IDLE  // experiment (power): after step 0 the shared-SIMD producer only
                              // keeps the flag protocol; the consumers hash stale W+K
    if constexpr (FLAGS && SIMPLE) {
      for (uint64_t k = 1; k <= steps; ++k) {
        if (k < steps && k >= 2) flag_wait_ge(&flags[1], uint32_t(k - 1), alive, A.err);
        S3H_SYNC_PRODUCED(uint32_t(k + 1));
      }
      return;
    }
#endif
    // Step k goes into buffer k & 1, which held step k - 2: FLAGS waits until the consumer
    // has released that step (the barrier of the other mode orders the same thing).
    for (uint64_t k = 1; k <= steps; k += 2) {
      if (k < steps) {
        if constexpr (FLAGS) {
          if (k >= 2) flag_wait_ge(&flags[1], uint32_t(k - 1), alive, A.err);
        }
        S3H_PROD_UNROLL
        for (uint32_t r = 0; r < kItems; ++r) {
          fetch_full(p[r] + kStride * (k + 1), bh[r] + kBps * (k + 1) < fend[r], A.zero, ra[r]);
          S3H_FETCH_ZY(p[r] + kStride * (k + 1), bh[r] + kBps * (k + 1) < fend[r], za[r]);
          S3H_PRODUCE(rb[r], zb[r], r, p[r] + kStride * k, bh[r] + kBps * k, rows(1, h[r]));
        }
      }
      S3H_SYNC_PRODUCED(uint32_t(k + 1));
      if (k + 1 > steps) break;
      if (k + 1 < steps) {
        if constexpr (FLAGS) flag_wait_ge(&flags[1], uint32_t(k), alive, A.err);
        S3H_PROD_UNROLL
        for (uint32_t r = 0; r < kItems; ++r) {
          fetch_full(p[r] + kStride * (k + 2), bh[r] + kBps * (k + 2) < fend[r], A.zero, rb[r]);
          S3H_FETCH_ZY(p[r] + kStride * (k + 2), bh[r] + kBps * (k + 2) < fend[r], zb[r]);
          S3H_PRODUCE(ra[r], za[r], r, p[r] + kStride * (k + 1), bh[r] + kBps * (k + 1), rows(0, h[r]));
        }
      }
      S3H_SYNC_PRODUCED(uint32_t(k + 2));
    }
    return;
  }
#undef S3H_PRODUCE
#undef S3H_ZY
#undef S3H_FETCH_ZY
#undef S3H_SYNC_PRODUCED
  // ------------------------------------------------------------------ consumer
#ifdef S3H_EXP_LONE_CONSUMER  // experiment: only consumer wave 0 works (wrong digests)
  if (role != 0) return;
#endif
#ifdef S3H_EXP_CONSUMER_IDLE  // experiment (power): the shared-SIMD consumers only keep the
                              // flag protocol; the producers run alone (wrong digests)
  if constexpr (FLAGS && SIMPLE) {
    for (uint32_t j = 0; j < uint32_t(steps); ++j) {
      flag_wait_ge(&flags[0], j + 1, alive, A.err);
      flag_publish(&flags[1], j + 1);
    }
    return;
  }
#endif
  __builtin_amdgcn_s_setprio(3);
  const bool ahalf = (lane >> 2) & 1u;
  const uint32_t k4 = lane & 3u;
  // quad: lanes 8c..8c+7 = chain c; pair: half-row h holds chains 4h..4h+3 (e-lane k, a-lane 7-k)
  const uint32_t part = kCpw * role + (PAIR ? 4 * (lane >> 3) + (ahalf ? 3 - k4 : k4) : lane >> 3);
  const uint32_t slot = slot0 + part;
  const bool valid = slot < A.n;
  const uint64_t nb = valid ? slot_blocks(A, A.slots[slot].len) : 0;
  const uint32_t last_slot = (slot0 + kParts <= A.n ? slot0 + kParts : A.n) - 1;
  const uint64_t live_end = slot_blocks(A, A.slots[last_slot].len);  // every chain live below
  // Rotation per lane: positions 0..2 of a quad take the three Sigma amounts, 3 repeats 0.
  // quad: one rotation per lane (positions 0..2 of a quad take the three Sigma amounts, 3
  // repeats 0); pair: all three in every lane
  const uint32_t am = PAIR ? (ahalf ? 2u : 6u)
                           : ahalf ? (k4 == 1 ? 22u : k4 == 2 ? 13u : 2u)
                                   : (k4 == 1 ? 11u : k4 == 2 ? 25u : 6u);
  const uint32_t am2 = ahalf ? 13u : 11u, am3 = ahalf ? 22u : 25u;
  const uint32_t mk = ahalf ? 0xffffffffu : 0u;
  const uint32_t one_a = ahalf ? 1u : 0u;
  uint32_t H[8];
  if (valid && resumes(A)) {
    const uint4* sp = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot]);
    const uint4 u = sp[0], v = sp[1];
    H[0] = u.x; H[1] = u.y; H[2] = u.z; H[3] = u.w; H[4] = v.x; H[5] = v.y; H[6] = v.z; H[7] = v.w;
  } else {
    init_state(H);
  }
  // Register image before block 0 (parity 0): gen_skew.py init_regs().  The a-quad's two
  // rounds of the (virtual) previous block compute zeros and its feed-forward adds H.
  uint32_t e13 = ahalf ? 0u : H[4], e12 = ahalf ? 0u : H[5], e11 = ahalf ? 0u : H[6],
           e10 = ahalf ? 0u : H[7];
  uint32_t e03 = ahalf ? H[2] : H[4], e02 = ahalf ? H[3] : 0u, e01 = 0, e00 = 0;
  uint32_t g11 = ahalf ? H[0] : 0u, g10 = ahalf ? H[1] : 0u, g01 = 0, g00 = 0;
  uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0, x0, x1 = 0;
  uint32_t q1, q2, q3, sl, cm, tt;
  // Per-lane LDS base (buffer 0, block 0, row 0, own column): block and buffer offsets are
  // immediates of the 16 ds_read_b128 that fetch one block's W+K.
  const uint4* lbase = &lds_wk[0][0][ahalf ? kParts : part];
  constexpr uint32_t kBlkStride = G::kBlkStride, kBufStride = kBps * G::kBlkStride;
  auto load = [&](uint32_t (&w)[64], const uint4* src) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint4 v = src[r * kCols];
      w[4 * r] = v.x; w[4 * r + 1] = v.y; w[4 * r + 2] = v.z; w[4 * r + 3] = v.w;
    }
  };
  // Final state of chains that end inside the pipeline: captured after the block that
  // follows their last one (a-half fed forward in its round 1).  Blocks below cap_from
  // (every chain of the workgroup still live) skip the check with one scalar branch.
  uint32_t f0 = 0, f1 = 0, f2 = 0, f3 = 0;
#define S3H_SKEW_CAPTURE(EP3, EP2, EP1, EP0, GQ1, GQ0) \
  do {                                                 \
    f0 = ahalf ? GQ1 : EP3;                            \
    f1 = ahalf ? GQ0 : EP2;                            \
    f2 = ahalf ? EP3 : EP1;                            \
    f3 = ahalf ? EP2 : EP0;                            \
  } while (0)

  const uint32_t it32 = uint32_t(iters);  // < 2^31: capi.hip runs longer ranges on the quad kernel
  // first block after which a chain can have ended (>= 1: block 0 ends none)
  const uint32_t cap_from = __builtin_amdgcn_readfirstlane(
      uint32_t(live_end > b0 + 1 ? live_end - b0 : 1));
  const uint32_t nb_rel = nb > b0 ? uint32_t(nb - b0) : 0u;

  uint32_t wa[64], wb[64];
  // consumer side of a step boundary: FLAGS releases the steps read so far and waits for the
  // next one (the barrier of the other mode)
#define S3H_SYNC_STEP(released, needed)                        \
  do {                                                         \
    if constexpr (FLAGS) {                                     \
      flag_publish(&flags[1], (released));                     \
      if ((needed) != 0u) flag_wait_ge(&flags[0], (needed), alive, A.err); \
    } else {                                                   \
      __syncthreads();                                         \
    }                                                          \
  } while (0)
  S3H_SYNC_STEP(0u, 1u);
  uint64_t clk0 = 0, rt0 = 0;
  if (A.clocks) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  load(wa, lbase);
  x0 = ahalf ? 0u : H[3] + H[7] + wa[0];
  // One block: rounds 0-15, then (after the step barrier when the next block lives in the
  // other LDS buffer) the next block's 16 rows are read while rounds 16-63 run; NEXT
  // consumes the next block's first word.  The a-quad lanes read the ones column, so their
  // NEXT word is 1 even past the last block.
  //
  // Fast steps -- none of whose blocks can end the launch or a chain -- run fully unrolled
  // with no per-block test; the remaining blocks (the ragged tail and the launch's last
  // block) run one at a time with the step barrier, capture and exit checks.
  // The next block's rows are read before this block's rounds 0-15 (the step barrier moves
  // with them), and rounds 16-63 + NEXT are one statement that takes every one of them as an
  // input: the compiler drains LDS once per block (the rows arrived ~500 cycles before) and a
  // block is two statements instead of three -- 543.88 -> 542.38 instructions per block, C2
  // 2,207.1 -> 2,202.8 cycles per block and C4 skews 2,238.3 -> 2,232.4 in one lease; the lane
  // pair layout (skewp) measured 2,476.1 -> 2,485.5 that way and keeps the three statements
  // (profiles/r06_skew_merge_next_ab.json).  S3H_EXP_SKEW_MERGE_NEXT: 0 never, 2 also skewp.
  constexpr bool kMergeNext = PAIR ? S3H_EXP_SKEW_MERGE_NEXT == 2 : S3H_EXP_SKEW_MERGE_NEXT >= 1;
  // Flag-synchronised groups (S3H_EXP_FLAG_PREFETCH, on in the product): the producer's step counter is
  // read without waiting, just before the next step's rows (LDS executes a wave's reads in
  // order, and the producer publishes a step only after its rows are written, so rows read
  // after a counter value that covers the step are that step's rows); it is checked after
  // rounds 0-15, and only a counter that did not cover the step costs a wait and a second read
  // of the rows.  Saves the counter read's latency at every step boundary: C3 2,217 -> 2,200
  // cycles per block, C4 skews 2,232 -> 2,220 (profiles/r06_flag_prefetch_ab.json).
  constexpr bool kFlagPrefetch = FLAGS && S3H_EXP_FLAG_PREFETCH != 0;
#define S3H_SKEW_FAST(L, P, CUR, NXT)                                                           \
  if constexpr (kMergeNext && kFlagPrefetch) {                                                  \
    /* the producer's step counter is read with the rows, checked after rounds 0-15 */          \
    uint32_t seen_prod = 0xffffffffu;                                                           \
    if (i == kBps - 1) {                                                                        \
      flag_publish(&flags[1], j + 1);                                                           \
      seen_prod = __hip_atomic_load(&flags[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
      asm volatile("" ::: "memory"); /* the rows are read after the counter */                  \
      load(NXT, nbuf);                                                                          \
    } else {                                                                                    \
      load(NXT, buf + (i + 1) * kBlkStride);                                                    \
    }                                                                                           \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_A_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    if (i == kBps - 1 && __builtin_amdgcn_readfirstlane(seen_prod) < j + 2) {                   \
      flag_wait_ge(&flags[0], j + 2, alive, A.err); /* not yet produced: wait, read again */    \
      load(NXT, nbuf);                                                                          \
    }                                                                                           \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_B_##P S3H_##L##_NEXT_##P                           \
                 : S3H_SKEW_STATE : S3H_SKEW_W(CUR), S3H_SKEW_WNEXT(NXT));                      \
  } else if constexpr (kMergeNext) {                                                            \
    if (i == kBps - 1) {                                                                        \
      S3H_SYNC_STEP(j + 1, j + 2);                                                              \
      load(NXT, nbuf);                                                                          \
    } else {                                                                                    \
      load(NXT, buf + (i + 1) * kBlkStride);                                                    \
    }                                                                                           \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_A_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_B_##P S3H_##L##_NEXT_##P                           \
                 : S3H_SKEW_STATE : S3H_SKEW_W(CUR), S3H_SKEW_WNEXT(NXT));                      \
  } else {                                                                                      \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_A_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    if (i == kBps - 1) {                                                                        \
      S3H_SYNC_STEP(j + 1, j + 2);                                                              \
      load(NXT, nbuf);                                                                          \
    } else {                                                                                    \
      load(NXT, buf + (i + 1) * kBlkStride);                                                    \
    }                                                                                           \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_B_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    asm volatile(S3H_ALIGN8 S3H_##L##_NEXT_##P                                                  \
                 : S3H_SKEW_STATE : [w0] "v"(NXT[0]), [am] "v"(am), [mk] "v"(mk));              \
  }
#define S3H_SKEW_SLOW(L, P, CUR, NXT)                                                           \
  {                                                                                             \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_A_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    const uint32_t nx = bb + 1;                                                                 \
    if (nx % kBps == 0 || nx >= it32) S3H_SYNC_STEP(nx / kBps, nx < it32 ? nx / kBps + 1 : 0u); \
    load(NXT, lbase + ((nx / kBps) & 1) * kBufStride + (nx % kBps) * kBlkStride);               \
    asm volatile(S3H_ALIGN8 S3H_##L##_ROUNDS_B_##P : S3H_SKEW_STATE : S3H_SKEW_W(CUR));         \
    if (bb >= cap_from) {                                                                       \
      asm volatile("; ragged tail: capture check");  /* keeps this branch scalar */           \
      if (nb_rel == bb) {                                                                       \
        if (P == 0) S3H_SKEW_CAPTURE(e13, e12, e11, e10, g01, g00);                             \
        else S3H_SKEW_CAPTURE(e03, e02, e01, e00, g11, g10);                                    \
      }                                                                                         \
    }                                                                                           \
    asm volatile(S3H_ALIGN8 S3H_##L##_NEXT_##P                                                  \
                 : S3H_SKEW_STATE : [w0] "v"(NXT[0]), [am] "v"(am), [mk] "v"(mk));              \
    if (nx >= it32) goto drain;                                                                 \
  }
  const uint32_t fast_end = cap_from < it32 ? cap_from : it32 - 1;  // blocks < it: no checks
  const uint32_t nfast = fast_end / kBps;                            // whole fast steps
#define S3H_SKEW_LOOPS(L)                                                                       \
  for (uint32_t j = 0; j < nfast; ++j) {                                                        \
    const uint4* buf = lbase + (j & 1) * kBufStride;                                            \
    const uint4* nbuf = lbase + ((j + 1) & 1) * kBufStride;                                     \
    _Pragma("unroll") for (uint32_t h = 0; h < kBps / 2; ++h) {                                 \
      {                                                                                         \
        const uint32_t i = 2 * h;                                                               \
        S3H_SKEW_FAST(L, 0, wa, wb)                                                             \
      }                                                                                         \
      {                                                                                         \
        const uint32_t i = 2 * h + 1;                                                           \
        S3H_SKEW_FAST(L, 1, wb, wa)                                                             \
      }                                                                                         \
    }                                                                                           \
  }                                                                                             \
  for (uint32_t bb = nfast * kBps;; bb += 2) { /* starts at an even block: parity 0 */          \
    S3H_SKEW_SLOW(L, 0, wa, wb)                                                                 \
    ++bb;                                                                                       \
    S3H_SKEW_SLOW(L, 1, wb, wa)                                                                 \
    --bb;                                                                                       \
  }
  if constexpr (PAIR) {
    S3H_SKEW_LOOPS(SKEWP)
  } else {
    S3H_SKEW_LOOPS(SKEW)
  }
drain:
  // The a-quad's last two rounds of the last block (parity (iters-1)&1) run as rounds 0-1
  // of a virtual block of the other parity (W = 1 in the a-quad); then every chain still
  // live is captured.
  {
    uint32_t wd[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) wd[i] = one_a;
    if (it32 & 1) {
      if constexpr (PAIR)
        asm volatile(S3H_ALIGN8 S3H_SKEWP_DRAIN_1 : S3H_SKEW_STATE : S3H_SKEW_W(wd));
      else
        asm volatile(S3H_ALIGN8 S3H_SKEW_DRAIN_1 : S3H_SKEW_STATE : S3H_SKEW_W(wd));
      if (nb_rel >= it32) S3H_SKEW_CAPTURE(e03, e02, e01, e00, g11, g10);
    } else {
      if constexpr (PAIR)
        asm volatile(S3H_ALIGN8 S3H_SKEWP_DRAIN_0 : S3H_SKEW_STATE : S3H_SKEW_W(wd));
      else
        asm volatile(S3H_ALIGN8 S3H_SKEW_DRAIN_0 : S3H_SKEW_STATE : S3H_SKEW_W(wd));
      if (nb_rel >= it32) S3H_SKEW_CAPTURE(e13, e12, e11, e10, g01, g00);
    }
  }
#undef S3H_SKEW_FAST
#undef S3H_SKEW_SLOW
#undef S3H_SKEW_LOOPS
#undef S3H_SKEW_CAPTURE
#undef S3H_SYNC_STEP
  if (A.clocks) {
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t* c = A.clocks + 4ull * (group * NC + role);
      c[0] = clk0; c[1] = clk1; c[2] = rt0; c[3] = rt1;
    }
  }
  if (valid && nb > b0 && (PAIR || k4 == 0)) {  // quad: one lane per quad writes its half
    const uint32_t w0 = ahalf ? 0u : 4u;
    if (emits(A, nb)) {
      uint4* o = reinterpret_cast<uint4*>(A.digests + 8ull * A.out_idx[slot] + w0);
      o[0] = make_uint4(bswap(f0), bswap(f1), bswap(f2), bswap(f3));
    } else if (A.state) {
      reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot] + w0)[0] = make_uint4(f0, f1, f2, f3);
    }
  }
}

template <int NC, bool PAIR = false>
__global__ __launch_bounds__(64 * (NC + 1)) void sha256_skew_kernel(LaunchArgs A) {
  __shared__ SkewLds<NC, PAIR> L;
  skew_body<NC, PAIR, false>(A, blockIdx.x, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L,
                             nullptr);
}

// Two independent (consumer, producer) groups per workgroup, flag-synchronised: waves 0 and 1
// consume groups 2b and 2b+1, waves 2 and 3 produce for them.  Four waves = one per SIMD, and
// neither consumer ever waits for the other (with one s_barrier for both, as in
// sha256_skew_kernel<2>, every step boundary waits for the slower of the two).
// Solo workgroups (A.solo > 0): with all four SIMDs of a CU busy each wave issues ~3 % slower
// than with two (4.18 vs 4.06 cycles/instruction), so the host gives the groups of the longest
// parts -- the ones that set the launch's time -- a workgroup (and, through a dynamic LDS pad
// that admits one workgroup per CU, a CU) of their own; see capi.hip plan_solo.
__global__ __launch_bounds__(256) void sha256_skew_pairs_kernel(LaunchArgs A) {
  __shared__ SkewLds<1, false> L[2];
  __shared__ uint32_t flags[2][2];
  if (threadIdx.x < 4) flags[threadIdx.x >> 1][threadIdx.x & 1] = 0;
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t g = wave & 1u;
  const uint32_t b = blockIdx.x;
  if (b < A.solo && g) return;  // a solo workgroup: waves 1 and 3 have no group
  skew_body<1, false, true>(A, b < A.solo ? b : A.solo + 2 * (b - A.solo) + g, wave >> 1, L[g],
                            flags[g]);
}

// Four (consumer, producer) groups per workgroup with every producer on its consumer's SIMD.
// The producer is written in the instruction classes that SIMD issues beside the round stream
// (skew_body SIMPLE), so one CU runs 32 chains at about the skew kernel's per-chain speed --
// four times the chains of sha256_skew_kernel<1> per CU, without skewp's extra VALU per round.
// Pairing by SIMD: every wave publishes its SIMD (HW_ID); on each SIMD the lower wave consumes
// and the higher one produces group = that SIMD.  The dispatcher places wave w on SIMD w % 4
// (tools/ubench_coissue*.hip), i.e. waves g and g + 4 -- the static fallback used if a
// placement ever is not two waves per SIMD.  LDS: 4 x 36 KiB = one workgroup per CU.
__global__ __launch_bounds__(512) void sha256_skew_shared_kernel(LaunchArgs A) {
  __shared__ SkewLds<1, false> L[4];
  __shared__ uint32_t flags[4][2];
  __shared__ uint32_t simd_of[8];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < 8) flags[threadIdx.x >> 1][threadIdx.x & 1] = 0;
  if ((threadIdx.x & 63u) == 0)
    simd_of[wave] = (__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3u;  // HW_REG_HW_ID.SIMD_ID
  __syncthreads();
  uint32_t per_simd[4] = {0, 0, 0, 0}, rank = 0;
  const uint32_t mine = __builtin_amdgcn_readfirstlane(simd_of[wave]);
#pragma unroll
  for (uint32_t w = 0; w < 8; ++w) {
    const uint32_t s = __builtin_amdgcn_readfirstlane(simd_of[w]);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) per_simd[k] += s == k;
    rank += (w < wave && s == mine);
  }
  const bool paired = per_simd[0] == 2 && per_simd[1] == 2 && per_simd[2] == 2 && per_simd[3] == 2;
  const uint32_t g = paired ? mine : wave & 3u;
  const uint32_t role = paired ? rank : wave >> 2;
  skew_body<1, false, true, true>(A, 4 * blockIdx.x + g, role, L[g], flags[g]);
}

// ------------------------------------------------------------- MD5 (producer/consumer)
// Batched MD5 for Content-MD5 / multipart-ETag verification (reference
// lib/hash/md5.cpp:71-116 for the step function, :158-172 for the padding).  Same
// workgroup shape as sha256_pc_kernel: the producer decodes little-endian words (one v_perm
// handles alignment), pads (64-bit LITTLE-endian bit length) and writes M[g(i)] + K[i] for
// the 64 steps to LDS; the consumer runs the chain: per step one bitop3 (F/G/H/I), one add3,
// one alignbit (rotate left) and one add.  State words are the digest words (no byte swap).

__device__ __forceinline__ void md5_tail(const uint8_t* p, uint64_t len, uint64_t bits,
                                         uint64_t blk, uint32_t w[16]) {
  const uint64_t nfull = len >> 6;
  const int rem = (blk == nfull) ? int(len & 63) : -1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = 4 * j + k;
      uint32_t byte = 0;
      if (i < rem) byte = p[i];
      else if (i == rem) byte = 0x80u;
      x |= byte << (8 * k);
    }
    w[j] = x;
  }
  if (blk == nblocks(len) - 1) {
    w[14] = uint32_t(bits);
    w[15] = uint32_t(bits >> 32);
  }
}

#define S3H_MD5_K(i) ((uint32_t)(                                                              \
  (i)==0?0xd76aa478u:(i)==1?0xe8c7b756u:(i)==2?0x242070dbu:(i)==3?0xc1bdceeeu:(i)==4?0xf57c0fafu: \
  (i)==5?0x4787c62au:(i)==6?0xa8304613u:(i)==7?0xfd469501u:(i)==8?0x698098d8u:(i)==9?0x8b44f7afu: \
  (i)==10?0xffff5bb1u:(i)==11?0x895cd7beu:(i)==12?0x6b901122u:(i)==13?0xfd987193u:              \
  (i)==14?0xa679438eu:(i)==15?0x49b40821u:(i)==16?0xf61e2562u:(i)==17?0xc040b340u:              \
  (i)==18?0x265e5a51u:(i)==19?0xe9b6c7aau:(i)==20?0xd62f105du:(i)==21?0x02441453u:              \
  (i)==22?0xd8a1e681u:(i)==23?0xe7d3fbc8u:(i)==24?0x21e1cde6u:(i)==25?0xc33707d6u:              \
  (i)==26?0xf4d50d87u:(i)==27?0x455a14edu:(i)==28?0xa9e3e905u:(i)==29?0xfcefa3f8u:              \
  (i)==30?0x676f02d9u:(i)==31?0x8d2a4c8au:(i)==32?0xfffa3942u:(i)==33?0x8771f681u:              \
  (i)==34?0x6d9d6122u:(i)==35?0xfde5380cu:(i)==36?0xa4beea44u:(i)==37?0x4bdecfa9u:              \
  (i)==38?0xf6bb4b60u:(i)==39?0xbebfbc70u:(i)==40?0x289b7ec6u:(i)==41?0xeaa127fau:              \
  (i)==42?0xd4ef3085u:(i)==43?0x04881d05u:(i)==44?0xd9d4d039u:(i)==45?0xe6db99e5u:              \
  (i)==46?0x1fa27cf8u:(i)==47?0xc4ac5665u:(i)==48?0xf4292244u:(i)==49?0x432aff97u:              \
  (i)==50?0xab9423a7u:(i)==51?0xfc93a039u:(i)==52?0x655b59c3u:(i)==53?0x8f0ccc92u:              \
  (i)==54?0xffeff47du:(i)==55?0x85845dd1u:(i)==56?0x6fa87e4fu:(i)==57?0xfe2ce6e0u:              \
  (i)==58?0xa3014314u:(i)==59?0x4e0811a1u:(i)==60?0xf7537e82u:(i)==61?0xbd3af235u:              \
  (i)==62?0x2ad7d2bbu:0xeb86d391u))

__device__ __forceinline__ constexpr int md5_g(int i) {
  return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}
__device__ __forceinline__ constexpr int md5_s(int i) {
  return i < 16 ? (i % 4 == 0 ? 7 : i % 4 == 1 ? 12 : i % 4 == 2 ? 17 : 22)
       : i < 32 ? (i % 4 == 0 ? 5 : i % 4 == 1 ? 9 : i % 4 == 2 ? 14 : 20)
       : i < 48 ? (i % 4 == 0 ? 4 : i % 4 == 1 ? 11 : i % 4 == 2 ? 16 : 23)
                : (i % 4 == 0 ? 6 : i % 4 == 1 ? 10 : i % 4 == 2 ? 15 : 21);
}

// F, G, H, I as single v_bitop3_b32 (truth table index = b<<2 | c<<1 | d): F = b?c:d (0xCA),
// G = d?b:c (0xE4), H = b^c^d (0x96), I = c^(b|~d) (0x39).  Written as builtins because the
// compiler otherwise splits F/G into disjoint and+add terms (one extra VALU per step).
template <int I>
__device__ __forceinline__ uint32_t md5_f(uint32_t b, uint32_t c, uint32_t d) {
  if constexpr (I < 16) return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
  else if constexpr (I < 32) return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE4);
  else if constexpr (I < 48) return __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
  else return __builtin_amdgcn_bitop3_b32(b, c, d, 0x39);
}

// One MD5 step in rotating names: the new b lands in `a` (a is dead after the add3).
template <int I>
__device__ __forceinline__ void md5_step(uint32_t& a, uint32_t b, uint32_t c, uint32_t d,
                                         uint32_t km) {
  const uint32_t t = a + md5_f<I>(b, c, d) + km;
  a = b + __builtin_amdgcn_alignbit(t, t, 32 - md5_s(I));
}

// The 64 steps straight from the message words (M[g(i)] + K[i] formed at each step, so no
// 64-word array is live at once: the self-fed MD5 wave keeps its register budget).
template <int I>
__device__ __forceinline__ void md5_steps_w(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                            const uint32_t w[16]) {
  if constexpr (I < 64) {
    md5_step<I>(a, b, c, d, w[md5_g(I)] + S3H_MD5_K(I));
    md5_steps_w<I + 1>(d, a, b, c, w);
  }
}

// MD5 steps in aligned 8-byte asm: every instruction 8 bytes (v_add_u32 in its VOP3
// encoding), each statement 8-byte aligned.  Step: f = F(b,c,d) (one bitop3), t = a + f +
// (M+K), t = rotl(t, s) (alignbit by 32 - s), a = b + t; the names rotate (a,b,c,d) ->
// (d,a,b,c).
#define S3H_MD5_ST(TT, A, B, C, D, K, R)                                                 \
  "v_bitop3_b32 %[f], %[" #B "], %[" #C "], %[" #D "] bitop3:" #TT "\n\t"               \
  "v_add3_u32 %[t], %[" #A "], %[f], %[" #K "]\n\t"                                     \
  "v_alignbit_b32 %[t], %[t], %[t], " #R "\n\t"                                         \
  "v_add_u32_e64 %[" #A "], %[" #B "], %[t]\n\t"
#define S3H_MD5_4(TT, K0, K1, K2, K3, R0, R1, R2, R3)                                    \
  S3H_MD5_ST(TT, a, b, c, d, K0, R0) S3H_MD5_ST(TT, d, a, b, c, K1, R1)                   \
  S3H_MD5_ST(TT, c, d, a, b, K2, R2) S3H_MD5_ST(TT, b, c, d, a, K3, R3)
// The first four steps read the block-start state s0..s3 and write fresh registers a..d, so
// the state survives for the feed-forward without four register copies.
#define S3H_MD5_ST_IO(TT, AIN, AOUT, B, C, D, K, R)                                      \
  "v_bitop3_b32 %[f], %[" #B "], %[" #C "], %[" #D "] bitop3:" #TT "\n\t"               \
  "v_add3_u32 %[t], %[" #AIN "], %[f], %[" #K "]\n\t"                                   \
  "v_alignbit_b32 %[t], %[t], %[t], " #R "\n\t"                                         \
  "v_add_u32_e64 %[" #AOUT "], %[" #B "], %[t]\n\t"

// The consumer's block with its M+K rows streamed in: five asm statements, each issuing the
// ds_read_b128 of the rows the NEXT statement needs, running its steps, and waiting for its
// reads in its last step (so its outputs are complete when it returns).  The compiler, left
// to itself, reads all 16 rows and waits for every one before the first step (it drains the
// LDS counter before an inline asm statement): 16 KiB per wave at 128 B/clk of LDS plus the
// latency exposed per block.  Statement boundaries cost an alignment s_nop whenever the
// compiler puts an odd number of 4-byte scalar instructions between two statements, so the
// block is cut into as few statements as the 30-operand limit allows: steps 0-7 | 8-23 |
// 24-39 | 40-55 | 56-63 (rows 0-1 | 2-5 | 6-9 | 10-13 | 14-15).  With kNext the fourth
// statement also reads rows 0-1 of the NEXT block (LDS byte address adn: the same producer
// step, so already published), so only a step's first block waits for rows after the barrier.
// `ad`: this lane's LDS byte address of row 0 (rows are 1,024 B apart: Md5Lds).
//
// S3H_MD5_ST_W ends a statement: its s_waitcnt (4 B) and the step's VOP2 add (4 B) keep the
// statement a multiple of 8 bytes (the reads were issued a statement earlier: nothing waits).
#define S3H_MD5_ST_W(TT, A, B, C, D, K, R)                                               \
  "v_bitop3_b32 %[f], %[" #B "], %[" #C "], %[" #D "] bitop3:" #TT "\n\t"               \
  "v_add3_u32 %[t], %[" #A "], %[f], %[" #K "]\n\t"                                     \
  "v_alignbit_b32 %[t], %[t], %[t], " #R "\n\t"                                         \
  "s_waitcnt lgkmcnt(0)\n\t"                                                            \
  "v_add_u32_e32 %[" #A "], %[" #B "], %[t]\n\t"
#define S3H_MD5_4W(TT, K0, K1, K2, K3, R0, R1, R2, R3)                                   \
  S3H_MD5_ST(TT, a, b, c, d, K0, R0) S3H_MD5_ST(TT, d, a, b, c, K1, R1)                   \
  S3H_MD5_ST(TT, c, d, a, b, K2, R2) S3H_MD5_ST_W(TT, b, c, d, a, K3, R3)
#define S3H_MD5_LD(N, ADR, OFF) "ds_read_b128 %[" #N "], %[" #ADR "] offset:" #OFF "\n\t"
#define S3H_MD5_K16(P0, P1, P2, P3)                                                       \
  [k0] "v"(P0.x), [k1] "v"(P0.y), [k2] "v"(P0.z), [k3] "v"(P0.w), [k4] "v"(P1.x),          \
      [k5] "v"(P1.y), [k6] "v"(P1.z), [k7] "v"(P1.w), [k8] "v"(P2.x), [k9] "v"(P2.y),      \
      [k10] "v"(P2.z), [k11] "v"(P2.w), [k12] "v"(P3.x), [k13] "v"(P3.y), [k14] "v"(P3.z), \
      [k15] "v"(P3.w)
#define S3H_MD5_STATE [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [f] "=&v"(f), [t] "=&v"(t)
#define S3H_MD5_NEXT4(N0, N1, N2, N3) [n0] "=&v"(N0), [n1] "=&v"(N1), [n2] "=&v"(N2), [n3] "=&v"(N3)
// 16 steps: two groups of 4 in round TT1 (rotations R*), two in TT2 (rotations Q*), the last
// step of the statement waiting for its reads
#define S3H_MD5_16(TT1, R0, R1, R2, R3, TT2, Q0, Q1, Q2, Q3)                               \
  S3H_MD5_4(TT1, k0, k1, k2, k3, R0, R1, R2, R3) S3H_MD5_4(TT1, k4, k5, k6, k7, R0, R1, R2, R3) \
  S3H_MD5_4(TT2, k8, k9, k10, k11, Q0, Q1, Q2, Q3)                                        \
  S3H_MD5_4W(TT2, k12, k13, k14, k15, Q0, Q1, Q2, Q3)
#define S3H_MD5_F 0xca, 25, 20, 15, 10  // F = b ? c : d;    s = 7, 12, 17, 22 (alignbit 32 - s)
#define S3H_MD5_G 0xe4, 27, 23, 18, 12  // G = d ? b : c;    s = 5, 9, 14, 20
#define S3H_MD5_H 0x96, 28, 21, 16, 9   // H = b ^ c ^ d;    s = 4, 11, 16, 23
#define S3H_MD5_I 0x39, 26, 22, 17, 11  // I = c ^ (b | ~d); s = 6, 10, 15, 21
#define S3H_MD5_16X(A, B) S3H_MD5_16(A, B)  // expands the round macros into arguments

template <bool kNext>
__device__ __forceinline__ void md5_block_streamed(uint32_t s0, uint32_t s1, uint32_t s2,
                                                   uint32_t s3, uint32_t& a, uint32_t& b,
                                                   uint32_t& c, uint32_t& d, v4u32 r0,
                                                   v4u32 r1, uint32_t ad, uint32_t adn,
                                                   v4u32& n0, v4u32& n1) {
  uint32_t f, t;
  v4u32 r2, r3, r4, r5, r6, r7, r8, r9, r10, r11, r12, r13, r14, r15;
  // steps 0-7 (F) from the block-start state (rows 0-1); rows 2-5 in flight
  asm volatile(S3H_ALIGN8 S3H_MD5_LD(n0, ad, 2048) S3H_MD5_LD(n1, ad, 3072)
               S3H_MD5_LD(n2, ad, 4096) S3H_MD5_LD(n3, ad, 5120)
               S3H_MD5_ST_IO(0xca, s0, a, s1, s2, s3, k0, 25)
               S3H_MD5_ST_IO(0xca, s3, d, a, s1, s2, k1, 20)
               S3H_MD5_ST_IO(0xca, s2, c, d, a, s1, k2, 15)
               S3H_MD5_ST_IO(0xca, s1, b, c, d, a, k3, 10)
               S3H_MD5_4W(0xca, k4, k5, k6, k7, 25, 20, 15, 10)
               : [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d), [f] "=&v"(f),
                 [t] "=&v"(t), S3H_MD5_NEXT4(r2, r3, r4, r5)
               : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [k0] "v"(r0.x),
                 [k1] "v"(r0.y), [k2] "v"(r0.z), [k3] "v"(r0.w), [k4] "v"(r1.x), [k5] "v"(r1.y),
                 [k6] "v"(r1.z), [k7] "v"(r1.w), [ad] "v"(ad)
               : "memory");
  // steps 8-23: F (rows 2-3), G (rows 4-5); rows 6-9 in flight
  asm volatile(S3H_ALIGN8 S3H_MD5_LD(n0, ad, 6144) S3H_MD5_LD(n1, ad, 7168)
               S3H_MD5_LD(n2, ad, 8192) S3H_MD5_LD(n3, ad, 9216)
               S3H_MD5_16X(S3H_MD5_F, S3H_MD5_G)
               : S3H_MD5_STATE, S3H_MD5_NEXT4(r6, r7, r8, r9)
               : S3H_MD5_K16(r2, r3, r4, r5), [ad] "v"(ad)
               : "memory");
  // steps 24-39: G (rows 6-7), H (rows 8-9); rows 10-13 in flight
  asm volatile(S3H_ALIGN8 S3H_MD5_LD(n0, ad, 10240) S3H_MD5_LD(n1, ad, 11264)
               S3H_MD5_LD(n2, ad, 12288) S3H_MD5_LD(n3, ad, 13312)
               S3H_MD5_16X(S3H_MD5_G, S3H_MD5_H)
               : S3H_MD5_STATE, S3H_MD5_NEXT4(r10, r11, r12, r13)
               : S3H_MD5_K16(r6, r7, r8, r9), [ad] "v"(ad)
               : "memory");
  // steps 40-55: H (rows 10-11), I (rows 12-13); rows 14-15 (+ the next block's 0-1) in flight
  if constexpr (kNext) {
    asm volatile(S3H_ALIGN8 S3H_MD5_LD(n0, ad, 14336) S3H_MD5_LD(n1, ad, 15360)
                 S3H_MD5_LD(n2, adn, 0) S3H_MD5_LD(n3, adn, 1024)
                 S3H_MD5_16X(S3H_MD5_H, S3H_MD5_I)
                 : S3H_MD5_STATE, S3H_MD5_NEXT4(r14, r15, n0, n1)
                 : S3H_MD5_K16(r10, r11, r12, r13), [ad] "v"(ad), [adn] "v"(adn)
                 : "memory");
  } else {
    asm volatile(S3H_ALIGN8 S3H_MD5_LD(n0, ad, 14336) S3H_MD5_LD(n1, ad, 15360)
                 S3H_MD5_16X(S3H_MD5_H, S3H_MD5_I)
                 : S3H_MD5_STATE, [n0] "=&v"(r14), [n1] "=&v"(r15)
                 : S3H_MD5_K16(r10, r11, r12, r13), [ad] "v"(ad)
                 : "memory");
  }
  // steps 56-63: I (rows 14-15)
  asm volatile(S3H_ALIGN8 S3H_MD5_4(0x39, k0, k1, k2, k3, 26, 22, 17, 11)
               S3H_MD5_4(0x39, k4, k5, k6, k7, 26, 22, 17, 11)
               : S3H_MD5_STATE
               : [k0] "v"(r14.x), [k1] "v"(r14.y), [k2] "v"(r14.z), [k3] "v"(r14.w),
                 [k4] "v"(r15.x), [k5] "v"(r15.y), [k6] "v"(r15.z), [k7] "v"(r15.w));
}

// The consumer's fast step: all kBps blocks of one producer step, fed forward, in ONE asm
// statement generated by tools/gen_md5.py (rows in fixed registers v[200:231] that never leave
// the statement; rows 0-1 of block 0 pinned to v[232:239], loaded after the step's barrier).
// The per-block statements above cost a wait state plus an alignment s_nop at each of their
// boundaries; this has one boundary per step.  `ad`: row 0 of block 0 of the step's buffer.
// Not for kBps = 1 (md5_pc_kernel<1>, several workgroups per CU): the fixed registers would
// raise its 128 VGPRs to 240 and cost it occupancy.
#ifdef S3H_EXP_MD5_INC  // experiment builds: another generated schedule (tools/gen_md5.py)
#include S3H_EXP_MD5_INC
#else
#include "md5_step_asm.inc"
#endif
#define S3H_MD5_STEP_OPERANDS                                                                 \
  : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [a] "=&v"(a), [b] "=&v"(b),   \
    [c] "=&v"(c), [d] "=&v"(d), [f] "=&v"(f), [t] "=&v"(t), "+{v[232:235]}"(r0),              \
    "+{v[236:239]}"(r1)                                                                       \
  : [ad] "v"(ad)                                                                              \
  : S3H_MD5_STEP_CLOBBERS, "memory"
template <int kBps>
__device__ __forceinline__ void md5_step_fused(uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                               uint32_t& s3, v4u32& r0, v4u32& r1, uint32_t ad) {
  uint32_t a, b, c, d, f, t;
  static_assert(kBps == 2 || kBps == 4, "fused MD5 steps are generated for 2 and 4 blocks");
  if constexpr (kBps == 4)
    asm volatile(S3H_ALIGN8 S3H_MD5_STEP_ASM_4 S3H_MD5_STEP_OPERANDS);
  else
    asm volatile(S3H_ALIGN8 S3H_MD5_STEP_ASM_2 S3H_MD5_STEP_OPERANDS);
}
#undef S3H_MD5_STEP_OPERANDS

// The rolling form of the fused step (tools/gen_md5.py roll_text, round 3): the statement reads
// every row itself, ROLL_DEPTH rows ahead into a ring of fixed registers, with counted waits
// every 4 rows -- no row read has less than ~20 steps to land, block boundaries included.
template <int kBps>
__device__ __forceinline__ void md5_step_roll(uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                              uint32_t& s3, uint32_t ad) {
  uint32_t a, b, c, d, f, t;
  static_assert(kBps == 2 || kBps == 4, "rolling MD5 steps are generated for 2 and 4 blocks");
#define S3H_MD5_ROLL_OPERANDS                                                                 \
  : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [a] "=&v"(a), [b] "=&v"(b),   \
    [c] "=&v"(c), [d] "=&v"(d), [f] "=&v"(f), [t] "=&v"(t)                                    \
  : [ad] "v"(ad)                                                                              \
  : S3H_MD5_ROLL_CLOBBERS, "memory"
#ifndef S3H_MD5_VMEM  // (the VMEM experiment's statements take other operands)
  if constexpr (kBps == 4)
    asm volatile(S3H_ALIGN8 S3H_MD5_ROLL_ASM_4 S3H_MD5_ROLL_OPERANDS);
  else
    asm volatile(S3H_ALIGN8 S3H_MD5_ROLL_ASM_2 S3H_MD5_ROLL_OPERANDS);
#endif
#undef S3H_MD5_ROLL_OPERANDS
}

#ifdef S3H_MD5_VMEM  // experiment (timing only; tools/gen_md5.py S3H_GEN_EXP=vmem): rows from L2
__device__ __forceinline__ void md5_step_vmem(uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                              uint32_t& s3, uint32_t voff, const uint8_t* region) {
  uint32_t a, b, c, d, f, t;
  const uint64_t r = uint64_t(reinterpret_cast<uintptr_t>(region));
#define S3H_SB(k) [sb##k] "s"(r + (k) * 4096ull)
  asm volatile(S3H_ALIGN8 S3H_MD5_ROLL_ASM_4
               : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [a] "=&v"(a),
                 [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d), [f] "=&v"(f), [t] "=&v"(t)
               : [voff] "v"(voff), S3H_SB(0), S3H_SB(1), S3H_SB(2), S3H_SB(3), S3H_SB(4),
                 S3H_SB(5), S3H_SB(6), S3H_SB(7), S3H_SB(8), S3H_SB(9), S3H_SB(10), S3H_SB(11),
                 S3H_SB(12), S3H_SB(13), S3H_SB(14), S3H_SB(15)
               : S3H_MD5_ROLL_CLOBBERS, "memory");
#undef S3H_SB
}
#endif

// Decoded message words of MD5 block `blk` (zeros at or past `limit` -- the launch's range or
// the lane's last block -- padding at the end).
__device__ __forceinline__ void md5_decode(const RawBlock& r, uint32_t sel, const uint8_t* bp,
                                           uint64_t len, uint64_t bits, uint64_t blk,
                                           uint64_t limit, uint32_t w[16]) {
  if (blk >= limit) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = 0;
  } else if (blk < (len >> 6)) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(r.d[j + 1], r.d[j], sel);
  } else {
    md5_tail(bp, len, bits, blk, w);
  }
}

// Rows Q.. of M[g(i)] + K[i] written to LDS, unrolled by recursion (a #pragma unroll over the
// 64 words was left rolled -- dynamic register indexing and a scratch array -- once the
// multi-block producer's loop grew past the unroller's budget).
template <int Q>
__device__ __forceinline__ void md5_km_rows(const uint32_t w[16], uint4 (*buf)[64], uint32_t lane) {
  if constexpr (Q < 16) {
    buf[Q][lane] = make_uint4(w[md5_g(4 * Q)] + S3H_MD5_K(4 * Q),
                              w[md5_g(4 * Q + 1)] + S3H_MD5_K(4 * Q + 1),
                              w[md5_g(4 * Q + 2)] + S3H_MD5_K(4 * Q + 2),
                              w[md5_g(4 * Q + 3)] + S3H_MD5_K(4 * Q + 3));
    md5_km_rows<Q + 1>(w, buf, lane);
  }
}

// kFull: the block is known to be a whole data block of every lane's part (the producer's
// fast steps), so only the v_perm decode is emitted -- not the padding path's 64 predicated
// byte loads, which, inlined at every unrolled produce site, made the multi-block producer's
// loop the bulk of the kernel's code.
template <bool kFull = false>
__device__ __forceinline__ void md5_produce(const RawBlock& r, uint32_t sel, const uint8_t* bp,
                                            uint64_t len, uint64_t bits, uint64_t blk,
                                            uint64_t limit, uint4 (*buf)[64], uint32_t lane) {
  uint32_t w[16];
  if constexpr (kFull) {
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(r.d[j + 1], r.d[j], sel);
  } else {
    md5_decode(r, sel, bp, len, bits, blk, limit, w);
  }
  md5_km_rows<0>(w, buf, lane);
}

// Self-fed MD5: one wave, one lane per chain (kChains <= 64, slots group*kChains...), each lane
// loads, decodes and hashes its own blocks -- no producer wave, no LDS, no synchronisation.
// ~350 instructions per block (64 M+K adds + 16 byte-order perms on top of the 4-VALU steps),
// i.e. well under a SHA-256 skew/skewp chain's 544-609, so it keeps pace with the SHA-256
// group it shares a workgroup with (sha256_md5_group_kernel).  Loads run kDepth blocks ahead
// (an MD5 block is ~0.6 us of chain time; HBM latency under a full-chip load is several).
//
// Paced (kPaceBps > 0, `pace` = the workgroup's SHA-256 producer step counter flags[0]): the
// SHA-256 group beside this wave reads the same parts, kPaceBps blocks per producer step, and
// issues a step's loads before it publishes the step.  Unpaced, the MD5 chain (~1.8x faster)
// ran ahead and both chains read every byte from HBM (C3 dual: 2.0017x the algorithmic bytes,
// profiles/r04_c3_dual_mixed_counters.json).  Paced, block B is fetched only once the producer
// has published step B / kPaceBps, i.e. after its own load of B was issued, microseconds
// earlier on the same CU: the MD5 read hits the CU's L1 or L2.  Pacing is a cache policy, not
// a dependency -- the MD5 digests never read the producer's output -- so a wait longer than
// kPaceWaitTicks just stops pacing for the rest of the launch.
//
// kXcd (experiment S3H_EXP_MD5_XCD_PACE; MD5 chains of skew groups that run on OTHER
// workgroups: the mixed grid's apart MD5 workgroups, the split grid's MD5 workgroups):
// workgroups b and b + 8 share an XCD (and its L2; MI355X_MICROARCH.md "Workgroup dispatch",
// tools/xcd_probe.hip), so an MD5 workgroup takes the skew groups of its own class
// blockIdx.x (mod 8) -- XcdChains -- and follows their producers' step counts in global
// memory (ShaPacer, skew_body GPROG).

// s_memrealtime ticks (100 MHz): 200 us, ~20-30 producer steps -- a producer that is not
// running (a shared device, the forced-stall build) turns pacing off instead of stalling MD5.
constexpr uint64_t kPaceWaitTicks = 20000;

// Where skew group g's producer step count lives in the progress array: the groups of one
// XCD class side by side, so the eight an MD5 wave follows share one 64-byte line (one L2
// read per poll).  < kProgressSlots (plan.cpp) for g < 1,024.
__device__ __forceinline__ uint32_t xcd_progress_slot(uint32_t g) { return (g & 7u) * 128u + (g >> 3); }

// Chains of an MD5 wave in XCD-class order: chain c = c0 + i (c0 = 64 x the wave's index among
// its class's waves) is part c % 8 of skew group g = xcls + 8 (c / 8), slot 8g + c % 8, over
// `ngroups` skew groups of 8 slots and `n` slots.  Slots ascend with i, so lane 0 holds the
// wave's longest part and its last valid lane the shortest, as in a contiguous group.
struct XcdChains {
  uint32_t xcls, c0, ngroups, n;
  __device__ uint32_t slot_of(uint32_t i) const {
    const uint32_t c = c0 + i;
    return 8u * (xcls + 8u * (c >> 3)) + (c & 7u);
  }
  __device__ uint32_t count() const {  // valid chains (a prefix of the lanes)
    const uint32_t in_cls = ngroups > xcls ? (ngroups - xcls + 7u) / 8u : 0u;
    const uint32_t first = c0 >> 3;
    if (in_cls <= first) return 0;
    const uint32_t k = in_cls - first < 8u ? in_cls - first : 8u;  // this wave's skew groups
    const uint32_t end = slot_of(8u * k - 1u) + 1u;                 // the last group may be partial
    return end <= n ? 8u * k : 8u * k - (end - n);
  }
};

// Waits, before the MD5 wave fetches block b0 + B, until the SHA-256 producer(s) of the same
// parts have published step B / kPaceBps (their loads of B are then issued).  LDS form: the
// workgroup's own producer counter; global form (kGlobal): the minimum over the wave's skew
// groups of gprog[group] = (epoch << 32 | steps), another launch's epoch reading as 0, over
// the lanes that still fetch data of their own part (B < `data_end`, blocks past b0): a lane
// whose part has ended -- or whose group has nothing in this launch's range -- waits for no
// producer (its group's producer stops publishing once the group's longest part ends).
template <uint32_t kPaceBps, bool kGlobal>
struct ShaPacer {
  const uint32_t* lds;
  const uint64_t* gprog;
  uint32_t epoch, group;  // global form: this lane's skew group (ignored where !valid)
  bool valid;
  uint64_t data_end;  // global form: this lane's part's blocks of data past b0
  uint32_t seen = 0;  // wave-uniform: the last step count read
  bool on = kPaceBps != 0;
  __device__ __forceinline__ void wait_for(uint64_t B) {
    if constexpr (kPaceBps != 0) {
      if (!on) return;
      const uint32_t need = (B < 2 * kPaceBps ? 1u : uint32_t(B / kPaceBps)) + S3H_EXP_PACE_LAG;
      uint64_t t0 = 0;
      while (seen < need) {
        if constexpr (kGlobal) {
          // the slowest of this wave's skew groups (a poll only happens when the wave has
          // caught up with them; its wait for the wave's own loads is then no extra stall)
          uint32_t m = 0xffffffffu;
          if (valid && B < data_end) {
            // agent scope: L2-served (no stale L1 line); the producer is on this XCD
            const uint64_t v = __hip_atomic_load(gprog + xcd_progress_slot(group), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            m = uint32_t(v >> 32) == epoch ? uint32_t(v) : 0u;
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            const uint32_t t = __shfl_xor(m, o);
            m = t < m ? t : m;
          }
          seen = __builtin_amdgcn_readfirstlane(m);
        } else {
          seen = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(lds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        }
        if (seen >= need) break;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) {
          t0 = now;
        } else if (now - t0 > kPaceWaitTicks) {
          on = false;
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
};

template <uint32_t kChains, uint32_t kPaceBps = 0, bool kXcd = false>
__device__ __forceinline__ void md5_self_body(const LaunchArgs& A, const uint32_t group,
                                              const uint32_t* pace = nullptr,
                                              const uint64_t* gprog = nullptr, uint32_t epoch = 0,
                                              uint32_t nskew = 0) {
  static_assert(!kXcd || (kChains == 64 && kPaceBps != 0), "XCD-class MD5 waves: 64 paced chains");
  const uint32_t lane = threadIdx.x & 63u;
  // chains of this wave: slot_of(i) for i < nvalid, ascending in i
  const XcdChains xc = {blockIdx.x & 7u, 64u * (group >> 3), nskew, A.n};
  auto slot_of = [&](uint32_t i) -> uint32_t {
    if constexpr (kXcd) return xc.slot_of(i);
    else return group * kChains + i;
  };
  uint32_t nvalid;
  if constexpr (kXcd) {
    nvalid = xc.count();
  } else {
    const uint32_t slot0 = group * kChains;
    nvalid = slot0 >= A.n ? 0u : (A.n - slot0 < kChains ? A.n - slot0 : kChains);
  }
  if (nvalid == 0) return;
  const uint32_t slot0 = slot_of(0);
  const bool valid = lane < nvalid;
  const uint32_t slot = valid ? slot_of(lane) : slot0;
  Slot s = {0, 0};
  if (valid) s = A.slots[slot];
  const uint64_t nb = valid ? slot_blocks(A, s.len) : 0;
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  const uint64_t b0 = A.blk_begin;
  if (wg_end <= b0) return;
  const uint64_t iters = wg_end - b0;
  const uint8_t* p = A.base + s.off + 64ull * (b0 - A.blk_origin);
  const uint32_t sel = le_selector(uint32_t(reinterpret_cast<uintptr_t>(p) & 3));
  const uint64_t fend = fetch_end(s.len, A.blk_end);
  const uint64_t bits = valid ? msg_bits(A, slot, s.len) : 0;
  __builtin_amdgcn_s_setprio(3);
  uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  if (valid && resumes(A)) {
    const uint4 v = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot])[0];
    st[0] = v.x; st[1] = v.y; st[2] = v.z; st[3] = v.w;
  }
  // ring[k % kRing] holds block k's raw bytes; block k + kDepth is fetched while block k is
  // hashed (the loops are unrolled by kRing so every ring index is a compile-time constant).
  // Blocks below every lane's first partial block (slots are sorted by length: the group's
  // last slot is the shortest) take the branch-free fast loop -- decode is one v_perm per
  // word -- so the compiler keeps counted vmcnt waits; the padding blocks at the end run the
  // general decode (its byte loads would otherwise force a full vmcnt drain every block).
  constexpr uint32_t kDepth = S3H_EXP_MD5_SELF_DEPTH, kRing = kDepth + 1;
  const uint32_t last = slot_of(nvalid - 1);
  const uint64_t full_end = (A.slots[last].len >> 6) < A.blk_end ? (A.slots[last].len >> 6) : A.blk_end;
  const uint64_t nfast = full_end > b0 ? (full_end - b0) / kRing * kRing : 0;  // whole rings
  RawBlock ring[kRing];
  ShaPacer<kPaceBps, kXcd> pacer = {pace, gprog, epoch, slot >> 3, valid, fend > b0 ? fend - b0 : 0};
  auto pace_to = [&](uint64_t B) {  // before fetching block b0 + B
    if (B < iters) pacer.wait_for(B);  // past the range: the zero page, nothing to share
  };
#pragma unroll
  for (uint32_t k = 0; k < kDepth; ++k) {
    pace_to(k);
    fetch_full(p + 64 * k, b0 + k < fend, A.zero, ring[k]);
  }
  auto hash_words = [&](const uint32_t w[16], uint64_t J) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    md5_steps_w<0>(a, b, c, d, w);
    const bool live = b0 + J < nb;
    st[0] = live ? st[0] + a : st[0];
    st[1] = live ? st[1] + b : st[1];
    st[2] = live ? st[2] + c : st[2];
    st[3] = live ? st[3] + d : st[3];
  };
  for (uint64_t j = 0; j < nfast; j += kRing) {
#pragma unroll
    for (uint32_t u = 0; u < kRing; ++u) {
      const uint64_t J = j + u;
      pace_to(J + kDepth);
      fetch_full(p + 64 * (J + kDepth), b0 + J + kDepth < fend, A.zero, ring[(u + kDepth) % kRing]);
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_perm(ring[u].d[k + 1], ring[u].d[k], sel);
      hash_words(w, J);
    }
  }
  for (uint64_t j = nfast;; j += kRing) {
#pragma unroll
    for (uint32_t u = 0; u < kRing; ++u) {
      const uint64_t J = j + u;
      if (J >= iters) goto md5_done;
      pace_to(J + kDepth);
      fetch_full(p + 64 * (J + kDepth), b0 + J + kDepth < fend, A.zero, ring[(u + kDepth) % kRing]);
      uint32_t w[16];
      md5_decode(ring[u], sel, p + 64 * J, decode_len(valid, s.len), bits, b0 + J,
                 nb < A.blk_end ? nb : A.blk_end, w);  // past the lane's last block: zeros
      hash_words(w, J);
    }
  }
md5_done:
  if (valid && nb > b0) {
    if (emits(A, nb))
      reinterpret_cast<uint4*>(A.digests + 4ull * A.out_idx[slot])[0] =
          make_uint4(st[0], st[1], st[2], st[3]);
    else if (A.state)
      reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot])[0] =
          make_uint4(st[0], st[1], st[2], st[3]);
  }
}

// MD5 group: one consumer wave (role 0) and one producer wave (role 1) over 64 chains (one
// lane each; slots group*64...).  The producer writes kBps blocks' M+K rows per step into one
// of two LDS buffers; one s_barrier per step.  Round 2 synchronised every block: the
// consumer's loop trip (a taken branch), the barrier and the first rows' LDS read cost ~150
// cycles per 1,200-cycle block on top of the 4-cycle issue of its 289 instructions
// (profiles/r03_exp_md5_rows.jsonl; a dependent MD5 step chain itself issues at 4.02 cycles
// per instruction, profiles/r03_ubench_dep.txt).  Now the consumer runs a step's blocks
// back to back, each block's last asm statement reading the next block's first rows.
template <int kBps>
struct Md5Lds {
  uint4 km[2][kBps][16][64];  // [buffer][block of the step][row][lane]: kBps x 32 KiB
};

// Experiments (timing only, wrong digests): S3H_EXP_MD5_NOSYNC drops every barrier of both
// waves (consumer speed with the producer's LDS traffic beside it but no waiting for it);
// S3H_EXP_MD5_NOPROD also removes the producer (the consumer alone).
#if defined(S3H_EXP_MD5_NOSYNC) || defined(S3H_EXP_MD5_NOPROD)
#define S3H_MD5_SYNC() ((void)0)
#else
#define S3H_MD5_SYNC() __syncthreads()
#endif
// kXcd (the split dual grid, sha256_md5_dual_kernel): the workgroup's 64 chains are those of
// the skew groups on its own XCD (XcdChains over `ngroups` groups), and the producer fetches a
// step only once those groups' producers have fetched it (ShaPacer, global form) -- one HBM
// read of every part for both digests.
template <int kBps, bool kXcd = false>
__device__ __forceinline__ void md5_pc_body(const LaunchArgs& A, const uint32_t group,
                                            const uint32_t role, Md5Lds<kBps>& L,
                                            const uint64_t* gprog = nullptr, uint32_t epoch = 0,
                                            uint32_t ngroups = 0) {
  auto& lds_km = L.km;
  const uint32_t lane = threadIdx.x & 63u;
  const XcdChains xc = {blockIdx.x & 7u, 64u * (group >> 3), ngroups, A.n};
  uint32_t slot0, slot;  // the first chain's and this lane's slot
  bool valid;
  if constexpr (kXcd) {
    const uint32_t nvalid = xc.count();
    if (nvalid == 0) return;  // uniform across the workgroup: both waves leave before any barrier
    slot0 = xc.slot_of(0);
    valid = lane < nvalid;
    slot = valid ? xc.slot_of(lane) : slot0;
  } else {
    slot0 = group * 64u;
    slot = slot0 + lane;
    valid = slot < A.n;
  }
  auto last_slot = [&]() -> uint32_t {  // the last valid chain's slot (the shortest part)
    if constexpr (kXcd) return xc.slot_of(xc.count() - 1);
    else return (slot0 + 64u <= A.n ? slot0 + 64u : A.n) - 1;
  };
  Slot s = {0, 0};
  if (valid) s = A.slots[slot];
  const uint64_t nb = valid ? slot_blocks(A, s.len) : 0;
  const uint64_t wg_nb = slot_blocks(A, A.slots[slot0].len);
  const uint64_t wg_end = wg_nb < A.blk_end ? wg_nb : A.blk_end;
  if (wg_end <= A.blk_begin) return;
  const uint64_t iters = wg_end - A.blk_begin;
  const uint64_t nsteps = (iters + kBps - 1) / kBps;  // the same in both waves: equal barriers

#ifdef S3H_EXP_MD5_NOPROD  // experiment (timing only, wrong digests): no producer at all
  if (role == 1) return;
#endif
  if (role == 1) {
    // Step k's blocks are fetched one step (kBps blocks, ~5 us of chain time) before they are
    // decoded: two named register sets alternate (no dynamic indexing -> no scratch).
    const uint64_t b0 = A.blk_begin;
    const uint8_t* p = A.base + s.off + 64ull * (b0 - A.blk_origin);
    const uint32_t sel = le_selector(uint32_t(reinterpret_cast<uintptr_t>(p) & 3));
    const uint64_t fend = fetch_end(s.len, A.blk_end);
    const uint64_t bits = valid ? msg_bits(A, slot, s.len) : 0;
    const uint64_t dl = decode_len(valid, s.len);
    // Blocks past this lane's last one (its padding included) are never consumed (the consumer
    // keeps only live chains' sums): decoded as zeros, like blocks past the launch's range.
    // Without this a ragged group's lanes that had finished took md5_decode's tail branch --
    // 64 predicated byte loads -- for every block after the shortest part's end, and the whole
    // wave ran it (MD5 of 300 parts of U[1, 16] MiB: 1.85x the longest chain's time).
    const uint64_t lim = nb < A.blk_end ? nb : A.blk_end;
    RawBlock ra[kBps], rb[kBps];
    ShaPacer<kXcd ? SkewGeom<1, false>::kBps : 0, true> pacer = {nullptr, gprog, epoch, slot >> 3, valid,
                                                                 fend > b0 ? fend - b0 : 0};
    // kXcd: step K's last block, once the skew producers have fetched it
#define S3H_MD5_FETCH(R, K)                                                                  \
    if constexpr (kXcd) {                                                                    \
      if (uint64_t(K) * kBps < iters)                                                        \
        pacer.wait_for(uint64_t(K) * kBps + kBps - 1 < iters ? uint64_t(K) * kBps + kBps - 1 \
                                                             : iters - 1);                   \
    }                                                                                        \
    _Pragma("unroll") for (int h = 0; h < kBps; ++h)                                        \
      fetch_full(p + 64 * ((K) * kBps + h), b0 + (K) * kBps + h < fend, A.zero, R[h]);
#define S3H_MD5_MAKE_T(R, K, FULL)                                                           \
    _Pragma("unroll") for (int h = 0; h < kBps; ++h)                                        \
      md5_produce<FULL>(R[h], sel, p + 64 * ((K) * kBps + h), dl, bits, b0 + (K) * kBps + h, \
                        lim, lds_km[(K) & 1][h], lane);
#define S3H_MD5_MAKE(R, K) S3H_MD5_MAKE_T(R, K, false)
    // Steps below `full_steps` hold whole data blocks of every lane's part (slots are sorted
    // by length; the group's last valid slot is the shortest; lanes past n decode_len past
    // everything): a compact loop with the perm-only decode runs them in pairs.
    const uint32_t lastv = last_slot();
    const uint64_t fabs = A.slots[lastv].len >> 6 < A.blk_end ? A.slots[lastv].len >> 6 : A.blk_end;
    const uint64_t full_steps = fabs > b0 ? (fabs - b0) / kBps : 0;
    // Register sets of raw blocks in flight: with 4-block steps (md5_pc_kernel<4>) two sets --
    // loads one step (~2 us of chain time) ahead -- hide the loads: three measured no faster
    // (C2 114.2-114.6 vs 114.4-114.7 GiB/s, C4 shard 811 vs 815; r03_exp_md5_roll.jsonl).
    // With 1-block steps (md5_pc_kernel<1>, grids beyond one workgroup per CU) one step of
    // lead is one block (~0.5 us), less than an HBM miss under load: three sets (two blocks
    // ahead) ran 20,480 x 256 KiB at 1,615.5 GiB/s against 1,435.0 with two
    // (profiles/r04_exp_md5_psets.jsonl).
    constexpr int kSets = kBps == 1 ? S3H_EXP_MD5_PSETS1 : S3H_EXP_MD5_PSETS;
    if constexpr (kSets == 3) {
    RawBlock rc[kBps];
    S3H_MD5_FETCH(ra, 0)
    S3H_MD5_FETCH(rb, 1)
    S3H_MD5_FETCH(rc, 2)
    S3H_MD5_MAKE(ra, 0)
    S3H_MD5_SYNC();
    uint64_t k = 1;  // step s lives in set s % 3: ra, rb, rc
    for (; k + 2 < full_steps; k += 3) {  // steps k, k + 1, k + 2: whole blocks
      S3H_MD5_FETCH(ra, k + 2)
      S3H_MD5_MAKE_T(rb, k, true)
      S3H_MD5_SYNC();
      S3H_MD5_FETCH(rb, k + 3)
      S3H_MD5_MAKE_T(rc, k + 1, true)
      S3H_MD5_SYNC();
      S3H_MD5_FETCH(rc, k + 4)
      S3H_MD5_MAKE_T(ra, k + 2, true)
      S3H_MD5_SYNC();
    }
    // k = 1 (mod 3): the same set roles.  One barrier per step k = 1 .. nsteps, as the
    // consumer's (one after each of its nsteps steps, the first after its state load).
    for (;; k += 3) {
      if (k < nsteps) {
        S3H_MD5_FETCH(ra, k + 2)
        S3H_MD5_MAKE(rb, k)
      }
      S3H_MD5_SYNC();
      if (k + 1 > nsteps) break;
      if (k + 1 < nsteps) {
        S3H_MD5_FETCH(rb, k + 3)
        S3H_MD5_MAKE(rc, k + 1)
      }
      S3H_MD5_SYNC();
      if (k + 2 > nsteps) break;
      if (k + 2 < nsteps) {
        S3H_MD5_FETCH(rc, k + 4)
        S3H_MD5_MAKE(ra, k + 2)
      }
      S3H_MD5_SYNC();
      if (k + 3 > nsteps) break;
    }
    } else {
    S3H_MD5_FETCH(ra, 0)
    S3H_MD5_FETCH(rb, 1)
    S3H_MD5_MAKE(ra, 0)
    S3H_MD5_SYNC();
    uint64_t k = 1;
    for (; k + 1 < full_steps; k += 2) {  // steps k and k + 1: whole blocks, both produced
      S3H_MD5_FETCH(ra, k + 1)
      S3H_MD5_MAKE_T(rb, k, true)
      S3H_MD5_SYNC();
      S3H_MD5_FETCH(rb, k + 2)
      S3H_MD5_MAKE_T(ra, k + 1, true)
      S3H_MD5_SYNC();
    }
    for (;; k += 2) {  // k odd: the same register roles as the loop above
      if (k < nsteps) {
        S3H_MD5_FETCH(ra, k + 1)
        S3H_MD5_MAKE(rb, k)
      }
      S3H_MD5_SYNC();
      if (k + 1 > nsteps) break;
      if (k + 1 < nsteps) {
        S3H_MD5_FETCH(rb, k + 2)
        S3H_MD5_MAKE(ra, k + 1)
      }
      S3H_MD5_SYNC();
      if (k + 2 > nsteps) break;
    }
    }
#undef S3H_MD5_FETCH
#undef S3H_MD5_MAKE
#undef S3H_MD5_MAKE_T
  } else {
    __builtin_amdgcn_s_setprio(3);
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (valid && resumes(A)) {
      const uint4 v = reinterpret_cast<const uint4*>(A.state + 8ull * A.out_idx[slot])[0];
      st[0] = v.x; st[1] = v.y; st[2] = v.z; st[3] = v.w;
    }
    S3H_MD5_SYNC();
    // slots are sorted by length: every chain of the group is live below the last one's end
    const uint32_t last = last_slot();
    const uint64_t live_end = slot_blocks(A, A.slots[last].len);
    uint64_t clk0 = 0, rt0 = 0;  // clock probe (s3h_plan_set_clock_probe), as in skew_body
    if (A.clocks) {
      clk0 = __builtin_amdgcn_s_memtime();
      rt0 = __builtin_amdgcn_s_memrealtime();
    }
    typedef __attribute__((address_space(3))) uint4 lds_u4;
    auto row_addr = [&](uint32_t buf, int h) {
      return uint32_t(reinterpret_cast<uintptr_t>((const lds_u4*)&lds_km[buf][h][0][lane]));
    };
    // One step: its kBps blocks back to back (`check`: only the chains still live are fed
    // forward, and blocks past the launch's range are skipped), then the step's barrier.
    // Steps whose every block lies below live_end -- every chain live -- run in their own loop
    // with no test (the loop tools/isa_counts.py counts); the ragged tail pays the selects.
    auto step = [&](uint64_t j, bool check) {
      const uint32_t buf = uint32_t(j & 1);
#ifdef S3H_MD5_VMEM
      if (kBps == 4 && !check) {  // timing only: rows from a 64 KiB region per workgroup
        md5_step_vmem(st[0], st[1], st[2], st[3], lane * 16u, A.base + 65536ull * group);
        S3H_MD5_SYNC();
        return;
      }
#endif
#if S3H_EXP_MD5_ROLL
      if (kBps > 1 && !check) {
        md5_step_roll<(kBps > 1 ? kBps : 2)>(st[0], st[1], st[2], st[3], row_addr(buf, 0));
        S3H_MD5_SYNC();
        return;
      }
#endif
      v4u32 r0 = *reinterpret_cast<const v4u32*>(&lds_km[buf][0][0][lane]);
      v4u32 r1 = *reinterpret_cast<const v4u32*>(&lds_km[buf][0][1][lane]);
#ifdef S3H_EXP_MD5_NOFUSE  // experiment: the per-block statements in the fast loop too
      if (false) {
#else
      if (kBps > 1 && !check) {
#endif
        md5_step_fused<(kBps > 1 ? kBps : 2)>(st[0], st[1], st[2], st[3], r0, r1, row_addr(buf, 0));
        S3H_MD5_SYNC();
        return;
      }
#pragma unroll
      for (int h = 0; h < kBps; ++h) {
        const uint64_t i = j * kBps + h;
        if (check && i >= iters) break;  // uniform: the launch's last step may be partial
        v4u32 n0, n1;
        uint32_t a, b, c, d;
        if (h + 1 < kBps)
          md5_block_streamed<true>(st[0], st[1], st[2], st[3], a, b, c, d, r0, r1,
                                   row_addr(buf, h), row_addr(buf, h + 1), n0, n1);
        else
          md5_block_streamed<false>(st[0], st[1], st[2], st[3], a, b, c, d, r0, r1,
                                    row_addr(buf, h), 0u, n0, n1);
        if (!check) {
          st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        } else {
          const bool live = (A.blk_begin + i) < nb;
          st[0] = live ? st[0] + a : st[0];
          st[1] = live ? st[1] + b : st[1];
          st[2] = live ? st[2] + c : st[2];
          st[3] = live ? st[3] + d : st[3];
        }
        r0 = n0;
        r1 = n1;
      }
      S3H_MD5_SYNC();
    };
    const uint64_t fast = live_end > A.blk_begin ? (live_end - A.blk_begin < iters
                                                    ? live_end - A.blk_begin : iters) : 0;
    uint64_t j = 0;
    for (; j < fast / kBps; ++j) step(j, false);
    for (; j < nsteps; ++j) step(j, true);
    if (A.clocks) {
      const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) {
        uint64_t* c = A.clocks + 4ull * group;
        c[0] = clk0; c[1] = clk1; c[2] = rt0; c[3] = rt1;
      }
    }
    if (valid && nb > A.blk_begin) {
      if (emits(A, nb))
        reinterpret_cast<uint4*>(A.digests + 4ull * A.out_idx[slot])[0] =
            make_uint4(st[0], st[1], st[2], st[3]);
      else if (A.state)
        reinterpret_cast<uint4*>(A.state + 8ull * A.out_idx[slot])[0] =
            make_uint4(st[0], st[1], st[2], st[3]);
    }
  }
}

// kBps = kMd5Bps (128 KiB of LDS: one workgroup per CU) while the grid fits one workgroup per
// CU (<= 64 x CUs parts); kBps = 1 (32 KiB, several per CU) for larger batches (capi.hip).
template <int kBps>
__global__ __launch_bounds__(kPcThreads) void md5_pc_kernel(LaunchArgs A) {
  __shared__ Md5Lds<kBps> L;
  md5_pc_body<kBps>(A, blockIdx.x, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L);
}

// ------------------------------------------------------------- dual digest (SHA-256 + MD5)
// x-amz-content-sha256 AND Content-MD5 of the same parts in one grid.
//
// sha256_md5_dual_kernel: workgroups [0, sha_grid) run the skew SHA-256 body (PAIR: skewp),
// the rest the MD5 body (128-thread workgroups each).  Two separate concurrent launches let
// the dispatcher stack MD5 workgroups onto CUs already running SHA-256 ones, where the two
// consumers share a SIMD's issue and both chains slow ~1.4-2.2x (kernel trace,
// profiles/r01_dual_kernel_trace.txt); one grid of <= 256 workgroups is placed one per CU
// (profiles/r01_placement.txt).  Used while sha_grid + md5_grid <= #CUs (skew, <= 2,048 parts).
static_assert(kPcThreads == 128, "dual kernel assumes 128-thread MD5 workgroups");
// Experiment S3H_EXP_MD5_XCD_PACE (kernel_abi.hpp kMd5XcdPace): the MD5 workgroups take the
// chains of the skew groups on their own XCD and fetch each step after those groups' producers
// have (md5_pc_body kXcd; the producers store their step counts to `progress`, tagged with
// `epoch`), so C2's parts are read from HBM about once for both digests -- measured 0.3 %
// slower, not the product.  Product: MD5 slots 64w.. per workgroup, unpaced.
template <bool PAIR>
__global__ __launch_bounds__(128) void sha256_md5_dual_kernel(LaunchArgs S, LaunchArgs M,
                                                              uint32_t sha_grid, uint64_t* progress,
                                                              uint32_t epoch) {
  __shared__ SkewLds<1, PAIR> LS;
  __shared__ Md5Lds<2> LM;  // 64 KiB beside the skew group's 36 KiB
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr bool kPaced = kMd5XcdPace && !PAIR;  // XcdChains assumes 8-part skew groups
  if (blockIdx.x < sha_grid)
    skew_body<1, PAIR, false, false, kPaced>(S, blockIdx.x, wave, LS, nullptr,
                                             progress ? progress + xcd_progress_slot(blockIdx.x) : nullptr,
                                             epoch);
  else
    md5_pc_body<2, kPaced>(M, blockIdx.x - sha_grid, wave, LM, progress, epoch, sha_grid);
}

// sha256_md5_group_kernel: every workgroup holds BOTH digests of the same kParts parts -- a
// SHA-256 group (wave 0 consumes, wave 2 produces, flag-synchronised) and a self-fed MD5 wave
// (wave 1, md5_self_body).  Three waves, one per SIMD: the MD5 chain runs on its own SIMD
// beside the SHA-256 chain, so a grid of <= 256 workgroups (skewp: <= 8,192 parts, BASELINE
// C4's per-GPU shard) gets both digests in about the SHA-256 time.  The MD5 plan must hold
// the same parts in the same order (plans of the same geometry do: stable sort).
// The self-fed MD5 wave of a group is paced by its SHA-256 producer (md5_self_body): it
// fetches each block after the producer has, so the part is read from HBM once.
#ifdef S3H_EXP_MD5_UNPACED  // experiment: round 3-5's unpaced MD5 wave (every byte read twice)
template <bool PAIR> constexpr uint32_t kMd5PaceBps = 0;
#else
template <bool PAIR> constexpr uint32_t kMd5PaceBps = SkewGeom<1, PAIR>::kBps;
#endif
template <bool PAIR>
__global__ __launch_bounds__(192) void sha256_md5_group_kernel(LaunchArgs S, LaunchArgs M) {
  __shared__ SkewLds<1, PAIR> LS;
  __shared__ uint32_t flags[2];
  if (threadIdx.x < 2) flags[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef S3H_EXP_GROUP_ONLY  // experiment: 1 = SHA-256 group only, 2 = MD5 wave only
  if ((S3H_EXP_GROUP_ONLY == 1 && wave == 1) || (S3H_EXP_GROUP_ONLY == 2 && wave != 1)) return;
#endif
  if (wave == 1)
    md5_self_body<SkewGeom<1, PAIR>::kParts, kMd5PaceBps<PAIR>>(M, blockIdx.x, &flags[0]);
  else
    skew_body<1, PAIR, true>(S, blockIdx.x, wave >> 1, LS, flags);
}

// sha256_md5_group_mixed_kernel: both digests of a RAGGED batch (2,049-8,192 parts, e.g.
// BASELINE C3) whose time is set by its longest parts.  The group kernel above runs every part
// at skewp's chain rate (2,476 cycles/block); here the first `F` workgroups take the 8F
// longest slots as skew-layout groups (8 parts, one consumer at the skew kernel's 8 VALU per
// round, ~2,280 cycles/block beside its MD5 wave), the rest the group kernel's 32-part skewp
// groups over slots 8F.. (their shorter parts finish in time at the slower rate).  The host
// picks F (capi.hip dual_mixed_solo) and launches at most one workgroup per CU (LDS pad).
// Both bodies index slots from their own group number, so the skewp half runs on LaunchArgs
// whose slot / out_idx arrays start at slot 8F; the clock probe is off (two group numberings).
// With `lead_md5` > 0 the 8F longest slots' MD5 chains run apart, on `lead_md5` workgroups
// after the G skewp ones (one self-fed MD5 wave of 64 chains each), so those skew groups run
// their SHA-256 alone on their CUs (plan.cpp dual_mixed_solo: when that grid fits).  The skewp
// groups' MD5 waves follow their own producer through LDS (one HBM read of those parts for both
// digests); the apart MD5 waves run unpaced -- pacing them across workgroups
// (S3H_EXP_MD5_XCD_PACE: each takes the skew groups of its own XCD and follows their
// producers' step counts in `progress`, tagged with this launch's `epoch`) cut C3's traffic
// 1.25x -> 1.18x but cost 3-4 % of its rate.
__global__ __launch_bounds__(192) void sha256_md5_group_mixed_kernel(LaunchArgs S, LaunchArgs M,
                                                                    uint32_t F, uint32_t G,
                                                                    uint32_t lead_md5,
                                                                    uint64_t* progress,
                                                                    uint32_t epoch) {
  __shared__ union {
    SkewLds<1, false> skew;
    SkewLds<1, true> skewp;
  } L;
  __shared__ uint32_t flags[2];
  if (threadIdx.x < 2) flags[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  S.clocks = nullptr;
  constexpr uint32_t kSolo = SkewGeom<1, false>::kParts;
  if (blockIdx.x < F) {
    if (wave != 1)
      skew_body<1, false, true, false, kMd5XcdPace && kMd5PaceBps<false> != 0>(
          S, blockIdx.x, wave >> 1, L.skew, flags,
          lead_md5 ? progress + xcd_progress_slot(blockIdx.x) : nullptr, epoch);
    else if (!lead_md5)
      md5_self_body<kSolo, kMd5PaceBps<false>>(M, blockIdx.x, &flags[0]);
    return;
  }
  if (lead_md5 && blockIdx.x >= F + G) {  // MD5 of slots 0 .. 8F-1, 64 chains per workgroup
    if (wave != 1) return;
    M.n = M.n < kSolo * F ? M.n : kSolo * F;
    if constexpr (kMd5XcdPace && kMd5PaceBps<false> != 0)
      // lead_md5 = mixed_lead_wgs(F): 8 XCD classes x ceil(F / 64) workgroups, each over the
      // skew groups that share its XCD, paced by their producers' global step counts
      md5_self_body<64, kMd5PaceBps<false>, true>(M, blockIdx.x - F - G, nullptr, progress, epoch, F);
    else
      md5_self_body<64>(M, blockIdx.x - F - G);  // slots 64w.., unpaced (the product)
    return;
  }
  const uint32_t shift = kSolo * F;
  if (shift >= S.n) return;
  S.slots += shift; S.out_idx += shift; S.n -= shift;
  M.slots += shift; M.out_idx += shift; M.n -= shift;
  if (wave == 1)
    md5_self_body<SkewGeom<1, true>::kParts, kMd5PaceBps<true>>(M, blockIdx.x - F, &flags[0]);
  else
    skew_body<1, true, true>(S, blockIdx.x - F, wave >> 1, L.skewp, flags);
}

// ------------------------------------------------------------- verification
// Download-side verification (ranged GETs of lib/src/download.cpp:88-103):
// mismatch[i] = digest(i) != expected(i), words compared as stored.
__global__ __launch_bounds__(256) void compare_digests_kernel(const uint32_t* got,
                                                              const uint32_t* want, uint64_t n,
                                                              uint32_t words, uint8_t* mismatch,
                                                              unsigned long long* count) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t diff = 0;
  for (uint32_t w = 0; w < words; ++w) diff |= got[words * i + w] ^ want[words * i + w];
  mismatch[i] = diff != 0;
  if (diff) atomicAdd(count, 1ull);
}

// ------------------------------------------------------------- multi-object streams
// Carry bookkeeping of one s3h_stream update, one thread per message (<= 127 bytes moved):
//   kSpliceHead : head[i] = carry[i][0:c] ++ chunk[0:h]   (c + h == 64: the block that
//                 straddles the previous update and this one, hashed by the head launch)
//   kSpliceGrow : carry[i][c:c+h] = chunk[0:h]           (still < 64 B buffered)
//   kSpliceReset: carry[i][0:r] = chunk[tail:tail+r]     (the new < 64-B remainder)
// The head block is built before the carry is overwritten (same thread, program order).
// (SpliceJob and its modes: kernel_abi.hpp)

__global__ __launch_bounds__(256) void stream_splice_kernel(const uint8_t* base,
                                                            const SpliceJob* jobs, uint8_t* carry,
                                                            uint8_t* head, uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  const SpliceJob j = jobs[i];
  uint8_t* cy = carry + 64 * i;
  if (j.mode & kSpliceHead) {
    uint8_t* hb = head + 64 * i;
    for (uint32_t k = 0; k < j.c; ++k) hb[k] = cy[k];
    for (uint32_t k = 0; k < j.h; ++k) hb[j.c + k] = base[j.src + k];
  }
  if (j.mode & kSpliceGrow)
    for (uint32_t k = 0; k < j.h; ++k) cy[j.c + k] = base[j.src + k];
  if (j.mode & kSpliceReset)
    for (uint32_t k = 0; k < j.r; ++k) cy[k] = base[j.tail + k];
}

// Chaining state of n empty messages (8-word stride for both algorithms).
__global__ __launch_bounds__(256) void stream_init_kernel(uint32_t* state, uint64_t n, int md5) {
  const uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (i >= n) return;
  uint4* s = reinterpret_cast<uint4*>(state + 8 * i);
  if (md5) {
    s[0] = make_uint4(0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u);
  } else {
    s[0] = make_uint4(0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au);
    s[1] = make_uint4(0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u);
  }
}

// ------------------------------------------------------------- synthetic input generator
// G(seed, p, L) of SURVEY.md 8(d): word j of part p is splitmix64(x0 + (j+1)*golden),
// x0 = seed ^ p*0xD1B54A32D192ED03, serialised little-endian.  Parts must start 8-B aligned.
// (GenPart: kernel_abi.hpp)

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
