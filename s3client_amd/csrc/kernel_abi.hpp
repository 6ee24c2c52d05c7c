// kernel_abi.hpp -- what the host side and the gfx950 kernels share: the launch argument block,
// the plan's part slots, the stream splice jobs, the generator's part records and the
// workgroup-shape constants the host sizes grids with.  Plain structs and constants: the
// host translation units (g++) and the kernel translation unit (launch.hip, hipcc) both include
// it, so a plan built on the host and the kernel that reads it agree by construction.
#pragma once
#include <stdint.h>

#include "exp_config.hpp"

#if defined(__HIPCC__)
#define S3H_HOST_DEVICE __host__ __device__ __forceinline__
#else
#define S3H_HOST_DEVICE inline
#endif

namespace s3h {

struct Slot {        // one upload part in a plan, slots sorted by block count (descending)
  uint64_t off;      // byte offset of the part relative to the launch's base pointer
  uint64_t len;      // part length in bytes (the full part, also for resumed launches)
};

// Number of 64-byte compressions for a message of `len` bytes: ceil((len + 9) / 64)
// (lib/hash/utility.cpp:42-56 alloc_padded: 0x80, zeros, 64-bit big-endian bit length).
S3H_HOST_DEVICE uint64_t nblocks(uint64_t len) { return (len + 72) >> 6; }

// LaunchArgs::flags
constexpr uint32_t kNoPad = 1;   // hash only the slot's whole 64-B blocks; never pad or emit
constexpr uint32_t kResume = 2;  // load the chaining state even at blk_begin == 0

// Bits of the device error word (LaunchArgs::err).  Every host entry point reads the word
// after its launches complete and fails the call when it is non-zero (plan.cpp plan_check):
// a launch whose digests may be wrong never returns S3H_OK.
constexpr uint32_t kErrSyncTimeout = 1;  // a producer/consumer flag wait timed out

struct LaunchArgs {
  const uint8_t* base;       // part p's block b is at base + slots[p].off + 64*(b - blk_origin)
  const Slot* slots;         // sorted by nblocks descending
  const uint32_t* out_idx;   // slot -> output part (message) index
  uint32_t* state;           // n*8 words (message order); may be null for single-launch plans
  uint32_t* digests;         // n*8 words (part order), bswap32(H_i) like lib/hash to_little
  const uint8_t* zero;       // 256 zero bytes: target of the loads of out-of-range lanes
  const uint64_t* bits;      // per-message bit length for the padding (null: 8 * slot length)
  uint64_t blk_begin, blk_end, blk_origin;
  uint32_t n;
  uint32_t flags;
  // Clock probe (s3h_plan_set_clock_probe; skew kernel): per consumer wave, shader-clock and
  // 100 MHz real-time counters at the start and end of its chain loop.  Null: off.
  uint64_t* clocks;
  // sha256_skew_pairs_kernel: the first `solo` workgroups run one group each (the longest
  // parts, on a CU of their own), the rest two.  0 elsewhere.
  uint32_t solo;
  // Device error word of the plan (kErr* bits OR-ed in by global atomics; cleared by the host).
  uint32_t* err;
};

// Cross-workgroup MD5 pacing (experiment S3H_EXP_MD5_XCD_PACE, sha256_kernels.hip ShaPacer /
// XcdChains): the MD5 workgroups of the split dual grid and the mixed grid's apart form take
// the chains of the skew groups on their own XCD and follow those groups' producers through
// step counts in global memory.  Measured: C2 dual traffic 2x -> 1.04-1.22x at -0.3 %, C3 dual
// 1.25x -> 1.18x at -3 to -4 % (profiles/r06_dual_xcd_pace_ab.json); the product keeps the
// in-workgroup (LDS) pacing only.
constexpr bool kMd5XcdPace = S3H_EXP_MD5_XCD_PACE != 0;

// sha256_md5_group_mixed_kernel, apart form: the MD5 workgroups of the F skew groups' chains,
// 64 chains each -- by XCD class under kMd5XcdPace (workgroups b and b + 8 share an XCD:
// ceil(F / 8) skew groups per class -> ceil(F / 64) workgroups per class, 8 classes).
S3H_HOST_DEVICE uint32_t mixed_lead_wgs(uint64_t F) {
  return kMd5XcdPace ? uint32_t(8 * ((F + 63) / 64)) : uint32_t((8 * F + 63) / 64);
}

// sha256_md5_dual_kernel (the split dual grid): MD5 workgroups after the `sha_groups` skew
// workgroups -- one per 64 parts, or by XCD class (8 x ceil(sha_groups / 64)) under kMd5XcdPace.
S3H_HOST_DEVICE uint32_t split_md5_wgs(uint64_t sha_groups, uint64_t n) {
  return kMd5XcdPace ? uint32_t(8 * ((sha_groups + 63) / 64)) : uint32_t((n + 63) / 64);
}

// Workgroup shapes (sha256_kernels.hip).
constexpr int kPcThreads = 128;          // producer/consumer: wave 0 consumer, wave 1 producer; 64 parts
constexpr int kPairThreads = 128;        // lane-pair kernel: 32 parts per workgroup
constexpr int kPairParts = 32;
constexpr int kQuadChainsPerWave = 8;    // skew / quad: 8 chains per consumer wave
// MD5 kernel: kMd5Bps-block producer steps (128 KiB of LDS, one workgroup per CU) while the
// grid fits one workgroup per CU (<= 64 x CUs parts); 1-block steps (32 KiB) beyond.
constexpr int kMd5Bps = S3H_EXP_MD5_BPS;

// ------------------------------------------------------------- multi-object streams
// Carry bookkeeping of one s3h_stream update, one thread per message (<= 127 bytes moved):
//   kSpliceHead : head[i] = carry[i][0:c] ++ chunk[0:h]   (c + h == 64: the block that
//                 straddles the previous update and this one, hashed by the head launch)
//   kSpliceGrow : carry[i][c:c+h] = chunk[0:h]           (still < 64 B buffered)
//   kSpliceReset: carry[i][0:r] = chunk[tail:tail+r]     (the new < 64-B remainder)
struct SpliceJob {
  uint64_t src, tail;  // chunk start / new-remainder start, offsets from the update's base
  uint32_t c, h, r, mode;
};
constexpr uint32_t kSpliceHead = 1, kSpliceGrow = 2, kSpliceReset = 4;

// ------------------------------------------------------------- synthetic input generator
// G(seed, p, L) of SURVEY.md 8(d): one record per part (byte offset, length, generator id).
struct GenPart { uint64_t off, len, id; };

}  // namespace s3h
