// exp_config.hpp -- every compile-time experiment switch of the kernels and the host plan, in
// one place, with the values the PRODUCT build uses.
//
// Experiment builds (`make exp TAG=... EXPFLAGS="-DS3H_EXP_..."`, timing studies under
// tools/exp/, never shipped) and the test-only forced-fault build (`make stall`) define
// S3H_EXPERIMENT_BUILD and may override anything below.  Without it -- the build of
// s3client_amd/lib/libs3hash.so -- every value switch must hold its default and no flag switch
// may be defined: the static_asserts and #errors below stop a product build that was
// compiled with an experiment's flags, so the shipped kernels are exactly the ones the
// measurements in DESIGN.md and the code hashes in kernel_isa_counts.json describe.
#pragma once

// ---- value switches: product defaults
#ifndef S3H_EXP_SKEW_BLK_PAD
#define S3H_EXP_SKEW_BLK_PAD 0  // skew layout: uint4 of LDS padding per block (SkewGeom)
#endif
#ifndef S3H_EXP_SKEW_BPS_NC2
#define S3H_EXP_SKEW_BPS_NC2 8  // skew NC=2: blocks per producer step
#endif
#ifndef S3H_EXP_PRODUCER_ROLLED
#define S3H_EXP_PRODUCER_ROLLED 0  // 1: skew producer loops over its items without unrolling
#endif
#ifndef S3H_EXP_MD5_SELF_DEPTH
#define S3H_EXP_MD5_SELF_DEPTH 4  // self-fed MD5: blocks fetched ahead
#endif
#ifndef S3H_EXP_MD5_BPS
#define S3H_EXP_MD5_BPS 4  // MD5 producer/consumer kernel: blocks per producer step
#endif
#ifndef S3H_EXP_MD5_ROLL
#define S3H_EXP_MD5_ROLL 1  // MD5 consumer: the rolling fused step (0: the chunked one)
#endif
#ifndef S3H_EXP_MD5_PSETS
#define S3H_EXP_MD5_PSETS 2  // MD5 producer, 4-block steps: raw-block register sets (3: two steps ahead)
#endif
#ifndef S3H_EXP_MD5_PSETS1
#define S3H_EXP_MD5_PSETS1 3  // the same for md5_pc_kernel<1> (1-block steps): two blocks ahead
#endif
#ifndef S3H_EXP_MIXED_MD5_APART
// ragged dual grid: 1 = the skew groups' MD5 chains on workgroups of their own when that grid
// fits (else in the skew groups), 0 = always in the skew groups (round 3)
#define S3H_EXP_MIXED_MD5_APART 1
#endif
#ifndef S3H_EXP_TAIL_RAMP_DIV
// host pipeline: once fewer than DIV slices are left, each slice carries 1/DIV of what is left
// (slices shrink by (DIV-1)/DIV each, down to 1/16 of a full slice)
#define S3H_EXP_TAIL_RAMP_DIV 8
#endif
#ifndef S3H_EXP_PACE_LAG
#define S3H_EXP_PACE_LAG 0  // MD5 pacing: extra producer steps to wait for beyond the block's own
#endif
#ifndef S3H_EXP_SKEW_MERGE_NEXT
// skew consumers read the next block's rows before rounds 0-15 and end a block with one
// statement (rounds 16-63 + NEXT): one LDS wait per block instead of two.  1: the quad layout
// (skew / skews), 0: never (rounds 1-6), 2: also the lane-pair layout (skewp)
#define S3H_EXP_SKEW_MERGE_NEXT 1
#endif
#ifndef S3H_EXP_FLAG_PREFETCH
// flag-synchronised skew consumers read the producer's step counter with the next step's rows
// and check it after rounds 0-15 (skew_body kFlagPrefetch; profiles/r06_flag_prefetch_ab.json:
// C3 2,217 -> 2,200 cycles per block, C4 skews 2,232 -> 2,220).  0: wait at the step boundary
#define S3H_EXP_FLAG_PREFETCH 1
#endif
#ifndef S3H_EXP_MD5_XCD_PACE
// 1: MD5 workgroups of the split / mixed dual grids paced by the skew groups on their XCD
// through global step counts (kernel_abi.hpp kMd5XcdPace)
#define S3H_EXP_MD5_XCD_PACE 0
#endif
#ifndef S3H_EXP_GPROG_OFF
#define S3H_EXP_GPROG_OFF 0  // 1: skew producers never store their global step counts (MD5 waits time out)
#endif
// ragged dual grid (plan.cpp dual_mixed_solo): cycles per block of a skewp group beside its MD5
// wave, and of a skew group with its MD5 apart / beside it -- the rates the split into skew
// and skewp groups is planned with.  2,650 from a sweep on C3 (profiles/
// r06_dual_mixed_planning_sweep.json: 2,550, calibrated on the C4 shard's equal parts, left
// C3's ragged skewp groups finishing last)
#ifndef S3H_EXP_DUAL_SKEWP_CYC
#define S3H_EXP_DUAL_SKEWP_CYC 2650
#endif
#ifndef S3H_EXP_DUAL_SKEW_CYC_APART
#define S3H_EXP_DUAL_SKEW_CYC_APART 2224
#endif
#ifndef S3H_EXP_DUAL_SKEW_CYC_INGROUP
#define S3H_EXP_DUAL_SKEW_CYC_INGROUP 2280
#endif
#ifndef S3H_EXP_SPIN_LIMIT
#define S3H_EXP_SPIN_LIMIT (1u << 24)  // flag waits: s_sleep 1 polls before a wait times out
#endif
#ifndef S3H_EXP_STALL_PRODUCER
// 1: flag-synchronised producers stop publishing after their first step, so every consumer
// wait times out (the forced-fault build `make stall`, tests/test_gpu_errors.py)
#define S3H_EXP_STALL_PRODUCER 0
#endif

#ifndef S3H_EXPERIMENT_BUILD
static_assert(S3H_EXP_SKEW_BLK_PAD == 0, "product build: S3H_EXP_SKEW_BLK_PAD must be 0");
static_assert(S3H_EXP_SKEW_BPS_NC2 == 8, "product build: S3H_EXP_SKEW_BPS_NC2 must be 8");
static_assert(S3H_EXP_PRODUCER_ROLLED == 0, "product build: unrolled skew producer");
static_assert(S3H_EXP_MD5_SELF_DEPTH == 4, "product build: self-fed MD5 loads 4 blocks ahead");
static_assert(S3H_EXP_MD5_BPS == 4, "product build: MD5 kernel with 4-block producer steps");
static_assert(S3H_EXP_MD5_ROLL == 1, "product build: rolling MD5 row reads");
static_assert(S3H_EXP_MD5_PSETS == 2, "product build: two MD5 producer register sets");
static_assert(S3H_EXP_MD5_PSETS1 == 3, "product build: three sets for 1-block MD5 steps");
static_assert(S3H_EXP_MIXED_MD5_APART == 1, "product build: skew groups' MD5 apart when it fits");
static_assert(S3H_EXP_TAIL_RAMP_DIV == 8, "product build: host tail slices shrink by 7/8");
static_assert(S3H_EXP_DUAL_SKEWP_CYC == 2650 && S3H_EXP_DUAL_SKEW_CYC_APART == 2224 &&
                  S3H_EXP_DUAL_SKEW_CYC_INGROUP == 2280,
              "product build: the dual grid's planning rates");
static_assert(S3H_EXP_SPIN_LIMIT == (1u << 24), "product build: flag waits give up after 2^24 polls");
static_assert(S3H_EXP_SKEW_MERGE_NEXT == 1, "product build: quad-layout blocks end in one statement");
static_assert(S3H_EXP_FLAG_PREFETCH == 1, "product build: step counters read with the rows");
static_assert(S3H_EXP_MD5_XCD_PACE == 0, "product build: MD5 paced within a workgroup only");
static_assert(S3H_EXP_GPROG_OFF == 0, "product build: skew producers publish their step counts");
static_assert(S3H_EXP_PACE_LAG == 0, "product build: MD5 waits for its block's own producer step");
static_assert(S3H_EXP_STALL_PRODUCER == 0, "product build: producers publish every step");

// ---- flag switches: experiments only (each changes a kernel's code or the plan's choices)
#if defined(S3H_EXP_FORCE_NC) || defined(S3H_EXP_SOLO) || defined(S3H_EXP_GROUP_SKEW) ||      \
    defined(S3H_EXP_NO_SPLIT) || defined(S3H_EXP_NO_GROUP_NC2) ||                            \
    defined(S3H_EXP_NO_DUAL_MIXED) || defined(S3H_EXP_PRODUCER_INC) ||                       \
    defined(S3H_EXP_PROD_ROWS) || defined(S3H_EXP_LONE_CONSUMER) ||                          \
    defined(S3H_EXP_MD5_INC) || defined(S3H_MD5_VMEM) || defined(S3H_EXP_MD5_NOSYNC) ||      \
    defined(S3H_EXP_MD5_NOPROD) || defined(S3H_EXP_MD5_NOFUSE) ||                            \
    defined(S3H_EXP_GROUP_ONLY) || defined(S3H_EXP_NONTEMPORAL_FETCH) ||                    \
    defined(S3H_EXP_GROUP_ANY) || defined(S3H_EXP_NO_TAIL_RAMP) ||                        \
    defined(S3H_EXP_PAGEABLE_DIRECT) || defined(S3H_EXP_PRODUCER_IDLE) ||                   \
    defined(S3H_EXP_CONSUMER_IDLE) || defined(S3H_EXP_MD5_UNPACED)
#error "an experiment switch is defined in a product build (define S3H_EXPERIMENT_BUILD: make exp)"
#endif
#endif  // S3H_EXPERIMENT_BUILD
