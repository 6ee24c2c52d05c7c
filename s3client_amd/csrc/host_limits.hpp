// host_limits.hpp -- sizes and thresholds of the host-resident path that more than one unit
// uses (the pipeline in host_path.cpp, the split planner in route_plan.cpp).  HIP-free.
#pragma once
#include <cstdint>

#include "../../include/s3hash.h"

namespace s3h::host {

// digest words per part: SHA-256 8, MD5 4
inline uint32_t digest_words(int algo) { return algo == S3H_ALGO_MD5 ? 4u : 8u; }

constexpr int kHostMaxAlgo = 2;  // algorithms one host-path call hashes (SHA-256 and/or MD5)
constexpr int kHostRing = 3;     // HBM ring slots / pinned staging slots

// Group mode (host_path.cpp run_host_groups) for many small parts: parts of at most
// kGroupMaxPart bytes go in groups of whole parts instead of slices of every part.
constexpr uint64_t kGroupMaxPart = 1ull << 20;
// Beyond this many ragged pinned parts the slice pipeline stages them (memcpy + one DMA per
// slice) instead of one DMA per part per slice.
constexpr uint64_t kPinnedStageMin = 256;

}  // namespace s3h::host
