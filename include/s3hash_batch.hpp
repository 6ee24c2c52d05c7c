// include/s3hash_batch.hpp -- C++ convenience layer over the C-ABI (include/s3hash.h) in the
// same `namespace sha256` as the lib/hash drop-in, for C++ callers such as the parallel
// upload (the reference's lib/src/upload.cpp:89-110 insertion point).  Header-only; every
// call goes to the GPU through libs3hash.so and throws on error (no CPU fallback) -- unless
// the caller passes Route::cpu or Route::automatic to payload_hashes / file_part_hashes.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "s3hash.h"
#include "sha256.h"

namespace sha256 {

struct batch_error : std::runtime_error {
  int code;
  batch_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void batch_check(int rc) {
  if (rc != S3H_OK) throw batch_error(rc, std::string("s3hash: ") + s3h_last_error());
}

// Digests of host-resident parts on the GPUs (0 = all visible devices), one uint32_t[8] per
// part in lib/hash's layout (hash[i] = bswap32(H_i)).
inline std::vector<uint32_t> sha256_batch(const std::vector<const uint8_t*>& parts,
                                          const std::vector<uint64_t>& lengths,
                                          int ndevices = 0, uint64_t slice_bytes = 0) {
  if (parts.size() != lengths.size()) throw std::invalid_argument("parts/lengths size mismatch");
  std::vector<uint32_t> out(8 * parts.size());
  if (!parts.empty())
    batch_check(s3h_sha256_batch_host(parts.data(), lengths.data(), parts.size(), out.data(),
                                      ndevices, slice_bytes));
  return out;
}

// Parts already in device memory at d_base + offsets[i]; digests written to d_digests.
inline void sha256_batch_device(int device, const void* d_base,
                                const std::vector<uint64_t>& offsets,
                                const std::vector<uint64_t>& lengths, uint32_t* d_digests,
                                void* stream = nullptr) {
  batch_check(s3h_sha256_batch_device(device, d_base, offsets.data(), lengths.data(),
                                      offsets.size(), d_digests, stream));
}

// Where a host batch is hashed (include/s3hash.h "size-aware routing"): gpu = the batched GPU
// path (default), cpu = the lib/hash drop-in on host threads, split = both at once (the
// longest parts on the CPU, the rest on the GPU), automatic = whichever a model measured once
// per process estimates to finish first (needs a GPU; never a fallback).
enum class Route { gpu = S3H_ROUTE_GPU, cpu = S3H_ROUTE_CPU, automatic = S3H_ROUTE_AUTO, split = S3H_ROUTE_SPLIT };

inline std::vector<std::string> to_hex(const std::vector<uint32_t>& d) {
  std::vector<std::string> out(d.size() / 8);
  for (size_t i = 0; i < out.size(); ++i) {
    char t[65];
    hash_to_text(const_cast<uint32_t*>(&d[8 * i]), t);
    out[i] = t;
  }
  return out;
}

// AUTO's decision for a batch of parts of `lengths` without running it (s3h_route_rates,
// measured on first use and kept current by routed calls, + s3h_route_choose): Route::gpu,
// Route::cpu or Route::split, and the GPU / CPU estimates.  `digests` is what the caller will
// compute (S3H_DIGESTS_SHA256, or S3H_DIGESTS_BOTH for Content-MD5 + x-amz-content-sha256: the
// CPU side is then priced at the MD5 + SHA-256 rate), `source` where the parts are
// (S3H_SOURCE_PINNED / _PAGEABLE / _FILE).  An uploader that hashes per job decides once for
// the whole upload with this, then hashes each job's parts on that route.
inline Route choose_route(const std::vector<uint64_t>& lengths, int ndevices = 0,
                          double* gpu_s = nullptr, double* cpu_s = nullptr,
                          int digests = S3H_DIGESTS_SHA256, int source = S3H_SOURCE_PINNED) {
  if (lengths.empty()) throw std::invalid_argument("choose_route: no parts");
  s3h_route_rates_t r{};
  r.size = sizeof r;
  batch_check(s3h_route_rates(&r));
  s3h_route_choice_t c{};
  batch_check(s3h_route_choose(&r, digests, lengths.data(), lengths.size(), ndevices, source, &c));
  if (gpu_s) *gpu_s = c.gpu_s;
  if (cpu_s) *cpu_s = c.cpu_s;
  return Route(c.route);
}

// 64-char lowercase hex per part: the `payloadHash` strings S3Api::UploadFilePart takes
// (lib/include/s3-api.h:447-452).  *taken (if non-null) receives the route that ran.
inline std::vector<std::string> payload_hashes(const std::vector<const uint8_t*>& parts,
                                               const std::vector<uint64_t>& lengths,
                                               int ndevices = 0, Route route = Route::gpu,
                                               Route* taken = nullptr) {
  if (parts.size() != lengths.size()) throw std::invalid_argument("parts/lengths size mismatch");
  if (route == Route::gpu) {
    if (taken) *taken = Route::gpu;
    return to_hex(sha256_batch(parts, lengths, ndevices));
  }
  std::vector<uint32_t> d(8 * parts.size());
  int t = S3H_ROUTE_GPU;
  if (!parts.empty())
    batch_check(s3h_sha256_batch_routed(parts.data(), lengths.data(), parts.size(), d.data(),
                                        ndevices, int(route), &t));
  if (taken) *taken = Route(t);
  return to_hex(d);
}

// Digests of byte ranges of a file -- the (file, offset, size) parts UploadFilePart sends --
// read by host threads straight into pinned staging (s3h_sha256_file_parts), as hex.
inline std::vector<std::string> file_part_hashes(const std::string& path,
                                                 const std::vector<uint64_t>& offsets,
                                                 const std::vector<uint64_t>& lengths,
                                                 int ndevices = 0, Route route = Route::gpu,
                                                 Route* taken = nullptr) {
  if (offsets.size() != lengths.size()) throw std::invalid_argument("offsets/lengths size mismatch");
  std::vector<uint32_t> d(8 * offsets.size());
  int t = S3H_ROUTE_GPU;
  if (!offsets.empty() && route == Route::gpu)
    batch_check(s3h_sha256_file_parts(path.c_str(), offsets.data(), lengths.data(), offsets.size(),
                                      d.data(), ndevices, 0));
  else if (!offsets.empty())
    batch_check(s3h_sha256_file_parts_routed(path.c_str(), offsets.data(), lengths.data(),
                                             offsets.size(), d.data(), ndevices, int(route), &t));
  if (taken) *taken = Route(t);
  return to_hex(d);
}

// Release the host path's cached per-device buffers (s3h_trim).
inline void trim() { batch_check(s3h_trim()); }

// Both upload headers per part from one pass (s3h_sha256_md5_batch_host): `sha256` gets the
// x-amz-content-sha256 hex, `md5` the 16 digest bytes of Content-MD5 (base64 them for the
// header) -- the replacement for one sha256::sha256 + one md5::md5 call per part.
struct DualDigests {
  std::vector<uint32_t> sha256;  // 8 words per part, lib/hash layout
  std::vector<uint32_t> md5;     // 4 words per part, digest bytes in memory order
};
inline DualDigests sha256_md5_batch(const std::vector<const uint8_t*>& parts,
                                    const std::vector<uint64_t>& lengths, int ndevices = 0,
                                    uint64_t slice_bytes = 0) {
  if (parts.size() != lengths.size()) throw std::invalid_argument("parts/lengths size mismatch");
  DualDigests d{std::vector<uint32_t>(8 * parts.size()), std::vector<uint32_t>(4 * parts.size())};
  if (!parts.empty())
    batch_check(s3h_sha256_md5_batch_host(parts.data(), lengths.data(), parts.size(),
                                          d.sha256.data(), d.md5.data(), ndevices, slice_bytes));
  return d;
}

// The same for (file, offset, size) parts (s3h_sha256_md5_file_parts): each slice is read once.
inline DualDigests file_part_sha256_md5(const std::string& path, const std::vector<uint64_t>& offsets,
                                        const std::vector<uint64_t>& lengths, int ndevices = 0) {
  if (offsets.size() != lengths.size()) throw std::invalid_argument("offsets/lengths size mismatch");
  DualDigests d{std::vector<uint32_t>(8 * offsets.size()), std::vector<uint32_t>(4 * offsets.size())};
  if (!offsets.empty())
    batch_check(s3h_sha256_md5_file_parts(path.c_str(), offsets.data(), lengths.data(),
                                          offsets.size(), d.sha256.data(), d.md5.data(), ndevices, 0));
  return d;
}

// Both digests on a route (s3h_sha256_md5_batch_routed / s3h_sha256_md5_file_parts_routed):
// Route::gpu = the one-grid dual pass, Route::cpu = SHA-256 + MD5 per part in one pass over
// memory on the host threads, Route::split = the longest parts on the CPU while the GPU hashes
// the rest, Route::automatic = the model's pick for both digests.  *taken: the route that ran.
inline DualDigests sha256_md5_routed(const std::vector<const uint8_t*>& parts,
                                     const std::vector<uint64_t>& lengths, int ndevices = 0,
                                     Route route = Route::automatic, Route* taken = nullptr) {
  if (parts.size() != lengths.size()) throw std::invalid_argument("parts/lengths size mismatch");
  DualDigests d{std::vector<uint32_t>(8 * parts.size()), std::vector<uint32_t>(4 * parts.size())};
  int t = int(route);
  if (!parts.empty())
    batch_check(s3h_sha256_md5_batch_routed(parts.data(), lengths.data(), parts.size(), d.sha256.data(),
                                            d.md5.data(), ndevices, int(route), &t));
  if (taken) *taken = Route(t);
  return d;
}
inline DualDigests file_part_sha256_md5_routed(const std::string& path, const std::vector<uint64_t>& offsets,
                                               const std::vector<uint64_t>& lengths, int ndevices = 0,
                                               Route route = Route::automatic, Route* taken = nullptr) {
  if (offsets.size() != lengths.size()) throw std::invalid_argument("offsets/lengths size mismatch");
  DualDigests d{std::vector<uint32_t>(8 * offsets.size()), std::vector<uint32_t>(4 * offsets.size())};
  int t = int(route);
  if (!offsets.empty())
    batch_check(s3h_sha256_md5_file_parts_routed(path.c_str(), offsets.data(), lengths.data(), offsets.size(),
                                                 d.sha256.data(), d.md5.data(), ndevices, int(route), &t));
  if (taken) *taken = Route(t);
  return d;
}

// Download-side check (s3h_verify_batch_host): true for every part whose SHA-256 differs from
// the expected hex digest (the x-amz-content-sha256 it was uploaded with).
inline std::vector<bool> verify_payloads(const std::vector<const uint8_t*>& parts,
                                         const std::vector<uint64_t>& lengths,
                                         const std::vector<std::string>& expected_hex,
                                         int ndevices = 0) {
  if (parts.size() != lengths.size() || parts.size() != expected_hex.size())
    throw std::invalid_argument("parts/lengths/expected size mismatch");
  std::vector<uint32_t> want(8 * parts.size());
  auto nibble = [](char c) -> int {
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10
           : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
  };
  for (size_t i = 0; i < parts.size(); ++i) {
    const std::string& h = expected_hex[i];
    // exactly 64 hex digits: no sign, whitespace or prefix is accepted
    bool ok = h.size() == 64;
    for (size_t k = 0; ok && k < 64; ++k) ok = nibble(h[k]) >= 0;
    if (!ok)
      throw std::invalid_argument("verify_payloads: expected digest of part " + std::to_string(i) +
                                  " is not 64 hex digits: \"" + h + "\"");
    uint8_t* w = reinterpret_cast<uint8_t*>(&want[8 * i]);
    for (int b = 0; b < 32; ++b) w[b] = uint8_t(nibble(h[2 * b]) << 4 | nibble(h[2 * b + 1]));
  }
  std::vector<uint8_t> bad(parts.size());
  uint64_t count = 0;
  if (!parts.empty())
    batch_check(s3h_verify_batch_host(S3H_ALGO_SHA256, parts.data(), lengths.data(), parts.size(),
                                      want.data(), bad.data(), &count, ndevices));
  return std::vector<bool>(bad.begin(), bad.end());
}

// n objects hashed as their bodies arrive (s3h_stream_*): append() one chunk per object
// (any length, 0 allowed), finish() -> n digests of everything appended since the last
// finish(), after which the object restarts with n empty messages.  The batched, on-device
// form of sha256_stream + the documented sha256_next contract (sha256.h:73-97).
class stream_batch {
 public:
  explicit stream_batch(uint64_t n, int device = 0, int algo = S3H_ALGO_SHA256)
      : n_(n), words_(algo == S3H_ALGO_MD5 ? 4 : 8) {
    batch_check(s3h_stream_create(device, algo, n, S3H_KERNEL_AUTO, &s_));
  }
  ~stream_batch() { s3h_stream_destroy(s_); }
  stream_batch(const stream_batch&) = delete;
  stream_batch& operator=(const stream_batch&) = delete;

  void append(const std::vector<const uint8_t*>& chunks, const std::vector<uint64_t>& lengths) {
    if (chunks.size() != n_ || lengths.size() != n_)
      throw std::invalid_argument("stream_batch: one chunk per object");
    batch_check(s3h_stream_update_host(s_, chunks.data(), lengths.data()));
  }
  std::vector<uint32_t> finish() {
    std::vector<uint32_t> out(words_ * n_);
    batch_check(s3h_stream_final_host(s_, out.data()));
    return out;
  }
  std::vector<std::string> finish_hex() {
    const std::vector<uint32_t> d = finish();
    std::vector<std::string> out(n_);
    static const char* hexd = "0123456789abcdef";
    for (uint64_t i = 0; i < n_; ++i) {
      const uint8_t* b = reinterpret_cast<const uint8_t*>(&d[words_ * i]);
      for (uint32_t k = 0; k < 4 * words_; ++k) {
        out[i] += hexd[b[k] >> 4];
        out[i] += hexd[b[k] & 15];
      }
    }
    return out;
  }
  uint64_t size() const { return n_; }

 private:
  s3h_stream_t s_ = nullptr;
  uint64_t n_;
  uint32_t words_;
};

}  // namespace sha256

namespace md5 {

// The multipart ETag an S3 endpoint returns from CompleteMultipartUpload
// (lib/src/api/multipart_upload.cpp:162-183), from the parts' MD5 digests in part order
// (4 words per part, as DualDigests::md5 / s3h_md5_batch_* return them): s3h_multipart_etag.
inline std::string multipart_etag(const std::vector<uint32_t>& part_md5s) {
  if (part_md5s.empty() || part_md5s.size() % 4)
    throw std::invalid_argument("multipart_etag: need 4 words per part and at least one part");
  char out[S3H_ETAG_MAX];
  sha256::batch_check(s3h_multipart_etag(part_md5s.data(), part_md5s.size() / 4, out, sizeof out));
  return out;
}

}  // namespace md5
