// stream.cpp -- multi-object streams (s3h_stream_*, include/s3hash.h): n messages hashed as
// their chunks arrive, the batched device-resident form of lib/hash's chunked API --
// sha256_stream (lib/hash/sha256.cpp:84-144) for the appends and the DOCUMENTED contract of
// sha256_next (sha256.h:73-89) for the finish.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <utility>
#include <vector>

#include "copy_pool.hpp"
#include "internal.hpp"

using namespace s3h::host;

// Multi-object stream (include/s3hash.h "multi-object streams").  Host bookkeeping: per
// message carry length (< 64) and total bytes.  Device: chaining state (message order),
// 64-B carry and head-block buffers, the splice jobs, three re-sortable plans.
struct s3h_stream_s {
  int device = 0, algo = 0;
  uint64_t n = 0;
  s3h_plan_s *head = nullptr, *body = nullptr, *fin = nullptr;
  uint32_t* d_state = nullptr;
  uint8_t* d_carry = nullptr;
  uint8_t* d_head = nullptr;
  s3h::SpliceJob* d_jobs = nullptr;
  uint64_t* d_bits = nullptr;
  // Host-form updates (s3h_stream_update_host): each update's chunks are packed at 64-B
  // aligned offsets into device staging set hb -- two sets, so update k+1's copy (on copy_s)
  // overlaps update k's hash (on own) -- by DMA straight from pinned chunks, or, for pageable
  // chunks, through pinned host pieces (two, kStreamPiece bytes) that copy threads on the
  // device's NUMA node fill while the previous piece's DMA runs.
  uint8_t* d_hs[2] = {nullptr, nullptr};
  uint64_t d_hs_cap[2] = {0, 0};
  uint8_t* h_piece[2] = {nullptr, nullptr};
  uint64_t h_piece_cap = 0;
  hipEvent_t hs_copied[2] = {nullptr, nullptr}, hs_hashed[2] = {nullptr, nullptr};
  hipEvent_t piece_copied[2] = {nullptr, nullptr};
  hipStream_t copy_s = nullptr;
  unsigned hs_set = 0, piece_next = 0;
  uint32_t* d_dig = nullptr;   // host-form final
  // Pinned staging of an update / final in two sets used alternately: set b is rewritten
  // only once the call that used it two calls ago has completed (staged[b]), so the host
  // prepares update k+1 while update k's kernels run (one set made every update wait for the
  // previous one's kernels: the GPU idled ~45 us per update, -4.7 % at 64 KiB chunks).
  uint8_t* h_pin = nullptr;
  s3h::SpliceJob* h_jobs[2] = {nullptr, nullptr};
  s3h::Slot* h_slots[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  uint32_t* h_order[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  uint64_t* h_bits[2] = {nullptr, nullptr};
  hipEvent_t staged[2] = {nullptr, nullptr};
  hipEvent_t done = nullptr;  // end of the last update / final: the next call's stream waits on it
  hipStream_t done_on = nullptr;  // the stream `done` was recorded on (same stream: no wait)
  bool done_set = false;
  unsigned set = 0;
  bool used_stage = false;  // this call copied from staging set `set ^ 1` (else no staged[] record)
  // What the head / body plans' device slots hold: an update whose lengths equal them and
  // whose offsets are them plus one constant (equal chunks appended in place) reuses the
  // slots with the launch base moved by that constant -- no re-sort, no copies.
  std::vector<uint64_t> up_offs[2], up_lens[2];
  bool up_valid[2] = {false, false};
  uint64_t slot_reuses = 0, slot_refills = 0;  // s3h_stream_stats: how updates found their slots
  // A call that failed after it started queueing work leaves the messages' host bookkeeping
  // (carries, totals) ahead of or behind the device state: the object refuses further calls.
  std::string failed;
  hipStream_t own = nullptr;
  std::vector<uint64_t> total;
  std::vector<uint32_t> carry;
  std::vector<uint64_t> offs, lens, offs2, lens2;
};

namespace {

// Host-form stream updates (s3h_stream_update_host): pinned host pieces of the staged copy
// (two, filled alternately); pinned ragged chunks DMA'd one by one only up to this many per
// update (more: staged -- a DMA per 1 MiB chunk costs more than a memcpy); updates above
// 2 x kStreamSubBytes are split into sub-updates of ~kStreamSubBytes (>= kStreamSubMin of
// every chunk) whose copies overlap the hash of the one before.
constexpr uint64_t kStreamPiece = 64ull << 20;
constexpr uint64_t kStreamDmaChunks = 64;
constexpr uint64_t kStreamSubBytes = 128ull << 20;
constexpr uint64_t kStreamSubMin = 64ull << 10;

// Test hook: S3H_TEST_STREAM_FAIL_SUB=k fails the k-th sub-update of the FIRST
// s3h_stream_update_host call that reaches it, before its copy (tests/test_gpu_stream.py).
const long g_fail_stream_sub = [] {
  const char* e = std::getenv("S3H_TEST_STREAM_FAIL_SUB");
  return e && *e ? std::atol(e) : -1L;
}();
std::atomic<bool> g_fail_stream_fired{false};

// Host-form staging of destroyed stream objects, kept per device for the next object (an
// uploader creates one per batch of objects: allocating, first-touching and registering 2 x 64
// MiB of pinned pieces plus the device sets cost ~35 ms per object, ~20 % of a C2-sized batch;
// profiles/r05_stream_vs_batch_ab.json).  At most kStagingKeep entries per device; s3h_trim
// frees them.
struct StreamStaging {
  uint8_t* d_hs[2] = {nullptr, nullptr};
  uint64_t d_hs_cap[2] = {0, 0};
  uint8_t* h_piece[2] = {nullptr, nullptr};
  uint64_t h_piece_cap = 0;
};
constexpr size_t kStagingKeep = 2;
struct StagingCache {
  std::mutex m;
  std::map<int, std::vector<StreamStaging>> free;
};
StagingCache& staging_cache() {
  static auto* c = new StagingCache();
  return *c;
}

void staging_release(int device, const StreamStaging& st) {
  DeviceGuard g(device);
  for (uint8_t* p : st.d_hs) (void)hipFree(p);
  pinned_free(st.h_piece[0]);
  pinned_free(st.h_piece[1]);
}


void stream_free(s3h_stream_s* S) {
  DeviceGuard g(S->device);
  if (S->own) (void)hipStreamSynchronize(S->own);
  if (S->copy_s) (void)hipStreamSynchronize(S->copy_s);
  for (hipEvent_t e : {S->staged[0], S->staged[1], S->done})
    if (e) (void)hipEventSynchronize(e);
  s3h_plan_destroy(S->head);
  s3h_plan_destroy(S->body);
  s3h_plan_destroy(S->fin);
  for (void* p : {(void*)S->d_state, (void*)S->d_carry, (void*)S->d_head, (void*)S->d_jobs,
                  (void*)S->d_bits, (void*)S->d_dig})
    (void)hipFree(p);
  pinned_free(S->h_pin);
  if (S->d_hs[0] || S->d_hs[1] || S->h_piece[0]) {  // idle now: keep it for the next object
    StreamStaging st;
    std::copy(S->d_hs, S->d_hs + 2, st.d_hs);
    std::copy(S->d_hs_cap, S->d_hs_cap + 2, st.d_hs_cap);
    std::copy(S->h_piece, S->h_piece + 2, st.h_piece);
    st.h_piece_cap = S->h_piece_cap;
    bool kept = false;
    {
      std::lock_guard<std::mutex> l(staging_cache().m);
      auto& v = staging_cache().free[S->device];
      if (v.size() < kStagingKeep) {
        v.push_back(st);
        kept = true;
      }
    }
    if (!kept) staging_release(S->device, st);
  }
  for (hipEvent_t e : {S->staged[0], S->staged[1], S->done, S->hs_copied[0], S->hs_copied[1],
                       S->hs_hashed[0], S->hs_hashed[1], S->piece_copied[0], S->piece_copied[1]})
    if (e) (void)hipEventDestroy(e);
  if (S->own) (void)hipStreamDestroy(S->own);
  if (S->copy_s) (void)hipStreamDestroy(S->copy_s);
  delete S;
}

int stream_reset(s3h_stream_s* S, hipStream_t s) {
  std::fill(S->total.begin(), S->total.end(), 0);
  std::fill(S->carry.begin(), S->carry.end(), 0u);
  (void)hipGetLastError();
  HIP_TRY(launch_stream_init(S->d_state, S->n, int(S->algo == S3H_ALGO_MD5), s));
  return S3H_OK;
}

// Claims the next staging set for a call on stream `s`: waits (host) until the set's previous
// use has completed, and orders `s` after the previous call's work on any stream (on the
// same stream, stream order does it; a handle reused after hipStreamDestroy is safe too, as
// destroying a stream waits for its work).
int stream_begin(s3h_stream_s* S, hipStream_t s, unsigned* b) {
  *b = S->set;
  S->set ^= 1u;
  S->used_stage = false;
  HIP_TRY(hipEventSynchronize(S->staged[*b]));
  if (!S->done_set || s != S->done_on) HIP_TRY(hipStreamWaitEvent(s, S->done, 0));
  return S3H_OK;
}

// staged[b] is recorded only when the call copied from set b (an update that reused the
// device slots copied nothing; the set's previous record still bounds its last use).
int stream_end(s3h_stream_s* S, hipStream_t s, unsigned b) {
  if (S->used_stage) HIP_TRY(hipEventRecord(S->staged[b], s));
  HIP_TRY(hipEventRecord(S->done, s));
  S->done_on = s;
  S->done_set = true;
  return S3H_OK;
}

// Launch base of update plan `which` (0 head, 1 body) for these slots: the device's slots
// moved by a constant when they fit (see up_offs), else after a refill from staging set b.
int stream_plan_base(s3h_stream_s* S, int which, s3h_plan_s* P, const uint8_t* base,
                     const std::vector<uint64_t>& offs, const std::vector<uint64_t>& lens,
                     unsigned b, hipStream_t s, const uint8_t** launch_base) {
  if (S->up_valid[which] && lens == S->up_lens[which]) {
    bool same = true, have = false;
    uint64_t delta = 0;
    for (uint64_t i = 0; i < S->n && same; ++i) {
      if (!lens[i]) continue;  // an empty slot is never read
      const uint64_t d = offs[i] - S->up_offs[which][i];
      if (!have) {
        delta = d;
        have = true;
      } else {
        same = d == delta;
      }
    }
    if (same) {  // base + off_now == (base + delta) + off_uploaded, modulo 2^64 like the slots
      *launch_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(base) + delta);
      ++S->slot_reuses;
      return S3H_OK;
    }
  }
  ++S->slot_refills;
  S->up_valid[which] = false;
  S->used_stage = true;
  if (int rc = plan_refill(P, offs.data(), lens.data(), true, S->h_slots[b][which], S->h_order[b][which], s))
    return rc;
  S->up_offs[which] = offs;
  S->up_lens[which] = lens;
  S->up_valid[which] = true;
  *launch_base = base;
  return S3H_OK;
}

// Runs one update / final body between stream_begin and stream_end.  stream_end runs on
// every exit after stream_begin succeeded -- staged[b] and `done` are recorded even when the
// body failed midway, so a later call never rewrites a staging set a queued copy still reads,
// nor skips waiting for partly queued work -- and a failed body marks the object failed.
template <typename Body>
int stream_call(s3h_stream_s* S, hipStream_t s, Body body) {
  if (!S->failed.empty())
    return fail(S3H_EINVAL, "stream object failed earlier (%s): destroy it", S->failed.c_str());
  unsigned b = 0;
  if (int rc = stream_begin(S, s, &b)) return rc;
  const int rc = body(b);
  const std::string err = g_err;
  const int rc_end = stream_end(S, s, b);
  if (rc) {
    S->failed = err;
    g_err = err;
    return rc;
  }
  if (rc_end) S->failed = g_err;
  return rc_end;
}

int stream_update_body(s3h_stream_s* S, const uint8_t* base, const uint64_t* offsets,
                       const uint64_t* lengths, hipStream_t s, unsigned b) {
  const uint64_t n = S->n;
  s3h::SpliceJob* const h_jobs = S->h_jobs[b];
  bool any_splice = false, any_head = false, any_body = false;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t L = lengths[i], off = L ? offsets[i] : 0;
    const uint32_t c = S->carry[i];
    s3h::SpliceJob j = {off, 0, c, 0, 0, 0};
    uint64_t body_off = off, B = 0;
    if (L == 0) {
    } else if (c > 0 && c + L < 64) {  // still inside one block: buffer it
      j.h = uint32_t(L);
      j.mode = s3h::kSpliceGrow;
      S->carry[i] = c + uint32_t(L);
    } else {
      j.h = c > 0 ? 64 - c : 0;  // bytes that complete the carried block
      body_off = off + j.h;
      B = (L - j.h) & ~uint64_t(63);
      j.r = uint32_t(L - j.h - B);
      j.tail = body_off + B;
      j.mode = (c > 0 ? s3h::kSpliceHead : 0) | (j.r ? s3h::kSpliceReset : 0);
      S->carry[i] = j.r;
    }
    S->total[i] += L;
    h_jobs[i] = j;
    any_splice |= j.mode != 0;
    any_head |= (j.mode & s3h::kSpliceHead) != 0;
    any_body |= B != 0;
    S->offs[i] = 64 * i;
    S->lens[i] = (j.mode & s3h::kSpliceHead) ? 64 : 0;
    S->offs2[i] = body_off;
    S->lens2[i] = B;
  }
  if (any_splice) {
    S->used_stage = true;
    HIP_TRY(hipMemcpyAsync(S->d_jobs, h_jobs, n * sizeof(s3h::SpliceJob), hipMemcpyHostToDevice, s));
    (void)hipGetLastError();
    HIP_TRY(launch_stream_splice(base, S->d_jobs, S->d_carry, S->d_head, n, s));
  }
  constexpr uint32_t kAppend = s3h::kNoPad | s3h::kResume;
  if (any_head) {  // the blocks straddling the previous update and this one come first
    const uint8_t* hb = nullptr;
    if (int rc = stream_plan_base(S, 0, S->head, S->d_head, S->offs, S->lens, b, s, &hb)) return rc;
    if (int rc = launch_args(S->head, hb, nullptr, S->d_state, 0, 1, 0, kAppend, nullptr, s)) return rc;
  }
  if (any_body) {
    const uint8_t* bb = nullptr;
    if (int rc = stream_plan_base(S, 1, S->body, base, S->offs2, S->lens2, b, s, &bb)) return rc;
    if (int rc = launch_args(S->body, bb, nullptr, S->d_state, 0, S->body->max_blocks, 0, kAppend, nullptr, s)) return rc;
  }
  return S3H_OK;
}

int stream_update(s3h_stream_s* S, const uint8_t* base, const uint64_t* offsets,
                  const uint64_t* lengths, hipStream_t s) {
  return stream_call(S, s, [&](unsigned b) { return stream_update_body(S, base, offsets, lengths, s, b); });
}

// The error words of the stream's three plans (head / body / final launches), once `s` has
// run everything before: plan_check.  Every plan's word is read and cleared (a fault of one
// must not be reported again by a later check), then the first failure is returned.
int stream_check(s3h_stream_s* S, hipStream_t s) {
  int first = S3H_OK;
  std::string msg;
  for (s3h_plan_s* P : {S->head, S->body, S->fin})
    if (int rc = plan_check(P, s); rc && !first) {
      first = rc;
      msg = g_err;
    }
  if (first) g_err = msg;
  return first;
}

int stream_final_body(s3h_stream_s* S, uint32_t* d_digests, hipStream_t s, unsigned b) {
  const uint64_t n = S->n;
  for (uint64_t i = 0; i < n; ++i) {
    S->offs[i] = 64 * i;
    S->lens[i] = S->carry[i];
    S->h_bits[b][i] = S->total[i] << 3;
  }
  S->used_stage = true;
  HIP_TRY(hipMemcpyAsync(S->d_bits, S->h_bits[b], n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  if (int rc = plan_refill(S->fin, S->offs.data(), S->lens.data(), false, S->h_slots[b][0], S->h_order[b][0], s)) return rc;
  // one or two padded blocks per message, starting from the appended state
  if (int rc = launch_args(S->fin, S->d_carry, d_digests, S->d_state, 0, S->fin->max_blocks, 0,
                           s3h::kResume, S->d_bits, s)) return rc;
  return stream_reset(S, s);
}

int stream_final(s3h_stream_s* S, uint32_t* d_digests, hipStream_t s) {
  return stream_call(S, s, [&](unsigned b) { return stream_final_body(S, d_digests, s, b); });
}

}  // namespace

namespace s3h::host {

void staging_trim() {
  std::map<int, std::vector<StreamStaging>> all;
  {
    std::lock_guard<std::mutex> l(staging_cache().m);
    all.swap(staging_cache().free);
  }
  for (auto& kv : all)
    for (auto& st : kv.second) staging_release(kv.first, st);
}

}  // namespace s3h::host

extern "C" {

int s3h_stream_create(int device, int algo, uint64_t n, int kernel, s3h_stream_t* out) {
  if (!out) return fail(S3H_EINVAL, "stream: null out-pointer");
  *out = nullptr;
  if (n == 0 || n > kMaxParts) return fail(S3H_EINVAL, "stream: need 0 < n <= 2^31");
  std::vector<uint64_t> zeros(n, 0);
  auto* S = new s3h_stream_s();
  S->device = device;
  S->algo = algo;
  S->n = n;
  S->total.assign(n, 0);
  S->carry.assign(n, 0);
  S->offs.assign(n, 0);
  S->lens.assign(n, 0);
  S->offs2.assign(n, 0);
  S->lens2.assign(n, 0);
  int rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->head);
  if (!rc) rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->body);
  if (!rc) rc = plan_build(device, algo, zeros.data(), zeros.data(), n, kernel, &S->fin);
  if (rc) {
    stream_free(S);
    return rc;
  }
  DeviceGuard g(device);
  const char* what = "chaining state";
  hipError_t e = hipMalloc(&S->d_state, n * 32);
  if (e == hipSuccess) e = hipMalloc(&S->d_carry, n * 64), what = "carries";
  if (e == hipSuccess) e = hipMalloc(&S->d_head, n * 64), what = "head blocks";
  if (e == hipSuccess) e = hipMalloc(&S->d_jobs, n * sizeof(s3h::SpliceJob)), what = "splice jobs";
  if (e == hipSuccess) e = hipMalloc(&S->d_bits, n * 8), what = "bit lengths";
  // per message and set: a splice job, two slots, the bit length, two order entries (8-B
  // aligned in this order)
  const size_t per = sizeof(s3h::SpliceJob) + 2 * sizeof(s3h::Slot) + 8 + 2 * 4;
  if (e == hipSuccess) {
    e = pinned_alloc(reinterpret_cast<void**>(&S->h_pin), 2 * n * per, device_place(device).node);
    what = e == hipSuccess ? "events / stream" : "pinned update staging";
  }
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    uint8_t* pin = S->h_pin + b * n * per;
    S->h_jobs[b] = reinterpret_cast<s3h::SpliceJob*>(pin);
    S->h_slots[b][0] = reinterpret_cast<s3h::Slot*>(pin + n * sizeof(s3h::SpliceJob));
    S->h_slots[b][1] = S->h_slots[b][0] + n;
    S->h_bits[b] = reinterpret_cast<uint64_t*>(S->h_slots[b][1] + n);
    S->h_order[b][0] = reinterpret_cast<uint32_t*>(S->h_bits[b] + n);
    S->h_order[b][1] = S->h_order[b][0] + n;
    e = hipEventCreateWithFlags(&S->staged[b], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&S->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&S->own, hipStreamNonBlocking);
  if (e == hipSuccess) {
    rc = stream_reset(S, S->own);
    // every event recorded once, so the first calls' waits have something to wait for
    for (hipEvent_t ev : {S->staged[0], S->staged[1], S->done})
      if (!rc && hipEventRecord(ev, S->own) != hipSuccess) rc = fail(S3H_EHIP, "stream: event record failed");
    if (!rc && hipStreamSynchronize(S->own) != hipSuccess) rc = fail(S3H_EHIP, "stream: init failed");
  } else {
    (void)hipGetLastError();
    rc = fail(e == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "stream (%llu messages): %s: %s",
              (unsigned long long)n, what, hipGetErrorString(e));
  }
  if (rc) {
    stream_free(S);
    return rc;
  }
  *out = S;
  return S3H_OK;
}

int s3h_stream_update_device(s3h_stream_t S, const void* d_base, const uint64_t* offsets,
                             const uint64_t* lengths, void* stream) {
  if (!S || !lengths || (!offsets && S->n)) return fail(S3H_EINVAL, "stream update: null argument");
  bool any = false;
  for (uint64_t i = 0; i < S->n; ++i) any |= lengths[i] != 0;
  if (any && !d_base) return fail(S3H_EINVAL, "stream update: null d_base");
  DeviceGuard g(S->device);
  return stream_update(S, static_cast<const uint8_t*>(d_base), offsets, lengths,
                       static_cast<hipStream_t>(stream));
}

int s3h_stream_final_device(s3h_stream_t S, uint32_t* d_digests, void* stream) {
  if (!S || !d_digests) return fail(S3H_EINVAL, "stream final: null argument");
  DeviceGuard g(S->device);
  return stream_final(S, d_digests, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {

// The copy threads of host-form stream updates: one pool per device, shared by every stream
// object on it (their copy phases take turns; each pool is as wide as the CPUs the process may
// use, on the device's NUMA node), created on first use and kept for the process.
struct StreamPools {
  std::mutex m;
  std::map<int, std::pair<std::unique_ptr<CopyPool>, std::unique_ptr<std::mutex>>> by_device;
};
StreamPools& stream_pools() {
  static auto* p = new StreamPools();  // never destroyed: threads may outlive static teardown
  return *p;
}

// fn(i) for i in [0, n) on `device`'s stream copy pool (exclusive while it runs)
void stream_pool_run(int device, uint64_t n, const std::function<void(uint64_t)>& fn) {
  StreamPools& P = stream_pools();
  CopyPool* pool;
  std::mutex* run_mu;
  {
    std::lock_guard<std::mutex> l(P.m);
    auto& e = P.by_device[device];
    if (!e.first) {
      e.first.reset(new CopyPool(host_threads_per_device(1) - 1, device_place(device)));
      e.second.reset(new std::mutex());
    }
    pool = e.first.get();
    run_mu = e.second.get();
  }
  std::lock_guard<std::mutex> l(*run_mu);
  pool->run(n, fn);
}

// One host-form update of at most a few hundred MiB (s3h_stream_update_host splits larger
// ones): the chunks are packed at 64-B aligned offsets into device staging set b and hashed on
// `own` once the set's copy has landed; the copy of the next update overlaps this hash.
//   pinned chunks of equal length at a constant stride -> one 2-D DMA;
//   a few other pinned chunks                          -> one DMA each;
//   anything else (pageable, or many ragged pinned)    -> copy threads fill pinned pieces,
//                                                         one DMA per piece.
// Returns once the chunks may be released by the caller.
// *queued is set once the call has queued work that reads the caller's chunks or advances the
// messages' bookkeeping (a failure after that leaves the object failed).
int stream_host_update_one(s3h_stream_s* S, const uint8_t* const* chunks, const uint64_t* lengths,
                           bool* queued) {
  const uint64_t n = S->n;
  std::vector<uint64_t> offs(n);
  uint64_t sum = 0, L0 = 0;
  bool equal = true;
  for (uint64_t i = 0; i < n; ++i) {
    offs[i] = sum;
    sum += (lengths[i] + 63) & ~uint64_t(63);
    if (i == 0) L0 = lengths[0];
    equal = equal && lengths[i] == L0;
  }
  const unsigned b = S->hs_set;
  S->hs_set ^= 1u;
  if (sum > S->d_hs_cap[b]) {
    HIP_TRY(hipEventSynchronize(S->hs_hashed[b]));  // the set's last hash has read it
    (void)hipFree(S->d_hs[b]);
    S->d_hs[b] = nullptr;
    S->d_hs_cap[b] = 0;
    HIP_TRY(hipMalloc(&S->d_hs[b], sum));
    S->d_hs_cap[b] = sum;
  }
  bool wait_copy = false;  // the DMA reads the caller's memory: wait for it before returning
  if (sum) {
    // set b is rewritten only after the hash that read it (two updates ago) has run
    HIP_TRY(hipStreamWaitEvent(S->copy_s, S->hs_hashed[b], 0));
    const bool pinned = all_pinned(chunks, lengths, nullptr, n);
    // equal non-empty chunks at one positive stride (ranges of one buffer): one 2-D DMA
    bool strided = pinned && equal && L0 > 0 && n > 1;
    const uintptr_t c0 = reinterpret_cast<uintptr_t>(chunks[0]);
    const uint64_t stride = strided ? uint64_t(reinterpret_cast<uintptr_t>(chunks[1]) - c0) : 0;
    strided = strided && stride >= L0 && stride < (uint64_t(1) << 62);
    for (uint64_t i = 2; strided && i < n; ++i)
      strided = uint64_t(reinterpret_cast<uintptr_t>(chunks[i]) - c0) == i * stride;
    if (strided) {
      *queued = true;
      HIP_TRY(hipMemcpy2DAsync(S->d_hs[b], (L0 + 63) & ~uint64_t(63), chunks[0], stride, L0, n,
                               hipMemcpyHostToDevice, S->copy_s));
      wait_copy = true;
    } else if (pinned && n <= kStreamDmaChunks) {
      *queued = true;
      for (uint64_t i = 0; i < n; ++i)
        if (lengths[i])
          HIP_TRY(hipMemcpyAsync(S->d_hs[b] + offs[i], chunks[i], lengths[i], hipMemcpyHostToDevice, S->copy_s));
      wait_copy = true;
    } else {
      // copy threads fill pinned piece q while piece q^1's DMA runs
      const uint64_t P = std::min<uint64_t>(sum, kStreamPiece);
      if (P > S->h_piece_cap) {
        for (hipEvent_t e : {S->piece_copied[0], S->piece_copied[1]}) HIP_TRY(hipEventSynchronize(e));
        pinned_free(S->h_piece[0]);
        pinned_free(S->h_piece[1]);
        S->h_piece[0] = S->h_piece[1] = nullptr;
        S->h_piece_cap = 0;
        const int node = device_place(S->device).node;
        for (uint8_t*& h : S->h_piece)
          HIP_TRY(pinned_alloc(reinterpret_cast<void**>(&h), P, node));
        S->h_piece_cap = P;
      }
      for (uint64_t lo = 0; lo < sum; lo += P) {
        const unsigned q = S->piece_next;  // alternates across updates too
        S->piece_next ^= 1u;
        const uint64_t hi = std::min(sum, lo + P);
        HIP_TRY(hipEventSynchronize(S->piece_copied[q]));  // its previous DMA has read it
        // the chunks overlapping [lo, hi) of the packed layout (offs ascending)
        const uint64_t i0 = uint64_t(std::upper_bound(offs.begin(), offs.end(), lo) - offs.begin()) - 1;
        const uint64_t i1 = uint64_t(std::lower_bound(offs.begin(), offs.end(), hi) - offs.begin());
        uint8_t* const dst = S->h_piece[q];
        stream_pool_run(S->device, i1 - i0, [&](uint64_t k) {
          const uint64_t i = i0 + k, a = std::max(offs[i], lo), e = std::min(offs[i] + lengths[i], hi);
          if (e > a) std::memcpy(dst + (a - lo), chunks[i] + (a - offs[i]), e - a);
        });
        *queued = true;
        HIP_TRY(hipMemcpyAsync(S->d_hs[b] + lo, dst, hi - lo, hipMemcpyHostToDevice, S->copy_s));
        HIP_TRY(hipEventRecord(S->piece_copied[q], S->copy_s));
      }
    }
    HIP_TRY(hipEventRecord(S->hs_copied[b], S->copy_s));
    HIP_TRY(hipStreamWaitEvent(S->own, S->hs_copied[b], 0));
  }
  *queued = true;
  const int rc = stream_update(S, S->d_hs[b], offs.data(), lengths, S->own);
  HIP_TRY(hipEventRecord(S->hs_hashed[b], S->own));
  if (wait_copy) HIP_TRY(hipEventSynchronize(S->hs_copied[b]));
  return rc;
}

}  // namespace

extern "C" {

// A large update is appended as consecutive sub-updates of at most `sl` bytes of every chunk
// (64-B multiples: no carry between them), so the copy of one overlaps the hash of the one
// before -- appending a chunk in pieces is the same as appending it whole.
int s3h_stream_update_host(s3h_stream_t S, const uint8_t* const* chunks, const uint64_t* lengths) {
  if (!S || !chunks || !lengths) return fail(S3H_EINVAL, "stream update: null argument");
  if (!S->failed.empty())
    return fail(S3H_EINVAL, "stream object failed earlier (%s): destroy it", S->failed.c_str());
  const uint64_t n = S->n;
  uint64_t sum = 0, longest = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (lengths[i] && !chunks[i]) return fail(S3H_EINVAL, "stream update: chunk %llu is null", (unsigned long long)i);
    sum += (lengths[i] + 63) & ~uint64_t(63);
    longest = std::max(longest, lengths[i]);
  }
  DeviceGuard g(S->device);
  if (!S->copy_s) {
    {  // staging left by an earlier object on this device, if any
      std::lock_guard<std::mutex> l(staging_cache().m);
      auto& v = staging_cache().free[S->device];
      if (!v.empty()) {
        const StreamStaging st = v.back();
        v.pop_back();
        std::copy(st.d_hs, st.d_hs + 2, S->d_hs);
        std::copy(st.d_hs_cap, st.d_hs_cap + 2, S->d_hs_cap);
        std::copy(st.h_piece, st.h_piece + 2, S->h_piece);
        S->h_piece_cap = st.h_piece_cap;
      }
    }
    HIP_TRY(hipStreamCreateWithFlags(&S->copy_s, hipStreamNonBlocking));
    for (hipEvent_t* e : {&S->hs_copied[0], &S->hs_copied[1], &S->hs_hashed[0], &S->hs_hashed[1],
                          &S->piece_copied[0], &S->piece_copied[1]})
      HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  const uint64_t sl = std::max<uint64_t>(kStreamSubMin, (kStreamSubBytes / std::max<uint64_t>(n, 1)) & ~uint64_t(63));
  // A sub-update that fails after an earlier one (or after queueing its own copies) leaves
  // the messages partly appended: the object is failed, so a retry cannot append the first
  // pieces twice, and the copy stream is drained before returning, so no DMA still reads the
  // caller's chunks (advisor r5).  A failure before anything was queued leaves it usable.
  uint64_t sub = 0;
  bool queued = false;
  auto one = [&](const uint8_t* const* c, const uint64_t* l) {
    int rc;
    if (g_fail_stream_sub >= 0 && sub == uint64_t(g_fail_stream_sub) &&  // test hook (env)
        !g_fail_stream_fired.exchange(true))
      rc = fail(S3H_ENOMEM, "stream update: injected failure of sub-update %llu", (unsigned long long)sub);
    else
      rc = stream_host_update_one(S, c, l, &queued);
    if (rc != S3H_OK) {
      const std::string err = g_err;
      (void)hipStreamSynchronize(S->copy_s);
      (void)hipGetLastError();
      if ((queued || sub > 0) && S->failed.empty()) S->failed = err;
      g_err = err;
    }
    ++sub;
    return rc;
  };
  if (sum <= 2 * kStreamSubBytes || longest <= sl) return one(chunks, lengths);
  std::vector<const uint8_t*> p(n);
  std::vector<uint64_t> l(n);
  for (uint64_t at = 0; at < longest; at += sl) {
    for (uint64_t i = 0; i < n; ++i) {
      l[i] = lengths[i] > at ? std::min(sl, lengths[i] - at) : 0;
      p[i] = l[i] ? chunks[i] + at : nullptr;
    }
    if (int rc = one(p.data(), l.data())) return rc;
  }
  return S3H_OK;
}

int s3h_stream_final_host(s3h_stream_t S, uint32_t* digests) {
  if (!S || !digests) return fail(S3H_EINVAL, "stream final: null argument");
  DeviceGuard g(S->device);
  const uint64_t bytes = S->n * digest_words(S->algo) * 4;
  if (!S->d_dig) HIP_TRY(hipMalloc(&S->d_dig, S->n * 32));
  int rc = stream_final(S, S->d_dig, S->own);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(digests, S->d_dig, bytes, hipMemcpyDeviceToHost, S->own));
  HIP_TRY(hipStreamSynchronize(S->own));
  return stream_check(S, S->own);
}

int s3h_stream_status(s3h_stream_t S, void* stream) {
  if (!S) return fail(S3H_EINVAL, "stream status: null stream");
  DeviceGuard g(S->device);
  return stream_check(S, static_cast<hipStream_t>(stream));
}

int s3h_stream_stats(s3h_stream_t S, uint64_t* slot_reuses, uint64_t* slot_refills) {
  if (!S) return fail(S3H_EINVAL, "stream stats: null stream");
  if (slot_reuses) *slot_reuses = S->slot_reuses;
  if (slot_refills) *slot_refills = S->slot_refills;
  return S3H_OK;
}

int s3h_stream_total(s3h_stream_t S, uint64_t i, uint64_t* total) {
  if (!S || !total || i >= S->n) return fail(S3H_EINVAL, "stream total: bad argument");
  *total = S->total[i];
  return S3H_OK;
}

int s3h_stream_destroy(s3h_stream_t S) {
  if (S) stream_free(S);
  return S3H_OK;
}

}  // extern "C"
