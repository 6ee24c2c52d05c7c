// host_path.cpp -- the host-resident path: parts in host memory (pinned or pageable) or byte
// ranges of a file are streamed through HBM and hashed on the way (s3h_*_batch_host,
// s3h_*_file_parts, s3h_verify_batch_host), sharded over devices with no collective, each
// device running one merged batch at a time through its cached context (host_queue.hpp).
//
// Pipeline per device shard: a plan over slot-strided offsets, a 3-slot HBM ring of n x slice
// bytes, one copy stream and one hash stream per algorithm; slice k of every part is copied
// while slice k-1 is hashed by a resumable launch (sha256_stream semantics, lib/hash/
// sha256.cpp:84-144).  Many small parts go in groups of whole parts instead (run_host_groups).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "copy_pool.hpp"
#include "host_queue.hpp"
#include "internal.hpp"

namespace s3h::host {

thread_local unsigned g_stage_threads_cap = 0;

namespace {

// ------------------------------------------------------------------ host-path context
// Everything one host-path call needs on a device -- streams, ring events, the copy-thread
// pool, plans, digest buffers, the pinned geometry staging, the HBM ring and the pinned
// staging ring -- is cached per device and reused by the next call (an uploader hashes file
// after file; creating and freeing these per call cost ~8 ms of a 27 ms call on a 512 MiB
// file, profiles/r01_app_upload_hash.txt).  Buffers only grow; an HBM ring above
// kKeepRingBytes is freed when the call returns, so a cached context holds at most
// kKeepRingBytes of HBM plus its staging; s3h_trim() frees idle contexts.
constexpr uint64_t kStageSlot = 32ull << 20;     // pinned staging bytes per ring slot
// Group mode (run_host_groups) for many small parts (<= kGroupMaxPart, host_limits.hpp): a
// group's copy must outlast its longest part's chain (~69 MB/s per chain vs ~52 GB/s of PCIe:
// 750 x), groups between kGroupMin and kGroupMax bytes.
// Groups of 1,536 x the longest part where two of them fit the HBM ring a context keeps
// between calls (release_large), else 768 x: 20,000 / 100,000 pinned parts of <= 128 KiB at
// 768 x 40.9 / 46.8 GiB/s, at 1,536 x 46.7 / 49.6 (profiles/r05_group_sweep.log).
constexpr uint64_t kGroupCopyPerChain = 1536, kGroupCopyPerChainMin = 768;
constexpr uint64_t kGroupMin = 64ull << 20, kGroupMax = 1ull << 30;
constexpr uint64_t kKeepRingBytes = 1ull << 30;  // largest HBM ring kept between calls
constexpr uint64_t kGroupChunk = 64ull << 20;    // group mode: pinned staging per packed chunk
// Staged slices are at least 32 KiB up to 4,096 parts per device (slots of up to 128 MiB),
// 128 MiB / n beyond: a file range's pread costs more than it moves below ~32 KiB, and each
// slice of memory parts costs a copy-thread dispatch and a launch (4,000 parts of U[256 KiB,
// 4 MiB] in 8 KiB slices: 512 slices, 26.6 GiB/s).
constexpr uint64_t kFileStageSlot = 128ull << 20;


struct HostCtx {
  int device = 0;
  Place place;  // NUMA node of the pinned staging and CPUs of the copy threads (device_place)
  hipStream_t copy_s = nullptr, hash_s[kHostMaxAlgo] = {};
  hipEvent_t copied[kHostRing] = {}, hashed[kHostRing][kHostMaxAlgo] = {};
  hipEvent_t chunk_copied[kHostRing] = {};  // group mode: a staging chunk's DMA has run
  std::unique_ptr<CopyPool> pool;
  s3h_plan_s* plan[kHostMaxAlgo] = {};
  uint32_t* d_dig[kHostMaxAlgo] = {};
  uint64_t dig_bytes[kHostMaxAlgo] = {};
  uint8_t* pin = nullptr;    // pinned slot/order staging of both plans' geometry
  uint64_t pin_bytes = 0;
  uint8_t* ring = nullptr;   // HBM ring: kHostRing slots of n * slice bytes
  uint64_t ring_bytes = 0;
  uint8_t* stage = nullptr;  // pinned staging ring (pageable and file sources)
  uint64_t stage_bytes = 0;
  // group mode (run_host_groups): two plans per algorithm (group k uses set k & 1) and their
  // pinned geometry staging
  s3h_plan_s* gplan[2][kHostMaxAlgo] = {};
  uint8_t* gpin = nullptr;
  uint64_t gpin_bytes = 0;

  hipError_t ensure_streams() {
    hipError_t e = hipSuccess;
    if (!copy_s) e = hipStreamCreateWithFlags(&copy_s, hipStreamNonBlocking);
    for (hipStream_t& st : hash_s)
      if (e == hipSuccess && !st) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int r = 0; r < kHostRing && e == hipSuccess; ++r) {
      if (!copied[r]) e = hipEventCreateWithFlags(&copied[r], hipEventDisableTiming);
      if (e == hipSuccess && !chunk_copied[r]) e = hipEventCreateWithFlags(&chunk_copied[r], hipEventDisableTiming);
      for (hipEvent_t& h : hashed[r])
        if (e == hipSuccess && !h) e = hipEventCreateWithFlags(&h, hipEventDisableTiming);
    }
    return e;
  }
  static hipError_t grow_dev(uint8_t** p, uint64_t* have, uint64_t want) {
    if (*have >= want) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    const hipError_t e = hipMalloc(p, want);
    if (e == hipSuccess) *have = want;
    return e;
  }
  // pinned host buffers on the context's NUMA node (place.node; < 0: the runtime's choice)
  hipError_t grow_pinned(uint8_t** p, uint64_t* have, uint64_t want) {
    if (*have >= want) return hipSuccess;
    pinned_free(*p);
    *p = nullptr;
    *have = 0;
    const hipError_t e = pinned_alloc(reinterpret_cast<void**>(p), want, place.node);
    if (e == hipSuccess) *have = want;
    return e;
  }
  hipError_t ensure_digests(int a, uint64_t bytes) {
    return grow_dev(reinterpret_cast<uint8_t**>(&d_dig[a]), &dig_bytes[a], bytes);
  }
  CopyPool* ensure_pool(unsigned workers) {  // exactly `workers` threads beside the caller
    if (!pool || pool->size() != workers) pool.reset(new CopyPool(workers, place));
    return pool.get();
  }
  // plan[a] for algorithm `algo` with room for n parts (reallocated only to grow)
  int ensure_plan(int a, int algo, uint64_t n) {
    if (plan[a] && plan[a]->algo == algo && plan[a]->cap >= n) return S3H_OK;
    s3h_plan_destroy(plan[a]);
    plan[a] = nullptr;
    return plan_alloc(device, algo, std::max<uint64_t>(n, 1024), &plan[a]);
  }
  // pinned geometry staging for plan a: cap slots + cap order entries
  s3h::Slot* h_slots(int a) {
    return reinterpret_cast<s3h::Slot*>(pin) + uint64_t(a) * pin_cap();
  }
  uint32_t* h_order(int a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<s3h::Slot*>(pin) + kHostMaxAlgo * pin_cap()) +
           uint64_t(a) * pin_cap();
  }
  uint64_t pin_cap() const { return pin_bytes / (kHostMaxAlgo * (sizeof(s3h::Slot) + 4)); }
  int ensure_gplan(int q, int a, int algo, uint64_t n) {
    s3h_plan_s*& P = gplan[q][a];
    if (P && P->algo == algo && P->cap >= n) return S3H_OK;
    s3h_plan_destroy(P);
    P = nullptr;
    return plan_alloc(device, algo, std::max<uint64_t>(n, 1024), &P);
  }
  uint64_t gpin_cap() const { return gpin_bytes / (2 * kHostMaxAlgo * (sizeof(s3h::Slot) + 4)); }
  hipError_t ensure_gpin(uint64_t n) {
    return grow_pinned(&gpin, &gpin_bytes, 2 * kHostMaxAlgo * std::max<uint64_t>(n, 1024) * (sizeof(s3h::Slot) + 4));
  }
  s3h::Slot* gslots(int q, int a) {
    return reinterpret_cast<s3h::Slot*>(gpin) + uint64_t(q * kHostMaxAlgo + a) * gpin_cap();
  }
  uint32_t* gorder(int q, int a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<s3h::Slot*>(gpin) + 2 * kHostMaxAlgo * gpin_cap()) +
           uint64_t(q * kHostMaxAlgo + a) * gpin_cap();
  }
  hipError_t ensure_pin(uint64_t n) {
    return grow_pinned(&pin, &pin_bytes, kHostMaxAlgo * std::max<uint64_t>(n, 1024) * (sizeof(s3h::Slot) + 4));
  }
  void sync() {
    if (copy_s) (void)hipStreamSynchronize(copy_s);
    for (hipStream_t st : hash_s)
      if (st) (void)hipStreamSynchronize(st);
  }
  void release_large() {  // after a call: do not keep a large HBM ring or staging ring
    if (ring_bytes > kKeepRingBytes) {
      (void)hipFree(ring);
      ring = nullptr;
      ring_bytes = 0;
    }
    if (stage_bytes > kHostRing * kFileStageSlot) {
      pinned_free(stage);
      stage = nullptr;
      stage_bytes = 0;
    }
  }
  ~HostCtx() {
    DeviceGuard g(device);
    sync();
    pool.reset();
    for (hipEvent_t e : copied)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : chunk_copied)
      if (e) (void)hipEventDestroy(e);
    for (auto& row : hashed)
      for (hipEvent_t e : row)
        if (e) (void)hipEventDestroy(e);
    if (copy_s) (void)hipStreamDestroy(copy_s);
    for (hipStream_t st : hash_s)
      if (st) (void)hipStreamDestroy(st);
    for (uint32_t* d : d_dig)
      if (d) (void)hipFree(d);
    for (s3h_plan_s* p : plan)
      if (p) s3h_plan_destroy(p);
    for (auto& row : gplan)
      for (s3h_plan_s* p : row)
        if (p) s3h_plan_destroy(p);
    if (ring) (void)hipFree(ring);
    pinned_free(stage);
    pinned_free(pin);
    pinned_free(gpin);
  }
};

// One cached context per device.  Host calls on a device run one batch at a time (the
// device queue below merges concurrent callers), so the context is normally free; a call that
// still finds it busy gets a private one.
struct HostCtxCache {
  std::mutex m;
  std::vector<HostCtx*> v;  // indexed by device
  std::vector<bool> busy;
  HostCtx* acquire(int device) {
    std::lock_guard<std::mutex> l(m);
    if (v.size() <= size_t(device)) {
      v.resize(device + 1, nullptr);
      busy.resize(device + 1, false);
    }
    if (busy[device]) {
      auto* p = new HostCtx();
      p->device = device;
      p->place = device_place(device);
      return p;
    }
    if (!v[device]) {
      v[device] = new HostCtx();
      v[device]->device = device;
      v[device]->place = device_place(device);
    }
    busy[device] = true;
    return v[device];
  }
  // ok: the call succeeded (keep the cached context); a failed call drops its context.
  void release(HostCtx* c, bool ok) {
    {
      DeviceGuard g(c->device);
      c->release_large();
    }
    {
      std::lock_guard<std::mutex> l(m);
      if (v[c->device] == c) {
        busy[c->device] = false;
        if (ok) return;
        v[c->device] = nullptr;
      }
    }
    delete c;
  }
  // NUMA record of device's cached context (false: none, or busy in a call right now)
  bool numa_of(int device, s3h_host_numa_t* info) {
    std::lock_guard<std::mutex> l(m);
    if (device < 0 || size_t(device) >= v.size() || !v[device] || busy[device]) return false;
    const HostCtx* c = v[device];
    info->staging_node = c->stage ? mem_node(c->stage) : -1;
    info->threads_node = c->pool ? c->pool->bound_node() : -1;
    info->copy_threads = c->pool ? int(c->pool->size()) : 0;
    return true;
  }
  void trim() {
    std::vector<HostCtx*> idle;
    {
      std::lock_guard<std::mutex> l(m);
      for (size_t d = 0; d < v.size(); ++d)
        if (v[d] && !busy[d]) {
          idle.push_back(v[d]);
          v[d] = nullptr;
        }
    }
    for (HostCtx* c : idle) delete c;
  }
};

HostCtxCache& host_ctx_cache() {
  static HostCtxCache* c = new HostCtxCache();  // never destroyed: HIP may be gone at exit
  return *c;
}

// S3H_TRACE_HOST=1: per-shard phase times of the host path on stderr (setup, pipeline, drain).
bool trace_host() {
  static const bool on = [] {
    const char* e = std::getenv("S3H_TRACE_HOST");
    return e && std::atoi(e) == 1;
  }();
  return on;
}


// Many small parts: slicing every part (run_host_shard) would cut them into slices of a few
// hundred bytes (the staging slot holds n slices) or issue one DMA per part and slice, so
// instead the parts go in GROUPS of consecutive parts (~kGroupCopyPerChain x the longest part,
// in [kGroupMin, kGroupMax] bytes): each group is packed into pinned staging by the copy
// threads (memcpy / pread; pinned parts that are one contiguous range of a buffer are DMA'd as
// that range instead), copied by one DMA into one of two HBM group buffers, and hashed WHOLE
// by one launch per algorithm while the next group is packed and copied.
int run_host_groups(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                    const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                    bool pinned) {
  const uint64_t n = sh.parts.size();
  std::vector<uint64_t> lens(n), poff(n);
  uint64_t longest = 0;
  for (uint64_t j = 0; j < n; ++j) {
    lens[j] = lengths[sh.parts[j]];
    longest = std::max(longest, lens[j]);
  }
  // the two group buffers stay within a quarter of the free HBM, as the slice ring does
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const uint64_t budget = std::min<uint64_t>(16ull << 30, (free_b + C.ring_bytes) / 4);
  const uint64_t longest64 = std::max<uint64_t>(64, (longest + 63) & ~uint64_t(63));
  uint64_t per_chain = kGroupCopyPerChain;
  if (const char* e = std::getenv("S3H_GROUP_COPY_PER_CHAIN"))  // measurements only
    if (std::atoll(e) > 0) per_chain = uint64_t(std::atoll(e));
  // beyond 768 x only while two groups fit the HBM ring a context keeps between calls
  // (release_large) -- reallocating it per call costs more than the overlap gains
  const uint64_t keep = kKeepRingBytes / 2;
  const uint64_t want = std::max(kGroupCopyPerChainMin * longest64, std::min(per_chain * longest64, keep));
  const uint64_t G = std::max(longest64, std::min({kGroupMax, std::max(kGroupMin, want), budget / 2 / 64 * 64}));
  std::vector<uint64_t> gstart{0}, gbytes;
  uint64_t acc = 0;
  for (uint64_t j = 0; j < n; ++j) {
    const uint64_t a = (lens[j] + 63) & ~uint64_t(63);
    if (acc + a > G && acc > 0) {
      gbytes.push_back(acc);
      gstart.push_back(j);
      acc = 0;
    }
    poff[j] = acc;
    acc += a;
  }
  gbytes.push_back(acc);
  gstart.push_back(n);
  const uint64_t ngroups = gbytes.size();
  uint64_t maxb = 64, maxparts = 1;
  for (uint64_t k = 0; k < ngroups; ++k) {
    maxb = std::max(maxb, gbytes[k]);
    maxparts = std::max(maxparts, gstart[k + 1] - gstart[k]);
  }
  // pinned parts that form one increasing range of a buffer with small gaps: DMA'd as is
  const uint8_t* const* parts = src.parts;
  auto contiguous = [&](uint64_t j0, uint64_t j1, uint64_t* span) {
    if (!pinned || !parts) return false;
    const uint8_t* lo = nullptr;
    const uint8_t* hi = nullptr;
    for (uint64_t j = j0; j < j1; ++j) {
      if (!lens[j]) continue;
      const uint8_t* p = parts[sh.parts[j]];
      if (hi && p < hi) return false;
      if (!lo) lo = p;
      hi = p + lens[j];
    }
    *span = lo ? uint64_t(hi - lo) : 0;
    // one DMA covers [lo, hi): it must lie inside ONE page-locked allocation -- parts from
    // separately pinned buffers in increasing address order have unregistered pages between
    // them (advisor r5), and are packed like pageable parts instead
    return *span <= maxb && (!lo || pinned_range(lo, *span));
  };
  HIP_TRY(C.ensure_streams());
  hipError_t ce = HostCtx::grow_dev(&C.ring, &C.ring_bytes, 2 * maxb);
  if (ce != hipSuccess) {
    (void)hipGetLastError();
    return fail(S3H_ENOMEM, "host group buffers (2 x %llu B of HBM): %s", (unsigned long long)maxb,
                hipGetErrorString(ce));
  }
  bool any_staged = false;
  for (uint64_t k = 0; k < ngroups && !any_staged; ++k) {
    uint64_t span = 0;
    any_staged = !contiguous(gstart[k], gstart[k + 1], &span);
  }
  // packed groups go through kHostRing pinned chunks of kGroupChunk bytes (a part always fits
  // one): the staging is sized for the copy in flight, not for the group the GPU hashes
  const uint64_t chunk = std::max(kGroupChunk, longest64);
  if (any_staged) {
    ce = C.grow_pinned(&C.stage, &C.stage_bytes, kHostRing * chunk);
    if (ce != hipSuccess) {
      (void)hipGetLastError();
      return fail(S3H_ENOMEM, "pinned group staging (%d x %llu B): %s", kHostRing,
                  (unsigned long long)chunk, hipGetErrorString(ce));
    }
  }
  bool chunk_used[kHostRing] = {};
  uint64_t chunk_next = 0;
  HIP_TRY(C.ensure_gpin(maxparts));
  for (int q = 0; q < 2; ++q)
    for (int a = 0; a < nalgo; ++a) {
      if (int rc = C.ensure_gplan(q, a, algos[a], maxparts)) return rc;
      HIP_TRY(hipMemsetAsync(C.gplan[q][a]->d_err, 0, sizeof(uint32_t), C.copy_s));
    }
  for (int a = 0; a < nalgo; ++a)
    HIP_TRY(C.ensure_digests(a, n * digest_words(algos[a]) * sizeof(uint32_t)));
  CopyPool* pool = any_staged ? C.ensure_pool(shard_threads(sh) - 1) : nullptr;
  std::vector<uint64_t> offs;
  for (uint64_t k = 0; k < ngroups; ++k) {
    const int q = int(k & 1);
    const uint64_t j0 = gstart[k], j1 = gstart[k + 1], ng = j1 - j0;
    uint8_t* const dgrp = C.ring + uint64_t(q) * maxb;
    // group k-2 used set q: its DMAs (host staging and geometry staging) must have run, and
    // its hashes (the HBM group buffer and the plans' device slots) before the copy stream
    // overwrites them
    if (k >= 2) {
      HIP_TRY(hipEventSynchronize(C.copied[q]));
      for (int a = 0; a < nalgo; ++a) HIP_TRY(hipStreamWaitEvent(C.copy_s, C.hashed[q][a], 0));
    }
    uint64_t span = 0;
    const bool direct = contiguous(j0, j1, &span);
    offs.assign(ng, 0);
    const uint8_t* base = nullptr;
    for (uint64_t t = 0; t < ng && direct; ++t)
      if (lens[j0 + t] && !base) base = parts[sh.parts[j0 + t]];
    for (uint64_t t = 0; t < ng; ++t)
      offs[t] = direct ? (lens[j0 + t] ? uint64_t(parts[sh.parts[j0 + t]] - base) : 0) : poff[j0 + t];
    for (int a = 0; a < nalgo; ++a)
      if (int rc = plan_geometry(C.gplan[q][a], offs.data(), lens.data() + j0, ng, S3H_KERNEL_AUTO,
                                 C.gslots(q, a), C.gorder(q, a), C.copy_s))
        return rc;
    if (direct) {
      if (span) HIP_TRY(hipMemcpyAsync(dgrp, base, span, hipMemcpyHostToDevice, C.copy_s));
    } else {  // packed chunk by chunk: parts [ja, jb) whose packed bytes fit one chunk
      for (uint64_t ja = j0, jb; ja < j1; ja = jb) {
        jb = ja + 1;
        while (jb < j1 && poff[jb] + ((lens[jb] + 63) & ~uint64_t(63)) - poff[ja] <= chunk) ++jb;
        const uint64_t bytes = (jb < j1 ? poff[jb] : gbytes[k]) - poff[ja];
        const int c = int(chunk_next++ % kHostRing);
        if (chunk_used[c]) HIP_TRY(hipEventSynchronize(C.chunk_copied[c]));  // its last DMA ran
        uint8_t* const hst = C.stage + uint64_t(c) * chunk;
        std::atomic<bool> bad{false};
        pool->run(jb - ja, [&](uint64_t t) {
          const uint64_t j = ja + t;
          if (lens[j] && !src.fill(sh.parts[j], 0, lens[j], hst + (poff[j] - poff[ja])))
            bad.store(true, std::memory_order_relaxed);
        });
        if (bad.load()) return fail(S3H_EINVAL, "reading a part failed (file shorter than a part?)");
        if (bytes) HIP_TRY(hipMemcpyAsync(dgrp + poff[ja], hst, bytes, hipMemcpyHostToDevice, C.copy_s));
        HIP_TRY(hipEventRecord(C.chunk_copied[c], C.copy_s));
        chunk_used[c] = true;
      }
    }
    HIP_TRY(hipEventRecord(C.copied[q], C.copy_s));
    for (int a = 0; a < nalgo; ++a) {
      s3h_plan_s* P = C.gplan[q][a];
      HIP_TRY(hipStreamWaitEvent(C.hash_s[a], C.copied[q], 0));
      if (int rc = plan_launch(P, dgrp, C.d_dig[a] + j0 * digest_words(algos[a]), 0, P->max_blocks, 0,
                               C.hash_s[a], false))
        return rc;
      HIP_TRY(hipEventRecord(C.hashed[q][a], C.hash_s[a]));
    }
  }
  int rc = S3H_OK;
  for (int a = 0; a < nalgo && rc == S3H_OK; ++a) {
    const uint32_t dw = digest_words(algos[a]);
    std::vector<uint32_t> local(n * dw);
    hipError_t e = hipMemcpyAsync(local.data(), C.d_dig[a], n * dw * 4, hipMemcpyDeviceToHost, C.hash_s[a]);
    if (e == hipSuccess) e = hipStreamSynchronize(C.hash_s[a]);
    if (e != hipSuccess) {
      rc = fail(S3H_EHIP, "D2H digests: %s", hipGetErrorString(e));
      break;
    }
    for (int q = 0; q < 2 && rc == S3H_OK; ++q) rc = plan_check(C.gplan[q][a], C.hash_s[a]);
    if (rc) break;
    for (uint64_t j = 0; j < n; ++j) std::memcpy(digests[a] + dw * sh.parts[j], &local[dw * j], dw * 4);
  }
  C.sync();
  if (trace_host())
    std::fprintf(stderr, "[s3h host] dev %d: %llu parts in %llu groups of <= %llu B (%s)\n", sh.device,
                 (unsigned long long)n, (unsigned long long)ngroups, (unsigned long long)maxb,
                 any_staged ? "staged" : "pinned ranges");
  return rc;
}

// Streams one device's parts through a 3-slot HBM ring; every slice is copied ONCE and
// hashed by each requested algorithm (SHA-256 and/or MD5) on its own stream, so a dual
// digest costs one PCIe pass.  digests[a] receives algo[a]'s digests (global part order).
// Copy modes per slice: pinned parts at a constant stride -> one 2-D DMA; other pinned parts
// -> one DMA per part; pageable parts and file ranges -> host threads fill a pinned staging
// slot (memcpy / pread) and one DMA moves it; more than kStageSlot/64 pageable parts (or no
// pinned memory) -> one pageable DMA per part.
int run_host_shard(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                   const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                   uint64_t slice) {
  if (nalgo < 1 || nalgo > kHostMaxAlgo) return fail(S3H_EINVAL, "host shard: %d algorithms", nalgo);
  const uint64_t n = sh.parts.size();
  if (n == 0) return S3H_OK;
  DeviceGuard g(sh.device);
  const double t_start = wall_s();
  std::vector<uint64_t> offs(n), lens(n);
  for (uint64_t j = 0; j < n; ++j) lens[j] = lengths[sh.parts[j]];
  const uint8_t* const* parts = src.parts;
  bool staged = !parts || !all_pinned(parts, lengths, sh.parts.data(), n);
  bool uniform = false;
  intptr_t stride = 0;
  if (!staged && n > 1) {  // equal-length parts at a constant positive host stride (file chunks)
    stride = parts[sh.parts[1]] - parts[sh.parts[0]];
    uniform = stride >= intptr_t(lens[0]) && lens[0] > 0;
    for (uint64_t j = 1; j < n && uniform; ++j)
      uniform = lens[j] == lens[0] && parts[sh.parts[j]] - parts[sh.parts[j - 1]] == stride;
  }
  // Many small parts (<= kGroupMaxPart): whole parts in groups instead of slices of every part
  // (run_host_groups) -- when staging would cut slices below 16 KiB (> 2,048 parts), or pinned
  // ragged parts would each take their own DMA per slice (> 64 parts: 4,000 pinned parts of
  // U[1 B, 1 MiB] spent 0.49 s draining 56,000 per-part DMAs for 1.9 GiB).  A caller's
  // explicit slice size keeps the slice pipeline.  Large parts beside them (an object's parts
  // batched with many small objects) run through the slice pipeline afterwards, on their own.
  if (slice == 0) {
    std::vector<uint64_t> small, large;
    for (uint64_t j = 0; j < n; ++j) (lens[j] <= kGroupMaxPart ? small : large).push_back(sh.parts[j]);
    const uint64_t ns = small.size();
    if ((staged && ns > 2048) || (!staged && !uniform && ns > 64)) {
      if (large.empty()) return run_host_groups(C, sh, algos, nalgo, src, lengths, digests, !staged);
      const HostShard hs{sh.device, sh.ndevices, std::move(small), sh.threads};
      const HostShard hl{sh.device, sh.ndevices, std::move(large), sh.threads};
      if (int rc = run_host_groups(C, hs, algos, nalgo, src, lengths, digests, !staged)) return rc;
      return run_host_shard(C, hl, algos, nalgo, src, lengths, digests, 0);
    }
  }
  // Many ragged pinned parts: packing them into staging (memcpy, one DMA per slice) beats one
  // DMA per part per slice (4,000 parts of U[256 KiB, 4 MiB]: 18.0 -> 30.2 GiB/s; 1,024 of
  // U[1, 8] MiB: 24.3 -> 27.8).
  if (!staged && !uniform && n > kPinnedStageMin) staged = true;
  // Too many pageable parts for the staging cap even at 64 B per slice: pageable DMAs.
#ifdef S3H_EXP_PAGEABLE_DIRECT  // tools/ experiment builds only: pageable DMAs, no staging
  bool direct_pageable = staged && parts;
#else
  bool direct_pageable = staged && parts && n * 64 > kStageSlot;
#endif
  if (direct_pageable) staged = false;
  if (slice == 0)
    slice = staged ? std::max<uint64_t>(std::max<uint64_t>(64, kStageSlot / n / 64 * 64),
                                        std::min<uint64_t>(32 << 10, kFileStageSlot / n / 64 * 64))
            : uniform ? (256ull << 10) : (2ull << 20);
  const uint64_t longest = *std::max_element(lens.begin(), lens.end());
  slice = std::min(slice, std::max<uint64_t>(64, (longest + 63) / 64 * 64));  // no idle slot bytes
  // The ring holds kHostRing*n*slice bytes of HBM: keep it within min(16 GiB, free/4).
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const uint64_t budget = std::min<uint64_t>(16ull << 30, (free_b + C.ring_bytes) / 4);
  if (kHostRing * n * slice > budget) slice = std::max<uint64_t>(64, budget / (kHostRing * n) / 64 * 64);
  for (uint64_t j = 0; j < n; ++j) offs[j] = j * slice;
  const uint64_t slot_bytes = n * slice;

  HIP_TRY(C.ensure_streams());
  hipError_t ce = hipSuccess;
  if (staged) {
    ce = C.grow_pinned(&C.stage, &C.stage_bytes, kHostRing * slot_bytes);
    if (ce != hipSuccess) {
      (void)hipGetLastError();
      if (!parts) return fail(S3H_ENOMEM, "pinned staging (%llu B): %s",
                              (unsigned long long)(kHostRing * slot_bytes), hipGetErrorString(ce));
      staged = false;  // memory parts: fall back to pageable DMAs
      direct_pageable = true;
    }
  }
  ce = HostCtx::grow_dev(&C.ring, &C.ring_bytes, kHostRing * slot_bytes);
  if (ce != hipSuccess) return fail(S3H_ENOMEM, "host ring (%llu B): %s",
                                    (unsigned long long)(kHostRing * slot_bytes), hipGetErrorString(ce));
  HIP_TRY(C.ensure_pin(n));
  uint64_t max_blocks = 0;
  for (int a = 0; a < nalgo; ++a) {
    if (int rc = C.ensure_plan(a, algos[a], n)) return rc;
    HIP_TRY(hipMemsetAsync(C.plan[a]->d_err, 0, sizeof(uint32_t), C.copy_s));  // before any launch
    HIP_TRY(C.ensure_digests(a, n * digest_words(algos[a]) * sizeof(uint32_t)));
    // geometry upload on the copy stream: every launch waits for a later copy on it
    if (int rc = plan_geometry(C.plan[a], offs.data(), lens.data(), n, S3H_KERNEL_AUTO,
                               C.h_slots(a), C.h_order(a), C.copy_s))
      return rc;
    max_blocks = std::max(max_blocks, C.plan[a]->max_blocks);
  }
  CopyPool* pool = nullptr;
  const unsigned threads = shard_threads(sh);  // the caller + workers
  if (staged) pool = C.ensure_pool(threads - 1);
  const uint64_t bps = slice / 64;  // blocks per slice
  s3h_plan_s* P0 = C.plan[0];
  s3h_plan_s* P1 = nalgo == 2 ? C.plan[1] : nullptr;
  const bool fused = nalgo == 2 && P0->max_blocks == P1->max_blocks &&
                     dual_mode(P0, P1, 0, bps) != kDualNone;
  int rc = S3H_OK;
  uint64_t k = 0;
  const double t_setup = wall_s();
  // Slices of bps blocks, then a geometric tail: the copies set the pace (PCIe; C2: a full
  // slice copies in ~4.7 ms and hashes in ~3.8) and slice k's hash runs beside slice k+1's
  // copy, so the hash keeps up only while hash(k) <= copy(k+1).  Once fewer than D slices are
  // left each slice takes 1/D of the rest (sizes shrink by (D-1)/D >= the hash/copy ratio,
  // ~0.81), down to bps/16, so the hash exposed after the last copy is one small slice's
  // (~0.24 ms).  Halving (D = 2) broke the condition at the first tail slice: 3.8 ms of
  // full-slice hash ran past the copies (tools/host_timeline.py trace).
  auto slice_blocks = [&](uint64_t b0) -> uint64_t {
    const uint64_t left = max_blocks - b0;
#ifndef S3H_EXP_NO_TAIL_RAMP  // tools/ experiment builds only: round-3 fixed slices
    constexpr uint64_t D = S3H_EXP_TAIL_RAMP_DIV;
    if (bps >= 256 && left < D * bps)
      return std::min(left, std::max<uint64_t>(bps / 16, (left + D - 1) / D));
#endif
    return std::min(left, bps);
  };
  for (uint64_t b0 = 0, step = 0; b0 < max_blocks && rc == S3H_OK; b0 += step, ++k) {
    step = slice_blocks(b0);
    const uint64_t sbytes = step * 64;  // bytes of each part this slice carries (<= slice)
    const int r = int(k % kHostRing);
    uint8_t* slot_base = C.ring + uint64_t(r) * slot_bytes;
    hipError_t e = hipSuccess;
    for (int a = 0; a < nalgo && k >= kHostRing && e == hipSuccess; ++a)
      e = hipStreamWaitEvent(C.copy_s, C.hashed[r][a], 0);  // slot reusable once all hashed it
    if (e != hipSuccess) { rc = fail(S3H_EHIP, "wait: %s", hipGetErrorString(e)); break; }
    const uint64_t byte0 = b0 * 64;
    if (staged) {
      // host slot r is free once the DMA that last read it (copied[r]) has finished
      uint8_t* hslot = C.stage + uint64_t(r) * slot_bytes;
      if (k >= kHostRing) e = hipEventSynchronize(C.copied[r]);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "stage wait: %s", hipGetErrorString(e)); break; }
      std::atomic<bool> bad{false};
      pool->run(n, [&](uint64_t j) {
        const uint64_t len = lens[j];
        if (byte0 < len && !src.fill(sh.parts[j], byte0, std::min(sbytes, len - byte0), hslot + j * slice))
          bad.store(true, std::memory_order_relaxed);
      });
      if (bad.load()) { rc = fail(S3H_EINVAL, "reading a part failed (file shorter than a part?)"); break; }
      e = step == bps ? hipMemcpyAsync(slot_base, hslot, slot_bytes, hipMemcpyHostToDevice, C.copy_s)
                      : hipMemcpy2DAsync(slot_base, slice, hslot, slice, sbytes, n,
                                         hipMemcpyHostToDevice, C.copy_s);
      if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D staged: %s", hipGetErrorString(e));
    } else if (uniform) {
      if (byte0 < lens[0]) {
        const uint64_t cnt = std::min(sbytes, lens[0] - byte0);
        e = hipMemcpy2DAsync(slot_base, slice, parts[sh.parts[0]] + byte0, stride, cnt, n,
                             hipMemcpyHostToDevice, C.copy_s);
        if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D 2D: %s", hipGetErrorString(e));
      }
    } else {
      for (uint64_t j = 0; j < n && rc == S3H_OK; ++j) {
        const uint64_t len = lens[j];
        if (byte0 >= len) continue;
        const uint64_t cnt = std::min(sbytes, len - byte0);
        e = hipMemcpyAsync(slot_base + j * slice, parts[sh.parts[j]] + byte0, cnt,
                           hipMemcpyHostToDevice, C.copy_s);
        if (e != hipSuccess) rc = fail(S3H_EHIP, "H2D: %s", hipGetErrorString(e));
      }
    }
    if (rc) break;
    e = hipEventRecord(C.copied[r], C.copy_s);
    if (fused) {  // both digests from one grid on one stream
      if (e == hipSuccess) e = hipStreamWaitEvent(C.hash_s[0], C.copied[r], 0);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e)); break; }
      rc = dual_launch(P0, P1, slot_base, C.d_dig[0], C.d_dig[1], b0, b0 + step, b0, true,
                       C.hash_s[0]);
      if (rc == S3H_OK) e = hipEventRecord(C.hashed[r][0], C.hash_s[0]);
      if (e == hipSuccess) e = hipEventRecord(C.hashed[r][1], C.hash_s[0]);
    }
    for (int a = 0; a < nalgo && rc == S3H_OK && !fused; ++a) {
      if (e == hipSuccess) e = hipStreamWaitEvent(C.hash_s[a], C.copied[r], 0);
      if (e != hipSuccess) { rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e)); break; }
      if (b0 < C.plan[a]->max_blocks)  // both pad 9 B, so equal block counts; guard anyway
        rc = plan_launch(C.plan[a], slot_base, C.d_dig[a], b0, b0 + step, b0, C.hash_s[a], true);
      if (rc == S3H_OK) e = hipEventRecord(C.hashed[r][a], C.hash_s[a]);
    }
    if (rc == S3H_OK && e != hipSuccess) rc = fail(S3H_EHIP, "event: %s", hipGetErrorString(e));
  }
  const double t_issue = wall_s();
  for (int a = 0; a < nalgo && rc == S3H_OK; ++a) {
    const uint32_t dw = digest_words(algos[a]);
    std::vector<uint32_t> local(n * dw);
    hipStream_t hs = C.hash_s[fused ? 0 : a];
    hipError_t e = hipMemcpyAsync(local.data(), C.d_dig[a], n * dw * 4, hipMemcpyDeviceToHost, hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    if (e != hipSuccess) { rc = fail(S3H_EHIP, "D2H digests: %s", hipGetErrorString(e)); break; }
    if ((rc = plan_check(C.plan[a], hs)) != S3H_OK) break;  // every slice's launch reported in
    for (uint64_t j = 0; j < n; ++j)
      std::memcpy(digests[a] + dw * sh.parts[j], &local[dw * j], dw * 4);
  }
  C.sync();  // nothing of this call may still run when the context is handed on
  if (trace_host())
    std::fprintf(stderr,
                 "[s3h host] dev %d: %llu parts, slice %llu B, %s, %llu slices: setup %.2f ms, "
                 "issue %.2f ms, drain %.2f ms; copy threads %u (%u CPUs over %d devices); "
                 "numa: device node %d, staging node %d, copy threads on %d CPUs of node %d\n",
                 sh.device, (unsigned long long)n, (unsigned long long)slice,
                 !parts ? "staged (file pread)" : staged ? "staged (pageable)"
                 : direct_pageable ? "pageable per-part" : uniform ? "pinned 2-D" : "pinned per-part",
                 (unsigned long long)k, 1e3 * (t_setup - t_start), 1e3 * (t_issue - t_setup),
                 1e3 * (wall_s() - t_issue), staged ? threads : 0u, host_cpus(), sh.ndevices,
                 C.place.dev_node, staged ? mem_node(C.stage) : -1, C.place.ncpus, C.place.node);
  return rc;
}

// File ranges and merged part references have no pageable-DMA fallback, and their staging
// slot is n x slice bytes with slices of at least 64 B: a shard of more than
// kMaxStagedRefs such parts runs in passes of that many, so the pinned staging ring never
// exceeds kHostRing x kFileStageSlot (384 MiB).
constexpr uint64_t kMaxStagedRefs = kFileStageSlot / 64;  // 2,097,152 parts

int run_host_shard_passes(HostCtx& C, const HostShard& sh, const int* algos, int nalgo,
                          const PartSource& src, const uint64_t* lengths, uint32_t* const* digests,
                          uint64_t slice) {
  if (src.parts || sh.parts.size() <= kMaxStagedRefs)
    return run_host_shard(C, sh, algos, nalgo, src, lengths, digests, slice);
  for (uint64_t s = 0; s < sh.parts.size(); s += kMaxStagedRefs) {
    const uint64_t e = std::min<uint64_t>(sh.parts.size(), s + kMaxStagedRefs);
    HostShard sub{sh.device, sh.ndevices,
                  std::vector<uint64_t>(sh.parts.begin() + s, sh.parts.begin() + e), sh.threads};
    if (int rc = run_host_shard(C, sub, algos, nalgo, src, lengths, digests, slice)) return rc;
  }
  return S3H_OK;
}

// The queue's executor: one shard on the device's cached context (or a private one when the
// cached one is busy); a failed call drops its context.
struct CtxExec {
  int operator()(const HostShard& sh, const int* algos, int nalgo, const PartSource& src,
                 const uint64_t* lengths, uint32_t* const* digests, uint64_t slice) {
    HostCtx* C = host_ctx_cache().acquire(sh.device);
    int rc = S3H_EHIP;
    try {
      rc = run_host_shard_passes(*C, sh, algos, nalgo, src, lengths, digests, slice);
    } catch (...) {
      host_ctx_cache().release(C, false);
      throw;  // run_guarded reports it
    }
    host_ctx_cache().release(C, rc == S3H_OK);
    return rc;
  }
};


}  // namespace

// Shard s (of nshards) gets parts i with i % nshards == s and runs on device devs[s]; a device
// may appear more than once (its shards run concurrently, each on its own context).

int batch_host_on(const int* algos, int nalgo, const PartSource& src,
                         const uint64_t* lengths, uint64_t n, uint32_t* const* digests,
                         const std::vector<int>& devs, uint64_t slice_bytes) {
  if (!lengths || n == 0) return fail(S3H_EINVAL, "batch_host: bad arguments");
  for (int a = 0; a < nalgo; ++a)
    if (!digests[a]) return fail(S3H_EINVAL, "batch_host: null digest array");
  int count = 0;
  if (int rc = s3h_device_count(&count)) return rc;
  if (devs.empty()) return fail(S3H_EINVAL, "batch_host: no devices");
  for (int d : devs)
    if (d < 0 || d >= count) return fail(S3H_EINVAL, "batch_host: device %d out of range [0,%d)", d, count);
  if (slice_bytes % 64) return fail(S3H_EINVAL, "slice_bytes must be a multiple of 64");
  if (src.parts)
    for (uint64_t i = 0; i < n; ++i)
      if (!src.parts[i] && lengths[i]) return fail(S3H_EINVAL, "batch_host: part %llu is null", (unsigned long long)i);
  const int nshards = int(std::min<uint64_t>(devs.size(), n));
  std::vector<HostShard> shards(nshards);
  for (int k = 0; k < nshards; ++k) shards[k] = {devs[k], nshards, {}, g_stage_threads_cap};
  for (uint64_t i = 0; i < n; ++i) shards[i % nshards].parts.push_back(i);
  std::vector<int> rcs(nshards, S3H_OK);
  std::vector<std::string> errs(nshards);
  auto run = [&](int k) {
    HostReq r{algos, nalgo, &src, lengths, digests, &shards[k], slice_bytes, S3H_OK, {}, false};
    CtxExec exec;
    submit(exec, r);
    rcs[k] = r.rc;
    errs[k] = r.err;
  };
  if (nshards == 1) {
    run(0);  // the caller's own thread: its affinity is the caller's business
  } else {   // one thread per device shard, on that device's node (it stages and issues DMAs)
    std::vector<std::thread> pool;
    for (int k = 0; k < nshards; ++k)
      pool.emplace_back([&run, k, place = device_place(shards[k].device)] {
        bind_self(place);
        run(k);
      });
    for (auto& t : pool) t.join();
  }
  for (int k = 0; k < nshards; ++k)
    if (rcs[k]) return fail(rcs[k], "device %d: %s", shards[k].device, errs[k].c_str());
  return S3H_OK;
}

// ndevices GPUs 0..ndevices-1 (0 or more than visible = all visible).
int batch_host(const int* algos, int nalgo, const PartSource& src,
                      const uint64_t* lengths, uint64_t n, uint32_t* const* digests, int ndevices,
                      uint64_t slice_bytes) {
  int count = 0;
  if (int rc = s3h_device_count(&count)) return rc;
  if (ndevices <= 0 || ndevices > count) ndevices = count;
  std::vector<int> devs(ndevices);
  std::iota(devs.begin(), devs.end(), 0);
  return batch_host_on(algos, nalgo, src, lengths, n, digests, devs, slice_bytes);
}

int batch_host(int algo, const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                      uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  if (!parts) return fail(S3H_EINVAL, "batch_host: null parts");
  uint32_t* const out[1] = {digests};
  PartSource src;
  src.parts = parts;
  return batch_host(&algo, 1, src, lengths, n, out, ndevices, slice_bytes);
}

// Open `path` and check that every range lies inside it -- before the call can be merged
// with other callers' (a batch fails as a whole).  Returns the descriptor or -1 (error set).
int open_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                           uint64_t n) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    fail(S3H_EINVAL, "file_parts: cannot open %s: %s", path, std::strerror(errno));
    return -1;
  }
  struct stat st {};
  if (fstat(fd, &st) != 0) {
    close(fd);
    fail(S3H_EINVAL, "file_parts: cannot stat %s", path);
    return -1;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i] > uint64_t(st.st_size) || lengths[i] > uint64_t(st.st_size) - offsets[i]) {
      close(fd);
      fail(S3H_EINVAL, "file_parts: part %llu [%llu, +%llu) is past the end of %s (%llu B)",
           (unsigned long long)i, (unsigned long long)offsets[i],
           (unsigned long long)lengths[i], path, (unsigned long long)st.st_size);
      return -1;
    }
  return fd;
}

int file_parts(const int* algos, int nalgo, const char* path, const uint64_t* offsets,
                      const uint64_t* lengths, uint64_t n, uint32_t* const* digests,
                      int ndevices, uint64_t slice_bytes) {
  if (!path || !offsets || !lengths || n == 0)
    return fail(S3H_EINVAL, "file_parts: bad arguments");
  for (int a = 0; a < nalgo; ++a)
    if (!digests[a]) return fail(S3H_EINVAL, "file_parts: null digest array");
  const int fd = open_file_parts(path, offsets, lengths, n);
  if (fd < 0) return S3H_EINVAL;
  PartSource src;
  src.fd = fd;
  src.file_off = offsets;
  const int rc = batch_host(algos, nalgo, src, lengths, n, digests, ndevices, slice_bytes);
  close(fd);
  return rc;
}

// Any algorithm list over memory parts or file ranges (route.cpp's GPU route).
int host_batch_algos(const int* algos, int nalgo, const uint8_t* const* parts, const char* path,
                     const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                     uint32_t* const* digests, int ndevices) {
  if (path) return file_parts(algos, nalgo, path, offsets, lengths, n, digests, ndevices, 0);
  if (!parts) return fail(S3H_EINVAL, "batch_host: null parts");
  PartSource src;
  src.parts = parts;
  return batch_host(algos, nalgo, src, lengths, n, digests, ndevices, 0);
}

}  // namespace s3h::host

using namespace s3h::host;

extern "C" {

int s3h_sha256_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                          uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  return batch_host(S3H_ALGO_SHA256, parts, lengths, n, digests, ndevices, slice_bytes);
}

int s3h_md5_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                       uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  return batch_host(S3H_ALGO_MD5, parts, lengths, n, digests, ndevices, slice_bytes);
}

int s3h_sha256_md5_batch_host(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                              uint32_t* sha256_digests, uint32_t* md5_digests, int ndevices,
                              uint64_t slice_bytes) {
  static const int algos[2] = {S3H_ALGO_SHA256, S3H_ALGO_MD5};
  uint32_t* const out[2] = {sha256_digests, md5_digests};
  if (!parts) return fail(S3H_EINVAL, "batch_host: null parts");
  PartSource src;
  src.parts = parts;
  return batch_host(algos, 2, src, lengths, n, out, ndevices, slice_bytes);
}

int s3h_sha256_batch_host_on(const uint8_t* const* parts, const uint64_t* lengths, uint64_t n,
                             uint32_t* digests, const int* devices, int ndevices,
                             uint64_t slice_bytes) {
  if (!parts || !devices || ndevices <= 0) return fail(S3H_EINVAL, "batch_host_on: bad arguments");
  static const int algo = S3H_ALGO_SHA256;
  uint32_t* const out[1] = {digests};
  PartSource src;
  src.parts = parts;
  return batch_host_on(&algo, 1, src, lengths, n, out, std::vector<int>(devices, devices + ndevices),
                       slice_bytes);
}

int s3h_sha256_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                          uint64_t n, uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  static const int algo = S3H_ALGO_SHA256;
  uint32_t* const out[1] = {digests};
  return file_parts(&algo, 1, path, offsets, lengths, n, out, ndevices, slice_bytes);
}

int s3h_md5_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                       uint64_t n, uint32_t* digests, int ndevices, uint64_t slice_bytes) {
  static const int algo = S3H_ALGO_MD5;
  uint32_t* const out[1] = {digests};
  return file_parts(&algo, 1, path, offsets, lengths, n, out, ndevices, slice_bytes);
}

int s3h_sha256_md5_file_parts(const char* path, const uint64_t* offsets, const uint64_t* lengths,
                              uint64_t n, uint32_t* sha256_digests, uint32_t* md5_digests,
                              int ndevices, uint64_t slice_bytes) {
  static const int algos[2] = {S3H_ALGO_SHA256, S3H_ALGO_MD5};
  uint32_t* const out[2] = {sha256_digests, md5_digests};
  return file_parts(algos, 2, path, offsets, lengths, n, out, ndevices, slice_bytes);
}

int s3h_verify_batch_host(int algo, const uint8_t* const* parts, const uint64_t* lengths,
                          uint64_t n, const uint32_t* expected, uint8_t* mismatch,
                          uint64_t* mismatches, int ndevices) {
  if (!expected || !mismatch || !mismatches) return fail(S3H_EINVAL, "verify: null argument");
  if (algo != S3H_ALGO_SHA256 && algo != S3H_ALGO_MD5)
    return fail(S3H_EINVAL, "verify: unknown algorithm %d", algo);
  const uint32_t dw = digest_words(algo);
  std::vector<uint32_t> got(n * dw);
  if (int rc = batch_host(algo, parts, lengths, n, got.data(), ndevices, 0)) return rc;
  uint64_t c = 0;
  for (uint64_t i = 0; i < n; ++i) {
    mismatch[i] = std::memcmp(&got[dw * i], expected + dw * i, dw * 4) != 0;
    c += mismatch[i];
  }
  *mismatches = c;
  return S3H_OK;
}

int s3h_trim(void) {
  host_ctx_cache().trim();
  staging_trim();
  return S3H_OK;
}

int s3h_host_numa(int mode, int* previous) {
  if (mode < kNumaOff || mode >= int(kMaxNumaNodes))
    return fail(S3H_EINVAL, "host numa: mode %d (want -1 local, -2 off, or a node)", mode);
  const int prev = g_numa_mode.exchange(mode);
  if (previous) *previous = prev;
  if (prev != mode) host_ctx_cache().trim();  // idle contexts re-place on their next call
  return S3H_OK;
}

int s3h_host_numa_info(int device, s3h_host_numa_t* info) {
  if (!info) return fail(S3H_EINVAL, "host numa info: null argument");
  *info = s3h_host_numa_t{-1, -1, 0, -1, -1, 0};
  if (int rc = check_device(device)) return rc;
  const Place P = device_place(device);
  info->device_node = P.dev_node;
  info->target_node = P.node;
  info->bound_cpus = P.ncpus;
  (void)host_ctx_cache().numa_of(device, info);
  return S3H_OK;
}


}  // extern "C"
