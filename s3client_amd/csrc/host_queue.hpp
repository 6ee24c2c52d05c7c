// host_queue.hpp -- concurrent host-path callers of one device meet in a queue and run merged.
//
// upload.cpp:136-140 hashes from cfg.jobs std::async threads, each call covering only its own
// job's parts.  Run as they come, 16 such calls of 32 parts put 16 small grids on the
// process's few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), which run them a few at a
// time: 4 GiB in 16 x 32 parts of 8 MiB took 1.3-1.4 s against 0.124 s for one call with all
// 512 parts (profiles/r02_app_per_job_coalesced.txt).  So the calls of one device meet in a
// queue: the first caller (the leader) takes every pending request with the same algorithms and
// slice size and runs them as ONE shard -- parts from memory and file ranges mixed -- then
// scatters the digests back; calls that arrive meanwhile form the next batch.  Once calls have
// been seen to overlap (within the last second), a leader first gathers the rest of the burst:
// it waits until no call has arrived for kGatherQuiet (at most kGatherMax).  A merged batch
// that fails is re-run one request at a time, so each caller gets its own status and message.
//
// HIP-free and templated on the executor that runs one shard (host_path.cpp: the device's
// cached context and the slice / group pipeline; tests/cpp/host_concurrency_test.cpp: a fake
// that sleeps, fails or throws), so the queue runs under ThreadSanitizer / AddressSanitizer on
// the CPU.
#pragma once
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/s3hash.h"
#include "host_limits.hpp"
#include "status.hpp"
#include "topology.hpp"

namespace s3h::host {

// One part of a merged batch (concurrent callers): host memory or a file range.
struct PartRef {
  const uint8_t* mem;
  int fd;
  uint64_t off;
};

// Where a shard's part bytes come from: host memory (pinned or pageable), byte ranges of an
// open file (read with pread straight into the pinned staging ring), or per-part references
// (a batch merged from concurrent calls whose sources differ).
struct PartSource {
  const uint8_t* const* parts = nullptr;  // memory parts, or null for a file / refs
  int fd = -1;                            // file parts: part i = [file_off[i], +lengths[i])
  const uint64_t* file_off = nullptr;
  const PartRef* refs = nullptr;
  PartRef ref(uint64_t i) const {
    if (parts) return {parts[i], -1, 0};
    if (refs) return refs[i];
    return {nullptr, fd, file_off[i]};
  }
  // bytes [byte0, byte0 + cnt) of part i into dst; false on a read error or a short file
  bool fill(uint64_t i, uint64_t byte0, uint64_t cnt, uint8_t* dst) const {
    const PartRef r = ref(i);
    if (r.mem) {
      std::memcpy(dst, r.mem + byte0, cnt);
      return true;
    }
    for (uint64_t done = 0; done < cnt;) {
      const ssize_t r2 = pread(r.fd, dst + done, cnt - done, off_t(r.off + byte0 + done));
      if (r2 < 0 && errno == EINTR) continue;
      if (r2 <= 0) return false;  // error or a part past the end of the file
      done += uint64_t(r2);
    }
    return true;
  }
};

struct HostShard {
  int device;
  int ndevices;                 // shards running concurrently (host threads are split between them)
  std::vector<uint64_t> parts;  // global part indices on this device
  unsigned threads = 0;         // staging threads cap (0: host_threads_per_device); the split
                                // route's GPU side leaves the rest of the CPUs to its CPU side
};

// The calling thread's staging-thread cap for the host batches it starts (the split route sets
// it around its GPU side; batch_host_on copies it into the shards).
extern thread_local unsigned g_stage_threads_cap;

// Staging threads of a shard (the calling thread included).
inline unsigned shard_threads(const HostShard& sh) {
  unsigned t = host_threads_per_device(sh.ndevices);
  if (const char* e = std::getenv("S3H_STAGE_THREADS"))  // measurements: cap every shard
    if (std::atoi(e) > 0) t = std::min(t, unsigned(std::atoi(e)));
  return sh.threads ? std::max(1u, std::min(sh.threads, t)) : t;
}

struct HostReq {
  const int* algos;
  int nalgo;
  const PartSource* src;
  const uint64_t* lengths;
  uint32_t* const* digests;
  const HostShard* sh;
  uint64_t slice;
  int rc = S3H_OK;
  std::string err;
  bool done = false;
};

struct DevQueue {
  std::mutex m;
  std::condition_variable cv;
  std::vector<HostReq*> pending;
  bool leader = false;
  double last_overlap = -1e9;  // when a call last found another one on this device
};

constexpr double kGatherQuiet = 300e-6, kGatherMax = 3e-3;

inline DevQueue& dev_queue(int device) {
  static std::mutex m;
  static auto* qs = new std::vector<std::unique_ptr<DevQueue>>();  // never destroyed
  std::lock_guard<std::mutex> l(m);
  if (qs->size() <= size_t(device)) qs->resize(size_t(device) + 1);
  if (!(*qs)[size_t(device)]) (*qs)[size_t(device)].reset(new DevQueue());
  return *(*qs)[size_t(device)];
}

inline bool same_work(const HostReq& a, const HostReq& b) {
  if (a.nalgo != b.nalgo || a.slice != b.slice) return false;
  for (int k = 0; k < a.nalgo; ++k)
    if (a.algos[k] != b.algos[k]) return false;
  return true;
}

// One shard: a single request as it is, several merged into one part list whose digests are
// scattered back to each request's own arrays.
//   exec(const HostShard&, const int* algos, int nalgo, const PartSource&,
//        const uint64_t* lengths, uint32_t* const* digests, uint64_t slice) -> s3h_status
template <class Exec>
int run_merged(Exec& exec, const std::vector<HostReq*>& batch) {
  const HostReq& f = *batch[0];
  if (batch.size() == 1) return exec(*f.sh, f.algos, f.nalgo, *f.src, f.lengths, f.digests, f.slice);
  uint64_t m = 0;
  bool mem = true;
  HostShard sh{f.sh->device, 1, {}, f.sh->threads};
  for (const HostReq* r : batch) {
    m += r->sh->parts.size();
    mem = mem && r->src->parts;
    sh.ndevices = std::max(sh.ndevices, r->sh->ndevices);
    sh.threads = sh.threads && r->sh->threads ? std::max(sh.threads, r->sh->threads) : 0;  // 0 = no cap
  }
  std::vector<uint64_t> lens(m);
  std::vector<const uint8_t*> ptrs(mem ? m : 0);
  std::vector<PartRef> refs(mem ? 0 : m);
  sh.parts.resize(m);
  uint64_t k = 0;
  for (const HostReq* r : batch)
    for (uint64_t g : r->sh->parts) {
      lens[k] = r->lengths[g];
      if (mem) ptrs[k] = r->src->parts[g];
      else refs[k] = r->src->ref(g);
      sh.parts[k] = k;
      ++k;
    }
  PartSource src;
  if (mem) src.parts = ptrs.data();
  else src.refs = refs.data();
  std::vector<uint32_t> out[kHostMaxAlgo];
  uint32_t* outp[kHostMaxAlgo] = {};
  for (int a = 0; a < f.nalgo; ++a) {
    out[a].resize(m * digest_words(f.algos[a]));
    outp[a] = out[a].data();
  }
  const int rc = exec(sh, f.algos, f.nalgo, src, lens.data(), outp, f.slice);
  if (rc != S3H_OK) return rc;
  k = 0;
  for (const HostReq* r : batch)
    for (uint64_t g : r->sh->parts) {
      for (int a = 0; a < f.nalgo; ++a) {
        const uint32_t dw = digest_words(f.algos[a]);
        std::memcpy(r->digests[a] + dw * g, outp[a] + dw * k, dw * 4);
      }
      ++k;
    }
  return S3H_OK;
}

// Runs a batch; nothing escapes.  *err receives the message of a failure.
template <class Exec>
int run_guarded(Exec& exec, const std::vector<HostReq*>& batch, std::string* err) {
  int rc;
  try {
    rc = run_merged(exec, batch);
  } catch (const std::bad_alloc&) {
    rc = fail(S3H_ENOMEM, "host batch: out of host memory");
  } catch (...) {
    rc = fail(S3H_EHIP, "host batch: unexpected exception");
  }
  *err = rc ? g_err : std::string();
  return rc;
}

// Runs a batch and hands every request its status, so the device queue's leader always gets
// to mark the batch done.  A merged batch that fails is re-run one request at a time: one
// caller's unreadable file range or allocation failure must not fail the other callers, and
// each caller gets its own status and message.
template <class Exec>
void run_batch(Exec& exec, const std::vector<HostReq*>& batch) {
  std::string err;
  const int rc = run_guarded(exec, batch, &err);
  if (rc != S3H_OK && batch.size() > 1) {
    for (HostReq* r : batch) r->rc = run_guarded(exec, {r}, &r->err);
    return;
  }
  for (HostReq* r : batch) {
    r->rc = rc;
    r->err = err;
  }
}

// Runs `r` (in a batch with the device's other pending calls); returns when it is done.
template <class Exec>
void submit(Exec& exec, HostReq& r) {
  DevQueue& q = dev_queue(r.sh->device);
  std::unique_lock<std::mutex> l(q.m);
  q.pending.push_back(&r);
  if (q.leader || q.pending.size() > 1) q.last_overlap = wall_s();
  q.cv.notify_all();  // a gathering leader counts arrivals
  q.cv.wait(l, [&] { return r.done || !q.leader; });
  if (r.done) return;
  q.leader = true;
  const double t0 = wall_s();
  for (double t_arr = t0; t0 - q.last_overlap < 1.0;) {
    const size_t had = q.pending.size();
    q.cv.wait_for(l, std::chrono::duration<double>(kGatherQuiet / 3));
    const double t = wall_s();
    if (q.pending.size() != had) t_arr = t;
    if (t - t_arr > kGatherQuiet || t - t0 > kGatherMax) break;
  }
  while (!r.done && !q.pending.empty()) {
    std::vector<HostReq*> batch;
    HostReq* first = q.pending.front();
    for (auto it = q.pending.begin(); it != q.pending.end();) {
      if (same_work(*first, **it)) {
        batch.push_back(*it);
        it = q.pending.erase(it);
      } else {
        ++it;
      }
    }
    l.unlock();
    run_batch(exec, batch);
    l.lock();
    for (HostReq* b : batch) b->done = true;
    q.cv.notify_all();
  }
  q.leader = false;  // a waiting caller takes over what is still pending
  q.cv.notify_all();
}

}  // namespace s3h::host
