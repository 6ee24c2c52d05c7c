// apps/s3_upload_hash.cpp -- parallel-upload counterpart with payload signing (config 5).
//
// The reference's s3-upload (apps/parallel_upload.cpp:55-167 -> sss::Upload ->
// lib/src/upload.cpp:113-149 UploadFile) slices a file into cfg.jobs x cfg.partsPerJob parts
// (upload.cpp:98-107, 133) and PUTs each with x-amz-content-sha256: UNSIGNED-PAYLOAD
// (upload.cpp:60 passes no payloadHash).  This tool computes the same part geometry, hashes
// every part in ONE batched GPU call (libs3hash.so, host-resident path: H2D included), and
// emits the signed UploadPart headers each part would carry, with the real digest in
// x-amz-content-sha256.  No network I/O (libcurl headers, Lyra and MinIO are not available
// in this environment): `--print-headers` shows what would be sent.
//
// Part sources (how the bytes reach the hash, mirroring the reference's two upload paths):
//   --source file    UploadFile (upload.cpp:113-149): parts are (file, offset, size) ranges as
//                    UploadFilePart sends them; s3h_sha256_file_parts preads each slice
//                    straight into pinned staging (default).
//   --source mmap    the file mmap'd, parts = pointers into the mapping (pageable memory).
//   --source memory  UploadData (upload.cpp:152-184): the object is a memory buffer (cfg.data)
//                    and parts go through S3Api::UploadPart -> DoUploadPart, which in the
//                    reference drops payloadHash (multipart_upload.cpp:131-136); here the digest
//                    is forwarded into the signature as DoUploadFilePart does (:81-86).
//   --per-job        one batch call per job thread at the same time (std::async per job, as
//                    upload.cpp:136-140 runs UploadParts), instead of one call for all parts.
//
//   s3-upload-hash -f FILE [-j JOBS] [-n PARTS_PER_JOB] [--source file|mmap|memory] [--per-job]
//                  [--cpu] [--verify] [--print-headers] [--devices N] [--repeat R]
//                  [--endpoint URL --bucket B --key K --access A --secret S --upload-id ID]
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <future>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "aws_sign.h"
#include "s3hash_batch.hpp"
#include "sha256.h"

namespace {

struct Part {
  int job, number;
  uint64_t offset, size;
};

// lib/src/upload.cpp:98-107 + :133, 136-140 (jobs x partsPerJob)
std::vector<Part> geometry(uint64_t size, int jobs, int parts_per_job) {
  std::vector<Part> out;
  const uint64_t per_job = (size + jobs - 1) / jobs;
  for (int j = 0; j < jobs; ++j) {
    uint64_t off = uint64_t(j) * per_job;
    if (off >= size) break;
    const uint64_t chunk = std::min(per_job, size - off);
    const uint64_t psz = (chunk + parts_per_job - 1) / parts_per_job;
    for (int k = 0; k < parts_per_job; ++k) {
      if (uint64_t(k) * psz >= chunk) break;
      const uint64_t s = std::min(psz, chunk - uint64_t(k) * psz);
      out.push_back({j, j * parts_per_job + k, off, s});
      off += s;
    }
  }
  return out;
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void usage() {
  std::fprintf(stderr,
               "usage: s3-upload-hash -f FILE [-j JOBS] [-n PARTS_PER_JOB] [--source file|mmap|memory]\n"
               "       [--per-job] [--cpu] [--verify] [--print-headers] [--endpoint URL --bucket B\n"
               "        --key K --access A --secret S --upload-id ID] [--devices N] [--repeat R]\n");
}

}  // namespace

int main(int argc, char** argv) {
  std::string file, endpoint = "http://127.0.0.1:9000", bucket = "bucket1", key = "key1";
  std::string access = "ACCESS", secret = "SECRET", upload_id = "UPLOAD-ID";
  std::string source = "file";
  int jobs = 1, ppj = 1, devices = 0, repeat = 1;
  bool cpu = false, verify = false, print_headers = false, per_job = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) { usage(); std::exit(2); }
      return argv[++i];
    };
    if (a == "-f") file = next();
    else if (a == "-j") jobs = std::atoi(next().c_str());
    else if (a == "-n") ppj = std::atoi(next().c_str());
    else if (a == "--cpu") cpu = true;
    else if (a == "--verify") verify = true;
    else if (a == "--print-headers") print_headers = true;
    else if (a == "--endpoint") endpoint = next();
    else if (a == "--bucket") bucket = next();
    else if (a == "--key") key = next();
    else if (a == "--access") access = next();
    else if (a == "--secret") secret = next();
    else if (a == "--upload-id") upload_id = next();
    else if (a == "--devices") devices = std::atoi(next().c_str());
    else if (a == "--repeat") repeat = std::atoi(next().c_str());
    else if (a == "--source") source = next();
    else if (a == "--per-job") per_job = true;
    else { usage(); return 2; }
  }
  if (file.empty() || jobs < 1 || ppj < 1 || repeat < 1 ||
      (source != "file" && source != "mmap" && source != "memory")) { usage(); return 2; }

  const int fd = open(file.c_str(), O_RDONLY);
  if (fd < 0) { std::perror(file.c_str()); return 1; }
  struct stat st {};
  fstat(fd, &st);
  const uint64_t size = uint64_t(st.st_size);
  if (size == 0) { std::fprintf(stderr, "empty file\n"); return 1; }
  // The object's bytes as the chosen upload path holds them: a private mapping (mmap), a
  // heap buffer read from the file (memory: the cfg.data of UploadData), or only the file
  // name (file: UploadFilePart reads by offset).  The CPU drop-in and --verify read the mapping.
  auto* data = static_cast<const uint8_t*>(mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0));
  if (data == MAP_FAILED) { std::perror("mmap"); return 1; }
  std::vector<uint8_t> object;
  const uint8_t* base = data;
  if (source == "memory") {
    object.resize(size);
    for (uint64_t got = 0; got < size;) {
      const ssize_t r = pread(fd, object.data() + got, size - got, off_t(got));
      if (r <= 0) { std::perror("read"); return 1; }
      got += uint64_t(r);
    }
    base = object.data();
  }

  const std::vector<Part> parts = geometry(size, jobs, ppj);
  std::vector<const uint8_t*> ptrs;
  std::vector<uint64_t> lens, offs;
  for (const auto& p : parts) {
    ptrs.push_back(base + p.offset);
    lens.push_back(p.size);
    offs.push_back(p.offset);
  }

  std::vector<std::string> hex(parts.size());
  // GPU runtime start-up (device discovery, code-object load) happens once per process in a
  // real uploader: do it before the timed hash stage with a one-part warm-up batch.
  double init_s = 0;
  if (!cpu) {
    const double ti = now();
    try {
      static const uint8_t warm[64] = {};
      (void)sha256::payload_hashes({warm}, {64}, devices);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s\n", e.what());
      return 1;
    }
    init_s = now() - ti;
  }
  // One hash pass over all parts: the CPU drop-in on one std::thread per job (as upload.cpp
  // runs its jobs), or one batched GPU call.
  auto hash_pass = [&]() -> bool {
    if (cpu) {
      std::vector<std::thread> pool;
      for (int j = 0; j < jobs; ++j)
        pool.emplace_back([&, j] {
          for (size_t i = 0; i < parts.size(); ++i)
            if (parts[i].job == j) {
              uint32_t h[8];
              sha256::sha256(ptrs[i], lens[i], h);
              char t[65];
              sha256::hash_to_text(h, t);
              hex[i] = t;
            }
        });
      for (auto& t : pool) t.join();
      return true;
    }
    // GPU: the parts of `idx` through the chosen source, hex digests into hex[idx[k]]
    auto gpu = [&](const std::vector<size_t>& idx) {
      std::vector<const uint8_t*> p;
      std::vector<uint64_t> l, o;
      for (size_t i : idx) {
        p.push_back(ptrs[i]);
        l.push_back(lens[i]);
        o.push_back(offs[i]);
      }
      const std::vector<std::string> h = source == "file"
                                             ? sha256::file_part_hashes(file, o, l, devices)
                                             : sha256::payload_hashes(p, l, devices);
      for (size_t k = 0; k < idx.size(); ++k) hex[idx[k]] = h[k];
    };
    try {
      if (per_job) {  // one concurrent batch call per job, like upload.cpp:136-140
        std::vector<std::future<void>> fut;
        for (int j = 0; j < jobs; ++j) {
          std::vector<size_t> idx;
          for (size_t i = 0; i < parts.size(); ++i)
            if (parts[i].job == j) idx.push_back(i);
          if (!idx.empty()) fut.push_back(std::async(std::launch::async, gpu, idx));
        }
        for (auto& f : fut) f.get();
      } else {
        std::vector<size_t> all(parts.size());
        for (size_t i = 0; i < all.size(); ++i) all[i] = i;
        gpu(all);
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s\n", e.what());
      return false;
    }
    return true;
  };
  // --repeat R: R passes (an uploader's steady state, buffers cached); the last pass is
  // reported, the first beside it.
  double t0 = 0, first = 0;
  for (int rep = 0; rep < repeat; ++rep) {
    t0 = now();
    if (!hash_pass()) return 1;
    if (rep == 0) first = now() - t0;
  }
  const double dt = now() - t0;

  int mismatches = 0;
  if (verify)
    for (size_t i = 0; i < parts.size(); ++i) {
      uint32_t h[8];
      sha256::sha256(ptrs[i], lens[i], h);
      char t[65];
      sha256::hash_to_text(h, t);
      mismatches += hex[i] != t;
    }

  std::printf("part,job,offset,size,sha256\n");
  for (size_t i = 0; i < parts.size(); ++i)
    std::printf("%d,%d,%llu,%llu,%s\n", parts[i].number, parts[i].job,
                (unsigned long long)parts[i].offset, (unsigned long long)parts[i].size,
                hex[i].c_str());
  if (print_headers)
    for (size_t i = 0; i < parts.size(); ++i) {
      s3h::sigv4::SignConfig c;
      c.access = access;
      c.secret = secret;
      c.endpoint = endpoint;
      c.method = "PUT";
      c.bucket = bucket;
      c.key = key;
      // instead of UNSIGNED-PAYLOAD (aws_sign.cpp:236-237); the memory path forwards it too,
      // where the reference's DoUploadPart drops it (multipart_upload.cpp:131-136)
      c.payloadHash = hex[i];
      // partNumber = i + 1 (multipart_upload.cpp:79, :126)
      c.parameters = {{"partNumber", std::to_string(parts[i].number + 1)}, {"uploadId", upload_id}};
      c.headers = {{"content-length", std::to_string(parts[i].size)}};
      for (const auto& kv : s3h::sigv4::SignHeaders(c))
        std::printf("# part %d %s: %s\n", parts[i].number, kv.first.c_str(), kv.second.c_str());
    }
  const std::string what = cpu ? std::string("cpu lib/hash drop-in")
                               : "gpu batch (H2D included, source " + source +
                                     (per_job ? ", one call per job" : ", one call") + ")";
  std::fprintf(stderr, "%s: %zu parts, %.3f GiB in %.3f s = %.3f GiB/s%s", what.c_str(), parts.size(),
               double(size) / (1 << 30), dt, double(size) / (1 << 30) / dt,
               verify ? (mismatches ? ", VERIFY FAILED" : ", verified vs CPU") : "");
  if (repeat > 1) std::fprintf(stderr, " (pass %d of %d; first pass %.3f s)", repeat, repeat, first);
  if (!cpu) std::fprintf(stderr, " (GPU runtime start-up before it: %.3f s)", init_s);
  std::fprintf(stderr, "\n");
  munmap(const_cast<uint8_t*>(data), size);
  close(fd);
  return mismatches ? 1 : 0;
}
