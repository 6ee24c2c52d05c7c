// apps/s3_upload_hash.cpp -- parallel-upload counterpart with payload signing (config 5).
//
// The reference's s3-upload (apps/parallel_upload.cpp:55-167 -> sss::Upload ->
// lib/src/upload.cpp:113-149 UploadFile) slices a file into cfg.jobs x cfg.partsPerJob parts
// (upload.cpp:98-107, 133) and PUTs each with x-amz-content-sha256: UNSIGNED-PAYLOAD
// (upload.cpp:60 passes no payloadHash).  This tool computes the same part geometry, hashes
// every part in ONE batched GPU call (libs3hash.so, host-resident path: H2D included), and
// emits the signed UploadPart headers each part would carry, with the real digest in
// x-amz-content-sha256.  `--print-headers` shows what would be sent.  `--send` PUTs every
// part with those headers to a plain-HTTP loopback endpoint (config 5: libcurl's headers and
// MinIO are absent from this image, so the endpoint is tests/s3_mock_server.py, which checks
// each body's SHA-256 against x-amz-content-sha256 and verifies the SigV4 signature): each job
// thread hashes (per-job mode) and PUTs its own parts in order, as upload.cpp:136-140 runs
// UploadParts, and the timed pass is then hash + upload.  By default only UploadPart requests
// are sent (to --upload-id), one connection per part; `--multipart` runs the whole
// UploadFile / UploadData flow (upload.cpp:113-149): CreateMultipartUpload (the upload ID from
// its XML), the parts, then CompleteMultipartUpload with every part's ETag
// (multipart_upload.cpp:48-61, 157-176), and checks the object ETag the server returns against
// the one the GPU MD5s give (with --content-md5 / --check-etag).  As in
// upload.cpp:94-95 each job sends to an endpoint drawn at random from the --endpoint list, and
// as DoUploadPart (upload.cpp:55-87) a failed part is sent again while a shared budget of
// --retries lasts.
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
//   --route R        gpu (default) | cpu | auto | split: where the hashing runs -- SHA-256, or
//                    SHA-256 + MD5 with --content-md5 / --check-etag.  auto decides once for the
//                    whole upload with the measured model, priced for the digests the upload
//                    computes (sha256::choose_route: a few large parts go to the CPU drop-in,
//                    hundreds to the GPU, the split in between); a CPU decision hashes per job as
//                    --cpu does, overlapped with the PUTs; split hashes each GPU call's longest
//                    parts on the CPU drop-in beside the GPU (S3H_ROUTE_SPLIT), both digests
//                    there too.
//
//   s3-upload-hash -f FILE [-j JOBS] [-n PARTS_PER_JOB] [--source file|mmap|memory] [--per-job]
//                  [--cpu] [--verify] [--print-headers] [--send] [--get-verify] [--retries N]
//                  [--content-md5] [--check-etag] [--multipart] [--route gpu|cpu|auto|split]
//                  [--devices N]
//                  [--repeat R] [--endpoint URL[,URL...] --bucket B --key K --access A
//                  --secret S --upload-id ID]
#include <fcntl.h>
#include <netdb.h>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <mutex>
#include <csignal>
#include <future>
#include <random>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "aws_sign.h"
#include "md5.h"
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

// Value of response header `name` (case-insensitive, up to the first blank: the reference's
// HTTPHeader regex "name\\s*:\\s*([^\\s]+)", response_parser.cpp:104-112) with its quotes
// trimmed as TrimETag does (response_parser.cpp:51-62); "" when absent.
std::string header_value(const std::string& head, const std::string& name) {
  std::string lower(head);
  for (char& c : lower) c = char(std::tolower(static_cast<unsigned char>(c)));
  std::string key = "\r\n" + name + ":";
  for (char& c : key) c = char(std::tolower(static_cast<unsigned char>(c)));
  const size_t k = lower.find(key);
  if (k == std::string::npos) return "";
  size_t b = k + key.size();
  while (b < head.size() && (head[b] == ' ' || head[b] == '\t')) ++b;
  size_t e = b;
  while (e < head.size() && !std::isspace(static_cast<unsigned char>(head[e]))) ++e;
  std::string v = head.substr(b, e - b);
  if (v.size() >= 2 && v.front() == '"') v = v.substr(1, v.size() - 2);
  else if (v.rfind("&#34;", 0) == 0 && v.size() >= 10) v = v.substr(5, v.size() - 10);
  return v;
}

// Text of the first <tag>...</tag> element (case-insensitive, attributes allowed), trimmed:
// the reference's XMLTag (response_parser.cpp:64-73); "" when absent.
std::string xml_tag(const std::string& xml, const std::string& tag) {
  std::string lower(xml), t(tag);
  for (char& c : lower) c = char(std::tolower(static_cast<unsigned char>(c)));
  for (char& c : t) c = char(std::tolower(static_cast<unsigned char>(c)));
  size_t b = lower.find("<" + t);
  while (b != std::string::npos && lower[b + 1 + t.size()] != '>' && lower[b + 1 + t.size()] != ' ')
    b = lower.find("<" + t, b + 1);
  if (b == std::string::npos) return "";
  b = lower.find('>', b);
  const size_t e = lower.find("</" + t, b);
  if (b == std::string::npos || e == std::string::npos) return "";
  std::string v = xml.substr(b + 1, e - b - 1);
  while (!v.empty() && std::isspace(static_cast<unsigned char>(v.back()))) v.pop_back();
  while (!v.empty() && std::isspace(static_cast<unsigned char>(v.front()))) v.erase(0, 1);
  return v;
}

// An ETag as CompleteMultipartUpload's XML carries it, its quotes trimmed: literal, &#34; or
// &quot; (S3Api::CompleteMultipartUpload, multipart_upload.cpp:165-175, handles the first two).
std::string trim_xml_etag(std::string v) {
  for (const char* q : {"\"", "&#34;", "&quot;"}) {
    const size_t n = std::strlen(q);
    if (v.size() >= 2 * n && v.compare(0, n, q) == 0 && v.compare(v.size() - n, n, q) == 0)
      return v.substr(n, v.size() - 2 * n);
  }
  return v;
}

int open_conn(const std::string& host, const std::string& port) {
  addrinfo hints{}, *ai = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), port.c_str(), &hints, &ai) != 0 || !ai) return -1;
  const int sock = socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
  const bool connected = sock >= 0 && connect(sock, ai->ai_addr, ai->ai_addrlen) == 0;
  freeaddrinfo(ai);
  if (!connected) {
    if (sock >= 0) close(sock);
    return -1;
  }
  // a stalled endpoint fails the request (and its retries) instead of hanging the upload
  const timeval tv{120, 0};
  (void)setsockopt(sock, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  (void)setsockopt(sock, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  return sock;
}

// One POST with a small body (CreateMultipartUpload's empty one, CompleteMultipartUpload's
// XML) over plain HTTP/1.1, Connection: close.  Returns the HTTP status (-1 on a socket error)
// and the response body in *out (a chunked body decoded).
int post_request(const std::string& host, const std::string& port, const std::string& target,
                 const s3h::sigv4::Map& headers, const std::string& body, std::string* out) {
  const int sock = open_conn(host, port);
  if (sock < 0) return -1;
  std::string req = "POST " + target + " HTTP/1.1\r\n";
  for (const auto& kv : headers) req += kv.first + ": " + kv.second + "\r\n";
  req += "Connection: close\r\n\r\n" + body;
  bool ok = true;
  for (size_t sent = 0; ok && sent < req.size();) {
    const ssize_t w = send(sock, req.data() + sent, req.size() - sent, MSG_NOSIGNAL);
    ok = w > 0;
    if (ok) sent += size_t(w);
  }
  std::string resp;
  char buf[4096];
  for (ssize_t r; ok && (r = recv(sock, buf, sizeof buf, 0)) > 0;) resp.append(buf, size_t(r));
  close(sock);
  int code = -1;
  const size_t he = resp.find("\r\n\r\n");
  if (!ok || he == std::string::npos || std::sscanf(resp.c_str(), "HTTP/%*d.%*d %d", &code) != 1)
    return -1;
  std::string head = resp.substr(0, he + 2), b = resp.substr(he + 4);
  for (char& c : head) c = char(std::tolower(static_cast<unsigned char>(c)));
  if (head.find("transfer-encoding: chunked") != std::string::npos) {
    std::string d;
    for (size_t i = 0; i < b.size();) {
      const size_t le = b.find("\r\n", i);
      if (le == std::string::npos) break;
      const size_t n = std::strtoul(b.c_str() + i, nullptr, 16);
      if (n == 0) break;
      d.append(b, le + 2, n);
      i = le + 2 + n + 2;
    }
    b.swap(d);
  }
  if (out) *out = b;
  return code;
}

// One UploadPart request over plain HTTP/1.1 (Connection: close): the signed headers, then
// the body from memory or, for file parts, by sendfile from the open file (what libcurl's
// read callback does in WebClient::UploadFile, webclient.cpp:331-355).  Returns the HTTP
// status, or -1 on a socket error; *etag receives the response's ETag (quotes trimmed), which
// S3Api::UploadFilePart / UploadPart return (multipart_upload.cpp:101-105, 138-143).
int put_part(const std::string& host, const std::string& port, const std::string& target,
             const s3h::sigv4::Map& headers, const uint8_t* mem, int fd, uint64_t off,
             uint64_t size, std::string* etag) {
  const int sock = open_conn(host, port);
  if (sock < 0) return -1;
  auto send_all = [&](const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
      const ssize_t w = send(sock, c, n, MSG_NOSIGNAL);
      if (w <= 0) return false;
      c += w;
      n -= size_t(w);
    }
    return true;
  };
  std::string req = "PUT " + target + " HTTP/1.1\r\n";
  for (const auto& kv : headers) req += kv.first + ": " + kv.second + "\r\n";
  req += "Connection: close\r\n\r\n";
  bool ok = send_all(req.data(), req.size());
  if (ok && mem) {
    ok = send_all(mem, size);
  } else if (ok) {
    off_t o = off_t(off);
    for (uint64_t left = size; ok && left > 0;) {
      const ssize_t w = sendfile(sock, fd, &o, left);
      ok = w > 0;
      if (ok) left -= uint64_t(w);
    }
  }
  std::string resp;  // the status line and every header
  char buf[4096];
  for (ssize_t r; ok && resp.find("\r\n\r\n") == std::string::npos &&
                  (r = recv(sock, buf, sizeof buf, 0)) > 0;)
    resp.append(buf, size_t(r));
  close(sock);
  int code = -1;
  if (ok && std::sscanf(resp.c_str(), "HTTP/%*d.%*d %d", &code) != 1) code = -1;
  if (etag) *etag = header_value(resp.substr(0, resp.find("\r\n\r\n") + 2), "ETag");
  return code;
}

// One ranged GetObject over plain HTTP/1.1 (Connection: close) into dst[0, size): the ranged
// GETs of DownloadPart (lib/src/download.cpp:72-85).  Returns the HTTP status, or -1 on a
// socket error or a body of another length.
int get_range(const std::string& host, const std::string& port, const std::string& target,
              const s3h::sigv4::Map& headers, uint8_t* dst, uint64_t size) {
  const int sock = open_conn(host, port);
  if (sock < 0) return -1;
  std::string req = "GET " + target + " HTTP/1.1\r\n";
  for (const auto& kv : headers) req += kv.first + ": " + kv.second + "\r\n";
  req += "Connection: close\r\n\r\n";
  bool ok = send(sock, req.data(), req.size(), MSG_NOSIGNAL) == ssize_t(req.size());
  std::string head;
  char buf[65536];
  size_t hdr_end = std::string::npos;
  uint64_t got = 0;
  for (ssize_t r; ok && (r = recv(sock, buf, sizeof buf, 0)) > 0;) {
    if (hdr_end == std::string::npos) {
      head.append(buf, size_t(r));
      hdr_end = head.find("\r\n\r\n");
      if (hdr_end == std::string::npos) continue;
      const size_t body0 = hdr_end + 4, n = std::min<uint64_t>(head.size() - body0, size);
      std::memcpy(dst, head.data() + body0, n);
      got = head.size() - body0;
    } else {
      const uint64_t n = got < size ? std::min<uint64_t>(uint64_t(r), size - got) : 0;
      std::memcpy(dst + got, buf, n);
      got += uint64_t(r);
    }
  }
  close(sock);
  int code = -1;
  if (!ok || std::sscanf(head.c_str(), "HTTP/%*d.%*d %d", &code) != 1) return -1;
  return got == size ? code : -1;
}

// Content-MD5 header value: base64 of the 16 digest bytes (RFC 1864).
std::string base64(const uint8_t* p, size_t n) {
  static const char k[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  for (size_t i = 0; i < n; i += 3) {
    const uint32_t v = uint32_t(p[i]) << 16 | (i + 1 < n ? uint32_t(p[i + 1]) << 8 : 0) |
                       (i + 2 < n ? p[i + 2] : 0);
    o += k[v >> 18];
    o += k[(v >> 12) & 63];
    o += i + 1 < n ? k[(v >> 6) & 63] : '=';
    o += i + 2 < n ? k[v & 63] : '=';
  }
  return o;
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void usage() {
  std::fprintf(stderr,
               "usage: s3-upload-hash -f FILE [-j JOBS] [-n PARTS_PER_JOB] [--source file|mmap|memory]\n"
               "       [--per-job] [--cpu] [--verify] [--print-headers] [--send] [--get-verify]\n"
               "       [--retries N] [--content-md5] [--check-etag] [--multipart] [--route gpu|cpu|auto|split]\n"
               "       [--endpoint URL[,URL...] --bucket B --key K --access A --secret S --upload-id ID]\n"
               "       [--devices N] [--repeat R]\n");
}

}  // namespace

int main(int argc, char** argv) {
  std::string file, endpoint = "http://127.0.0.1:9000", bucket = "bucket1", key = "key1";
  std::string access = "ACCESS", secret = "SECRET", upload_id = "UPLOAD-ID";
  std::string source = "file";
  std::string route_name = "gpu";
  int jobs = 1, ppj = 1, devices = 0, repeat = 1, max_retries = 0;
  bool cpu = false, verify = false, print_headers = false, per_job = false, send_parts = false;
  bool content_md5 = false;  // also send Content-MD5: both digests from one pass
  // --check-etag: each UploadPart's ETag must equal the part's MD5 (plain buckets).  Off by
  // default, as in the reference (DoUploadFilePart / DoUploadPart only require an ETag,
  // multipart_upload.cpp:101-105, 138-143): SSE-KMS / SSE-C parts have non-MD5 ETags, and a
  // Content-MD5 header already makes the server check the body.
  bool check_etag = false;
  bool get_verify = false;   // after the upload, GET every part back and verify it
  bool multipart = false;    // --send: CreateMultipartUpload before the parts, Complete after
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
    else if (a == "--send") send_parts = true;
    else if (a == "--retries") max_retries = std::atoi(next().c_str());
    else if (a == "--content-md5") content_md5 = true;
    else if (a == "--check-etag") check_etag = true;
    else if (a == "--get-verify") get_verify = true;
    else if (a == "--multipart") multipart = true;
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
    else if (a == "--route") route_name = next();
    else { usage(); return 2; }
  }
  std::signal(SIGPIPE, SIG_IGN);  // a closed connection fails its PUT (sendfile has no MSG_NOSIGNAL)
  if (file.empty() || jobs < 1 || ppj < 1 || repeat < 1 ||
      (source != "file" && source != "mmap" && source != "memory") ||
      (route_name != "gpu" && route_name != "cpu" && route_name != "auto" && route_name != "split")) {
    usage();
    return 2;
  }
  const sha256::Route route = route_name == "cpu"     ? sha256::Route::cpu
                              : route_name == "auto"  ? sha256::Route::automatic
                              : route_name == "split" ? sha256::Route::split
                                                      : sha256::Route::gpu;
  sha256::Route route_taken = route;

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

  const bool want_md5 = content_md5 || check_etag;  // MD5s: Content-MD5 and/or the ETag check
  std::vector<std::string> hex(parts.size()), md5b64(want_md5 ? parts.size() : 0);
  std::vector<uint32_t> md5w(want_md5 ? 4 * parts.size() : 0);  // GPU MD5s
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
  // --route: ONE decision for the whole upload, made here before the timed passes (the first
  // decision measures the model, once per process, like the runtime start-up above).  A CPU
  // decision hashes exactly as --cpu does -- each job thread hashes its own parts with the
  // drop-in and PUTs them as it goes, so hashing overlaps the uploads -- and a GPU decision as
  // the default GPU path.
  // The decision prices what this upload computes: with --content-md5 (or --check-etag) each
  // part needs both digests, and the CPU side runs MD5 as well as SHA-256 (pricing
  // only SHA-256 under-priced the CPU near the crossover).  AUTO may also pick the split.
  double est_gpu = 0, est_cpu = 0;
  if (!cpu && route != sha256::Route::gpu && route != sha256::Route::split) {
    try {
      route_taken = route == sha256::Route::cpu
                        ? sha256::Route::cpu
                        : sha256::choose_route(lens, devices, &est_gpu, &est_cpu,
                                               want_md5 ? S3H_DIGESTS_BOTH : S3H_DIGESTS_SHA256,
                                               source == "file" ? S3H_SOURCE_FILE : S3H_SOURCE_PAGEABLE);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s\n", e.what());
      return 1;
    }
  }
  const bool cpu_hash_mode = cpu || route_taken == sha256::Route::cpu;
  // Signed UploadPart headers of part i: its digest in x-amz-content-sha256 instead of
  // UNSIGNED-PAYLOAD (aws_sign.cpp:236-237); the memory path forwards it too, where the
  // reference's DoUploadPart drops it (multipart_upload.cpp:131-136).
  std::vector<std::string> endpoints;  // cfg.endpoints (s3-client.h), comma-separated here
  for (size_t b = 0, e; b <= endpoint.size(); b = e + 1) {
    e = endpoint.find(',', b);
    if (e == std::string::npos) e = endpoint.size();
    if (e > b) endpoints.push_back(endpoint.substr(b, e - b));
  }
  if (endpoints.empty()) { usage(); return 2; }
  auto part_config = [&](size_t i, const std::string& ep) {
    s3h::sigv4::SignConfig c;
    c.access = access;
    c.secret = secret;
    c.endpoint = ep;
    c.method = "PUT";
    c.bucket = bucket;
    c.key = key;
    c.payloadHash = hex[i];
    // partNumber = i + 1 (multipart_upload.cpp:79, :126)
    c.parameters = {{"partNumber", std::to_string(parts[i].number + 1)}, {"uploadId", upload_id}};
    c.headers = {{"content-length", std::to_string(parts[i].size)}};
    if (content_md5) c.headers["Content-MD5"] = md5b64[i];  // sent, not signed (aws_sign.cpp:266-271)
    return c;
  };
  std::vector<std::pair<std::string, std::string>> hostport;
  for (const std::string& ep : endpoints) {  // http://HOST:PORT only (loopback, no TLS)
    const size_t h0 = ep.find("://"), c = ep.rfind(':');
    if (send_parts && (ep.rfind("http://", 0) != 0 || c == std::string::npos || c <= h0 + 3)) {
      std::fprintf(stderr, "--send needs --endpoint http://HOST:PORT[,...]\n");
      return 2;
    }
    hostport.emplace_back(send_parts ? ep.substr(h0 + 3, c - h0 - 3) : "", send_parts ? ep.substr(c + 1) : "");
  }
  std::atomic<int> put_failed{0}, retries{0};
  std::mutex fail_mu;
  std::vector<std::string> failures;  // "part N: why", for every part that failed for good
  // Part i to endpoint e, signed afresh (new x-amz-date) on every attempt; a failed attempt
  // is repeated while the shared retry budget lasts (retriesG, upload.cpp:55-69).  As
  // DoUploadFilePart / DoUploadPart (multipart_upload.cpp:101-105, 138-143) a 200 without an
  // ETag fails the attempt; with --check-etag the ETag must also equal the part's MD5 from
  // the GPU (S3 returns a plain part's body MD5 as its ETag), else the attempt fails.
  std::vector<std::string> part_etags(parts.size());  // UploadPart ETags, for --multipart's Complete
  auto put = [&](size_t i, size_t e) {
    const uint8_t* mem = source == "file" ? nullptr : ptrs[i];
    std::string why;
    for (;;) {
      const s3h::sigv4::SignConfig c = part_config(i, endpoints[e]);
      const std::string target = "/" + bucket + "/" + key + "?" + s3h::sigv4::UrlEncode(c.parameters);
      std::string etag;
      const int code = put_part(hostport[e].first, hostport[e].second, target,
                                s3h::sigv4::SignHeaders(c), mem, fd, offs[i], lens[i], &etag);
      if (code == 200 && etag.empty()) {
        why = "no ETag found in the HTTP header";
      } else if (code == 200 && check_etag) {
        char want[33];
        md5::hash_to_text(&md5w[4 * i], want);
        std::string got(etag);
        for (char& ch : got) ch = char(std::tolower(static_cast<unsigned char>(ch)));
        if (got == want) {
          part_etags[i] = etag;
          return;
        }
        why = "ETag \"" + etag + "\" != the part's MD5 " + want;
      } else if (code == 200) {
        part_etags[i] = etag;
        return;
      } else {
        why = "HTTP status " + std::to_string(code);
      }
      if (retries++ >= max_retries) break;
    }
    ++put_failed;
    std::lock_guard<std::mutex> lk(fail_mu);
    failures.push_back("part " + std::to_string(parts[i].number + 1) + ": " + why);
  };
  std::mt19937 rng{std::random_device{}()};
  std::vector<std::vector<size_t>> job_parts(jobs);
  for (size_t i = 0; i < parts.size(); ++i) job_parts[parts[i].job].push_back(i);
  auto cpu_hash = [&](size_t i) {
    uint32_t h[8];
    sha256::sha256(ptrs[i], lens[i], h);
    char t[65];
    sha256::hash_to_text(h, t);
    hex[i] = t;
    if (want_md5) {
      uint32_t* m = &md5w[4 * i];
      md5::md5(ptrs[i], lens[i], m);
      md5b64[i] = base64(reinterpret_cast<const uint8_t*>(m), 16);
    }
  };
  // GPU: the parts of `idx` through the chosen source, hex digests into hex[idx[k]]
  auto gpu = [&](const std::vector<size_t>& idx) {
    std::vector<const uint8_t*> p;
    std::vector<uint64_t> l, o;
    for (size_t i : idx) {
      p.push_back(ptrs[i]);
      l.push_back(lens[i]);
      o.push_back(offs[i]);
    }
    if (want_md5) {  // both digests, each slice read and copied once; --route split (or
                     // AUTO's split) puts each call's longest parts on the CPU, both digests there too
      const bool split = route_taken == sha256::Route::split;
      const sha256::DualDigests d =
          source == "file" ? (split ? sha256::file_part_sha256_md5_routed(file, o, l, devices, sha256::Route::split)
                                    : sha256::file_part_sha256_md5(file, o, l, devices))
                           : (split ? sha256::sha256_md5_routed(p, l, devices, sha256::Route::split)
                                    : sha256::sha256_md5_batch(p, l, devices));
      for (size_t k = 0; k < idx.size(); ++k) {
        char t[65];
        sha256::hash_to_text(const_cast<uint32_t*>(&d.sha256[8 * k]), t);
        hex[idx[k]] = t;
        md5b64[idx[k]] = base64(reinterpret_cast<const uint8_t*>(&d.md5[4 * k]), 16);
        std::copy(&d.md5[4 * k], &d.md5[4 * k] + 4, &md5w[4 * idx[k]]);
      }
      return;
    }
    // --route split: each call's longest parts on the CPU drop-in while the GPU hashes the rest
    const sha256::Route r = route_taken == sha256::Route::split ? sha256::Route::split : sha256::Route::gpu;
    const std::vector<std::string> h = source == "file"
                                           ? sha256::file_part_hashes(file, o, l, devices, r)
                                           : sha256::payload_hashes(p, l, devices, r);
    for (size_t k = 0; k < idx.size(); ++k) hex[idx[k]] = h[k];
  };
  // --multipart: the POSTs around the parts (S3Api::CreateMultipartUpload /
  // CompleteMultipartUpload, multipart_upload.cpp:157-204), on one endpoint drawn at random as
  // UploadFile's S3Api is (upload.cpp:124-128).  Each is signed with its body's SHA-256 (the
  // CPU drop-in: a few hundred bytes) where the reference sends UNSIGNED-PAYLOAD.
  std::string object_etag, complete_error;
  auto signed_post = [&](size_t e, const s3h::sigv4::Map& params, const std::string& body,
                         std::string* out) {
    uint32_t h[8];
    sha256::sha256(reinterpret_cast<const uint8_t*>(body.data()), body.size(), h);
    char t[65];
    sha256::hash_to_text(h, t);
    s3h::sigv4::SignConfig c;
    c.access = access;
    c.secret = secret;
    c.endpoint = endpoints[e];
    c.method = "POST";
    c.bucket = bucket;
    c.key = key;
    c.payloadHash = t;
    c.parameters = params;
    c.headers = {{"content-length", std::to_string(body.size())}};
    const std::string target = "/" + bucket + "/" + key + "?" + s3h::sigv4::UrlEncode(params);
    return post_request(hostport[e].first, hostport[e].second, target, s3h::sigv4::SignHeaders(c),
                        body, out);
  };
  auto create_upload = [&](size_t e) -> bool {
    std::string xml;
    const int code = signed_post(e, {{"uploads", ""}}, "", &xml);
    upload_id = xml_tag(xml, "UploadId");  // XMLTag(xml, "uploadId"), multipart_upload.cpp:203
    if (code == 200 && !upload_id.empty()) return true;
    complete_error = "CreateMultipartUpload: HTTP status " + std::to_string(code) + (upload_id.empty() ? ", no UploadId" : "");
    return false;
  };
  auto complete_upload = [&](size_t e) -> bool {
    // BuildEndUploadXML (multipart_upload.cpp:48-61): every part's ETag in part-number order
    std::string xml = "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<CompleteMultipartUpload "
                      "xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\">\n";
    for (size_t i = 0; i < parts.size(); ++i)
      xml += "<Part><ETag>" + part_etags[i] + "</ETag><PartNumber>" +
             std::to_string(parts[i].number + 1) + "</PartNumber></Part>";
    xml += "</CompleteMultipartUpload>";
    std::string resp;
    const int code = signed_post(e, {{"uploadId", upload_id}}, xml, &resp);
    object_etag = trim_xml_etag(xml_tag(resp, "ETag"));
    if (code == 200 && !object_etag.empty()) return true;
    complete_error = "CompleteMultipartUpload: HTTP status " + std::to_string(code) +
                     (object_etag.empty() ? ", no ETag" : "") + (resp.empty() ? "" : ": " + resp.substr(0, 200));
    return false;
  };
  // One pass over all parts.  Job threads as upload.cpp:136-140 runs them: the CPU drop-in
  // hashes each part of its job (and, with --send, PUTs it right after); on the GPU either one
  // batched call for all parts (then the jobs PUT) or, --per-job, one concurrent batch call per
  // job, each job then PUTting its own parts.
  auto hash_pass = [&]() -> bool {
    const size_t ep0 = std::uniform_int_distribution<size_t>(0, endpoints.size() - 1)(rng);
    if (send_parts && multipart && !create_upload(ep0)) return false;
    try {
      if (!cpu_hash_mode && !per_job) {
        std::vector<size_t> all(parts.size());
        for (size_t i = 0; i < all.size(); ++i) all[i] = i;
        gpu(all);
        if (!send_parts) return true;
      }
      std::vector<std::future<void>> fut;
      for (int j = 0; j < jobs; ++j) {
        if (job_parts[j].empty()) continue;
        // RandomIndex(0, cfg.endpoints.size() - 1) per job (upload.cpp:94-95)
        const size_t ep = std::uniform_int_distribution<size_t>(0, endpoints.size() - 1)(rng);
        fut.push_back(std::async(std::launch::async, [&, j, ep] {
          if (!cpu_hash_mode && per_job) gpu(job_parts[j]);
          for (size_t i : job_parts[j]) {
            if (cpu_hash_mode) cpu_hash(i);
            if (send_parts) put(i, ep);
          }
        }));
      }
      for (auto& f : fut) f.get();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s\n", e.what());
      return false;
    }
    // the reference's UploadParts throws on a part that failed for good, so no Complete
    if (send_parts && multipart && !put_failed.load() && !complete_upload(ep0)) return false;
    return true;
  };
  // --repeat R: R passes (an uploader's steady state, buffers cached); the last pass is
  // reported, the first beside it.
  double t0 = 0, first = 0;
  for (int rep = 0; rep < repeat; ++rep) {
    t0 = now();
    if (!hash_pass()) {
      if (!complete_error.empty()) std::fprintf(stderr, "upload failed: %s\n", complete_error.c_str());
      return 1;
    }
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

  // --get-verify: the download side (DownloadFile / DownloadParts, download.cpp:88-130): each
  // job GETs its parts by byte range into one buffer, then every part is checked against the
  // digest it was uploaded with -- on the GPU in one s3h_verify_batch_host call (the CPU
  // drop-in with --cpu).
  int get_failed = 0;
  uint64_t down_bad = 0;
  double t_get = 0, t_check = 0;
  if (send_parts && get_verify) {
    std::vector<uint8_t> down(size);
    std::atomic<int> failed{0};
    const double g0 = now();
    std::vector<std::future<void>> fut;
    for (int j = 0; j < jobs; ++j) {
      if (job_parts[j].empty()) continue;
      const size_t e = std::uniform_int_distribution<size_t>(0, endpoints.size() - 1)(rng);
      fut.push_back(std::async(std::launch::async, [&, j, e] {
        for (size_t i : job_parts[j]) {
          s3h::sigv4::SignConfig c;
          c.access = access;
          c.secret = secret;
          c.endpoint = endpoints[e];
          c.method = "GET";
          c.bucket = bucket;
          c.key = key;
          c.headers = {{"Range", "bytes=" + std::to_string(offs[i]) + "-" +
                                     std::to_string(offs[i] + lens[i] - 1)}};
          if (get_range(hostport[e].first, hostport[e].second, "/" + bucket + "/" + key,
                        s3h::sigv4::SignHeaders(c), down.data() + offs[i], lens[i]) != 206)
            ++failed;
        }
      }));
    }
    for (auto& f : fut) f.get();
    get_failed = failed.load();
    const double g1 = now();
    std::vector<const uint8_t*> dp(parts.size());
    for (size_t i = 0; i < parts.size(); ++i) dp[i] = down.data() + offs[i];
    if (cpu) {
      for (size_t i = 0; i < parts.size(); ++i) {
        uint32_t h[8];
        sha256::sha256(dp[i], lens[i], h);
        char t[65];
        sha256::hash_to_text(h, t);
        down_bad += hex[i] != t;
      }
    } else {
      try {
        for (bool b : sha256::verify_payloads(dp, lens, hex, devices)) down_bad += b;
      } catch (const std::exception& e) {
        std::fprintf(stderr, "verify: %s\n", e.what());
        return 1;
      }
    }
    t_get = g1 - g0;
    t_check = now() - g1;
  }

  std::printf("part,job,offset,size,sha256\n");
  for (size_t i = 0; i < parts.size(); ++i)
    std::printf("%d,%d,%llu,%llu,%s\n", parts[i].number, parts[i].job,
                (unsigned long long)parts[i].offset, (unsigned long long)parts[i].size,
                hex[i].c_str());
  if (print_headers)
    for (size_t i = 0; i < parts.size(); ++i)
      for (const auto& kv : s3h::sigv4::SignHeaders(part_config(i, endpoints[0])))
        std::printf("# part %d %s: %s\n", parts[i].number, kv.first.c_str(), kv.second.c_str());
  std::string what = cpu ? std::string("cpu lib/hash drop-in")
                         : "gpu batch (H2D included, source " + source +
                               (per_job ? ", one call per job" : ", one call") +
                               (route == sha256::Route::gpu ? std::string()
                                : std::string(", route ") + route_name + " -> " +
                                      (route_taken == sha256::Route::cpu     ? "cpu"
                                       : route_taken == sha256::Route::split ? "split"
                                                                             : "gpu")) +
                               (route == sha256::Route::automatic
                                    ? " (model: gpu " + std::to_string(est_gpu) + " s, cpu " +
                                          std::to_string(est_cpu) + " s)"
                                    : std::string()) + ")";
  if (send_parts) what = "upload (hash + PUT to " + endpoint + ", " + std::to_string(jobs) + " jobs), " + what;
  std::fprintf(stderr, "%s: %zu parts, %.3f GiB in %.3f s = %.3f GiB/s%s", what.c_str(), parts.size(),
               double(size) / (1 << 30), dt, double(size) / (1 << 30) / dt,
               verify ? (mismatches ? ", VERIFY FAILED" : ", verified vs CPU") : "");
  if (send_parts)
    std::fprintf(stderr, " (%d of %zu PUTs not 200, %d retries)", put_failed.load(),
                 parts.size() * size_t(repeat), retries.load());
  if (repeat > 1) std::fprintf(stderr, " (pass %d of %d; first pass %.3f s)", repeat, repeat, first);
  if (!cpu) std::fprintf(stderr, " (GPU runtime start-up before it: %.3f s)", init_s);
  std::fprintf(stderr, "\n");
  for (const std::string& f : failures) std::fprintf(stderr, "upload failed: %s\n", f.c_str());
  bool etag_mismatch = false;
  std::string local_etag;
  if (want_md5) {  // the ETag CompleteMultipartUpload would return, from the GPU MD5s
    try {
      local_etag = md5::multipart_etag(md5w);
      std::fprintf(stderr, "multipart etag: %s\n", local_etag.c_str());
    } catch (const std::exception& e) {
      std::fprintf(stderr, "multipart etag: %s\n", e.what());
      return 1;
    }
  }
  if (send_parts && multipart && !put_failed.load()) {
    // the object's ETag from the server's CompleteMultipartUpload, checked against the one the
    // local MD5s give: the server hashed what it received, so equality closes the loop
    std::string lower(object_etag);
    for (char& ch : lower) ch = char(std::tolower(static_cast<unsigned char>(ch)));
    etag_mismatch = want_md5 && lower != local_etag;
    std::fprintf(stderr, "complete: upload id %s, object etag %s%s\n", upload_id.c_str(),
                 object_etag.c_str(),
                 !want_md5 ? "" : etag_mismatch ? " != the local multipart etag (MISMATCH)"
                                                : " == the local multipart etag");
  }
  if (send_parts && get_verify)
    std::fprintf(stderr, "download verify: %zu parts, %d GETs failed, %llu mismatches (GET %.3f s, %s check %.3f s)\n",
                 parts.size(), get_failed, (unsigned long long)down_bad, t_get, cpu ? "CPU" : "GPU",
                 t_check);
  munmap(const_cast<uint8_t*>(data), size);
  close(fd);
  return mismatches || put_failed.load() || get_failed || down_bad || etag_mismatch ? 1 : 0;
}
