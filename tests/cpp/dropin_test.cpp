// tests/cpp/dropin_test.cpp -- the lib/hash drop-in linked exactly as the reference's callers
// link lib/hash: only include/sha256.h + utility.h and libs3hash.so.  Mirrors the reference's
// in-file known-answer tests (lib/hash/sha256.cpp:236-399, which do not compile upstream) and
// exercises every exported symbol.  `--gpu` also runs the batched C++ API on the GPU.
// Output: CSV "Hash,<action>,0|1," like the reference tests (test/utility.cpp:87-95).
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <future>
#include <string>
#include <vector>

#include "md5.h"
#include "s3hash_batch.hpp"
#include "sha256.h"

static int fails = 0;
static void report(const char* action, bool ok) {
  std::printf("Hash,%s,%d,\n", action, int(ok));
  fails += !ok;
}

static std::string text(uint32_t h[8]) {
  char t[65];
  sha256::hash_to_text(h, t);
  return t;
}

static std::string digest(const std::string& s) {
  uint32_t h[8];
  sha256::sha256(reinterpret_cast<const uint8_t*>(s.data()), s.size(), h);
  return text(h);
}

int main(int argc, char** argv) {
  std::string s6, s14, s15;
  for (int i = 0; i < 15; ++i) {
    if (i < 6) s6 += "12345678";
    if (i < 14) s14 += "12345678";
    s15 += "12345678";
  }
  s14 += "1234567";
  // KATs of lib/hash/sha256.cpp:248-249, 284-285, 331-332
  report("sha256 48 bytes", digest(s6) == "dd7f20ca4910f937c3e560427de36fea7c37eed94899b3a9bf286905860d17ae");
  report("sha256 119 bytes", digest(s14) == "0c65765f1b9fff74bb831fa24c63d9ab0513c881fc7b4919b43f72f5487a24fd");
  report("sha256 120 bytes", digest(s15) == "979e3016a670a5b1308dba2d715f75201eebcef0adc4a1ac99877fad91ce3ff6");
  report("sha256 empty", digest("") == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");

  // sha256_stream over an alloc_padded buffer == sha256 (sha256.cpp:147-160 composition)
  {
    size_t sz = 0;
    uint8_t* buf = alloc_padded(s15.size(), s15.size(), &sz, nullptr);
    std::memcpy(buf, s15.data(), s15.size());
    uint32_t h[8];
    sha256::init_hash(h);
    sha256::sha256_stream(h, buf, sz);
    sha256::to_little(h);
    std::free(buf);
    report("alloc_padded+stream", sz == 192 && text(h) == digest(s15));
  }
  // chunked: whole blocks with total_length 0, then the final chunk with the total length
  {
    std::string big(1000, 'x');
    for (size_t i = 0; i < big.size(); ++i) big[i] = char(i * 7 + 3);
    uint32_t h[8];
    sha256::init_hash(h);
    sha256::sha256_next(reinterpret_cast<const uint8_t*>(big.data()), 640, h, 0, nullptr);
    std::vector<uint8_t> tmp(512);
    sha256::sha256_next(reinterpret_cast<const uint8_t*>(big.data()) + 640, 360, h, 1000, tmp.data());
    sha256::to_little(h);
    report("sha256_next chunked", text(h) == digest(big));
  }
  // sha256_file == sha256 of the same bytes (incl. exactly 16 MiB, the reference buffer size)
  for (size_t n : {size_t(0), size_t(1), size_t(100000), size_t(16) << 20}) {
    std::string path = "/tmp/s3h_dropin_" + std::to_string(n);
    std::vector<uint8_t> v(n);
    for (size_t i = 0; i < n; ++i) v[i] = uint8_t(i * 31 + 7);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (n) std::fwrite(v.data(), 1, n, f);
    std::fclose(f);
    uint32_t a[8], b[8];
    sha256::sha256_file(path.c_str(), a);
    sha256::sha256(v.data(), n, b);
    std::remove(path.c_str());
    report(("sha256_file " + std::to_string(n)).c_str(), std::memcmp(a, b, 32) == 0);
  }
  // hmac256 RFC 4231 test case 2 ("Jefe")
  {
    const std::string key = "Jefe", msg = "what do ya want for nothing?";
    uint8_t mac[32];
    hmac256(reinterpret_cast<const uint8_t*>(msg.data()), msg.size(),
            reinterpret_cast<const uint8_t*>(key.data()), key.size(), mac);
    char t[65];
    for (int i = 0; i < 32; ++i) std::snprintf(t + 2 * i, 3, "%02x", mac[i]);
    report("hmac256 rfc4231", std::string(t) == "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843");
  }
  // md5 drop-in (lib/hash/md5.h): RFC 1321 test suite values, md5_file == md5
  {
    auto m = [](const std::string& x) {
      uint32_t h[4];
      md5::md5(reinterpret_cast<const uint8_t*>(x.data()), x.size(), h);
      char t[33];
      md5::hash_to_text(h, t);
      return std::string(t);
    };
    report("md5 rfc1321", m("") == "d41d8cd98f00b204e9800998ecf8427e" &&
                              m("abc") == "900150983cd24fb0d6963f7d28e17f72" &&
                              m("message digest") == "f96b697d7cb7938d525a2f31aaf161d0");
    std::vector<uint8_t> v(1000003);
    for (size_t i = 0; i < v.size(); ++i) v[i] = uint8_t(i * 13 + 1);
    FILE* f = std::fopen("/tmp/s3h_md5_dropin", "wb");
    std::fwrite(v.data(), 1, v.size(), f);
    std::fclose(f);
    uint32_t a[4], b[4];
    md5::md5_file("/tmp/s3h_md5_dropin", a);
    md5::md5(v.data(), v.size(), b);
    std::remove("/tmp/s3h_md5_dropin");
    report("md5_file", std::memcmp(a, b, 16) == 0);
  }
  // utility.h helpers
  report("utility", to_big_endian(0x0102030405060708ull) == 0x0807060504030201ull &&
                        to_little_endian(0x11223344u) == 0x44332211u &&
                        next_div_by(129, 64) == 192 && next_div_by(128, 64) == 128 &&
                        right_rotate(1u, 1) == 0x80000000u && lshift(0xff, 8) == 0xff00u);
  // verify_payloads rejects a malformed expected digest -- a sign, whitespace, a 0x prefix, a
  // non-hex digit, a wrong length -- before any GPU call, naming the part (CPU-only check)
  {
    const std::string good(64, 'a');
    const std::string bad[] = {"-1" + std::string(62, '0'), " f" + std::string(62, '0'),
                               "0x" + std::string(62, '0'), std::string(63, '0') + "g",
                               std::string(63, '0')};
    bool all_rejected = true;
    for (const std::string& b : bad) {
      const uint8_t byte = 0;
      try {
        (void)sha256::verify_payloads({&byte, &byte}, {1, 1}, {good, b});
        all_rejected = false;
      } catch (const std::invalid_argument& e) {
        all_rejected &= std::string(e.what()).find("part 1") != std::string::npos;
      } catch (...) {
        all_rejected = false;  // the parse must fail first, not the (absent) GPU
      }
    }
    report("verify_payloads rejects malformed hex", all_rejected);
  }
  if (argc > 1 && std::string(argv[1]) == "--gpu") {
    std::vector<std::string> msgs = {s6, s14, s15, "", std::string(5 << 20, 'q')};
    std::vector<const uint8_t*> ptrs;
    std::vector<uint64_t> lens;
    for (auto& m : msgs) {
      ptrs.push_back(reinterpret_cast<const uint8_t*>(m.data()));
      lens.push_back(m.size());
    }
    const auto hex = sha256::payload_hashes(ptrs, lens);
    bool ok = true;
    for (size_t i = 0; i < msgs.size(); ++i) ok &= hex[i] == digest(msgs[i]);
    report("gpu batch payload_hashes", ok);
    // both upload headers in one pass == the single-buffer drop-ins
    const sha256::DualDigests dd = sha256::sha256_md5_batch(ptrs, lens);
    bool dual_ok = true;
    for (size_t i = 0; i < msgs.size(); ++i) {
      uint32_t h[8], m5[4];
      sha256::sha256(ptrs[i], lens[i], h);
      md5::md5(ptrs[i], lens[i], m5);
      dual_ok &= std::memcmp(h, &dd.sha256[8 * i], 32) == 0 && std::memcmp(m5, &dd.md5[4 * i], 16) == 0;
    }
    report("gpu sha256_md5_batch", dual_ok);
    // the same messages streamed in ragged chunks through sha256::stream_batch
    sha256::stream_batch sb(msgs.size());
    std::vector<size_t> pos(msgs.size(), 0);
    const size_t steps[] = {1, 63, 64, 65, 1000, 1 << 20};
    for (int round = 0;; ++round) {
      bool more = false;
      std::vector<const uint8_t*> cp(msgs.size());
      std::vector<uint64_t> cl(msgs.size());
      for (size_t i = 0; i < msgs.size(); ++i) {
        const size_t take = std::min(steps[(round + i) % 6], msgs[i].size() - pos[i]);
        cp[i] = reinterpret_cast<const uint8_t*>(msgs[i].data()) + pos[i];
        cl[i] = take;
        pos[i] += take;
        more |= take > 0;
      }
      if (!more) break;
      sb.append(cp, cl);
    }
    const auto sh = sb.finish_hex();
    bool sok = true;
    for (size_t i = 0; i < msgs.size(); ++i) sok &= sh[i] == digest(msgs[i]);
    report("gpu stream_batch", sok);

    // Concurrent callers in the shape of lib/src/upload.cpp:89-110 + 136-140: the transfer
    // test's object (test/parallel-file-transfer-test.cpp:50-59, bytes i % 128) sliced into
    // 3 jobs x 2 parts; each job is a std::async thread that hashes ITS parts with its own
    // batch call while the others do (the calls meet in the device's queue and run as merged
    // batches), plus a fourth job hashing the same parts from a file.
    {
      const uint64_t size = 38000007;
      std::vector<uint8_t> obj(size);
      for (uint64_t i = 0; i < size; ++i) obj[i] = uint8_t(i % 128);
      const char* want[6] = {
          "6dcb77e2b805f5cf4962377e29401180e87ee214d469a71d2c9b14f7a99cc52c",
          "f9b1736fa43ac57591e39848316506aa821605e047ba754955d58cd322a3ea35",
          "61da16a2a47588d0ce1395076a3d238235bd76001af269e378b2b74fb9777776",
          "f8ebaab206806551bcb184b6626cbabb017ab968c5c34db7231fa548fbbb94a3",
          "272da9db8caf86bf7e463fca5f7b002dd158eaa49b6f992b41e3593f37ff95fb",
          "0aa12676f0770a0be4618bb2992d5e48ebef5c4858965bb8f3f2ee417ffbc1cb"};
      std::vector<uint64_t> offs, lens;  // upload.cpp:98-107 + :133
      const uint64_t per_job = (size + 2) / 3;
      for (int j = 0; j < 3; ++j) {
        uint64_t off = j * per_job;
        const uint64_t chunk = std::min(per_job, size - off), psz = (chunk + 1) / 2;
        for (int k = 0; k < 2; ++k) {
          const uint64_t sz = std::min(psz, chunk - k * psz);
          offs.push_back(off);
          lens.push_back(sz);
          off += sz;
        }
      }
      const std::string path = "/tmp/s3h_dropin_xfer.bin";
      FILE* f = std::fopen(path.c_str(), "wb");
      std::fwrite(obj.data(), 1, size, f);
      std::fclose(f);
      bool cok = true;
      for (int rep = 0; rep < 3 && cok; ++rep) {
        std::vector<std::future<std::vector<std::string>>> jobs;
        for (int j = 0; j < 3; ++j)
          jobs.push_back(std::async(std::launch::async, [&, j] {
            return sha256::payload_hashes({obj.data() + offs[2 * j], obj.data() + offs[2 * j + 1]},
                                          {lens[2 * j], lens[2 * j + 1]});
          }));
        auto file_job = std::async(std::launch::async, [&] {
          return sha256::file_part_hashes(path, offs, lens);
        });
        for (int j = 0; j < 3; ++j) {
          const auto h = jobs[j].get();
          cok &= h.size() == 2 && h[0] == want[2 * j] && h[1] == want[2 * j + 1];
        }
        const auto fh = file_job.get();
        for (int i = 0; i < 6; ++i) cok &= fh[i] == want[i];
      }
      report("gpu concurrent jobs", cok);

      // Size-aware routing through the C++ layer: one decision for the upload
      // (choose_route), then each route explicitly, memory parts and file ranges alike --
      // every route returns the reference's digests.
      bool rok = true;
      double g = 0, c = 0;
      const sha256::Route pick = sha256::choose_route(lens, 0, &g, &c);
      rok &= g > 0 && c > 0 && (pick == sha256::Route::cpu) == (c < g);
      std::vector<const uint8_t*> parts;
      for (uint64_t o : offs) parts.push_back(obj.data() + o);
      for (sha256::Route r : {sha256::Route::gpu, sha256::Route::cpu, sha256::Route::automatic}) {
        sha256::Route t1 = sha256::Route::automatic, t2 = sha256::Route::automatic;
        const auto hm = sha256::payload_hashes(parts, lens, 0, r, &t1);
        const auto hf = sha256::file_part_hashes(path, offs, lens, 0, r, &t2);
        for (int i = 0; i < 6; ++i) rok &= hm[i] == want[i] && hf[i] == want[i];
        rok &= t1 != sha256::Route::automatic && t2 != sha256::Route::automatic;
        if (r == sha256::Route::automatic) rok &= t1 == pick && t2 == pick;
        else rok &= t1 == r && t2 == r;
      }
      report("gpu routed payload_hashes", rok);
      std::remove(path.c_str());
    }
    sha256::trim();
  }
  return fails ? 1 : 0;
}
