/*
 * oracle/cpu_baseline.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline that bench.py times
 * (cpu_baseline, kind "port").  Never linked into the product.
 *
 * A from-scratch restatement of lib/hash's sha256::sha256 that keeps lib/hash's COST
 * STRUCTURE, so that timing it on the GPU box's host is a faithful "lib/hash on these cores"
 * number without shipping the reference (BASELINE.md "CPU baseline plan"):
 *   - one-shot sha256 (lib/hash/sha256.cpp:147-160): a thread-local 4 KiB scratch when the
 *     padded message fits (next_div_by(len + 9, 64) <= 4096), otherwise a calloc'd padded copy
 *     (alloc_padded, utility.cpp:42-56) filled by memcpy, freed afterwards;
 *   - compression (sha256.cpp:84-144): scalar, big-endian words assembled byte by byte
 *     (lshift, utility.h:121-123) inside the first 16 rounds, then a 16-word ring schedule
 *     updated in place during rounds 16-63; Ch/Maj/Sigma in lib/hash's boolean forms;
 *   - output words bswap32(H_i) (to_little, sha256.h:103-106).
 * Built by bench.py on the box with the reference's release flags
 * `-Ofast -march=native -flto` (lib/CMakeLists.txt:45); calibrated against the real lib/hash
 * in the build container (tools/calibrate_cpu_baseline.py ->
 * profiles/r02_cpu_baseline_calibration.json).  Digests are checked against the golden
 * fixtures (tests/test_oracle.py) and, in bench.py, against the GPU's.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t RC[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

static inline uint32_t ror32(uint32_t v, unsigned s) { return (v >> s) | (v << (32 - s)); }
static inline uint32_t big_s0(uint32_t v) { return ror32(v, 2) ^ ror32(v, 13) ^ ror32(v, 22); }
static inline uint32_t big_s1(uint32_t v) { return ror32(v, 6) ^ ror32(v, 11) ^ ror32(v, 25); }
static inline uint32_t choose(uint32_t s, uint32_t x, uint32_t y) { return (s & x) | ((~s) & y); }
static inline uint32_t major(uint32_t x, uint32_t y, uint32_t z) { return (x & y) ^ (x & z) ^ (y & z); }

#define BASE_ROUND(KW)                                  \
  do {                                                  \
    const uint32_t t1 = hh + big_s1(e) + choose(e, f, g) + (KW); \
    const uint32_t t2 = big_s0(a) + major(a, b, c);     \
    hh = g; g = f; f = e; e = d + t1;                   \
    d = c; c = b; b = a; a = t1 + t2;                   \
  } while (0)

/* compression of whole 64-byte blocks, lib/hash's loop shape (sha256.cpp:88-143) */
static void base_compress(uint32_t st[8], const uint8_t *p, uint64_t nbytes) {
  for (uint64_t left = nbytes >> 6; left; --left) {
    uint32_t ring[16];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], hh = st[7];
    for (int r = 0; r < 16; ++r, p += 4) {
      ring[r] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
      BASE_ROUND(RC[r] + ring[r]);
    }
    for (int r = 16; r < 64; ++r) {
      const uint32_t x = ring[(r + 1) & 15], y = ring[(r + 14) & 15];
      ring[r & 15] += (ror32(x, 7) ^ ror32(x, 18) ^ (x >> 3)) +
                      (ror32(y, 17) ^ ror32(y, 19) ^ (y >> 10)) + ring[(r + 9) & 15];
      BASE_ROUND(ring[r & 15] + RC[r]);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += hh;
  }
}

void base_sha256(const uint8_t *data, uint64_t len, uint32_t out[8]) {
  static __thread uint8_t scratch[4096];
  static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  memcpy(out, iv, sizeof iv);
  const uint64_t padded = (len + 9 + 63) & ~(uint64_t)63;
  uint8_t *msg = padded <= sizeof scratch ? scratch : (uint8_t *)calloc(padded, 1);
  if (msg == scratch) memset(msg, 0, padded);
  memcpy(msg, data, len);
  msg[len] = 0x80;
  for (int i = 0; i < 8; ++i) msg[padded - 1 - i] = (uint8_t)((len << 3) >> (8 * i));
  base_compress(out, msg, padded);
  if (msg != scratch) free(msg);
  for (int i = 0; i < 8; ++i) out[i] = __builtin_bswap32(out[i]);
}

struct base_job {
  const uint8_t *base;
  const uint64_t *off, *len;
  uint64_t n, first, step;
  uint32_t *out;
};

static void *base_worker(void *arg) {
  const struct base_job *j = (const struct base_job *)arg;
  for (uint64_t i = j->first; i < j->n; i += j->step) base_sha256(j->base + j->off[i], j->len[i], j->out + 8 * i);
  return NULL;
}

/* n parts on `threads` POSIX threads, parts round-robin (one std::thread per core in the
 * BASELINE plan); returns 0, or -1 if a thread could not be started. */
int base_sha256_batch(const uint8_t *base, const uint64_t *offsets, const uint64_t *lengths,
                      uint64_t n, uint32_t *out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof *tid);
  struct base_job *jobs = (struct base_job *)calloc((size_t)threads, sizeof *jobs);
  int rc = 0, started = 0;
  for (int t = 0; t < threads; ++t, ++started) {
    jobs[t] = (struct base_job){base, offsets, lengths, n, (uint64_t)t, (uint64_t)threads, out};
    if (pthread_create(&tid[t], NULL, base_worker, &jobs[t])) { rc = -1; break; }
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
  return rc;
}
