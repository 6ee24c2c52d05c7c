// tools/ubench_coissue.hip -- can a second wave on the SAME SIMD issue beside a SHA-256
// consumer wave without slowing it?  (Design question for C4-sized batches: skew consumers
// (8 VALU/round, mostly 3-source VOP3) on every SIMD with a producer wave beside each.)
//
// One workgroup per CU, 8 waves: waves 0-3 run the skew-like consumer round stream (the
// quad/skew round mix: alignbit, bitop3, bfi, 2 x xor_dpp, 3 x add_dpp / add3) for a fixed
// count; waves 4-7 are partners of kind P that run until their SIMD's consumer is done (LDS
// flag) and count what they issued:
//   0 none (exit)            1 VOP2 only: lshl/lshr/xor/add/or, 2-source, independent
//   2 VOP3 3-source mix      3 VOP2 mix + one ds_write_b128 per 16 VALU (producer-like)
//   4 VOP2 mix with v_perm (byte swap) per 8            5 the consumer stream itself
// Every wave records its SIMD (HW_ID) so pairs are matched by (CU, SIMD), not by index.
// Result (profiles/r02_ubench_coissue*.txt): every partner here was starved -- but each of these
// streams contains "complex" instructions (left shifts, alignbit, perm, add3, DPP).  The
// per-class sweep in tools/ubench_coissue2.hip shows that partners made only of simple ones
// (add/sub, xor/or/and, right shifts, mov) DO issue beside the round stream at the lone-wave
// rate; sha256_skew_shared_kernel's producer is built on that.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_coissue tools/ubench_coissue.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define QR(a, b, c, d, x, xn)                                                                 \
  "v_alignbit_b32 %[q1], %[" #a "], %[" #a "], %[h1]\n\t"                                     \
  "v_bitop3_b32 %[q4], %[" #a "], %[" #b "], %[m] bitop3:0xd2\n\t"                            \
  "v_bfi_b32 %[q2], %[q4], %[" #b "], %[" #c "]\n\t"                                          \
  "v_xor_b32_dpp %[q3], %[q1], %[q1] quad_perm:[1,2,0,1] row_mask:0xf bank_mask:0xf\n\t"     \
  "v_xor_b32_dpp %[q3], %[q1], %[q3] quad_perm:[2,0,1,2] row_mask:0xf bank_mask:0xf\n\t"     \
  "v_add3_u32 %[q3], %[" #x "], %[q3], %[q2]\n\t"                                             \
  "v_add_u32_dpp %[" #xn "], %[w], %[" #c "] quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0x5\n\t" \
  "v_add_u32_dpp %[" #d "], %[" #d "], %[q3] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"       \
  "v_add_u32_dpp %[" #d "], %[q3], %[q3] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
#define Q4 QR(s0, s1, s2, s3, xa, xb) QR(s3, s0, s1, s2, xb, xa) QR(s2, s3, s0, s1, xa, xb) QR(s1, s2, s3, s0, xb, xa)
#define Q16 Q4 Q4 Q4 Q4
#define Q64 Q16 Q16 Q16 Q16
constexpr int kQ64Instr = 64 * 9;

// partner bodies: 16 instructions each, on 6 independent registers
#define V2_8 "v_lshlrev_b32 %0, 7, %1\n\tv_lshrrev_b32 %2, 25, %3\n\tv_xor_b32 %4, %0, %2\n\tv_add_u32 %5, %5, %4\n\t" \
             "v_or_b32 %1, %1, %5\n\tv_lshrrev_b32 %3, 3, %3\n\tv_xor_b32 %2, %3, %4\n\tv_add_u32 %0, %0, %1\n\t"
#define V3_8 "v_alignbit_b32 %0, %1, %1, 7\n\tv_alignbit_b32 %2, %3, %3, 18\n\tv_bitop3_b32 %4, %0, %2, %5 bitop3:0x96\n\t" \
             "v_add3_u32 %5, %5, %4, %1\n\tv_alignbit_b32 %1, %4, %4, 17\n\tv_bitop3_b32 %3, %1, %2, %0 bitop3:0x96\n\t" \
             "v_add3_u32 %0, %0, %3, %5\n\tv_alignbit_b32 %2, %5, %5, 19\n\t"
#define VP_8 "v_perm_b32 %0, %1, %3, %6\n\tv_lshrrev_b32 %2, 25, %3\n\tv_xor_b32 %4, %0, %2\n\tv_add_u32 %5, %5, %4\n\t" \
             "v_or_b32 %1, %1, %5\n\tv_lshrrev_b32 %3, 3, %3\n\tv_xor_b32 %2, %3, %4\n\tv_add_u32 %0, %0, %1\n\t"

template <int P, int CPRIO, int PPRIO>
__global__ __launch_bounds__(512) void coissue(uint32_t* out, uint64_t* rec, int iters) {
  __shared__ volatile uint32_t done[5];  // [simd] = that SIMD's consumer finished; [4] = count
  __shared__ uint4 scratch[8][64];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_REG_HW_ID
  const uint32_t simd = (hw >> 4) & 3;
  if (threadIdx.x < 5) done[threadIdx.x] = 0;
  __syncthreads();
  uint64_t t0, t1, count = 0;
  uint32_t sink = 0;
  if (wave < 4) {
    if (CPRIO) __builtin_amdgcn_s_setprio(3);
    uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
    uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
    const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < iters; ++i)
      asm volatile(".p2align 3\n\t" Q64
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                     [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                   : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    count = uint64_t(iters) * kQ64Instr;
    done[simd] = 1;  // every SIMD's consumer flags its own slot
    if (lane == 0) atomicAdd(const_cast<uint32_t*>(&done[4]), 1u);
    sink = s0 ^ s1 ^ s2 ^ s3;
  } else {
    if (PPRIO) __builtin_amdgcn_s_setprio(3);
    if (P == 0) {
      t0 = t1 = 0;
    } else {
      uint32_t a = lane, b = lane * 7, c = lane * 13, d = lane * 17, e = lane * 19, f = lane * 23;
      const uint32_t sel = 0x00010203u;
      uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
      uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
      const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
      // exit when this SIMD's consumer is done, when all four are (odd placement), or after
      // a cap -- every partner wave terminates whatever the placement
      const uint64_t cap = 8ull * uint64_t(iters) * kQ64Instr;
      while (!done[simd] && done[4] < 4 && count < cap) {
        if (P == 1) {
          for (int k = 0; k < 8; ++k)
            asm volatile(".p2align 3\n\t" V2_8 V2_8 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "v"(sel));
          count += 128;
        } else if (P == 2) {
          for (int k = 0; k < 8; ++k)
            asm volatile(".p2align 3\n\t" V3_8 V3_8 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "v"(sel));
          count += 128;
        } else if (P == 3) {
          for (int k = 0; k < 8; ++k) {
            asm volatile(".p2align 3\n\t" V2_8 V2_8 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "v"(sel));
            scratch[k][lane] = make_uint4(a, b, c, d);
          }
          count += 128;
        } else if (P == 4) {
          for (int k = 0; k < 8; ++k)
            asm volatile(".p2align 3\n\t" VP_8 VP_8 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f) : "v"(sel));
          count += 128;
        } else {
          asm volatile(".p2align 3\n\t" Q64
                       : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                         [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                       : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
          count += kQ64Instr;
        }
      }
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
      sink = a ^ b ^ c ^ d ^ e ^ f ^ s0 ^ s1 ^ s2 ^ s3;
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = sink;
  if (lane == 0) {
    uint64_t* r = rec + 4 * (blockIdx.x * 8 + wave);
    r[0] = t1 - t0;
    r[1] = count;
    r[2] = hw;
    r[3] = wave;
  }
}

template <int P, int CPRIO = 1, int PPRIO = 0>
int run(int grid, const char* label) {
  const int iters = 300;
  uint32_t* out;
  uint64_t* rec;
  CHECK(hipMalloc(&out, size_t(grid) * 512 * 4));
  CHECK(hipMalloc(&rec, size_t(grid) * 8 * 4 * 8));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((coissue<P, CPRIO, PPRIO>), dim3(grid), dim3(512), 0, 0, out, rec, iters);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint64_t> h(size_t(grid) * 8 * 4);
  CHECK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
  double ccpi = 0, cmax = 0, pipc = 0;
  int nc = 0, np = 0, paired = 0;
  for (int g = 0; g < grid; ++g) {
    std::map<int, int> simd_of;
    for (int w = 0; w < 8; ++w) {
      const uint64_t* r = &h[4 * (g * 8 + w)];
      simd_of[w] = int((r[2] >> 4) & 3);
      if (w < 4) {
        const double cpi = double(r[0]) / double(r[1]);
        ccpi += cpi;
        cmax = std::max(cmax, cpi);
        ++nc;
      } else if (P != 0 && r[0]) {
        pipc += double(r[1]) / double(r[0]);
        ++np;
      }
    }
    for (int w = 4; w < 8; ++w)
      for (int c = 0; c < 4; ++c) paired += simd_of[w] == simd_of[c];
  }
  printf("%-40s prio c%d/p%d grid=%3d consumer cyc/instr mean %.3f max %.3f | partner instr/cycle %.3f "
         "(= %.2f cyc/instr) | partners sharing a consumer's SIMD %d/%d\n",
         label, CPRIO * 3, PPRIO * 3, grid, ccpi / nc, cmax, np ? pipc / np : 0.0, np && pipc > 0 ? np / pipc : 0.0,
         paired, 4 * grid);
  CHECK(hipFree(out));
  CHECK(hipFree(rec));
  return 0;
}

int main() {
  for (int grid : {1, 256}) {
    if (run<0>(grid, "partner: none")) return 1;
    if (run<1>(grid, "partner: VOP2 (lshl/lshr/xor/add/or)")) return 1;
    if (run<2>(grid, "partner: VOP3 (alignbit/bitop3/add3)")) return 1;
    if (run<3>(grid, "partner: VOP2 + ds_write_b128 / 16")) return 1;
    if (run<4>(grid, "partner: VOP2 + v_perm / 8")) return 1;
    if (run<5>(grid, "partner: consumer stream")) return 1;
  }
  // equal priorities (both 0, both 3): does a partner get slots, and at what cost?
  for (int grid : {256}) {
    if (run<1, 0, 0>(grid, "partner: VOP2 (lshl/lshr/xor/add/or)")) return 1;
    if (run<3, 0, 0>(grid, "partner: VOP2 + ds_write_b128 / 16")) return 1;
    if (run<2, 0, 0>(grid, "partner: VOP3 (alignbit/bitop3/add3)")) return 1;
    if (run<5, 0, 0>(grid, "partner: consumer stream")) return 1;
    if (run<1, 1, 1>(grid, "partner: VOP2 (lshl/lshr/xor/add/or)")) return 1;
    if (run<5, 1, 1>(grid, "partner: consumer stream")) return 1;
  }
  return 0;
}
