// tools/ubench_round.hip -- cycles per lane-pair SHA-256 round for different instruction
// orders (one wave alone on its SIMD, like the pair kernel's consumer).  Orders keep the DPP
// read-after-VALU-write distance (>= 2 instructions between t and the a-half DPP add).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_round tools/ubench_round.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define I_R1(a) "v_alignbit_b32 %[q1], %[" #a "], %[" #a "], %[h1]\n\t"
#define I_R2(a) "v_alignbit_b32 %[q2], %[" #a "], %[" #a "], %[h2]\n\t"
#define I_R3(a) "v_alignbit_b32 %[q3], %[" #a "], %[" #a "], %[h3]\n\t"
#define I_SEL(a, b) "v_bitop3_b32 %[q4], %[" #a "], %[" #b "], %[m] bitop3:0xd2\n\t"
#define I_S "v_bitop3_b32 %[q1], %[q1], %[q2], %[q3] bitop3:0x96\n\t"
#define I_S5 "v_bitop3_b32 %[q5], %[q1], %[q2], %[q3] bitop3:0x96\n\t"
#define I_F(b, c) "v_bfi_b32 %[q2], %[q4], %[" #b "], %[" #c "]\n\t"
#define I_F6(b, c) "v_bfi_b32 %[q6], %[q4], %[" #b "], %[" #c "]\n\t"
#define I_T(x) "v_add3_u32 %[q3], %[" #x "], %[q1], %[q2]\n\t"
#define I_T56(x) "v_add3_u32 %[q3], %[" #x "], %[q5], %[q6]\n\t"
#define I_XN(c, xn, wn) "v_add_u32_dpp %[" #xn "], %[" #c "], %[" #wn "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t"
#define I_E(d) "v_add_u32_dpp %[" #d "], %[" #d "], %[q3] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
#define I_A(d) "v_add_u32_dpp %[" #d "], %[q3], %[q3] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

// V0: current kernel order
#define V0(a, b, c, d, x, xn, wn) I_R1(a) I_R2(a) I_R3(a) I_SEL(a, b) I_S I_F(b, c) I_T(x) I_XN(c, xn, wn) I_E(d) I_A(d)
// V1: sel between rotations, F before S
#define V1(a, b, c, d, x, xn, wn) I_R1(a) I_R2(a) I_SEL(a, b) I_R3(a) I_F6(b, c) I_S5 I_T56(x) I_XN(c, xn, wn) I_E(d) I_A(d)
// V2: sel first
#define V2(a, b, c, d, x, xn, wn) I_SEL(a, b) I_R1(a) I_R2(a) I_R3(a) I_F6(b, c) I_S5 I_T56(x) I_XN(c, xn, wn) I_E(d) I_A(d)
// V3: e-add before xn
#define V3(a, b, c, d, x, xn, wn) I_R1(a) I_R2(a) I_R3(a) I_SEL(a, b) I_S I_F(b, c) I_T(x) I_E(d) I_XN(c, xn, wn) I_A(d)

// VA: DPP adds replaced by plain VOP2 adds (wrong math; timing only)
#define I_XNP(c, xn, wn) "v_add_u32_e32 %[" #xn "], %[" #c "], %[" #wn "]\n\t"
#define I_EP(d) "v_add_u32_e32 %[" #d "], %[" #d "], %[q3]\n\t"
#define I_AP(d) "v_add_u32_e32 %[" #d "], %[q3], %[" #d "]\n\t"
#define VA(a, b, c, d, x, xn, wn) I_R1(a) I_R2(a) I_R3(a) I_SEL(a, b) I_S I_F(b, c) I_T(x) I_XNP(c, xn, wn) I_EP(d) I_AP(d)
// VB: same opcodes, no dependencies between instructions of a round (pure issue rate)
#define VB(a, b, c, d, x, xn, wn) \
  "v_alignbit_b32 %[q1], %[" #a "], %[" #a "], %[h1]\n\t" "v_alignbit_b32 %[q2], %[" #b "], %[" #b "], %[h2]\n\t" \
  "v_alignbit_b32 %[q3], %[" #c "], %[" #c "], %[h3]\n\t" "v_bitop3_b32 %[q4], %[" #a "], %[" #b "], %[m] bitop3:0xd2\n\t" \
  "v_bitop3_b32 %[q5], %[" #b "], %[" #c "], %[" #x "] bitop3:0x96\n\t" "v_bfi_b32 %[q6], %[" #c "], %[" #b "], %[" #a "]\n\t" \
  "v_add3_u32 %[q1], %[" #x "], %[" #a "], %[" #b "]\n\t" "v_add_u32_dpp %[q2], %[" #c "], %[" #wn "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t" \
  "v_add_u32_dpp %[q3], %[" #a "], %[" #b "] row_shl:4 row_mask:0xf bank_mask:0x5\n\t" "v_add_u32_dpp %[q4], %[" #b "], %[" #c "] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

#define KERNEL(NAME, V)                                                                      \
  __global__ void NAME(uint32_t* out, uint64_t* cyc, int iters) {                            \
    const uint32_t lane = threadIdx.x;                                                       \
    const bool ah = (lane >> 2) & 1;                                                         \
    uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;    \
    uint32_t xa = 0, xb = 0, q1, q2, q3, q4, q5, q6;                                         \
    const uint32_t w1 = lane ^ 0x1234, w2 = lane ^ 0x5678, w3 = lane ^ 0x9abc, w4 = lane;    \
    const uint32_t sh1 = ah ? 2 : 6, sh2 = ah ? 13 : 11, sh3 = ah ? 22 : 25;                 \
    const uint32_t msk = ah ? ~0u : 0u;                                                      \
    uint64_t t0;                                                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");               \
    for (int i = 0; i < iters; ++i) {                                                        \
      asm volatile(V(s0, s1, s2, s3, xa, xb, w1) V(s3, s0, s1, s2, xb, xa, w2)               \
                   V(s2, s3, s0, s1, xa, xb, w3) V(s1, s2, s3, s0, xb, xa, w4)               \
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3),             \
                     [xa] "+v"(xa), [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2),           \
                     [q3] "=&v"(q3), [q4] "=&v"(q4), [q5] "=&v"(q5), [q6] "=&v"(q6)           \
                   : [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4), [h1] "v"(sh1), \
                     [h2] "v"(sh2), [h3] "v"(sh3), [m] "v"(msk));                            \
    }                                                                                        \
    uint64_t t1;                                                                             \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");               \
    out[lane] = s0 ^ s1 ^ s2 ^ s3;                                                           \
    if (lane == 0) *cyc = t1 - t0;                                                           \
  }

KERNEL(k_v0, V0)
KERNEL(k_v1, V1)
KERNEL(k_v2, V2)
KERNEL(k_v3, V3)
KERNEL(k_va, VA)
KERNEL(k_vb, VB)

int main() {
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 256));
  CHECK(hipMalloc(&cyc, 8));
  const int iters = 4096;
  struct { const char* n; void (*k)(uint32_t*, uint64_t*, int); } T[] = {
      {"V0 r1 r2 r3 sel S F t xn e a", k_v0}, {"V1 r1 r2 sel r3 F S t xn e a", k_v1},
      {"V2 sel r1 r2 r3 F S t xn e a", k_v2}, {"V3 r1 r2 r3 sel S F t e xn a", k_v3},
      {"VA no-DPP adds", k_va}, {"VB independent (issue rate)", k_vb}};
  for (auto& t : T) {
    uint64_t c = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(t.k, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      CHECK(hipDeviceSynchronize());
    }
    CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    printf("%-32s cycles/round=%.2f  cycles/instr=%.3f\n", t.n, double(c) / (iters * 4.0),
           double(c) / (iters * 40.0));
  }
  return 0;
}
