// tools/ubench_issue.hip -- lone-wave issue cost per opcode with NO compiler padding: each
// loop trip is ONE asm statement of 32 independent instructions of one opcode (the compiler
// pads between asm statements, which contaminated the first ubench's absolute numbers).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define X4(s) s s s s
#define X32(s) X4(X4(s)) X4(s) X4(s)
// 8 independent destinations rotate through %0..%7, sources %8..%10
#define OPS8(op, tail) \
  op " %0, " tail "\n\t" op " %1, " tail "\n\t" op " %2, " tail "\n\t" op " %3, " tail "\n\t" \
  op " %4, " tail "\n\t" op " %5, " tail "\n\t" op " %6, " tail "\n\t" op " %7, " tail "\n\t"

#define KERNEL(NAME, BODY)                                                                    \
  __global__ void NAME(uint32_t* out, uint64_t* cyc, int iters) {                             \
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, \
             r6 = r0 + 6, r7 = r0 + 7;                                                        \
    const uint32_t a = threadIdx.x * 3u, b = threadIdx.x * 5u + 7u, c = 9u;                   \
    uint64_t t0, t1;                                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");                \
    for (int i = 0; i < iters; ++i)                                                           \
      asm volatile(BODY BODY BODY BODY                                                        \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6),    \
                     "+v"(r7)                                                                 \
                   : "v"(a), "v"(b), "v"(c));                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");                \
    out[threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;                                 \
    if (threadIdx.x == 0) *cyc = t1 - t0;                                                     \
  }

KERNEL(k_alignbit, OPS8("v_alignbit_b32", "%8, %9, %10"))
KERNEL(k_bitop3, OPS8("v_bitop3_b32", "%8, %9, %10 bitop3:0x96"))
KERNEL(k_add3, OPS8("v_add3_u32", "%8, %9, %10"))
KERNEL(k_bfi, OPS8("v_bfi_b32", "%8, %9, %10"))
KERNEL(k_perm, OPS8("v_perm_b32", "%8, %9, %10"))
KERNEL(k_add_e32, OPS8("v_add_u32_e32", "%8, %9"))
KERNEL(k_xor_e32, OPS8("v_xor_b32_e32", "%8, %9"))
KERNEL(k_add_e64, OPS8("v_add_u32_e64", "%8, %9"))
KERNEL(k_add_dpp, OPS8("v_add_u32_dpp", "%8, %9 row_shl:4 row_mask:0xf bank_mask:0x5"))
KERNEL(k_mov_dpp, OPS8("v_mov_b32_dpp", "%8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"))
KERNEL(k_lshl_add, OPS8("v_lshl_add_u32", "%8, 3, %10"))
KERNEL(k_mix_round, "v_alignbit_b32 %0, %8, %8, %9\n\tv_alignbit_b32 %1, %8, %8, %10\n\t"
                    "v_alignbit_b32 %2, %8, %8, %9\n\tv_bitop3_b32 %3, %8, %9, %10 bitop3:0xd2\n\t"
                    "v_bitop3_b32 %4, %9, %10, %8 bitop3:0x96\n\tv_bfi_b32 %5, %8, %9, %10\n\t"
                    "v_add3_u32 %6, %8, %9, %10\n\tv_add_u32_dpp %7, %8, %9 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t")

// dependent chains: every instruction reads the previous one's result (%0)
#define DEP8(op, tail) op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" \
                       op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t"
KERNEL(k_dep_add_e32, DEP8("v_add_u32_e32", "%8, %0"))
KERNEL(k_dep_add3, DEP8("v_add3_u32", "%0, %8, %9"))
KERNEL(k_dep_alignbit, DEP8("v_alignbit_b32", "%0, %0, 7"))
KERNEL(k_dep_bitop3, DEP8("v_bitop3_b32", "%0, %8, %9 bitop3:0xca"))
// MD5-like step: bitop3 -> add3 -> alignbit -> add, each dependent (x2 per 8)
KERNEL(k_dep_md5, "v_bitop3_b32 %1, %0, %8, %9 bitop3:0xca\n\tv_add3_u32 %1, %1, %10, %9\n\t"
                  "v_alignbit_b32 %1, %1, %1, 25\n\tv_add_u32_e32 %0, %0, %1\n\t"
                  "v_bitop3_b32 %1, %0, %8, %9 bitop3:0xca\n\tv_add3_u32 %1, %1, %10, %9\n\t"
                  "v_alignbit_b32 %1, %1, %1, 25\n\tv_add_u32_e32 %0, %0, %1\n\t")
// same with VOP2 add instead of add3 (a+K+M precomputed off the chain)
KERNEL(k_dep_md5b, "v_bitop3_b32 %1, %0, %8, %9 bitop3:0xca\n\tv_add_u32_e32 %1, %10, %1\n\t"
                   "v_alignbit_b32 %1, %1, %1, 25\n\tv_add_u32_e32 %0, %0, %1\n\t"
                   "v_bitop3_b32 %1, %0, %8, %9 bitop3:0xca\n\tv_add_u32_e32 %1, %10, %1\n\t"
                   "v_alignbit_b32 %1, %1, %1, 25\n\tv_add_u32_e32 %0, %0, %1\n\t")

int main() {
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMalloc(&cyc, 8));
  const int iters = 2048;
  struct { const char* n; void (*k)(uint32_t*, uint64_t*, int); } T[] = {
      {"v_alignbit_b32", k_alignbit}, {"v_bitop3_b32", k_bitop3}, {"v_add3_u32", k_add3},
      {"v_bfi_b32", k_bfi}, {"v_perm_b32", k_perm}, {"v_add_u32_e32", k_add_e32},
      {"v_xor_b32_e32", k_xor_e32}, {"v_add_u32_e64", k_add_e64}, {"v_add_u32_dpp", k_add_dpp},
      {"v_mov_b32_dpp", k_mov_dpp}, {"v_lshl_add_u32", k_lshl_add}, {"round mix (8)", k_mix_round},
      {"DEP v_add_u32_e32", k_dep_add_e32}, {"DEP v_add3_u32", k_dep_add3},
      {"DEP v_alignbit", k_dep_alignbit}, {"DEP v_bitop3", k_dep_bitop3},
      {"DEP md5 step (add3)", k_dep_md5}, {"DEP md5 step (add)", k_dep_md5b}};
  for (auto& t : T) {
    for (int threads : {64, 512}) {
      uint64_t c = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(t.k, dim3(1), dim3(threads), 0, 0, out, cyc, iters);
        CHECK(hipDeviceSynchronize());
      }
      CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
      printf("%-18s waves/SIMD=%d  cycles/instr (wave 0) = %.3f\n", t.n, threads == 64 ? 1 : 2,
             double(c) / (iters * 32.0));
    }
  }
  return 0;
}
