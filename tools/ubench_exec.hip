// tools/ubench_exec.hip -- does a lone wave issue faster when EXEC has fewer live lanes?
// (gfx950 SIMDs are 32 lanes wide: a wave64 VALU op takes 2 passes.  If a half-EXEC wave
// issued every 2 cycles, a chain layout confined to 32 lanes would run twice as fast.)
// Streams: 8 independent v_add3 (3-source), 8 independent v_add_u32 (2-source), and a
// dependent v_add3 chain; EXEC = 64 / 32 / 16 / 8 live lanes (low lanes), one wave per CU.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_exec tools/ubench_exec.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define X4(s) s s s s
#define OPS8(op, tail) \
  op " %0, " tail "\n\t" op " %1, " tail "\n\t" op " %2, " tail "\n\t" op " %3, " tail "\n\t" \
  op " %4, " tail "\n\t" op " %5, " tail "\n\t" op " %6, " tail "\n\t" op " %7, " tail "\n\t"
#define DEP8(op, tail) op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" \
                       op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t" op " %0, " tail "\n\t"

// 64 instructions per asm statement, statement 8-byte aligned
#define KERNEL(NAME, BODY)                                                                    \
  __global__ void NAME(uint32_t* out, uint64_t* cyc, int iters, int live) {                   \
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, \
             r6 = r0 + 6, r7 = r0 + 7;                                                        \
    const uint32_t a = threadIdx.x * 3u, b = threadIdx.x * 5u + 7u, c = 9u;                   \
    uint64_t t0 = 0, t1 = 0;                                                                  \
    if (int(threadIdx.x) < live) {                                                            \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");              \
      for (int i = 0; i < iters; ++i)                                                         \
        asm volatile(".p2align 3\n\t" X4(X4(BODY)) X4(BODY) X4(BODY) X4(BODY) X4(BODY)        \
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6),  \
                       "+v"(r7)                                                               \
                     : "v"(a), "v"(b), "v"(c));                                               \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");              \
    }                                                                                         \
    out[threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;                                 \
    if (threadIdx.x == 0) *cyc = t1 - t0;                                                     \
  }

KERNEL(k_add3, OPS8("v_add3_u32", "%8, %9, %10"))
KERNEL(k_add_e32, OPS8("v_add_u32_e32", "%8, %9"))
KERNEL(k_dep_add3, DEP8("v_add3_u32", "%0, %8, %9"))
KERNEL(k_xor_dpp, OPS8("v_xor_b32_dpp", "%8, %9 quad_perm:[1,2,0,1] row_mask:0xf bank_mask:0xf"))

int main() {
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMalloc(&cyc, 8));
  const int iters = 1024;
  const double per = 32.0 * 8;  // instructions per asm statement
  struct { const char* n; void (*k)(uint32_t*, uint64_t*, int, int); } T[] = {
      {"v_add3_u32 indep", k_add3}, {"v_add_u32_e32 indep", k_add_e32},
      {"v_add3_u32 DEP", k_dep_add3}, {"v_xor_b32_dpp indep", k_xor_dpp}};
  for (auto& t : T) {
    for (int live : {64, 32, 16, 8}) {
      uint64_t c = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(t.k, dim3(1), dim3(64), 0, 0, out, cyc, iters, live);
        CHECK(hipDeviceSynchronize());
      }
      CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
      printf("%-22s live lanes=%2d  cycles/instr = %.3f\n", t.n, live, double(c) / (iters * per));
    }
  }
  return 0;
}
