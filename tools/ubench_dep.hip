// tools/ubench_dep.hip -- dependent-issue latency of the MD5 step's instructions on gfx950.
// One wave; each loop trip is one asm statement, 8-byte aligned, of 8-byte instructions only
// (VOP3 encodings), so the numbers carry no misalignment penalty, and 2,048 instructions long,
// so the loop's taken branch (tens of cycles: a 32-instruction trip measured 5.0 cycles per
// instruction for anything) is amortised away.  Prints cycles per
// instruction (s_memtime) for independent streams, dependent chains of one opcode, the MD5
// step (bitop3 -> add3 -> alignbit -> add, each reading the previous result) and two MD5
// chains interleaved.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_dep tools/ubench_dep.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define X4(s) s s s s
#define KERNEL(NAME, NI, BODY)                                                                \
  __global__ void NAME(uint32_t* out, uint64_t* cyc, int iters) {                             \
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, \
             r6 = r0 + 6, r7 = r0 + 7;                                                        \
    const uint32_t a = threadIdx.x * 3u, b = threadIdx.x * 5u + 7u, c = 9u;                   \
    uint64_t t0, t1;                                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");                \
    for (int i = 0; i < iters; ++i)                                                           \
      asm volatile(".p2align 3\n\t" X4(X4(X4(X4(BODY))))                                      \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6),    \
                     "+v"(r7)                                                                 \
                   : "v"(a), "v"(b), "v"(c));                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");                \
    out[threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;                                 \
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = 256ull * (NI); }                        \
  }

// independent: 8 destinations, no instruction reads an earlier one's result
#define IND8(op, tail)                                                                        \
  op " %0, " tail "\n\t" op " %1, " tail "\n\t" op " %2, " tail "\n\t" op " %3, " tail "\n\t" \
  op " %4, " tail "\n\t" op " %5, " tail "\n\t" op " %6, " tail "\n\t" op " %7, " tail "\n\t"
// dependent: every instruction reads the previous one's result
#define DEP8(op, tail) X4(op " %0, " tail "\n\t" op " %0, " tail "\n\t")
KERNEL(k_ind_add, 8, IND8("v_add_u32_e64", "%8, %9"))
KERNEL(k_ind_alignbit, 8, IND8("v_alignbit_b32", "%8, %9, %10"))
KERNEL(k_ind_mix, 8, "v_bitop3_b32 %0, %8, %9, %10 bitop3:0xca\n\tv_add3_u32 %1, %8, %9, %10\n\t"
                     "v_alignbit_b32 %2, %8, %8, 25\n\tv_add_u32_e64 %3, %8, %9\n\t"
                     "v_bitop3_b32 %4, %8, %9, %10 bitop3:0xca\n\tv_add3_u32 %5, %8, %9, %10\n\t"
                     "v_alignbit_b32 %6, %8, %8, 25\n\tv_add_u32_e64 %7, %8, %9\n\t")
KERNEL(k_dep_add, 8, DEP8("v_add_u32_e64", "%0, %8"))
KERNEL(k_dep_alignbit, 8, DEP8("v_alignbit_b32", "%0, %0, 7"))
KERNEL(k_dep_bitop3, 8, DEP8("v_bitop3_b32", "%0, %8, %9 bitop3:0xca"))
KERNEL(k_dep_add3, 8, DEP8("v_add3_u32", "%0, %8, %9"))
// MD5 step as md5_block_streamed runs it: f = F(b,c,d); t = a + f + mk; t = rotl(t); a = b + t
#define MD5STEP(A, B, C, D)                                                                   \
  "v_bitop3_b32 %6, " B ", " C ", " D " bitop3:0xca\n\tv_add3_u32 %7, " A ", %6, %8\n\t"      \
  "v_alignbit_b32 %7, %7, %7, 25\n\tv_add_u32_e64 " A ", " B ", %7\n\t"
KERNEL(k_md5_one, 8, MD5STEP("%0", "%1", "%2", "%3") MD5STEP("%3", "%0", "%1", "%2"))
// two independent MD5 chains, instruction by instruction interleaved: chain 1 on %0-%3 with
// temporaries %8/%9, chain 2 on %4-%7 with %10/%11 (each rotating its names like the first)
#define MD5STEP2(A, B, C, D, A2, B2, C2, D2)                                                  \
  "v_bitop3_b32 %8, " B ", " C ", " D " bitop3:0xca\n\t"                                      \
  "v_bitop3_b32 %10, " B2 ", " C2 ", " D2 " bitop3:0xca\n\t"                                  \
  "v_add3_u32 %9, " A ", %8, %12\n\tv_add3_u32 %11, " A2 ", %10, %12\n\t"                     \
  "v_alignbit_b32 %9, %9, %9, 25\n\tv_alignbit_b32 %11, %11, %11, 25\n\t"                     \
  "v_add_u32_e64 " A ", " B ", %9\n\tv_add_u32_e64 " A2 ", " B2 ", %11\n\t"
__global__ void k_md5_two(uint32_t* out, uint64_t* cyc, int iters) {
  uint32_t r[12];
  for (int k = 0; k < 12; ++k) r[k] = threadIdx.x + k;
  const uint32_t mk = threadIdx.x * 3u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i)
    asm volatile(".p2align 3\n\t" X4(X4(X4(X4(
                     MD5STEP2("%0", "%1", "%2", "%3", "%4", "%5", "%6", "%7")
                     MD5STEP2("%3", "%0", "%1", "%2", "%7", "%4", "%5", "%6")))))
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11])
                 : "v"(mk));
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  uint32_t x = 0;
  for (int k = 0; k < 12; ++k) x ^= r[k];
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = 256ull * 16; }
}

int main() {
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMalloc(&cyc, 16));
  const int iters = 256;
  struct { const char* n; void (*k)(uint32_t*, uint64_t*, int); } T[] = {
      {"IND v_add_u32_e64", k_ind_add}, {"IND v_alignbit_b32", k_ind_alignbit},
      {"IND md5 mix (no dependences)", k_ind_mix},
      {"DEP v_add_u32_e64", k_dep_add}, {"DEP v_alignbit_b32", k_dep_alignbit},
      {"DEP v_bitop3_b32", k_dep_bitop3}, {"DEP v_add3_u32", k_dep_add3},
      {"MD5 step, one chain", k_md5_one}, {"MD5 step, two chains interleaved", k_md5_two}};
  for (auto& t : T) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(t.k, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      CHECK(hipDeviceSynchronize());
    }
    uint64_t h[2];
    CHECK(hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost));
    printf("%-34s cycles/instr = %.3f\n", t.n, double(h[0]) / (double(iters) * double(h[1])));
  }
  return 0;
}
