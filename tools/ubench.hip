// tools/ubench.hip -- microbenchmarks that pin down the VALU issue model the SHA-256
// kernels are designed against (DESIGN.md "Issue model").  Standalone HIP program:
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip && tools/ubench
// Every kernel loops 256 times over a 128-instruction body (32 x a 4-instruction asm group,
// small enough to stay in the instruction cache)
// and reports shader cycles per instruction per wave from s_memtime, plus the in-kernel
// clock from s_memrealtime (100 MHz).  Workgroups of 64 / 256 / 512 / 1024 threads put
// 1 / 1 / 2 / 4 waves on each SIMD of one CU (dispatch order 0->2->1->3).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int N = 2048 * 16;  // 256 trips of a 128-instruction body (i-cache resident)

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}
__device__ __forceinline__ uint64_t rstamp() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

#define UB_KERNEL(NAME, ASM)                                                              \
  __global__ void NAME(uint32_t* out, uint64_t* cyc) {                                    \
    uint32_t a = threadIdx.x, b = a * 3u + 1u, c = a * 7u + 2u, d = a * 11u + 3u;         \
    float fa = float(a), fb = 1.0001f, fc = 0.5f;                                         \
    const uint64_t r0 = rstamp();                                                         \
    const uint64_t t0 = stamp();                                                          \
    _Pragma("unroll 1") for (int o = 0; o < N / 128; ++o) {                               \
      _Pragma("unroll") for (int i = 0; i < 32; ++i) {                                    \
        asm volatile(ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(fa) : "v"(fb), "v"(fc)); \
      }                                                                                   \
    }                                                                                     \
    const uint64_t t1 = stamp();                                                          \
    const uint64_t r1 = rstamp();                                                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ __float_as_uint(fa);     \
    if (threadIdx.x % 64 == 0) {                                                          \
      cyc[2 * (threadIdx.x / 64)] = t1 - t0;                                              \
      cyc[2 * (threadIdx.x / 64) + 1] = r1 - r0;                                          \
    }                                                                                     \
  }

// dependent chains (each instruction reads the previous one's result)
UB_KERNEL(k_alignbit_dep, "v_alignbit_b32 %0, %0, %0, 7\n\tv_alignbit_b32 %0, %0, %0, 7\n\tv_alignbit_b32 %0, %0, %0, 7\n\tv_alignbit_b32 %0, %0, %0, 7")
UB_KERNEL(k_add3_dep, "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2")
UB_KERNEL(k_add_e32_dep, "v_add_u32_e32 %0, %1, %0\n\tv_add_u32_e32 %0, %1, %0\n\tv_add_u32_e32 %0, %1, %0\n\tv_add_u32_e32 %0, %1, %0")
UB_KERNEL(k_fma_dep, "v_fma_f32 %4, %4, %5, %6\n\tv_fma_f32 %4, %4, %5, %6\n\tv_fma_f32 %4, %4, %5, %6\n\tv_fma_f32 %4, %4, %5, %6")
// independent (4 chains interleaved)
UB_KERNEL(k_alignbit_ind, "v_alignbit_b32 %0, %0, %0, 7\n\tv_alignbit_b32 %1, %1, %1, 7\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_alignbit_b32 %3, %3, %3, 7")
UB_KERNEL(k_bitop3_ind, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %3, %0 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %0, %1 bitop3:0x96")
UB_KERNEL(k_add3_ind, "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %1, %1, %2, %3\n\tv_add3_u32 %2, %2, %3, %0\n\tv_add3_u32 %3, %3, %0, %1")
UB_KERNEL(k_add_e32_ind, "v_add_u32_e32 %0, %1, %0\n\tv_add_u32_e32 %1, %2, %1\n\tv_add_u32_e32 %2, %3, %2\n\tv_add_u32_e32 %3, %0, %3")
UB_KERNEL(k_xor_e32_ind, "v_xor_b32_e32 %0, %1, %0\n\tv_xor_b32_e32 %1, %2, %1\n\tv_xor_b32_e32 %2, %3, %2\n\tv_xor_b32_e32 %3, %0, %3")
UB_KERNEL(k_add_e64_ind, "v_add_u32_e64 %0, %1, %0\n\tv_add_u32_e64 %1, %2, %1\n\tv_add_u32_e64 %2, %3, %2\n\tv_add_u32_e64 %3, %0, %3")
UB_KERNEL(k_perm_ind, "v_perm_b32 %0, %1, %0, %2\n\tv_perm_b32 %1, %2, %1, %3\n\tv_perm_b32 %2, %3, %2, %0\n\tv_perm_b32 %3, %0, %3, %1")
UB_KERNEL(k_bfi_ind, "v_bfi_b32 %0, %1, %0, %2\n\tv_bfi_b32 %1, %2, %1, %3\n\tv_bfi_b32 %2, %3, %2, %0\n\tv_bfi_b32 %3, %0, %3, %1")
UB_KERNEL(k_fma_ind, "v_fma_f32 %4, %4, %5, %6\n\tv_fma_f32 %0, %0, %5, %6\n\tv_fma_f32 %1, %1, %5, %6\n\tv_fma_f32 %2, %2, %5, %6")
UB_KERNEL(k_mix_ind, "v_alignbit_b32 %0, %0, %0, 7\n\tv_add_u32_e32 %1, %2, %1\n\tv_bitop3_b32 %2, %2, %3, %0 bitop3:0x96\n\tv_xor_b32_e32 %3, %0, %3")
// DPP cross-lane (row_shr:1) add, used by the lane-pair formulation
UB_KERNEL(k_add_dpp_ind, "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\tv_add_u32_dpp %1, %2, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1")

typedef void (*KFn)(uint32_t*, uint64_t*);

int run(const char* name, KFn k, int threads) {
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 4096 * 4));
  CHECK(hipMalloc(&cyc, 64 * 8));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, out, cyc);
    CHECK(hipDeviceSynchronize());
  }
  uint64_t h[64];
  const int waves = threads / 64;
  CHECK(hipMemcpy(h, cyc, 2 * waves * 8, hipMemcpyDeviceToHost));
  double mn = 1e30, mx = 0, ghz = 0;
  for (int w = 0; w < waves; ++w) {
    const double cpi = double(h[2 * w]) / N;
    mn = cpi < mn ? cpi : mn;
    mx = cpi > mx ? cpi : mx;
    ghz += double(h[2 * w]) / (double(h[2 * w + 1]) * 10.0) / waves;
  }
  const int per_simd = threads <= 256 ? 1 : threads / 256;
  // SIMD throughput: instructions retired per SIMD per cycle, from the slowest wave
  printf("%-16s waves/SIMD=%d  cyc/instr/wave min=%.2f max=%.2f  SIMD cyc/instr=%.2f  clk=%.2f GHz\n",
         name, per_simd, mn, mx, mx / per_simd, ghz);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

int main() {
  struct { const char* n; KFn k; } T[] = {
      {"alignbit dep", k_alignbit_dep}, {"add3 dep", k_add3_dep}, {"add_e32 dep", k_add_e32_dep},
      {"fma dep", k_fma_dep}, {"alignbit ind", k_alignbit_ind}, {"bitop3 ind", k_bitop3_ind},
      {"add3 ind", k_add3_ind}, {"add_e32 ind", k_add_e32_ind}, {"xor_e32 ind", k_xor_e32_ind},
      {"add_e64 ind", k_add_e64_ind}, {"perm ind", k_perm_ind}, {"bfi ind", k_bfi_ind},
      {"fma ind", k_fma_ind}, {"mix ind", k_mix_ind}, {"add_dpp+nop", k_add_dpp_ind}};
  int rc = 0;
  for (auto& t : T)
    for (int th : {64, 512, 1024}) rc |= run(t.n, t.k, th);
  return rc;
}
