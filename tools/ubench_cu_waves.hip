// tools/ubench_cu_waves.hip -- does a wave's issue rate depend on how many OTHER SIMDs of its
// CU are busy?  One workgroup per CU (grid <= 256), W waves per workgroup (one per SIMD for
// W <= 4); waves whose bit is set in `active` run a long straight-line stream of quad-kernel
// rounds (9 VALU each, 64 rounds per asm statement), the others exit at once.  Each active
// wave reports its own cycles per instruction.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_cu_waves tools/ubench_cu_waves.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
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

template <int W>
__global__ __launch_bounds__(64 * W) void stream(uint32_t* out, uint32_t* cyc, int iters,
                                                 uint32_t active) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!((active >> wave) & 1)) return;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
  uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
  const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i)
    asm volatile(Q64
                 : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                   [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                 : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 64 * W + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
  if (lane == 0) cyc[blockIdx.x * W + wave] = uint32_t(t1 - t0);
}

template <int W>
int run(int grid, uint32_t active, const char* label) {
  const int iters = 400;
  uint32_t *out, *cyc;
  CHECK(hipMalloc(&out, size_t(grid) * 64 * W * 4));
  CHECK(hipMalloc(&cyc, size_t(grid) * W * 4));
  CHECK(hipMemset(cyc, 0, size_t(grid) * W * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream<W>, dim3(grid), dim3(64 * W), 0, 0, out, cyc, iters, active);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> h(size_t(grid) * W);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 4, hipMemcpyDeviceToHost));
  double sum = 0, mx = 0;
  int cnt = 0;
  for (uint32_t c : h)
    if (c) {
      const double cpi = double(c) / (double(iters) * 64 * 9);
      sum += cpi;
      mx = std::max(mx, cpi);
      ++cnt;
    }
  printf("%-34s W=%d grid=%3d active=0x%02x: waves %4d  cycles/instr mean %.3f max %.3f\n", label,
         W, grid, active, cnt, sum / cnt, mx);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

// Wave 0 runs the round stream; wave 1 is a "pacer" of kind P that runs until wave 0 sets an
// LDS flag: 0 exits at once, 1 VALU adds (different code), 2 s_nop loop, 3 s_sleep loop,
// 4 LDS polling only, 5 SALU loop, 6 v_mov loop (1 VALU per flag poll of 16).
template <int P>
__global__ __launch_bounds__(128) void paced(uint32_t* out, uint32_t* cyc, int iters) {
  __shared__ volatile uint32_t flag;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) flag = 0;
  __syncthreads();
  if (wave == 1) {
    if (P == 0) return;
    uint32_t v = lane, u = lane * 7;
    while (flag == 0) {
      if (P == 1) {
        for (int k = 0; k < 16; ++k) asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %1, %1, %0" : "+v"(v), "+v"(u));
      } else if (P == 2) {
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
      } else if (P == 3) {
        __builtin_amdgcn_s_sleep(2);
      } else if (P == 5) {
        uint32_t sc = 0;
        for (int k = 0; k < 16; ++k) asm volatile("s_add_u32 %0, %0, 1" : "+s"(sc));
      } else if (P == 6) {
        asm volatile("v_mov_b32 %0, %1\n\ts_nop 7\n\ts_nop 7" : "=v"(v) : "v"(u));
      }
    }
    out[gridDim.x * 64 + blockIdx.x * 64 + lane] = v ^ u;
    return;
  }
  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
  uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
  const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i)
    asm volatile(Q64
                 : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                   [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                 : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) flag = 1;
  out[blockIdx.x * 64 + lane] = s0 ^ s1 ^ s2 ^ s3;
  if (lane == 0) cyc[blockIdx.x] = uint32_t(t1 - t0);
}

template <int P>
int run_paced(int grid, const char* label) {
  const int iters = 400;
  uint32_t *out, *cyc;
  CHECK(hipMalloc(&out, size_t(grid) * 128 * 4));
  CHECK(hipMalloc(&cyc, size_t(grid) * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(paced<P>, dim3(grid), dim3(128), 0, 0, out, cyc, iters);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> h(grid);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 4, hipMemcpyDeviceToHost));
  double sum = 0, mx = 0;
  for (uint32_t c : h) {
    const double cpi = double(c) / (double(iters) * 64 * 9);
    sum += cpi;
    mx = std::max(mx, cpi);
  }
  printf("pacer %-28s grid=%3d: main wave cycles/instr mean %.3f max %.3f\n", label, grid,
         sum / grid, mx);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

// Two waves, each running a round stream; wave 1 starts D cycles late (s_sleep units of 64
// cycles) and runs either the SAME code (kSame) or a separate copy of it (different addresses).
template <int D, bool kSame>
__global__ __launch_bounds__(128) void pair2(uint32_t* out, uint32_t* cyc, int iters) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
  uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
  const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
  if (wave == 1)
    for (int k = 0; k < D; ++k) __builtin_amdgcn_s_sleep(1);
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (kSame || wave == 0) {
    for (int i = 0; i < iters; ++i)
      asm volatile(Q64
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                     [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                   : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
  } else {
    for (int i = 0; i < iters; ++i)
      asm volatile("s_nop 0\n\t" Q64
                   : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                     [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                   : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 128 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
  if (lane == 0) cyc[blockIdx.x * 2 + wave] = uint32_t(t1 - t0);
}

template <int D, bool kSame>
int run_pair2(const char* label) {
  const int iters = 400, grid = 64;
  uint32_t *out, *cyc;
  CHECK(hipMalloc(&out, size_t(grid) * 128 * 4));
  CHECK(hipMalloc(&cyc, size_t(grid) * 2 * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((pair2<D, kSame>), dim3(grid), dim3(128), 0, 0, out, cyc, iters);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> h(grid * 2);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 4, hipMemcpyDeviceToHost));
  double s0 = 0, s1 = 0;
  for (int b = 0; b < grid; ++b) {
    s0 += double(h[2 * b]) / (double(iters) * 64 * 9);
    s1 += double(h[2 * b + 1]) / (double(iters) * 64 * 9);
  }
  printf("pair2 %-26s delay=%4d x64cyc: wave0 %.3f  wave1 %.3f cycles/instr\n", label, D,
         s0 / grid, s1 / grid);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

// Same-code pair with a workgroup barrier per iteration (B = 1), plus 8 ds_read_b128 and an
// lgkmcnt(0) wait before it (B = 2): the consumer loop's synchronisation, without producers.
template <int B>
__global__ __launch_bounds__(128) void pair_sync(uint32_t* out, uint32_t* cyc, int iters) {
  __shared__ uint4 lds[512];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  lds[threadIdx.x] = make_uint4(lane, lane, lane, lane);
  __syncthreads();
  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
  uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
  uint32_t w = lane ^ 0x1234;
  const uint32_t sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i) {
    if (B == 2) {
      uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4 v = lds[(lane & 3) + 4 * k + 64 * (i & 1)];
        acc.x ^= v.x; acc.y ^= v.y;
      }
      w ^= acc.x ^ acc.y;
    }
    asm volatile(Q64
                 : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                   [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                 : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
    __syncthreads();
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 128 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
  if (lane == 0) cyc[blockIdx.x * 2 + wave] = uint32_t(t1 - t0);
}

template <int B>
int run_sync(const char* label) {
  const int iters = 400, grid = 64;
  uint32_t *out, *cyc;
  CHECK(hipMalloc(&out, size_t(grid) * 128 * 4));
  CHECK(hipMalloc(&cyc, size_t(grid) * 2 * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(pair_sync<B>, dim3(grid), dim3(128), 0, 0, out, cyc, iters);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> h(grid * 2);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 4, hipMemcpyDeviceToHost));
  double s0 = 0, s1 = 0;
  for (int b = 0; b < grid; ++b) {
    s0 += double(h[2 * b]) / (double(iters) * 64 * 9);
    s1 += double(h[2 * b + 1]) / (double(iters) * 64 * 9);
  }
  printf("sync %-34s: wave0 %.3f  wave1 %.3f cycles/instr (incl. sync)\n", label, s0 / grid, s1 / grid);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

// Same-code pair with a barrier per iteration; after each barrier wave 1 waits D extra cycles
// (s_nop D-1, D in 1..8; D = 9..16: two s_nops) before its rounds: does a phase offset
// restore the paired issue rate?
template <int D>
__global__ __launch_bounds__(128) void pair_phase(uint32_t* out, uint32_t* cyc, int iters) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4;
  uint32_t xa = 0, xb = 0, q1, q2, q3, q4;
  const uint32_t w = lane ^ 0x1234, sh = 6 + (lane & 3), msk = (lane & 4) ? ~0u : 0u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i) {
    if (wave == 1) {
      if (D >= 1 && D <= 8) asm volatile("s_nop %0" ::"i"(D >= 1 && D <= 8 ? D - 1 : 0));
      if (D > 8) asm volatile("s_nop 7\n\ts_nop %0" ::"i"(D > 8 ? D - 9 : 0));
    }
    asm volatile(Q64
                 : [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [xa] "+v"(xa),
                   [xb] "+v"(xb), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4)
                 : [w] "v"(w), [h1] "v"(sh), [m] "v"(msk));
    __syncthreads();
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 128 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
  if (lane == 0) cyc[blockIdx.x * 2 + wave] = uint32_t(t1 - t0);
}

template <int D>
int run_phase() {
  const int iters = 400, grid = 64;
  uint32_t *out, *cyc;
  CHECK(hipMalloc(&out, size_t(grid) * 128 * 4));
  CHECK(hipMalloc(&cyc, size_t(grid) * 2 * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(pair_phase<D>, dim3(grid), dim3(128), 0, 0, out, cyc, iters);
    CHECK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> h(grid * 2);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 4, hipMemcpyDeviceToHost));
  double s0 = 0, s1 = 0;
  for (int b = 0; b < grid; ++b) {
    s0 += double(h[2 * b]) / (double(iters) * 64 * 9);
    s1 += double(h[2 * b + 1]) / (double(iters) * 64 * 9);
  }
  printf("phase wave1 +%2d nop-cycles after barrier: wave0 %.3f  wave1 %.3f cycles/instr\n", D,
         s0 / grid, s1 / grid);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

int main() {
  for (int grid : {1, 64, 256}) {
    run<1>(grid, 0x1, "1 wave/CU");
    run<2>(grid, 0x3, "2 busy SIMDs");
    run<3>(grid, 0x7, "3 busy SIMDs");
    run<4>(grid, 0xf, "4 busy SIMDs");
    run<4>(grid, 0x7, "3 busy of a 4-wave WG");
    run<8>(grid, 0xff, "8 waves (2 per SIMD)");
  }
  run_phase<0>(); run_phase<1>(); run_phase<2>(); run_phase<3>(); run_phase<4>();
  run_phase<5>(); run_phase<6>(); run_phase<7>(); run_phase<8>(); run_phase<10>();
  run_phase<12>(); run_phase<14>(); run_phase<16>();
  run_sync<1>("same code + s_barrier/iter");
  run_sync<2>("same code + 8 ds_read + barrier/iter");
  run_pair2<0, true>("same code");
  run_pair2<1, true>("same code");
  run_pair2<4, true>("same code");
  run_pair2<32, true>("same code");
  run_pair2<0, false>("separate code copies");
  run_pair2<4, false>("separate code copies");
  for (int grid : {1}) {
    run_paced<0>(grid, "none (exits)");
    run_paced<1>(grid, "VALU add/xor loop");
    run_paced<2>(grid, "s_nop loop");
    run_paced<3>(grid, "s_sleep loop");
    run_paced<4>(grid, "LDS flag poll only");
    run_paced<5>(grid, "SALU loop");
    run_paced<6>(grid, "1 v_mov per 2 s_nop 7");
  }
  return 0;
}
