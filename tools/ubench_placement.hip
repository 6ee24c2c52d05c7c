// tools/ubench_placement.hip -- where does the dispatcher put the waves of small grids?
// Each wave records HW_ID (SIMD, CU, SH, SE) and XCC_ID while every wave spins long enough for
// the whole grid to be co-resident.  Prints, per (waves per workgroup, grid): CUs used, max
// workgroups per CU, max waves per SIMD.  Same LDS footprint per workgroup as the quad kernel.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_placement tools/ubench_placement.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int W, bool kBigVgpr>
__global__ __launch_bounds__(64 * W) void probe(uint32_t* out, long long spin) {
  __shared__ uint4 lds[2 * 2 * 16 * 8 * (W - 1 > 0 ? W - 1 : 1)];
  if (kBigVgpr) asm volatile("s_nop 0" ::: "v159");  // allocate 160 VGPRs like the quad kernel
  if (threadIdx.x < 16) lds[threadIdx.x] = make_uint4(threadIdx.x, 0, 0, 0);
  __syncthreads();
  const long long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if ((threadIdx.x & 63) == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
    const uint32_t w = blockIdx.x * W + (threadIdx.x >> 6);
    out[2 * w] = hw;
    out[2 * w + 1] = xcc + lds[0].x;
  }
}

template <int W, bool kBigVgpr = false>
int run(int grid) {
  uint32_t* d;
  const size_t nw = size_t(grid) * W;
  CHECK(hipMalloc(&d, nw * 8));
  hipLaunchKernelGGL((probe<W, kBigVgpr>), dim3(grid), dim3(64 * W), 0, 0, d, 2000000LL);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> h(nw * 2);
  CHECK(hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost));
  CHECK(hipFree(d));
  std::map<std::tuple<int, int, int, int>, std::map<int, int>> cu;  // (xcc,se,sh,cu) -> simd->waves
  std::map<std::tuple<int, int, int, int>, std::map<int, int>> cu_wgs;
  std::map<int, int> per_xcc;
  for (size_t w = 0; w < nw; ++w) {
    const uint32_t hw = h[2 * w], xcc = h[2 * w + 1] & 0xf;
    const int simd = (hw >> 4) & 3, cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    auto key = std::make_tuple(int(xcc), se, sh, cuid);
    cu[key][simd]++;
    cu_wgs[key][int(w / W)] = 1;
    per_xcc[xcc]++;
  }
  int max_simd = 0, max_wg = 0, hist[9] = {0};
  for (auto& kv : cu) {
    for (auto& s : kv.second) max_simd = std::max(max_simd, s.second);
    const int wgs = int(cu_wgs[kv.first].size());
    max_wg = std::max(max_wg, wgs);
    hist[std::min(wgs, 8)]++;
  }
  int shared_simd_waves = 0;
  for (auto& kv : cu)
    for (auto& s : kv.second)
      if (s.second > 1) shared_simd_waves += s.second;
  printf("%s waves/WG=%d grid=%4d: CUs used %3zu, max WGs/CU %d, max waves/SIMD %d, waves on shared "
         "SIMDs %4d, CUs with 1/2/3/4 WGs: %d/%d/%d/%d, XCDs:", kBigVgpr ? "vgpr160" : "vgpr-lo", W, grid, cu.size(), max_wg,
         max_simd, shared_simd_waves, hist[1], hist[2], hist[3], hist[4]);
  for (auto& x : per_xcc) printf(" %d:%d", x.first, x.second);
  printf("\n");
  return 0;
}

int main() {
  for (int grid : {32, 43, 64, 128, 171, 256, 512}) {
    run<2>(grid);
    run<3>(grid);
    run<4>(grid);
    run<5>(grid);
  }
  for (int grid : {32, 43, 128, 256, 512}) {
    run<2, true>(grid);
    run<3, true>(grid);
    run<4, true>(grid);
    run<5, true>(grid);
  }
  return 0;
}
