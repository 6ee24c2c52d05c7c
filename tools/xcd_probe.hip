// xcd_probe.hip -- which XCD each workgroup of a dual-grid-shaped launch runs on.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/xcd_probe tools/xcd_probe.hip && tools/xcd_probe
//
// The split and mixed dual grids (sha256_kernels.hip) give each MD5 workgroup the chains of the
// skew groups with blockIdx.x == its own (mod 8), assuming workgroups are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md "Workgroup dispatch").  This launches grids of the same
// shapes (128 / 192 threads, ~100 KiB of LDS: one workgroup per CU) and prints, per grid, how
// many workgroups share an XCD with every workgroup 8 apart, and the XCC id of the first 16.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

template <int kLdsWords>
__global__ __launch_bounds__(192) void probe(unsigned* xcc, unsigned* cu) {
  __shared__ unsigned lds[kLdsWords];
  const unsigned id = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID[15:0]
  lds[threadIdx.x] = id;
  __syncthreads();
  if (threadIdx.x == 0) {
    xcc[blockIdx.x] = lds[0] & 0xf;
    cu[blockIdx.x] = __builtin_amdgcn_s_getreg((15 << 11) | 4);  // HW_REG_HW_ID
  }
  // hold the CU for a while so the grid is resident at once, as the hash kernels are
  const long long t0 = clock64();
  while (clock64() - t0 < 2000000) __builtin_amdgcn_s_sleep(10);
}

int main() {
  const int grids[] = {144, 199, 256, 36, 9};
  unsigned *dx, *dc;
  if (hipMalloc(&dx, 4096) != hipSuccess || hipMalloc(&dc, 4096) != hipSuccess) return 1;
  for (int g : grids) {
    for (int threads : {128, 192}) {
      hipLaunchKernelGGL(probe<25600>, dim3(g), dim3(threads), 0, 0, dx, dc);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      std::vector<unsigned> x(g);
      if (hipMemcpy(x.data(), dx, 4 * g, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      int same = 0, pairs = 0;
      for (int b = 0; b + 8 < g; ++b, ++pairs) same += x[b] == x[b + 8];
      std::printf("grid %3d x %3d threads: %d of %d pairs (b, b+8) share an XCD; xcc of blocks 0..15:",
                  g, threads, same, pairs);
      for (int b = 0; b < 16 && b < g; ++b) std::printf(" %u", x[b]);
      std::printf("\n");
    }
  }
  return 0;
}
