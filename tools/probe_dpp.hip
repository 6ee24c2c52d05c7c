// Semantics probe for the instructions the skew kernel adds: v_add_u32_dpp row_half_mirror,
// v_subrev_u32_dpp with bank masks, v_xad_u32.  Prints lane values of one 16-lane row.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  uint32_t a = 100 + l, b = 1000 * (l + 1), c = 0, d = 5000 + l, e = 7, f = (l >> 2) & 1 ? ~0u : 0u;
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n\ts_nop 4"
               : "=v"(c) : "v"(a), "v"(b));
  out[l] = c;
  uint32_t x = d;
  asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %0 row_half_mirror row_mask:0xf bank_mask:0xa\n\ts_nop 4"
               : "+v"(x) : "v"(a));
  out[64 + l] = x;
  uint32_t y;
  asm volatile("v_xad_u32 %0, %1, %2, %3" : "=v"(y) : "v"(e), "v"(f), "v"(b));
  out[128 + l] = y;
  uint32_t z = d;
  asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %0 row_half_mirror row_mask:0xf bank_mask:0x5\n\ts_nop 4"
               : "+v"(z) : "v"(a));
  out[192 + l] = z;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[4] = {"add_dpp mirror  c = a[mirror] + b", "subrev_dpp mirror banks 1,3: x = d - a[mirror]",
                          "xad (7 ^ f) + b  (f = ~0 on lanes 4-7)", "add_dpp mirror banks 0,2: z = a[mirror] + d"};
  for (int k = 0; k < 4; ++k) {
    printf("%s\n", names[k]);
    for (int l = 0; l < 16; ++l) printf("  lane %2d: %u (%d)\n", l, h[64 * k + l], (int)h[64 * k + l]);
  }
  return 0;
}
