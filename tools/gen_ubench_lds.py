#!/usr/bin/env python3
"""Generates tools/ubench_lds.hip: what an LDS row read costs a lone wave that runs the MD5
consumer's dependent step chain.

The MD5 consumer (md5_step_asm.inc) reads each block's 16 M+K rows with 16 ds_read_b128 -- 64
distinct 16-byte columns per instruction, one per chain -- between 256 dependent step VALU.
Timing-only builds put the reads at ~6.5 cycles each beyond their issue slot.  The rows are
laid out [row][lane] (uint4), which for ds_read_b128's four 16-lane groups is bank-conflict-
free (each group covers 256 contiguous bytes), so bank conflicts do not explain it.  This
benchmark isolates the read: one wave, the MD5 step chain (bitop3 -> add3(mk) -> alignbit ->
add) with the row reads of the consumer's rolling schedule (each row re-read for the next
block right after its last use, a counted lgkmcnt(8) before every 8th row), and the same
schedule with:
  none    every read replaced by an 8-byte v_mov, every wait by s_nops (the issue floor)
  b128    per-lane distinct 16 B (addr = row*1024 + lane*16): the MD5 consumer's reads
  b128q   quad broadcast (addr = row*1024 + (lane/4)*16): the SHA-256 skew consumer's shape
  b128s   one address for all lanes
  b64x2   two ds_read_b64 per row (distinct 8 B per lane each)
  none2 / b128_2   TWO independent MD5 chains interleaved instruction by instruction, each
          with its own rows (32 reads per block pair): does instruction-level parallelism hide
          the read cost that a single dependency chain pays?

Prints cycles per 64-step block (s_memtime) for 1 workgroup and for 16 (one per CU, like C2).

    python3 tools/gen_ubench_lds.py && hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds tools/ubench_lds.hip
"""
import os

ROUNDS = [(0xca, (25, 20, 15, 10)), (0xe4, (27, 23, 18, 12)), (0x96, (28, 21, 16, 9)),
          (0x39, (26, 22, 17, 11))]
RING = 100  # v[100:163]: 16 rows x 4 words
BLOCKS_PER_STMT = 2


def block(variant: str) -> list[str]:
    ops = []
    names = ["%0", "%1", "%2", "%3"]
    for r in range(16):
        if r % 8 == 0:
            ops += (["s_nop 0", "s_nop 0"] if variant == "none"
                    else ["s_waitcnt lgkmcnt(8)", "s_nop 0"])  # 8 bytes either way
        for q in range(4):
            i = 4 * r + q
            tt, rot = ROUNDS[i // 16]
            A, B, C, D = (names[(4 - i + k) % 4] for k in range(4))
            ops += [f"v_bitop3_b32 %4, {B}, {C}, {D} bitop3:0x{tt:02x}",
                    f"v_add3_u32 %5, {A}, %4, v{RING + 4 * r + q}",
                    f"v_alignbit_b32 %5, %5, %5, {rot[i % 4]}",
                    f"v_add_u32_e64 {A}, {B}, %5"]
        # row r was used by steps 4r..4r+3: read the next block's row r into the same registers
        reg = f"v[{RING + 4 * r}:{RING + 4 * r + 3}]"
        if variant == "none":
            ops += [f"v_mov_b32_e64 v{RING + 4 * r}, %6"]
        elif variant == "b64x2":
            ops += [f"ds_read_b64 v[{RING + 4 * r}:{RING + 4 * r + 1}], %6 offset:{r * 1024}",
                    f"ds_read_b64 v[{RING + 4 * r + 2}:{RING + 4 * r + 3}], %6 offset:{r * 1024 + 512}"]
        else:
            ops += [f"ds_read_b128 {reg}, %6 offset:{r * 1024}"]
    return ops


RING2 = 164  # v[164:227]: the second chain's rows


def block2(variant: str) -> list[str]:
    """Two chains: chain 1 on %0-%3 (f %4, t %5), chain 2 on %7-%10 (f %11, t %12)."""
    ops = []
    n1, n2 = ["%0", "%1", "%2", "%3"], ["%7", "%8", "%9", "%10"]
    for r in range(16):
        if r % 8 == 0:
            ops += (["s_nop 0", "s_nop 0"] if variant == "none2"
                    else ["s_waitcnt lgkmcnt(15)", "s_nop 0"])
        for q in range(4):
            i = 4 * r + q
            tt, rot = ROUNDS[i // 16]
            st = []
            for names, f, t, ring in ((n1, "%4", "%5", RING), (n2, "%11", "%12", RING2)):
                A, B, C, D = (names[(4 - i + k) % 4] for k in range(4))
                st.append([f"v_bitop3_b32 {f}, {B}, {C}, {D} bitop3:0x{tt:02x}",
                           f"v_add3_u32 {t}, {A}, {f}, v{ring + 4 * r + q}",
                           f"v_alignbit_b32 {t}, {t}, {t}, {rot[i % 4]}",
                           f"v_add_u32_e64 {A}, {B}, {t}"])
            for k in range(4):
                ops += [st[0][k], st[1][k]]
        for ring, base in ((RING, 0), (RING2, 16384)):
            if variant == "none2":
                ops += [f"v_mov_b32_e64 v{ring + 4 * r}, %6"]
            else:
                ops += [f"ds_read_b128 v[{ring + 4 * r}:{ring + 4 * r + 3}], %6 offset:{base + r * 1024}"]
    return ops


def kernel2(variant: str) -> str:
    body = "\\n\\t".join(op for op in block2(variant))
    clob = ", ".join(f'"v{RING + k}"' for k in range(128))
    return f'''
__global__ void __launch_bounds__(64) k_{variant}(uint32_t* out, uint64_t* cyc, int iters) {{
  __shared__ uint4 lds[2 * 16 * 64 + 64];
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = lane; k < 2 * 16 * 64 + 64; k += 64) lds[k] = make_uint4(k, k * 3u, k * 5u, k * 7u);
  __syncthreads();
  uint32_t a = lane, b = lane + 1, c = lane + 2, d = lane + 3, f = 0, t = 0;
  uint32_t a2 = lane + 9, b2 = lane + 10, c2 = lane + 11, d2 = lane + 12, f2 = 0, t2 = 0;
  uint32_t ad = (uint32_t)(uintptr_t)lds + lane * 16u;
  uint64_t t0, t1;
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i)
    asm volatile(".p2align 3\\n\\t{body}"
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&v"(f), "=&v"(t), "+v"(ad), "+v"(a2),
                   "+v"(b2), "+v"(c2), "+v"(d2), "=&v"(f2), "=&v"(t2)
                 :
                 : {clob}, "memory");
  asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 64 + lane] = a ^ b ^ c ^ d ^ a2 ^ b2 ^ c2 ^ d2;
  if (lane == 0) {{ cyc[2 * blockIdx.x] = t1 - t0; cyc[2 * blockIdx.x + 1] = (uint64_t)iters; }}
}}
'''


def kernel(variant: str) -> str:
    if variant in ("none2", "b128_2"):
        return kernel2(variant)
    body = "\\n\\t".join(op for _ in range(BLOCKS_PER_STMT) for op in block(variant))
    clob = ", ".join(f'"v{RING + k}"' for k in range(64))
    if variant in ("b128", "b128s", "b128q"):
        addr = {"b128": "lane * 16u", "b128q": "(lane >> 2) * 16u", "b128s": "0u"}[variant]
    elif variant == "b128x":
        addr = "lane * 16u"  # the XOR is per row: applied through the row offset below
    elif variant == "b64x2":
        addr = "lane * 8u"
    else:
        addr = "lane * 16u"
    return f'''
__global__ void __launch_bounds__(64) k_{variant}(uint32_t* out, uint64_t* cyc, int iters) {{
  __shared__ uint4 lds[16 * 64 + 64];
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = lane; k < 16 * 64 + 64; k += 64) lds[k] = make_uint4(k, k * 3u, k * 5u, k * 7u);
  __syncthreads();
  uint32_t a = lane, b = lane + 1, c = lane + 2, d = lane + 3, f = 0, t = 0;
  const uint32_t ad = (uint32_t)(uintptr_t)lds + {addr};
  uint64_t t0, t1;
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < iters; ++i)
    asm volatile(".p2align 3\\n\\t{body}"
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&v"(f), "=&v"(t)
                 : "v"(ad)
                 : {clob}, "memory");
  asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * 64 + lane] = a ^ b ^ c ^ d;
  if (lane == 0) {{ cyc[2 * blockIdx.x] = t1 - t0; cyc[2 * blockIdx.x + 1] = (uint64_t)iters * {BLOCKS_PER_STMT}; }}
}}
'''


def main():
    variants = ["none", "b128", "b128q", "b128s", "b64x2", "none2", "b128_2"]
    src = ['// GENERATED by tools/gen_ubench_lds.py -- do not edit.',
           '#include <hip/hip_runtime.h>', '#include <cstdint>', '#include <cstdio>', '#include <vector>',
           '#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { '
           'printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)']
    src += [kernel(v) for v in variants]
    table = ", ".join(f'{{"{v}", k_{v}}}' for v in variants)
    src.append(f'''
typedef void (*K)(uint32_t*, uint64_t*, int);
int main() {{
  struct {{ const char* name; K k; }} ks[] = {{{table}}};
  uint32_t* out; uint64_t* cyc;
  CHECK(hipMalloc(&out, 256 * 64 * 4));
  CHECK(hipMalloc(&cyc, 256 * 2 * 8));
  const int iters = 4096;
  printf("variant  grid  cycles/block (64 MD5 steps = 256 VALU + 16 row reads + 2 waits; "
         "*2: per block PAIR of two interleaved chains)\\n");
  for (auto& v : ks) {{
    for (int grid : {{1, 16}}) {{
      double best = 1e30;
      for (int rep = 0; rep < 3; ++rep) {{
        hipLaunchKernelGGL(v.k, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
        CHECK(hipDeviceSynchronize());
        std::vector<uint64_t> h(2 * grid);
        CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
        double worst = 0;
        for (int g = 0; g < grid; ++g) worst = std::max(worst, double(h[2 * g]) / double(h[2 * g + 1]));
        best = std::min(best, worst);
      }}
      printf("%-7s  %4d  %.1f\\n", v.name, grid, best);
    }}
  }}
  return 0;
}}
''')
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench_lds.hip")
    with open(path, "w") as f:
        f.write("\n".join(src))
    print(path)


if __name__ == "__main__":
    main()
