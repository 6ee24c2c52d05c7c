#!/usr/bin/env python3
"""Generates tools/ubench_coissue2.hip (optional argv[1]: comma-separated B streams to run
beside A = skew_round): wave A (one per SIMD) runs a consumer-like stream, wave B
(a partner on the same SIMD) a candidate producer stream; reports both waves' cycles per
instruction, lone and paired, with and without s_setprio 3 on A."""
# skew round (gen_skew.py round_ops opcode sequence) on rotating state s0..s3, x0/x1
def rnd(s0, s1, s2, s3, x, xn):
    return [f"v_alignbit_b32 %[q1], %[{s0}], %[{s0}], %[am]",
            f"v_bitop3_b32 %[sl], %[{s0}], %[{s1}], %[mk] bitop3:0xd2",
            f"v_bfi_b32 %[cm], %[sl], %[{s1}], %[{s2}]",
            "v_xor_b32_dpp %[q3], %[q1], %[q1] quad_perm:[1,2,0,1] row_mask:0xf bank_mask:0xf",
            f"v_add_u32_dpp %[t], %[{s0}], %[w] row_half_mirror row_mask:0xf bank_mask:0xf",
            "v_xor_b32_dpp %[q3], %[q1], %[q3] quad_perm:[2,0,1,2] row_mask:0xf bank_mask:0xf",
            f"v_xad_u32 %[{xn}], %[{s2}], %[mk], %[t]",
            f"v_add3_u32 %[{s3}], %[{x}], %[q3], %[cm]"]
ROUND = []
for r in range(16):
    st = ["s0", "s1", "s2", "s3"]
    k = r % 4
    s0, s1, s2, s3 = st[(0 - k) % 4], st[(1 - k) % 4], st[(2 - k) % 4], st[(3 - k) % 4]
    ROUND += rnd(s0, s1, s2, s3, "x0" if r % 2 == 0 else "x1", "x1" if r % 2 == 0 else "x0")
BLOCK = []
for r in range(64):
    BLOCK += ROUND[8 * (r % 16): 8 * (r % 16) + 8]
    if r % 4 == 3:
        BLOCK.append(f"ds_read_b128 %[v{(r // 4) % 4}], %[la] offset:{16 * (r // 4)}")
    if r % 16 == 15:
        BLOCK.append("s_waitcnt lgkmcnt(0)")
A_STREAMS = {"skew_block": BLOCK, "skew_round": ROUND, "add3_only": ["v_add3_u32 %[s0], %[s1], %[s2], %[s0]",
             "v_add3_u32 %[s1], %[s2], %[s3], %[s1]", "v_add3_u32 %[s2], %[s3], %[s0], %[s2]",
             "v_add3_u32 %[s3], %[s0], %[s1], %[s3]"] * 32}
# partner streams on b0..b7 (independent), 128 instructions
def simple_sigma(x, y, t0, t1, t2):
    # sigma0-like from shifts by immediates + bitop3 xor3 (all 'simple' class) + adds
    return [f"v_lshrrev_b32 %[{t0}], 7, %[{x}]", f"v_lshlrev_b32 %[{t1}], 25, %[{x}]",
            f"v_lshrrev_b32 %[{t2}], 18, %[{x}]", f"v_bitop3_b32 %[{t0}], %[{t0}], %[{t1}], %[{t2}] bitop3:0x96",
            f"v_lshlrev_b32 %[{t1}], 14, %[{x}]", f"v_lshrrev_b32 %[{t2}], 3, %[{x}]",
            f"v_bitop3_b32 %[{t0}], %[{t0}], %[{t1}], %[{t2}] bitop3:0x96", f"v_add_u32 %[{y}], %[{y}], %[{t0}]"]
B_STREAMS = {
    "none": [],
    "add_u32": [f"v_add_u32 %[b{i}], %[b{(i+1)%8}], %[b{(i+2)%8}]" for i in range(8)] * 16,
    "old_V2_8": ["v_lshlrev_b32 %[b0], 7, %[b1]", "v_lshrrev_b32 %[b2], 25, %[b3]", "v_xor_b32 %[b4], %[b0], %[b2]",
                 "v_add_u32 %[b5], %[b5], %[b4]", "v_or_b32 %[b1], %[b1], %[b5]", "v_lshrrev_b32 %[b3], 3, %[b3]",
                 "v_xor_b32 %[b2], %[b3], %[b4]", "v_add_u32 %[b0], %[b0], %[b1]"] * 16,
    "simple_sigma": (simple_sigma("b0", "b1", "b2", "b3", "b4") + simple_sigma("b5", "b6", "b7", "b2", "b3")) * 8,
    "alignbit_sigma": (["v_alignbit_b32 %[b2], %[b0], %[b0], 7", "v_alignbit_b32 %[b3], %[b0], %[b0], 18",
                        "v_lshrrev_b32 %[b4], 3, %[b0]", "v_bitop3_b32 %[b2], %[b2], %[b3], %[b4] bitop3:0x96",
                        "v_add3_u32 %[b1], %[b1], %[b2], %[b5]", "v_alignbit_b32 %[b6], %[b5], %[b5], 17",
                        "v_alignbit_b32 %[b7], %[b5], %[b5], 19", "v_add_u32 %[b0], %[b0], %[b1]"]) * 16,
    "skew_round": None,  # the A stream itself on the partner
}
def pure(tmpl, dist=2):
    return [tmpl.format(d=f"b{i}", a=f"b{(i+1)%8}", b=f"b{(i+dist)%8}") for i in range(8)] * 16
for name, tmpl in [("xor", "v_xor_b32 %[{d}], %[{a}], %[{b}]"), ("or", "v_or_b32 %[{d}], %[{a}], %[{b}]"),
                   ("and", "v_and_b32 %[{d}], %[{a}], %[{b}]"), ("sub_u32", "v_sub_u32 %[{d}], %[{a}], %[{b}]"),
                   ("bitop3", "v_bitop3_b32 %[{d}], %[{a}], %[{b}], %[{d}] bitop3:0x96"),
                   ("lshrrev_imm", "v_lshrrev_b32 %[{d}], 7, %[{a}]"), ("lshlrev_imm", "v_lshlrev_b32 %[{d}], 25, %[{a}]"),
                   ("mov", "v_mov_b32 %[{d}], %[{a}]"), ("fma_f32", "v_fma_f32 %[{d}], %[{a}], %[{b}], %[{d}]"),
                   ("add_lit", "v_add_u32 %[{d}], 0x428a2f98, %[{a}]"), ("mul_u24", "v_mul_u32_u24 %[{d}], %[{a}], %[{b}]"),
                   ("add_e64", "v_add_u32_e64 %[{d}], %[{a}], %[{b}]"), ("xor_e64", "v_xor_b32_e64 %[{d}], %[{a}], %[{b}]"),
                   ("add_f32", "v_add_f32 %[{d}], %[{a}], %[{b}]"), ("mul_f32", "v_mul_f32 %[{d}], %[{a}], %[{b}]"),
                   ("pk_add_u16", "v_pk_add_u16 %[{d}], %[{a}], %[{b}]"), ("lshl_or", "v_lshl_or_b32 %[{d}], %[{a}], 7, %[{b}]"),
                   ("add_co", "v_add_co_u32 %[{d}], vcc, %[{a}], %[{b}]"), ("xnor", "v_xnor_b32 %[{d}], %[{a}], %[{b}]"),
                   ("mad_u24", "v_mad_u32_u24 %[{d}], %[{a}], %[{b}], %[{d}]"), ("ashr_imm", "v_ashrrev_i32 %[{d}], 7, %[{a}]")]:
    B_STREAMS[name] = pure(tmpl)
def expansion(x15, x2, x7, x16, w, lshl=True):
    """one message-schedule expansion W = s1(x2) + x7 + s0(x15) + x16, then W + K; left shifts as
    v_lshlrev (lshl=True) or the rotations as v_alignbit (lshl=False)"""
    if lshl:
        s0 = [f"v_lshrrev_b32 %[t0], 7, %[{x15}]", f"v_lshrrev_b32 %[t1], 18, %[{x15}]",
              f"v_lshrrev_b32 %[t2], 3, %[{x15}]", f"v_lshlrev_b32 %[t3], 25, %[{x15}]",
              "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96", f"v_lshlrev_b32 %[t1], 14, %[{x15}]",
              "v_bitop3_b32 %[u0], %[t0], %[t3], %[t1] bitop3:0x96"]
        s1 = [f"v_lshrrev_b32 %[t0], 17, %[{x2}]", f"v_lshrrev_b32 %[t1], 19, %[{x2}]",
              f"v_lshrrev_b32 %[t2], 10, %[{x2}]", f"v_lshlrev_b32 %[t3], 15, %[{x2}]",
              "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96", f"v_lshlrev_b32 %[t1], 13, %[{x2}]",
              "v_bitop3_b32 %[u1], %[t0], %[t3], %[t1] bitop3:0x96"]
    else:
        s0 = [f"v_alignbit_b32 %[t0], %[{x15}], %[{x15}], 7", f"v_alignbit_b32 %[t1], %[{x15}], %[{x15}], 18",
              f"v_lshrrev_b32 %[t2], 3, %[{x15}]", "v_bitop3_b32 %[u0], %[t0], %[t1], %[t2] bitop3:0x96"]
        s1 = [f"v_alignbit_b32 %[t0], %[{x2}], %[{x2}], 17", f"v_alignbit_b32 %[t1], %[{x2}], %[{x2}], 19",
              f"v_lshrrev_b32 %[t2], 10, %[{x2}]", "v_bitop3_b32 %[u1], %[t0], %[t1], %[t2] bitop3:0x96"]
    return s0 + s1 + ["v_add_u32 %[u0], %[u0], %[u1]", f"v_add_u32 %[u0], %[u0], %[{x7}]",
                      f"v_add_u32 %[{w}], %[u0], %[{x16}]", f"v_add_u32 %[{w}], 0x428a2f98, %[{w}]"]
def producer(lshl):
    out = []
    for t in range(8):  # ring of 8 W registers b0..b7 (positions mod 8 stand in for t-15, t-2 ...)
        out += expansion(f"b{(t+1)%8}", f"b{(t+6)%8}", f"b{(t+1)%8}", f"b{t%8}", f"b{t%8}", lshl)
    return out
for name, tmpl in [("bfrev", "v_bfrev_b32 %[{d}], %[{a}]"), ("not", "v_not_b32 %[{d}], %[{a}]"),
                   ("mov_sdwa_w1", "v_mov_b32_sdwa %[{d}], %[{a}] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0"),
                   ("add_sdwa", "v_add_u32_sdwa %[{d}], %[{a}], %[{b}] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"),
                   ("lshrrev_reg", "v_lshrrev_b32 %[{d}], %[{b}], %[{a}]"), ("min_u32", "v_min_u32 %[{d}], %[{a}], %[{b}]"),
                   ("cvt_f32_u32", "v_cvt_f32_u32 %[{d}], %[{a}]"), ("subrev", "v_subrev_u32 %[{d}], %[{a}], %[{b}]")]:
    B_STREAMS[name] = pure(tmpl)
# round 2, candidates for left shifts / byte placement without doublings
for name, tmpl in [("mul_lo_u32", "v_mul_lo_u32 %[{d}], %[{a}], %[{b}]"), ("mul_hi_u32", "v_mul_hi_u32 %[{d}], %[{a}], %[{b}]"),
                   ("ldexp_f32", "v_ldexp_f32 %[{d}], %[{a}], %[{b}]"), ("exp_f32", "v_exp_f32 %[{d}], %[{a}]"),
                   ("cvt_f32_ubyte0", "v_cvt_f32_ubyte0 %[{d}], %[{a}]"), ("cvt_u32_f32", "v_cvt_u32_f32 %[{d}], %[{a}]"),
                   ("max_u32", "v_max_u32 %[{d}], %[{a}], %[{b}]"), ("cndmask", "v_cndmask_b32 %[{d}], %[{a}], %[{b}], vcc"),
                   ("sub_f32", "v_sub_f32 %[{d}], %[{a}], %[{b}]"), ("lshlrev_b16", "v_lshlrev_b16 %[{d}], %[{b}], %[{a}]"),
                   ("add_u16", "v_add_u16 %[{d}], %[{a}], %[{b}]"), ("mul_f32_lit", "v_mul_f32 %[{d}], 0x42000000, %[{a}]"),
                   ("fmac_f32", "v_fmac_f32 %[{d}], %[{a}], %[{b}]"), ("mul_legacy", "v_mul_legacy_f32 %[{d}], %[{a}], %[{b}]"),
                   ("ashr_reg", "v_ashrrev_i32 %[{d}], %[{b}], %[{a}]"), ("bfe_u32", "v_bfe_u32 %[{d}], %[{a}], 8, 8"),
                   ("mul_lo_u16", "v_mul_lo_u16 %[{d}], %[{a}], %[{b}]"), ("max_f32", "v_max_f32 %[{d}], %[{a}], %[{b}]"),
                   ("subrev_f32", "v_subrev_f32 %[{d}], %[{a}], %[{b}]"), ("mov_dpp", "v_mov_b32_dpp %[{d}], %[{a}] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")]:
    B_STREAMS[name] = pure(tmpl)
for name, op in [("pk_mul_f32", "v_pk_mul_f32"), ("pk_add_f32", "v_pk_add_f32"), ("pk_fma_f32", "v_pk_fma_f32"),
                 ("lshlrev_b64", "v_lshlrev_b64")]:
    if name == "lshlrev_b64":
        B_STREAMS[name] = [f"v_lshlrev_b64 %[p{i%4}], 7, %[p{(i+1)%4}]" for i in range(128)]
    elif name == "pk_fma_f32":
        B_STREAMS[name] = [f"{op} %[p{i%4}], %[p{(i+1)%4}], %[p{(i+2)%4}], %[p{i%4}]" for i in range(128)]
    else:
        B_STREAMS[name] = [f"{op} %[p{i%4}], %[p{(i+1)%4}], %[p{(i+2)%4}]" for i in range(128)]
# 64-bit right shift of a {x, x} pair -> rotr in the low word: pairs (b0,b1), (b2,b3), ...
B_STREAMS["lshrrev_b64"] = [f"v_lshrrev_b64 %[p{i%4}], 7, %[p{(i+1)%4}]" for i in range(128)]
def expansion2(i):
    """expansion with 2 left shifts per new W (a = W<<13, b = W<<25 kept beside W): s0's x<<14 =
    a+a, s1's y<<15 = 4a; ring registers b0-b7 stand for W, u-regs for temporaries"""
    x, y, w = f"b{(i+1)%8}", f"b{(i+6)%8}", f"b{i%8}"
    return [f"v_lshrrev_b32 %[t0], 7, %[{x}]", f"v_lshrrev_b32 %[t1], 18, %[{x}]", f"v_lshrrev_b32 %[t2], 3, %[{x}]",
            "v_add_u32 %[t3], %[u0], %[u0]", "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96",
            "v_bitop3_b32 %[u1], %[t0], %[t3], %[u2] bitop3:0x96",                       # s0
            f"v_lshrrev_b32 %[t0], 17, %[{y}]", f"v_lshrrev_b32 %[t1], 19, %[{y}]", f"v_lshrrev_b32 %[t2], 10, %[{y}]",
            "v_add_u32 %[t3], %[u0], %[u0]", "v_add_u32 %[t3], %[t3], %[t3]",
            "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96", "v_bitop3_b32 %[t0], %[t0], %[t3], %[u0] bitop3:0x96",  # s1
            "v_add_u32 %[u1], %[u1], %[t0]", f"v_add_u32 %[u1], %[u1], %[{y}]", f"v_add_u32 %[{w}], %[u1], %[{x}]",
            f"v_lshlrev_b32 %[u0], 13, %[{w}]", f"v_lshlrev_b32 %[u2], 25, %[{w}]",   # the 2 left shifts
            f"v_add_u32 %[t1], 0x428a2f98, %[{w}]"]
B_STREAMS["producer_2c"] = [op for i in range(8) for op in expansion2(i)]
B_STREAMS["producer_2c_perm"] = B_STREAMS["producer_2c"] + ["v_perm_b32 %[b0], %[b1], %[b1], %[b2]"] * 3
B_STREAMS["producer_lshl"] = producer(True)
B_STREAMS["producer_alignbit"] = producer(False)
B_STREAMS["add_u32_dep1"] = [f"v_add_u32 %[b0], %[b0], %[b{i%7+1}]" for i in range(128)]
B_STREAMS["xor_dep1"] = [f"v_xor_b32 %[b0], %[b0], %[b{i%7+1}]" for i in range(128)]
def asm_block(lines, regs):
    body = "\\n\\t".join(lines)
    ops = ", ".join(f'[{r}] "=&v"({r})' if r in ("v0", "v1", "v2", "v3") else f'[{r}] "+v"({r})' for r in regs)
    return f'asm volatile(".p2align 3\\n\\t{body}" : {ops} : [am] "v"(am), [mk] "v"(mk), [w] "v"(w), [la] "v"(la) : "vcc", "memory");'
A_REGS = ["s0", "s1", "s2", "s3", "x0", "x1", "q1", "q3", "sl", "cm", "t", "v0", "v1", "v2", "v3"]
B_REGS = [f"b{i}" for i in range(8)] + ["t0", "t1", "t2", "t3", "u0", "u1", "u2"]
out = ['''// tools/ubench_coissue2.hip -- GENERATED by tools/gen_ubench_coissue2.py (see its docstring).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_coissue2 tools/ubench_coissue2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \\
  printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
''']
an, bn = list(A_STREAMS), list(B_STREAMS)
out.append("const char* kA[] = {" + ", ".join(f'"{n}"' for n in an) + "};")
out.append("__device__ constexpr int kAPer[] = {" + ", ".join(str(sum(1 for l in A_STREAMS[n] if not l.startswith("s_"))) for n in an) + "};")
out.append("const char* kB[] = {" + ", ".join(f'"{n}"' for n in bn) + "};")
out.append("template <int TA> __device__ __forceinline__ uint32_t run_a(int iters, uint32_t am, uint32_t mk, uint32_t w, uint32_t lane) {")
out.append("  uint32_t s0 = lane * 3 + 1, s1 = lane * 5 + 2, s2 = lane * 7 + 3, s3 = lane * 11 + 4, x0 = 0, x1 = 0, q1 = 0, q3 = 0, sl = 0, cm = 0, t = 0;\n  uint4 v0, v1, v2, v3; const uint32_t la = lane * 16;")
for i, n in enumerate(an):
    kw = "if constexpr" if i == 0 else "else if constexpr"
    out.append(f"  {kw} (TA == {i}) for (int i = 0; i < iters; ++i) {asm_block(A_STREAMS[n], A_REGS)}")
out.append("  return s0 ^ s1 ^ s2 ^ s3 ^ x0 ^ x1;\n}")
out.append("template <int TB> __device__ __forceinline__ uint32_t run_b(int iters, uint32_t am, uint32_t mk, uint32_t w, uint32_t lane, int& per) {")
out.append("  uint32_t " + ", ".join(f"b{i} = lane * {2*i+3} + {i}" for i in range(8)) + ", t0 = 0, t1 = 0, t2 = 0, t3 = 0, u0 = 0, u1 = 0, u2 = 0;\n  uint64_t p0 = lane * 0x100000001ull, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3; const uint32_t la = lane * 16;")
for i, n in enumerate(bn):
    kw = "if constexpr" if i == 0 else "else if constexpr"
    if n == "none":
        out.append(f"  {kw} (TB == {i}) {{ per = 0; return 0; }}")
    elif n == "skew_round":
        out.append(f"  {kw} (TB == {i}) {{ per = {len(ROUND)}; return run_a<0>(iters, am, mk, w, lane); }}")
    else:
        regs = ["p0", "p1", "p2", "p3"] if n in ("lshrrev_b64", "lshlrev_b64") or n.startswith("pk_") and n.endswith("f32") else B_REGS
        out.append(f"  {kw} (TB == {i}) {{ per = {len(B_STREAMS[n])}; for (int i = 0; i < iters; ++i) {asm_block(B_STREAMS[n], regs)} }}")
out.append("  return " + " ^ ".join(f"b{i}" for i in range(8)) + " ^ u0 ^ uint32_t(p0 ^ p1 ^ p2 ^ p3);\n}")
out.append('''
template <int TA, int TB, bool PRIO>
__global__ __launch_bounds__(512) void k(uint32_t* out, uint64_t* rec, int ia, int ib) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  const uint32_t am = 6 + (lane & 3), mk = (lane & 4) ? ~0u : 0u, w = lane ^ 0x1234;
  __shared__ uint4 lds_pad[128];
  lds_pad[threadIdx.x & 127] = make_uint4(lane, 0, 0, 0);
  __syncthreads();
  uint64_t t0, t1;
  int per = 0;
  uint32_t s;
  if (wave < 4 && PRIO) __builtin_amdgcn_s_setprio(3);
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (wave < 4) { s = run_a<TA>(ia, am, mk, w, lane); per = kAPer[TA]; }
  else s = run_b<TB>(ib, am, mk, w, lane, per);
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[threadIdx.x] = s;
  if (lane == 0) { rec[3 * wave] = t1 - t0; rec[3 * wave + 1] = hw; rec[3 * wave + 2] = uint64_t(per) * (wave < 4 ? ia : ib); }
}

template <int TA, int TB, bool PRIO>
int run(const char* tag) {
  // B runs about as long as A alone would (A: 200 x 128 instr); its own count is scaled so both
  // overlap for most of the run
  const int ia = 200, ib = 200;
  uint32_t* out; uint64_t* rec;
  CHECK(hipMalloc(&out, 512 * 4)); CHECK(hipMalloc(&rec, 24 * 8));
  const int waves = TB == 0 ? 4 : 8;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((k<TA, TB, PRIO>), dim3(1), dim3(64 * waves), 0, 0, out, rec, ia, ib);
    CHECK(hipDeviceSynchronize());
  }
  uint64_t h[24];
  CHECK(hipMemcpy(h, rec, 24 * 8, hipMemcpyDeviceToHost));
  double a = 0, b = 0; int same = 0;
  for (int w = 0; w < waves; ++w) {
    const double cpi = double(h[3 * w]) / double(h[3 * w + 2] ? h[3 * w + 2] : 1);
    if (w < 4) a += cpi / 4; else b += cpi / 4;
  }
  for (int w = 4; w < waves; ++w) for (int c = 0; c < 4; ++c) same += ((h[3*w+1] >> 4) & 3) == ((h[3*c+1] >> 4) & 3);
  printf("A=%-11s B=%-15s prio=%d  A %.3f cyc/instr  B %.3f cyc/instr  (B overlap %s, same-SIMD pairs %d)  %s\\n",
         kA[TA], kB[TB], PRIO ? 3 : 0, a, b, "", same, tag);
  CHECK(hipFree(out)); CHECK(hipFree(rec));
  return 0;
}
int main() {''')
out.append('  if (run<0, 0, true>("(warm-up, clocks ramping)")) return 1;')
import sys
PAIRS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["none", "add_u32", "producer_2c", "producer_2c_perm", "producer_lshl"]
for ta in ([1] if len(sys.argv) > 1 else range(2)):   # with a list: A = skew_round only
    for tb in [bn.index(x) for x in PAIRS]:
        for prio in ("true",):
            out.append(f'  if (run<{ta}, {tb}, {prio}>("")) return 1;')
out.append("  return 0;\n}")
open("/root/repo/tools/ubench_coissue2.hip", "w").write("\n".join(out) + "\n")
