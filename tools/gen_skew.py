#!/usr/bin/env python3
"""Generator (and lane-level simulator) of the skewed lane-octet SHA-256 round schedule.

One SHA-256 chain lives on 8 lanes of a wave: an e-quad (lanes 0-3 of the half-row, DPP banks
0/2) holding e,f,g,h and an a-quad (lanes 4-7, banks 1/3) holding a,b,c,d, as in the quad
kernel.  The a-quad runs TWO ROUNDS BEHIND the e-quad.  With that skew both halves' updates
become "own nonlinear part + one precomputed sum" and the exchange between the quads needs
no extra instruction:

    e-quad, round t:  e[t+1]   = x_e + Sigma1(e[t])   + Ch(e[t], e[t-1], e[t-2])
                      x_e      = a[t-3] + e[t-3] + W[t]+K[t]
    a-quad, round t:  a[t-1]   = x_a + Sigma0(a[t-2]) + Maj(a[t-2], a[t-3], a[t-4])
                      x_a      = e[t-1] - a[t-5]            (a[r+1] = T1[r] + T2[r],
                                                             T1[r] = e[r+1] - a[r-3])

and the NEXT round's x needs, in the e-quad, the a-quad's current s0 (a[t-2]) plus its own s2
(e[t-2]) plus W+K; in the a-quad, the e-quad's current s0 (e[t]) minus its own s2 (a[t-4]).
The cross term is one `v_add_u32_dpp row_half_mirror` (lane i <-> lane 7-i swaps the quads)
and the per-quad sign of the own term is one `v_xad_u32` with a per-lane mask (x ^ 0 = x,
x ^ ~0 = -x - 1; the a-quad's W register holds 1 to restore the +1).  A round is

    v_alignbit_b32  q1, s0, s0, amt        ; one rotation per lane (e: 6,11,25,6  a: 2,13,22,2)
    v_bitop3_b32    sel, s0, s1, mk 0xd2   ; e: s0 ; a: ~(s0 ^ s1)
    v_bfi_b32       cm, sel, s1, s2        ; e: Ch  ; a: Maj
    v_xor_b32_dpp   q3, q1, q1 quad_perm:[1,2,0,1]
    v_add_u32_dpp   t, s0, w row_half_mirror          ; cross + W (next round)
    v_xor_b32_dpp   q3, q1, q3 quad_perm:[2,0,1,2]    ; q3 = Sigma
    v_xad_u32       xn, s2, mk, t                     ; +/- own s2
    v_add3_u32      new, x, q3, cm

8 VALU per round (the quad kernel needs 9), and the pipeline runs across block boundaries:
the a-quad finishes block k's rounds 62-63 during block k+1's rounds 0-1.  The feed-forward
(H += state) costs 4 bank-masked adds per half per block, and three more masked DPP adds
correct the precomputed sums that straddle a block boundary (C1, C2, C4 below).

Registers (per lane): the ring R(r) written by round r of a block of parity p is
    R(0), R(1) = G[p][0], G[p][1];  R(2..59) = N[r % 4];  R(60..63) = E[p][0..3]
and R(-1..-4) = E[q][3..0] with q = 1 - p (the previous block's last four).  After a block's
e-feed-forward E[p][3..0] (e-lanes) are H_e..H_h; after the next block's a-feed-forward the
a-half H_a..H_d are (G[q][1], G[q][0], E[p][3], E[p][2]) (a-lanes).

The same schedule runs on a lane-PAIR layout (layout="pair"): a chain on e-lane k and a-lane
7-k of a half-row -- the same row_half_mirror partner -- with Sigma as three per-lane rotations
and one xor3 (9 VALU per round, four chains per half-row, 32 per wave).

This module emits the asm text (`emit_inc`) consumed by s3client_amd/csrc/sha256_kernels.hip
and simulates the same instruction lists lane by lane (`simulate_chains`), which
tests/test_skew_schedule.py checks against hashlib on multi-block messages.
"""
import argparse
import os
import struct

M32 = 0xFFFFFFFF
K256 = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]

E_MASK, A_MASK = 0x5, 0xA   # DPP bank masks: banks 0/2 = e-quad, 1/3 = a-quad
PERM1, PERM2 = (1, 2, 0, 1), (2, 0, 1, 2)


# ----------------------------------------------------------------------------- instruction lists
# Each instruction is a tuple: (op, dst, srcs..., extra).  Register names are symbolic:
#   gP_I (G[p][i]), eP_I (E[p][i]), n0..n3, x0, x1, q1, q3, sl, cm, t, am, mk, w0..w63.

def R(r, p):
    q = 1 - p
    if r < 0:
        return f"e{q}_{4 + r}"          # R(-1..-4) = E[q][3..0]
    if r < 2:
        return f"g{p}_{r}"
    if r < 60:
        return f"n{r % 4}"
    return f"e{p}_{r - 60}"


def round_ops(r, p, wreg, layout="quad"):
    """Instructions of round r (0..63) of a block of parity p.  wreg: W+K register of round r+1
    (None at r = 63: the next block's first word is consumed by next_ops).

    layout "quad": a chain on 8 lanes (e-quad + a-quad), Sigma = one per-lane rotation folded
    by two quad_perm xor_dpp.  layout "pair": a chain on 2 lanes (e-lane k, a-lane 7-k of a
    half-row: the same row_half_mirror partner), Sigma = three per-lane rotations + xor3, four
    chains per half-row (9 VALU per round)."""
    q = 1 - p
    s0, s1, s2 = R(r - 1, p), R(r - 2, p), R(r - 3, p)
    xc, xn = f"x{r % 2}", f"x{(r + 1) % 2}"
    pair = layout == "pair"
    ops = [("align", "q1", s0, "am")]
    if pair:
        ops += [("align", "q2", s0, "am2"), ("align", "q3", s0, "am3")]
    ops.append(("sel", "sl", s0, s1, "mk"))
    if r == 1:
        # a-feed-forward of the previous block's raw a63 (s0 here) once SEL has read it, so that
        # P1 below already hands the e-quad H_b.
        ops.append(("ffa", f"g{p}_0", f"g{q}_0"))
    ops.append(("bfi", "cm", "sl", s1, s2))
    if r == 0:
        # C4: the a-quad's cross term below is e's fed-forward H_e; it needs the raw e64 =
        # H_e - H_e(old).  A DPP operand can only be the minuend of a subtraction on this
        # hardware (v_subrev_u32_dpp swizzles its minuend: tools/probe_dpp.hip), so the old
        # H_e is added to the own term instead: ~(a60 + H_e(old)) = ~a60 - H_e(old).  s2's
        # a-part (raw a60) is dead after BFI and P2.
        ops.append(("adda", s2, f"e{p}_3"))
    if r == 1:
        ops.append(("ffa", f"e{q}_3", f"e{p}_3"))   # raw a62 -> H_c (s1: last read by BFI)
        ops.append(("ffa", f"e{q}_2", f"e{p}_2"))   # raw a61 -> H_d (read by P2 below)
    if pair:
        ops.append(("xor3", "q3", "q1", "q2", "q3"))
        if wreg is not None:
            ops += [("p1", "t", s0, wreg), ("p2", xn, s2, "mk", "t")]
    else:
        ops.append(("xor1", "q3", "q1"))
        if wreg is not None:
            ops.append(("p1", "t", s0, wreg))
        ops.append(("xor2", "q3", "q1"))
        if wreg is not None:
            ops.append(("p2", xn, s2, "mk", "t"))
    if r == 0:
        # C2: the e-quad's cross term was the previous block's raw a62: add its H_c.
        ops.append(("adde", xn, f"e{p}_3"))
    ops.append(("add3", R(r, p), xc, "q3", "cm"))
    if r == 1:
        ops.append(("ffa", f"g{p}_1", f"g{q}_1"))   # raw a64 -> H_a
    if r == 63:
        for i in (0, 1, 3):
            ops.append(("ffe", f"e{p}_{i}", f"e{q}_{i}"))
    return ops


def rounds_ops(p, first=0, last=64, layout="quad"):
    return [op for r in range(first, last)
            for op in round_ops(r, p, f"w{r + 1}" if r < 63 else None, layout)]


def next_ops(p, wreg="w0"):
    """After round 63: x for the next block's round 0 (needs its W[0]+K[0])."""
    q = 1 - p
    return [("p1", "t", f"e{p}_2", wreg),          # cross: a-quad gets raw e63, e-quad raw a61
            ("ffe", f"e{p}_2", f"e{q}_2"),
            ("p2", "x0", f"e{p}_0", "mk", "t"),    # own: e-quad H_h (fed forward), a-quad a59
            ("adde", "x0", f"e{q}_2")]             # C1: + H_d (a-quad, fed forward at round 1)


# ----------------------------------------------------------------------------- simulator
def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def bank(lane):
    return (lane >> 2) & 3


def simulate_ops(ops, regs):
    """Execute an instruction list on 8-lane register vectors (dict name -> list of 8 ints)."""
    for ins in ops:
        op = ins[0]
        if op == "align":
            _, d, s, a = ins
            regs[d] = [rotr(regs[s][i], regs[a][i] & 31) for i in range(8)]
        elif op == "sel":
            _, d, a, b, m = ins
            regs[d] = [(regs[a][i] & ~regs[m][i] | ~(regs[a][i] ^ regs[b][i]) & regs[m][i]) & M32
                       for i in range(8)]
        elif op == "bfi":
            _, d, s, a, b = ins
            regs[d] = [(regs[s][i] & regs[a][i] | ~regs[s][i] & regs[b][i]) & M32 for i in range(8)]
        elif op == "xor3":
            _, d, a, b, c = ins
            regs[d] = [regs[a][i] ^ regs[b][i] ^ regs[c][i] for i in range(8)]
        elif op in ("xor1", "xor2"):
            _, d, s = ins
            perm = PERM1 if op == "xor1" else PERM2
            other = regs[s] if op == "xor1" else regs[d]
            regs[d] = [regs[s][(i & ~3) + perm[i & 3]] ^ other[i] for i in range(8)]
        elif op == "p1":
            _, d, s, w = ins
            regs[d] = [(regs[s][7 - i] + regs[w][i]) & M32 for i in range(8)]
        elif op == "p2":
            _, d, s, m, t = ins
            regs[d] = [((regs[s][i] ^ regs[m][i]) + regs[t][i]) & M32 for i in range(8)]
        elif op == "add3":
            _, d, a, b, c = ins
            regs[d] = [(regs[a][i] + regs[b][i] + regs[c][i]) & M32 for i in range(8)]
        elif op in ("ffe", "ffa"):
            _, d, s = ins
            msk = E_MASK if op == "ffe" else A_MASK
            regs[d] = [(regs[s][i] + regs[d][i]) & M32 if msk >> bank(i) & 1 else regs[d][i]
                       for i in range(8)]
        elif op == "adde":
            _, d, s = ins
            regs[d] = [(regs[s][7 - i] + regs[d][i]) & M32 if E_MASK >> bank(i) & 1 else regs[d][i]
                       for i in range(8)]
        elif op == "adda":
            _, d, s = ins
            regs[d] = [(regs[s][7 - i] + regs[d][i]) & M32 if A_MASK >> bank(i) & 1 else regs[d][i]
                       for i in range(8)]
        else:
            raise ValueError(op)


def schedule(block_words):
    out = []
    for w in block_words:
        ws = list(w)
        for t in range(16, 64):
            s0 = rotr(ws[t - 15], 7) ^ rotr(ws[t - 15], 18) ^ (ws[t - 15] >> 3)
            s1 = rotr(ws[t - 2], 17) ^ rotr(ws[t - 2], 19) ^ (ws[t - 2] >> 10)
            ws.append((ws[t - 16] + s0 + ws[t - 7] + s1) & M32)
        out.append([(ws[t] + K256[t]) & M32 for t in range(64)])
    return out


def lane_chain(i, layout):
    """Chain index of lane i (0..7) of a half-row: quad = one chain, pair = four (e-lane k and
    a-lane 7-k)."""
    if layout == "quad":
        return 0
    return i if i < 4 else 7 - i


def init_regs(Hs, wk0s, layout="quad"):
    """Kernel prologue: register contents before block 0 (parity 0), per lane.  Hs[c] = 8-word
    state (a..h) of chain c, wk0s[c] = W[0]+K[0] of its block 0."""
    def lanes(f):  # f(chain state, ahalf, wk0) -> value
        return [f(Hs[lane_chain(i, layout)], i >= 4, wk0s[lane_chain(i, layout)]) & M32
                for i in range(8)]
    regs = {n: [0] * 8 for n in
            ["g0_0", "g0_1", "g1_0", "g1_1", "n0", "n1", "n2", "n3", "x1", "q1", "q2", "q3", "sl",
             "cm", "t"] + [f"e{p}_{i}" for p in (0, 1) for i in range(4)]}
    if layout == "quad":
        regs["am"] = [6, 11, 25, 6, 2, 22, 13, 2]  # lanes 4-7 mirror lanes 3-0: any order works
    else:
        regs["am"], regs["am2"], regs["am3"] = [6] * 4 + [2] * 4, [11] * 4 + [13] * 4, [25] * 4 + [22] * 4
    regs["mk"] = [0] * 4 + [M32] * 4
    regs["e1_3"] = lanes(lambda H, a, w: 0 if a else H[4])
    regs["e1_2"] = lanes(lambda H, a, w: 0 if a else H[5])
    regs["e1_1"] = lanes(lambda H, a, w: 0 if a else H[6])
    regs["e1_0"] = lanes(lambda H, a, w: 0 if a else H[7])
    regs["e0_3"] = lanes(lambda H, a, w: H[2] if a else H[4])  # C4 / C2 of block 0: old H_e / H_c
    regs["e0_2"] = lanes(lambda H, a, w: H[3] if a else 0)     # a-feed-forward source for H_d
    regs["g1_1"] = lanes(lambda H, a, w: H[0] if a else 0)
    regs["g1_0"] = lanes(lambda H, a, w: H[1] if a else 0)
    regs["x0"] = lanes(lambda H, a, w: 0 if a else H[3] + H[7] + w)
    return regs


def extract(regs, p_last, chain=0, layout="quad"):
    """Final state of a chain after the drain (rounds 0-1 of a virtual block of parity
    1 - p_last)."""
    q = 1 - p_last
    el = chain if layout == "pair" else 0
    al = 7 - chain if layout == "pair" else 4
    e = [regs[f"e{p_last}_{i}"][el] for i in (3, 2, 1, 0)]
    a = [regs[f"g{q}_1"][al], regs[f"g{q}_0"][al], regs[f"e{p_last}_3"][al], regs[f"e{p_last}_2"][al]]
    return a + e


def simulate_chains(Hs, blocks, layout="quad"):
    """Run the generated schedule lane by lane over the chains of one half-row (1 for quad, 4 for
    pair; all with the same block count); return their final states."""
    nchains = 1 if layout == "quad" else 4
    wks = [schedule(b) for b in blocks]
    nb = len(wks[0])
    assert all(len(w) == nb for w in wks)
    regs = init_regs(Hs, [w[0][0] for w in wks], layout)

    def wreg(k, r):
        return [wks[lane_chain(i, layout)][k][r] if i < 4 else 1 for i in range(8)]
    for k in range(nb):
        p = k & 1
        for r in range(64):
            regs[f"w{r}"] = wreg(k, r)
        simulate_ops(rounds_ops(p, layout=layout), regs)
        regs["w0"] = wreg(k + 1, 0) if k + 1 < nb else [0] * 4 + [1] * 4
        simulate_ops(next_ops(p), regs)
    # drain: the a-half's last two rounds (+ its feed-forward) in a virtual block
    p = nb & 1
    regs["w1"] = regs["w2"] = [0] * 4 + [1] * 4
    simulate_ops(rounds_ops(p, 0, 2, layout), regs)
    return [extract(regs, 1 - p, c, layout) for c in range(nchains)]


def simulate_chain(H, blocks_words):
    """Quad layout, one chain."""
    return simulate_chains([H], [blocks_words])[0]


def ref_compress(H, blocks_words):
    H = list(H)
    for wk in schedule(blocks_words):
        a, b, c, d, e, f, g, h = H
        for t in range(64):
            t1 = (h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + wk[t]) & M32
            t2 = ((rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M32
            h, g, f, e, d, c, b, a = g, f, e, (d + t1) & M32, c, b, a, (t1 + t2) & M32
        H = [(x + y) & M32 for x, y in zip(H, [a, b, c, d, e, f, g, h])]
    return H


def pad_words(msg):
    ml = len(msg) * 8
    m = msg + b"\x80" + b"\x00" * ((55 - len(msg)) % 64) + struct.pack(">Q", ml)
    return [list(struct.unpack(">16I", m[i:i + 64])) for i in range(0, len(m), 64)]


# ----------------------------------------------------------------------------- hazards
DPP_OPS = ("xor1", "xor2", "p1", "ffe", "ffa", "adde", "adda")


def dpp_src(ins):
    """The VGPR a DPP instruction reads through the DPP lane network (its src0)."""
    return ins[2]


def dpp_hazards(ops, wait_states=2):
    """gfx9: a VALU write of a VGPR followed by a DPP read of it needs 2 wait states (other
    instructions).  Returns (index, instruction, distance) for every violation in `ops`."""
    bad = []
    for i, ins in enumerate(ops):
        if ins[0] not in DPP_OPS:
            continue
        src = dpp_src(ins)
        for d in range(1, wait_states + 1):
            if i - d >= 0 and ops[i - d][1] == src:
                bad.append((i, ins, d))
    return bad


def block_stream(p, layout="quad"):
    """Instruction order of one block of parity p followed by the next block's first rounds."""
    return rounds_ops(p, layout=layout) + next_ops(p) + rounds_ops(1 - p, 0, 4, layout)


# ----------------------------------------------------------------------------- asm emission
def asm_of(ins):
    op = ins[0]
    r = lambda n: "%[" + n + "]"   # noqa: E731
    if op == "align":
        return f"v_alignbit_b32 {r(ins[1])}, {r(ins[2])}, {r(ins[2])}, {r(ins[3])}"
    if op == "sel":
        return f"v_bitop3_b32 {r(ins[1])}, {r(ins[2])}, {r(ins[3])}, {r(ins[4])} bitop3:0xd2"
    if op == "bfi":
        return f"v_bfi_b32 {r(ins[1])}, {r(ins[2])}, {r(ins[3])}, {r(ins[4])}"
    if op == "xor3":
        return f"v_bitop3_b32 {r(ins[1])}, {r(ins[2])}, {r(ins[3])}, {r(ins[4])} bitop3:0x96"
    if op == "xor1":
        return (f"v_xor_b32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[2])} quad_perm:[1,2,0,1] "
                "row_mask:0xf bank_mask:0xf")
    if op == "xor2":
        return (f"v_xor_b32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[1])} quad_perm:[2,0,1,2] "
                "row_mask:0xf bank_mask:0xf")
    if op == "p1":
        return (f"v_add_u32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[3])} row_half_mirror "
                "row_mask:0xf bank_mask:0xf")
    if op == "p2":
        return f"v_xad_u32 {r(ins[1])}, {r(ins[2])}, {r(ins[3])}, {r(ins[4])}"
    if op == "add3":
        return f"v_add3_u32 {r(ins[1])}, {r(ins[2])}, {r(ins[3])}, {r(ins[4])}"
    if op in ("ffe", "ffa"):
        m = E_MASK if op == "ffe" else A_MASK
        return (f"v_add_u32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[1])} quad_perm:[0,1,2,3] "
                f"row_mask:0xf bank_mask:{m:#x}")
    if op == "adde":
        return (f"v_add_u32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[1])} row_half_mirror "
                f"row_mask:0xf bank_mask:{E_MASK:#x}")
    if op == "adda":
        return (f"v_add_u32_dpp {r(ins[1])}, {r(ins[2])}, {r(ins[1])} row_half_mirror "
                f"row_mask:0xf bank_mask:{A_MASK:#x}")
    raise ValueError(op)


SPLIT = 16  # rounds in the first asm statement of a block


def c_string(ops):
    return "\n".join(f'  "{asm_of(i)}\\n\\t"' for i in ops)


def emit_inc(path):
    out = ["// GENERATED by tools/gen_skew.py -- do not edit.  Skewed SHA-256 rounds: S3H_SKEW_*",
           "// lane-octet layout (8 VALU per round), S3H_SKEWP_* lane-pair layout (9 VALU per",
           "// round); see the generator's docstring for the schedule.", ""]
    for layout, tag in (("quad", "SKEW"), ("pair", "SKEWP")):
        for p in (0, 1):
            # split after round SPLIT-1: the next block's W+K reads are issued between the halves
            out.append(f"#define S3H_{tag}_ROUNDS_A_{p} \\")
            out.append(c_string(rounds_ops(p, 0, SPLIT, layout)).replace("\n", " \\\n"))
            out.append("")
            out.append(f"#define S3H_{tag}_ROUNDS_B_{p} \\")
            out.append(c_string(rounds_ops(p, SPLIT, 64, layout)).replace("\n", " \\\n"))
            out.append("")
            out.append(f"#define S3H_{tag}_NEXT_{p} \\")
            out.append(c_string(next_ops(p)).replace("\n", " \\\n"))
            out.append("")
            out.append(f"#define S3H_{tag}_DRAIN_{p} \\")
            out.append(c_string(rounds_ops(p, 0, 2, layout)).replace("\n", " \\\n"))
            out.append("")
    with open(path, "w") as f:
        f.write("\n".join(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "s3client_amd",
                                                  "csrc", "sha256_skew_rounds.inc"))
    ap.add_argument("--check", action="store_true", help="simulate vs the reference compression")
    a = ap.parse_args()
    if a.check:
        import hashlib
        import random
        rng = random.Random(1)
        for n in (0, 1, 55, 56, 64, 119, 120, 200, 1000):
            msg = bytes(rng.randrange(256) for _ in range(n))
            got = simulate_chain(IV, pad_words(msg))
            want = list(struct.unpack(">8I", hashlib.sha256(msg).digest()))
            print(n, "quad ok" if got == want else f"MISMATCH {got} {want}")
            msgs = [bytes(rng.randrange(256) for _ in range(n)) for _ in range(4)]
            got = simulate_chains([IV] * 4, [pad_words(m) for m in msgs], "pair")
            want = [list(struct.unpack(">8I", hashlib.sha256(m).digest())) for m in msgs]
            print(n, "pair ok" if got == want else "PAIR MISMATCH")
    emit_inc(a.out)
    for layout in ("quad", "pair"):
        n = len(rounds_ops(0, layout=layout)) + len(next_ops(0))
        print(f"{layout}: {n} VALU per block")
    print(f"wrote {a.out}")


if __name__ == "__main__":
    main()
