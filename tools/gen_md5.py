#!/usr/bin/env python3
"""Generator (and lane-level simulator) of the MD5 consumer's fused step: the kBps blocks of one
producer step in ONE inline-asm statement (s3client_amd/csrc/md5_step_asm.inc).

Why one statement.  With one statement per 8-16 MD5 steps (round 3's md5_block_streamed) the
compiler puts, at every statement boundary, one wait state (it assumes an asm statement's
outputs may carry gfx950's dst-forwarding hazard into the next statement that reads them) and
then an alignment s_nop to bring the next statement back to 8 bytes: 9.5 s_nop per block, 3 %
of the loop.  The operand limit (30 per statement) is what kept statements short: 16 M+K
words of a block as separate operands.  Here the rows live in FIXED registers the statement
clobbers (they never leave it), so a whole step needs only the state, the temporaries, the
LDS address and the block's first two rows:

    operands  s0..s3 (+v: chaining state, fed forward in the statement), a, b, c, d, f, t
              (=&v), ad (v: LDS byte address of this lane's row 0 of block 0 of the step),
              rows 0-1 of block 0 pinned to v[232:235], v[236:239] (+: loaded by the compiler
              after the step's barrier; each block's fourth chunk reads the NEXT block's rows
              0-1 into the same registers)
    clobbers  v[200:231]: ring A = v[200:215] (rows 2-5, then 10-13), ring B = v[216:231]
              (rows 6-9, then 14-15)

Per block: five chunks of steps 0-7 | 8-23 | 24-39 | 40-55 | 56-63; every chunk first issues
the ds_read_b128 of the rows the NEXT chunk needs and waits for them (s_waitcnt lgkmcnt(0))
before its own last add, so no row is in flight at a chunk boundary and none at the end of the
statement.  Every instruction is 8 bytes (VOP3 adds) except the wait + VOP2 add pair that ends
a chunk, so the statement stays 8-byte aligned throughout.  Row r of block h is at LDS byte
offset h*16384 + r*1024 from `ad` (Md5Lds: uint4 km[2][kBps][16][64]); 3*16384 + 15*1024 =
64,512 fits the 16-bit DS offset.

`simulate()` executes the emitted text for one lane (register file + LDS image, reads landing
only at a wait -- a register read before its wait is an error) so tests/test_md5_schedule.py
checks the generated statement against hashlib's MD5 on the CPU.

    python tools/gen_md5.py [OUT.inc]
"""
from __future__ import annotations

import os
import re
import struct
import sys

BLOCK_BYTES = 16384          # one block's 16 rows x 64 lanes x 16 B in Md5Lds
ROW_BYTES = 1024
RING_A = 200                 # rows 2-5 / 10-13
RING_B = 216                 # rows 6-9 / 14-15
PIN0, PIN1 = 232, 236        # rows 0 and 1 (operands)
CLOBBERS = [f"v{r}" for r in range(RING_A, RING_B + 16)]
# round function (bitop3 truth table over b, c, d) and alignbit amounts (32 - s)
ROUNDS = [(0xca, (25, 20, 15, 10)),   # F = b ? c : d
          (0xe4, (27, 23, 18, 12)),   # G = d ? b : c
          (0x96, (28, 21, 16, 9)),    # H = b ^ c ^ d
          (0x39, (26, 22, 17, 11))]   # I = c ^ (b | ~d)
CHUNKS = [(0, 8), (8, 24), (24, 40), (40, 56), (56, 64)]


def row_reg(r: int) -> int:
    """First VGPR of row r (4 consecutive registers: steps 4r..4r+3)."""
    if r == 0:
        return PIN0
    if r == 1:
        return PIN1
    if 2 <= r <= 5:
        return RING_A + 4 * (r - 2)
    if 6 <= r <= 9:
        return RING_B + 4 * (r - 6)
    if 10 <= r <= 13:
        return RING_A + 4 * (r - 10)
    return RING_B + 4 * (r - 14)


def chunk_reads(c: int, h: int, nxt: bool) -> list[tuple[int, int]]:
    """(first VGPR, LDS offset) of the rows chunk c issues (for the chunk after it)."""
    rows = [[2, 3, 4, 5], [6, 7, 8, 9], [10, 11, 12, 13], [14, 15], []][c]
    out = [(row_reg(r), h * BLOCK_BYTES + r * ROW_BYTES) for r in rows]
    if c == 3 and nxt:
        out += [(PIN0, (h + 1) * BLOCK_BYTES), (PIN1, (h + 1) * BLOCK_BYTES + ROW_BYTES)]
    return out


def step_ops(i: int, wait: bool) -> list[str]:
    ops = step_ops_k(i, f"v{row_reg(i // 4) + i % 4}")
    if wait:
        ops[3:] = ["s_waitcnt lgkmcnt(0)", ops[3].replace("_e64", "_e32")]
    return ops


def step_ops_k(i: int, k: str) -> list[str]:
    """MD5 step i: f = F(b,c,d); t = a + f + (M+K)[i]; t = rotl(t, s); a = b + t.  The names
    rotate (a,b,c,d) -> (d,a,b,c) each step; steps 0-3 read the block-start state s0..s3 and
    write fresh a..d (so s0..s3 survive for the feed-forward)."""
    tt, rot = ROUNDS[i // 16]
    names = "abcd"
    if i < 4:
        # live value of each name before step i: s-registers until written
        cur = {"a": "%[s0]", "b": "%[s1]", "c": "%[s2]", "d": "%[s3]"}
        for j in range(i):
            cur[names[(4 - j) % 4]] = f"%[{names[(4 - j) % 4]}]"
        A, B, C, D = (cur[names[(4 - i + q) % 4]] for q in range(4))
        out = f"%[{names[(4 - i) % 4]}]"
    else:
        A, B, C, D = (f"%[{names[(4 - i + q) % 4]}]" for q in range(4))
        out = A
    return [f"v_bitop3_b32 %[f], {B}, {C}, {D} bitop3:0x{tt:02x}",
            f"v_add3_u32 %[t], {A}, %[f], {k}",
            f"v_alignbit_b32 %[t], %[t], %[t], {rot[i % 4]}",
            f"v_add_u32_e64 {out}, {B}, %[t]"]


def block_ops(h: int, nxt: bool) -> list[str]:
    ops = []
    for c, (lo, hi) in enumerate(CHUNKS):
        reads = chunk_reads(c, h, nxt)
        ops += [f"ds_read_b128 v[{r}:{r + 3}], %[ad] offset:{off}" for r, off in reads]
        for i in range(lo, hi):
            ops += step_ops(i, wait=bool(reads) and i == hi - 1)
    ops += [f"v_add_u32_e64 %[s{q}], %[s{q}], %[{n}]" for q, n in enumerate("abcd")]
    return ops


def step_text(bps: int) -> list[str]:
    ops = []
    for h in range(bps):
        ops += block_ops(h, h + 1 < bps)
    return ops


# ----------------------------------------------------------------------------- rolling schedule
# Round 3 (later): the chunked statement above waits at the end of every chunk for ALL the rows
# it issued; chunk 0's rows 2-5 have only steps 0-7 (~130 cycles) to land, and the chunked
# reads leave nothing in flight at a block boundary.  The rolling statement keeps ROLL_DEPTH
# rows in flight: row g (counting rows over the whole step, 16 per block) is read into slot
# g % (ROLL_DEPTH + 1) when row g - ROLL_DEPTH starts, and a counted `s_waitcnt lgkmcnt(n)`
# (LDS reads of one wave return in order) before every ROLL_WAIT-th row lands the next
# ROLL_WAIT rows, each read >= ROLL_DEPTH - ROLL_WAIT + 1 rows (>= 20 steps) earlier.  Only the
# step's first row waits a whole LDS latency (the producer writes the step's buffer before
# the barrier).  Depth 12 / a wait every 8 rows was the best of eight shapes measured
# (profiles/r03_exp_md5_roll.jsonl: waits cost issue slots, short leads cost stalls):
# C2 1,278-1,286 -> 1,246 cycles per block (114.2 -> 116.8-117.1 GiB/s), C4 shard 815 -> 845.
ROLL_DEPTH = int(os.environ.get("S3H_GEN_ROLL_DEPTH", 12))  # (env: experiment builds only)
ROLL_WAIT = int(os.environ.get("S3H_GEN_ROLL_WAIT", 8))
ROLL_BASE = min(200, 256 - 4 * (ROLL_DEPTH + 1))  # the ring ends at or below v255
ROLL_CLOBBERS = [f"v{r}" for r in range(ROLL_BASE, ROLL_BASE + 4 * (ROLL_DEPTH + 1))]


def roll_text(bps: int, depth: int = ROLL_DEPTH, wait: int = ROLL_WAIT) -> list[str]:
    total = 16 * bps
    slots = depth + 1
    assert 1 <= wait <= depth <= 15

    def reg(g: int) -> int:
        return ROLL_BASE + 4 * (g % slots)

    def read(g: int) -> str:
        off = (g // 16) * BLOCK_BYTES + (g % 16) * ROW_BYTES
        return f"ds_read_b128 v[{reg(g)}:{reg(g) + 3}], %[ad] offset:{off}"

    def land(b: int) -> str | None:
        """The wait before row b, or None: rows below `upto` must have landed, and the
        reads issued so far are rows below min(b + depth, total) (in order)."""
        if b == 0:
            upto = 1
        elif b == 1 or b % wait == 0:
            upto = min(total, (b // wait + 1) * wait)
        else:
            return None
        return f"s_waitcnt lgkmcnt({min(b + depth, total) - upto})"

    ops = [read(g) for g in range(min(depth, total))]
    ops += [land(0), "s_nop 0"]  # 4 + 4 bytes: the statement stays 8-byte aligned
    ops = _exp(ops + _roll_body(bps, depth, total, read, land, reg))
    return ops


def _exp(ops: list[str]) -> list[str]:
    """Timing-only experiment variants (S3H_GEN_EXP; wrong digests, never the product):
    nowait0 -- the step's first wait removed; nolds -- every ds_read_b128 becomes an 8-byte
    v_mov_b32_e64 of its first register (one issue slot, no LDS traffic) and every wait an
    s_nop 0."""
    mode = os.environ.get("S3H_GEN_EXP", "")
    if mode == "vmem":
        # rows from global memory instead of LDS (timing only): row g of the step is at byte
        # g * 1024 of a per-workgroup region; base %[sb<g//4>] (SGPR pair) + lane offset
        # %[voff] + immediate (g % 4) * 1024 (the 13-bit signed immediate holds < 4 KiB)
        out = []
        for o in ops:
            if o.startswith("ds_read"):
                reg = o.split(" ")[1].rstrip(",")
                off = int(o.rsplit(":", 1)[1])
                g = (off // BLOCK_BYTES) * 16 + (off % BLOCK_BYTES) // ROW_BYTES
                out.append(f"global_load_dwordx4 {reg}, %[voff], %[sb{g // 4}] offset:{(g % 4) * 1024}")
            elif o.startswith("s_waitcnt lgkmcnt"):
                out.append(o.replace("lgkmcnt", "vmcnt"))
            else:
                out.append(o)
        return out
    if mode == "nowait0":
        i = next(k for k, o in enumerate(ops) if o.startswith("s_waitcnt"))
        return ops[:i] + ["s_nop 0"] + ops[i + 1:]
    if mode == "nolds":
        out = []
        for o in ops:
            if o.startswith("ds_read"):
                out.append(f"v_mov_b32_e64 v{o.split('v[')[1].split(':')[0]}, 0")
            elif o.startswith("s_waitcnt"):
                out.append("s_nop 0")
            else:
                out.append(o)
        return out
    return ops


def _roll_body(bps, depth, total, read, land, reg) -> list[str]:
    ops = []
    for h in range(bps):
        for i in range(64):
            g = 16 * h + i // 4
            if i % 4 == 0 and g + depth < total:
                ops.append(read(g + depth))
            step = step_ops_k(i, f"v{reg(g) + i % 4}")
            w = land(g + 1) if i % 4 == 3 and i < 63 else None
            # a wait goes before the step's last add, re-encoded as 4-byte VOP2 (pairs of 4 B)
            ops += step if w is None else step[:3] + [w, step[3].replace("_e64", "_e32")]
        ff = [f"v_add_u32_e64 %[s{q}], %[s{q}], %[{n}]" for q, n in enumerate("abcd")]
        w = land(16 * (h + 1)) if h + 1 < bps else None
        ops += ff if w is None else ff[:3] + [w, ff[3].replace("_e64", "_e32")]
    return ops


def emit_inc(path: str) -> None:
    lines = ["// Generated by tools/gen_md5.py -- do not edit.  The MD5 consumer's fused step: all",
             "// kBps blocks of one producer step in one asm statement (rows in fixed registers; see",
             "// the generator's docstring for the register map and the chunk schedule).",
             f"#define S3H_MD5_STEP_CLOBBERS {', '.join(chr(34) + c + chr(34) for c in CLOBBERS)}"]
    for bps in (2, 4):  # (md5_pc_kernel<1> keeps the per-block statements: occupancy)
        ops = step_text(bps)
        lines.append(f"#define S3H_MD5_STEP_ASM_{bps} \\")
        lines += [f'  "{op}\\n\\t" \\' for op in ops]
        lines.append('  ""')
    if os.environ.get("S3H_GEN_EXP") == "vmem":
        lines.append("#define S3H_MD5_VMEM 1")
    lines.append(f"#define S3H_MD5_ROLL_CLOBBERS {', '.join(chr(34) + c + chr(34) for c in ROLL_CLOBBERS)}")
    for bps in (2, 4):
        lines.append(f"#define S3H_MD5_ROLL_ASM_{bps} \\")
        lines += [f'  "{op}\\n\\t" \\' for op in roll_text(bps)]
        lines.append('  ""')
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


# ----------------------------------------------------------------------------- simulator
M32 = 0xFFFFFFFF


def _bitop3(tt: int, x: int, y: int, z: int) -> int:
    r = 0
    for bit in range(32):
        idx = (((x >> bit) & 1) << 2) | (((y >> bit) & 1) << 1) | ((z >> bit) & 1)
        r |= ((tt >> idx) & 1) << bit
    return r


def simulate(ops: list[str], regs: dict[str, int], lds: dict[int, int]) -> dict[str, int]:
    """Execute `ops` for one lane.  `regs`: named operands ('%[s0]', '%[ad]', ...) and 'vN'
    registers; `lds`: byte address -> 32-bit word.  A ds_read lands at the next
    s_waitcnt lgkmcnt(n) that leaves at most n newer reads in flight: reading or overwriting one of its registers before that is an error,
    as is a read still in flight at the end."""
    regs = dict(regs)
    pending: dict[str, int] = {}
    fifo: list[list[str]] = []  # registers of each read in flight, oldest first

    def get(x: str) -> int:
        x = x.strip()
        if x in pending:
            raise AssertionError(f"register {x} read before its LDS read was waited for")
        if re.fullmatch(r"-?\d+", x):
            return int(x) & M32
        return regs[x]

    def put(x: str, v: int) -> None:
        if x in pending:
            raise AssertionError(f"register {x} written while an LDS read into it is in flight")
        regs[x] = v & M32

    for op in ops:
        m = re.match(r"(\S+)\s+(.*)$", op)
        name, rest = m.group(1), m.group(2)
        if name == "s_waitcnt":
            n = int(re.fullmatch(r"lgkmcnt\((\d+)\)", rest).group(1))
            assert n <= 15, "lgkmcnt is a 4-bit counter"
            while len(fifo) > n:  # LDS reads of one wave return in order
                for reg in fifo.pop(0):
                    regs[reg] = pending.pop(reg)
            continue
        if name == "s_nop":
            continue
        if name == "ds_read_b128":
            mm = re.fullmatch(r"v\[(\d+):(\d+)\], (\S+) offset:(\d+)", rest)
            r0, r1, adr, off = int(mm.group(1)), int(mm.group(2)), mm.group(3), int(mm.group(4))
            assert r1 == r0 + 3 and off < 65536
            base = get(adr) + off
            for q in range(4):
                reg = f"v{r0 + q}"
                if reg in pending:
                    raise AssertionError(f"two LDS reads in flight into {reg}")
                pending[reg] = lds[base + 4 * q]
            fifo.append([f"v{r0 + q}" for q in range(4)])
            assert len(fifo) <= 15, "more LDS reads in flight than lgkmcnt can count"
            continue
        tt = None
        if " bitop3:" in rest:
            rest, t = rest.split(" bitop3:")
            tt = int(t, 16)
        args = [a.strip() for a in rest.split(",")]
        d, src = args[0], args[1:]
        if name == "v_bitop3_b32":
            put(d, _bitop3(tt, get(src[0]), get(src[1]), get(src[2])))
        elif name == "v_add3_u32":
            put(d, get(src[0]) + get(src[1]) + get(src[2]))
        elif name == "v_alignbit_b32":
            s = get(src[2]) & 31
            put(d, ((get(src[0]) << 32 | get(src[1])) >> s))
        elif name in ("v_add_u32_e32", "v_add_u32_e64"):
            put(d, get(src[0]) + get(src[1]))
        else:
            raise AssertionError(f"unexpected instruction {op}")
    assert not pending, f"LDS reads in flight at the end: {sorted(pending)}"
    return regs


def md5_mk_rows(block: bytes) -> list[int]:
    """The 64 words the producer writes for one block: M[g(i)] + K[i] (RFC 1321 order)."""
    import math
    m = struct.unpack("<16I", block)
    out = []
    for i in range(64):
        g = [i, (5 * i + 1) % 16, (3 * i + 5) % 16, (7 * i) % 16][i // 16]
        out.append((m[g] + int(abs(math.sin(i + 1)) * 2 ** 32)) & M32)
    return out


def lds_image(blocks: list[bytes], ad: int) -> dict[int, int]:
    lds = {}
    for h, blk in enumerate(blocks):
        mk = md5_mk_rows(blk)
        for i in range(64):
            lds[ad + h * BLOCK_BYTES + (i // 4) * ROW_BYTES + 4 * (i % 4)] = mk[i]
    return lds


def simulate_step(state: list[int], blocks: list[bytes], ad: int = 0x400,
                  roll: bool = False) -> list[int]:
    """MD5 state after the fused step over len(blocks) whole blocks (as the kernel runs it:
    chunked -- rows 0-1 of block 0 in the pinned registers before the statement; rolling --
    the statement reads every row itself)."""
    lds = lds_image(blocks, ad)
    regs = {f"%[s{q}]": state[q] for q in range(4)}
    regs["%[ad]"] = ad
    if roll:
        out = simulate(roll_text(len(blocks)), regs, lds)
        return [out[f"%[s{q}]"] for q in range(4)]
    for q in range(4):
        regs[f"v{PIN0 + q}"] = lds[ad + 4 * q]
        regs[f"v{PIN1 + q}"] = lds[ad + ROW_BYTES + 4 * q]
    out = simulate(step_text(len(blocks)), regs, lds)
    return [out[f"%[s{q}]"] for q in range(4)]


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    emit_inc(sys.argv[1] if len(sys.argv) > 1 else
             os.path.join(here, "..", "s3client_amd", "csrc", "md5_step_asm.inc"))
