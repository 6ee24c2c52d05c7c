"""CPU checks of the shared-SIMD producer (tools/gen_producer.py), the asm statement that
sha256_skew_shared_kernel's producer wave runs per block: simulated on one lane, its W[t]+K[t]
drive a plain 64-round compression to hashlib's digest for multi-block messages; the
committed .inc is the generator's output; it uses only the instruction classes a SIMD
issues beside the consumer's round stream (no left shift, alignbit, perm, add3: those would
stall it -- profiles/r02_ubench_coissue_classes*.txt); and the kernel that runs it keeps f32
denormals, which its v_mul_f32 left shifts need."""
import hashlib
import os
import random
import re
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_producer  # noqa: E402

M32 = 0xFFFFFFFF
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _compress(h, wk):
    a, b, c, d, e, f, g, hh = h
    for t in range(64):
        t1 = (hh + (_rotr(e, 6) ^ _rotr(e, 11) ^ _rotr(e, 25)) + ((e & f) ^ (~e & g)) + wk[t]) & M32
        t2 = ((_rotr(a, 2) ^ _rotr(a, 13) ^ _rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M32
        a, b, c, d, e, f, g, hh = (t1 + t2) & M32, a, b, c, (d + t1) & M32, e, f, g
    return [(x + y) & M32 for x, y in zip(h, [a, b, c, d, e, f, g, hh])]


def _padded(msg):
    return msg + b"\x80" + b"\0" * ((55 - len(msg)) % 64) + struct.pack(">Q", 8 * len(msg))


@pytest.mark.parametrize("n,fill", [(0, None), (3, None), (55, None), (56, None), (64, None),
                                    (119, None), (200, None), (1000, None), (640, 0xFF),
                                    (640, 0x80), (640, 0x7F), (640, 0x01)])
def test_producer_drives_compression_to_hashlib(n, fill):
    """fill: constant bytes, the extremes of the masked denormal multiplies (mulf_ok asserts
    every product stays below 2^24)."""
    rng = random.Random(n)
    msg = bytes(rng.randrange(256) if fill is None else fill for _ in range(n))
    p = _padded(msg)
    h = IV
    for i in range(0, len(p), 64):
        blk = p[i:i + 64]
        le = [int.from_bytes(blk[4 * j:4 * j + 4], "little") for j in range(16)]  # as loaded
        out = gen_producer.simulate(le)
        assert len(out) == 64
        h = _compress(h, [out[(t // 4) * gen_producer.ROW + (t % 4) * 4] for t in range(64)])
    assert h == list(struct.unpack(">8I", hashlib.sha256(msg).digest()))


def test_committed_inc_is_generated(tmp_path):
    out = tmp_path / "p.inc"
    gen_producer.emit_inc(str(out))
    with open(os.path.join(ROOT, "s3client_amd", "csrc", "sha256_producer_simple.inc")) as f:
        assert f.read() == out.read_text()


def test_only_coissuable_instruction_classes():
    with open(os.path.join(ROOT, "s3client_amd", "csrc", "sha256_producer_simple.inc")) as f:
        ops = re.findall(r'"([a-z_0-9]+) ', f.read())
    allowed = {"v_add_u32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_lshrrev_b32", "v_bitop3_b32",
               "v_mul_f32", "ds_write_b32", "s_waitcnt"}
    assert set(ops) <= allowed, set(ops) - allowed
    # left shifts: one denormal v_mul_f32 + doublings (v_add_u32 x, x) each
    assert ops.count("v_mul_f32") == 93 and ops.count("ds_write_b32") == 64
    assert 2100 < len(ops) - 65 < 2300


def test_shared_kernel_keeps_f32_denormals():
    """v_mul_f32 on a denormal bit pattern is a left shift only if f32 denormals are neither
    flushed on input nor on output: .amdhsa_float_denorm_mode_32 3 in the built code object."""
    s_file = os.path.join(ROOT, "build", "isa", "capi-hip-amdgcn-amd-amdhsa-gfx950.s")
    if not os.path.exists(s_file):
        pytest.skip("no build/isa (make builds it)")
    text = open(s_file).read()
    m = re.search(r"\.amdhsa_kernel _ZN3s3h25sha256_skew_shared_kernel\w*\n(.*?)\.end_amdhsa_kernel", text, re.S)
    assert m, "skews kernel descriptor not found"
    assert re.search(r"\.amdhsa_float_denorm_mode_32 3\b", m.group(1))


@pytest.mark.parametrize("variant", [{"perm": True}, {"lds": True}, {"mulf": False, "merge3": False},
                                     {"perm": True, "mulf": False, "merge3": False},
                                     {"lds": True, "mulf": False, "merge3": False},
                                     {"zyv": True}, {"zyv": "plain"}])
def test_experiment_variants_compute_the_same_schedule(variant):
    """The v_perm and LDS-pipe byte-swap variants, the doublings-only first version
    (experiments, profiles/r02_exp_producer_*) and the byte swap from unaligned in-block loads
    (--zyv / --zyv-plain, profiles/r05_exp_producer_zyv.jsonl; the simulator forms the loads'
    values from the block's bytes, gen_producer.zyv_inputs)."""
    rng = random.Random(9)
    for _ in range(10):
        blk = bytes(rng.randrange(256) for _ in range(64))
        le = [int.from_bytes(blk[4 * j:4 * j + 4], "little") for j in range(16)]
        out = gen_producer.simulate(le, **variant)
        assert [out[gen_producer.wk_offset(t)] for t in range(64)] == gen_producer.reference_wk(blk)


def test_zyv_loads_stay_inside_the_block():
    """The --zyv statement's loads (kernel fetch_zy: bytes 1..60 and 3..62 of the block) are the
    values zyv_inputs forms from the block's own bytes: no byte before or after it is read."""
    blk = bytes(range(64))
    le = [int.from_bytes(blk[4 * j:4 * j + 4], "little") for j in range(16)]
    regs = gen_producer.zyv_inputs(le)
    for k in range(15):
        assert regs[gen_producer.ZR[k]] == int.from_bytes(blk[4 * k + 1:4 * k + 5], "little")
    for j in range(1, 16):
        assert regs[gen_producer.YR[j - 1]] == int.from_bytes(blk[4 * j - 1:4 * j + 3], "little")
