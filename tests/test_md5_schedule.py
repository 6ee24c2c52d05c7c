"""CPU checks of the MD5 consumer's fused step (tools/gen_md5.py), the asm statements that
s3client_amd/csrc/md5_step_asm.inc holds (the chunked form and the rolling form the product
runs): executed lane by lane against hashlib's MD5, with every LDS read landing only at its
counted wait, and the committed .inc equal to the generator's."""
import hashlib
import os
import random
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_md5  # noqa: E402

IV = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476]


def _padded_blocks(msg: bytes) -> list[bytes]:
    m = msg + b"\x80" + b"\0" * ((55 - len(msg)) % 64) + struct.pack("<Q", 8 * len(msg))
    return [m[i:i + 64] for i in range(0, len(m), 64)]


@pytest.mark.parametrize("roll", [False, True])
@pytest.mark.parametrize("bps", [1, 2, 4])
def test_fused_step_matches_hashlib(bps, roll):
    if roll and bps == 1:
        pytest.skip("the rolling step is generated for 2 and 4 blocks")
    rng = random.Random(bps)
    for n in (55, 64 * bps - 9, 64 * 3 * bps - 9, 64 * 2 * bps + 7):
        msg = bytes(rng.getrandbits(8) for _ in range(n))
        blocks = _padded_blocks(msg)
        blocks += [None] * (-len(blocks) % bps)  # pad the last step (not hashed, see below)
        st = list(IV)
        for j in range(0, len(blocks), bps):
            step = blocks[j:j + bps]
            if None in step:
                # the kernel's last partial step runs the checked per-block path; here a step
                # of only the real blocks (a 1-block step is the same statement for bps 1)
                for b in (b for b in step if b is not None):
                    st = gen_md5.simulate_step(st, [b])
            else:
                st = gen_md5.simulate_step(st, step, roll=roll)
        assert struct.pack("<4I", *st) == hashlib.md5(msg).digest(), (bps, n, roll)


def test_reads_never_used_or_overwritten_in_flight():
    ops = gen_md5.step_text(4)
    regs = {f"%[s{q}]": 0 for q in range(4)}
    regs["%[ad]"] = 0
    lds = gen_md5.lds_image([bytes(64)] * 4, 0)
    # drop one wait: the simulator must catch the row used before it landed
    i = next(k for k, op in enumerate(ops) if op.startswith("s_waitcnt"))
    with pytest.raises(AssertionError, match="read before"):
        gen_md5.simulate(ops[:i] + ops[i + 1:], dict(regs, **{f"v{gen_md5.PIN0 + q}": 0 for q in range(8)}), lds)


@pytest.mark.parametrize("k", [0, 1, 4, -1])
def test_rolling_waits_are_exact(k):
    """Loosen any one counted wait by one: some row is then read before it landed."""
    ops = gen_md5.roll_text(4)
    regs = {f"%[s{q}]": 0 for q in range(4)}
    regs["%[ad]"] = 0
    lds = gen_md5.lds_image([bytes(64)] * 4, 0)
    waits = [i for i, op in enumerate(ops) if op.startswith("s_waitcnt")]
    i = waits[k]
    n = int(ops[i].split("(")[1].rstrip(")"))
    loose = ops[:i] + [f"s_waitcnt lgkmcnt({n + 1})"] + ops[i + 1:]
    with pytest.raises(AssertionError, match="read before"):
        gen_md5.simulate(loose, regs, lds)


def test_rolling_statement_shape():
    for bps in (2, 4):
        ops = gen_md5.roll_text(bps)
        assert sum(o.startswith("v_") for o in ops) == bps * (256 + 4)
        assert sum(o.startswith("ds_read_b128") for o in ops) == bps * 16
        # waits: the step's first row, rows 1..W-1, then every W rows
        assert sum(o.startswith("s_waitcnt") for o in ops) == 2 + (bps * 16 - 1) // gen_md5.ROLL_WAIT
        small = [o.startswith(("s_waitcnt", "v_add_u32_e32", "s_nop")) for o in ops]
        assert sum(small) % 2 == 0
        for k, o in enumerate(ops):
            if o.startswith("s_waitcnt"):
                assert ops[k + 1].startswith(("v_add_u32_e32", "s_nop"))
        regs = {int(o.split("v[")[1].split(":")[0]) for o in ops if o.startswith("ds_read")}
        assert regs <= {int(c[1:]) for c in gen_md5.ROLL_CLOBBERS[::4]}


def test_statement_shape():
    for bps in (1, 2, 4):
        ops = gen_md5.step_text(bps)
        valu = [o for o in ops if o.startswith("v_")]
        assert len(valu) == bps * (256 + 4)
        assert sum(o.startswith("ds_read_b128") for o in ops) == bps * 16 - 2
        assert sum(o.startswith("s_waitcnt") for o in ops) == bps * 4
        # 8-byte alignment: every 4-byte instruction (the wait, the VOP2 add) comes in a pair
        small = [o.startswith(("s_waitcnt", "v_add_u32_e32")) for o in ops]
        assert sum(small) % 2 == 0
        for k, s in enumerate(small):
            if ops[k].startswith("s_waitcnt"):
                assert ops[k + 1].startswith("v_add_u32_e32")
        offs = [int(o.rsplit(":", 1)[1]) for o in ops if o.startswith("ds_read")]
        assert max(offs) < 65536


def test_inc_is_current(tmp_path):
    out = tmp_path / "md5_step_asm.inc"
    gen_md5.emit_inc(str(out))
    with open(os.path.join(ROOT, "s3client_amd", "csrc", "md5_step_asm.inc")) as f:
        assert f.read() == out.read_text()
