"""CPU checks of the skewed lane-octet SHA-256 schedule (tools/gen_skew.py), the instruction
stream that sha256_skew_kernel runs as inline asm: simulated lane by lane (DPP quad_perm,
row_half_mirror and bank masks included) it must reproduce SHA-256 bit-exactly across block
boundaries, from any chaining state; the committed .inc must be the generator's output; and
no DPP read may follow the VALU write of its source within 2 instructions."""
import hashlib
import os
import random
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_skew  # noqa: E402


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 119, 120, 127, 128, 200, 1000, 4096 + 7])
def test_schedule_matches_hashlib(n):
    rng = random.Random(n)
    msg = bytes(rng.randrange(256) for _ in range(n))
    got = gen_skew.simulate_chain(gen_skew.IV, gen_skew.pad_words(msg))
    assert got == list(struct.unpack(">8I", hashlib.sha256(msg).digest()))


@pytest.mark.parametrize("n", [0, 55, 56, 64, 200, 1000])
def test_pair_layout_four_chains(n):
    """Lane-pair layout: four independent chains per half-row (e-lane k, a-lane 7-k)."""
    rng = random.Random(100 + n)
    msgs = [bytes(rng.randrange(256) for _ in range(n)) for _ in range(4)]
    got = gen_skew.simulate_chains([gen_skew.IV] * 4, [gen_skew.pad_words(m) for m in msgs], "pair")
    assert got == [list(struct.unpack(">8I", hashlib.sha256(m).digest())) for m in msgs]


def test_schedule_from_arbitrary_state():
    """Resumed launches start from a loaded chaining state, not the IV."""
    rng = random.Random(5)
    for _ in range(5):
        H = [rng.getrandbits(32) for _ in range(8)]
        blocks = [[rng.getrandbits(32) for _ in range(16)] for _ in range(rng.randrange(1, 6))]
        assert gen_skew.simulate_chain(H, blocks) == gen_skew.ref_compress(H, blocks)


def test_instruction_counts():
    # 8 (quad) / 9 (pair) VALU per round; feed-forward (8) and boundary corrections (3) per block
    assert len(gen_skew.rounds_ops(0)) + len(gen_skew.next_ops(0)) == 64 * 8 + 11
    assert len(gen_skew.rounds_ops(0, layout="pair")) + len(gen_skew.next_ops(0)) == 64 * 9 + 11


@pytest.mark.parametrize("layout", ["quad", "pair"])
@pytest.mark.parametrize("p", [0, 1])
def test_no_dpp_hazards(p, layout):
    assert gen_skew.dpp_hazards(gen_skew.block_stream(p, layout)) == []
    assert gen_skew.dpp_hazards(gen_skew.rounds_ops(p, 0, 2, layout)) == []


def test_committed_inc_is_generated(tmp_path):
    out = tmp_path / "skew.inc"
    gen_skew.emit_inc(str(out))
    committed = os.path.join(ROOT, "s3client_amd", "csrc", "sha256_skew_rounds.inc")
    with open(committed) as f:
        assert f.read() == out.read_text()
