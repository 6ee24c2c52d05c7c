"""Host-side plan rules that need no GPU (s3h_dual_layout): which form of the SHA-256 + MD5
mixed grid a batch gets (capi.hip dual_mixed_solo)."""
import numpy as np

import s3client_amd as s3

L0 = 64 * 1024


def test_mixed_grid_forms():
    rng = np.random.default_rng(5)
    # C3-like ragged batches: the apart form while its grid fits 256 CUs, round 3's beyond
    F, apart = s3.dual_layout(5 * 1024 + rng.integers(0, 59 * 1024 + 1, 3000))
    assert F > 0 and apart
    F, apart = s3.dual_layout(5 * 1024 + rng.integers(0, 59 * 1024 + 1, 5500))
    assert F > 0 and not apart
    # fewer CUs: the same batch no longer fits the apart grid
    F1, a1 = s3.dual_layout(5 * 1024 + rng.integers(0, 59 * 1024 + 1, 3000), cus=120)
    assert not a1


def test_lengths_between_the_two_ratios_keep_a_mixed_grid():
    """Every part within 2650/2224 of the longest but some within 2650/2280 (the planning rates,
    exp_config.hpp): the apart form would need a skew group for every part, round 3's form needs
    one (advisor r4: the loop returned 0 instead of trying the smaller ratio)."""
    lens = [L0] + [int(L0 * 0.85)] * 2099
    assert s3.dual_layout(lens) == (1, False)


def test_no_mixed_grid():
    assert s3.dual_layout([L0] * 3000) == (0, False)              # equal lengths
    assert s3.dual_layout([L0] * 2000) == (0, False)              # below the group range
    assert s3.dual_layout([L0] * 9000, cus=256) == (0, False)     # beyond 32 x CUs parts
