"""XCD-class chain mapping of the cross-workgroup MD5 pacing experiment (S3H_EXP_MD5_XCD_PACE;
sha256_kernels.hip XcdChains, kernel_abi.hpp mixed_lead_wgs / split_md5_wgs), restated: the
MD5 workgroups of a dual grid must cover every slot of the skew groups exactly once, each
workgroup's chains must come from skew groups on its own XCD class (blockIdx mod 8), and each
wave's valid chains must ascend in slot order (lane 0 the longest part, as the kernel's
fast-loop bounds assume).  Pure arithmetic: runs on the CPU."""
import pytest


def slot_of(xcls, c0, i):
    c = c0 + i
    return 8 * (xcls + 8 * (c >> 3)) + (c & 7)


def count(xcls, c0, ngroups, n):
    in_cls = (ngroups - xcls + 7) // 8 if ngroups > xcls else 0
    first = c0 >> 3
    if in_cls <= first:
        return 0
    k = min(in_cls - first, 8)
    end = slot_of(xcls, c0, 8 * k - 1) + 1
    return 8 * k if end <= n else 8 * k - (end - n)


def md5_wgs(ngroups):
    return 8 * ((ngroups + 63) // 64)


@pytest.mark.parametrize("ngroups,n,first_block", [
    (1, 1, 1), (1, 8, 1), (7, 50, 7), (73, 4096, 183), (128, 1024, 128), (128, 1020, 128),
    (200, 1597, 200), (224, 1792, 224), (256, 2048, 256)])
def test_md5_workgroups_cover_the_skew_slots_once(ngroups, n, first_block):
    """first_block: blockIdx of the first MD5 workgroup (F + G in the mixed grid, sha_grid in
    the split grid): its class decides which skew groups each MD5 workgroup takes."""
    seen = []
    for w in range(md5_wgs(ngroups)):
        b = first_block + w
        xcls, c0 = b & 7, 64 * (w >> 3)
        nv = count(xcls, c0, ngroups, min(n, 8 * ngroups))
        slots = [slot_of(xcls, c0, i) for i in range(nv)]
        assert slots == sorted(slots)
        for s in slots:
            assert (s // 8) % 8 == b % 8, (w, s)  # the skew group shares this workgroup's XCD
            assert s // 8 < ngroups and s < n
        seen += slots
    assert sorted(seen) == list(range(min(n, 8 * ngroups)))
