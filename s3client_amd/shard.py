"""Multi-GPU sharding of upload parts.

Parts are independent SHA-256 chains, so a batch shards with NO collective on the data path:
global part p goes to rank (device) p % world, local slot p // world; every rank hashes only
bytes in its own HBM and writes 32 B per part.  The only cross-rank traffic is timing (a
barrier and a max-reduction in bench.py) and, when a caller wants one digest list on one
host, an all-gather of the 32-byte digests (``gather_digests``; 32 B per part, verification
and reporting only -- xGMI stays idle while hashing).
"""
from __future__ import annotations

import numpy as np


def shard_ids(n_total: int, rank: int, world: int) -> np.ndarray:
    """Global part ids owned by ``rank``: p % world == rank, in increasing order."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return np.arange(rank, n_total, world, dtype=np.uint64)


def pack_offsets(lengths, align: int = 256) -> np.ndarray:
    """Offsets of parts packed back to back in one HBM buffer, each `align`-byte aligned."""
    lens = np.asarray(lengths, dtype=np.uint64)
    if lens.size == 0:
        return lens
    padded = (lens + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    return np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.uint64)


def gather_digests(local: np.ndarray, ids: np.ndarray, n_total: int, group=None) -> np.ndarray:
    """Reassemble the (n_total, 8) uint32 digest table from every rank's shard."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, (np.asarray(ids, dtype=np.uint64),
                                   np.asarray(local, dtype=np.uint32)), group=group)
    out = np.zeros((n_total, 8), dtype=np.uint32)
    seen = np.zeros(n_total, dtype=bool)
    for pid, dig in parts:
        out[pid.astype(np.int64)] = dig
        seen[pid.astype(np.int64)] = True
    if not seen.all():
        raise RuntimeError("some parts were not hashed by any rank")
    return out
