"""Game sharding across ranks (one process per GPU) and the result gather.

Games are independent and every per-game seed is a pure function of (run seed, game
index) (analytics/tournament/arena_runner.py:241-254), so rank r of W plays the games
with index == r (mod W) (configs 4 and 5: a fixed job split over the ranks) or the
contiguous block r (config 3: each rank adds its own block of games, weak scaling), and
the only collective is one gather of fixed-size 32-byte bk_result records at the end
(SURVEY 8e).  On GPUs the process group is RCCL
(backend "nccl"); the same code runs on gloo over CPU tensors in the tests.
"""
from __future__ import annotations

import numpy as np

RESULT_BYTES = 32


def shard_indices(n_total: int, rank: int, world: int) -> np.ndarray:
    """Global game indices owned by `rank`: rank, rank + W, rank + 2W, ..."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return np.arange(rank, n_total, world, dtype=np.int64)


def gather_results(local, n_total: int, rank: int, world: int, dist, device=None):
    """All-gather every rank's result records (uint8 [n_local, 32], torch tensor) and
    return them in global game order as a torch uint8 tensor [n_total, 32] on `device`.
    Ranks own index == rank (mod W), so shard sizes differ by at most one: pad to the
    largest, gather, then interleave."""
    import torch
    per = (n_total + world - 1) // world
    buf = torch.zeros((per, RESULT_BYTES), dtype=torch.uint8, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = torch.empty((n_total, RESULT_BYTES), dtype=torch.uint8, device=device or local.device)
    for r in range(world):
        idx = shard_indices(n_total, r, world)
        out[torch.from_numpy(idx).to(out.device)] = parts[r][: len(idx)].to(out.device)
    return out


def gather_blocks(local, rank: int, world: int, dist, device=None):
    """All-gather equal-sized contiguous blocks (rank r holds global records r * n ..
    (r + 1) * n - 1, uint8 [n, 32] torch tensor) and return them in global order,
    uint8 [world * n, 32] on `device`."""
    import torch
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous())
    return torch.cat([p.to(device or local.device) for p in parts], dim=0)


def check_indices(local_ids, n_total: int, world: int, dist):
    """Every global index 0..n_total-1 arrived from exactly one rank: all-gather each
    rank's index list (after the timed region) and count.  Returns, on every rank,
    {"indices": n_total, "every_index_once": bool, "missing": k, "duplicates": k}."""
    ids = [int(i) for i in np.asarray(local_ids, dtype=np.int64).ravel()]
    parts = [None] * world
    if dist is not None:
        dist.all_gather_object(parts, ids)
    else:
        parts = [ids]
    allv = np.concatenate([np.asarray(p, dtype=np.int64) for p in parts]) if parts else np.zeros(0, np.int64)
    inside = allv[(allv >= 0) & (allv < n_total)]
    cnt = np.bincount(inside, minlength=n_total)
    missing = int((cnt == 0).sum())
    dup = int((cnt > 1).sum()) + int(len(allv) - len(inside))
    return {"indices": int(n_total), "every_index_once": missing == 0 and dup == 0, "missing": missing,
            "duplicates": dup}


def records_sha256(records) -> str:
    """SHA-256 of gathered records in global order (a torch tensor or bytes)."""
    import hashlib
    if hasattr(records, "cpu"):
        records = records.contiguous().cpu().numpy().tobytes()
    return hashlib.sha256(bytes(records)).hexdigest()
