"""Multi-GPU layout of a demodulation batch: one process per GPU, frames
sharded by index, no collective on the data path; the only exchange is the
gather of decoded payloads (RCCL all_gather over xGMI; gloo on CPU in the
tests).  Frames are independent, so scaling is weak: each rank owns its
frames' IQ in its own HBM."""
from __future__ import annotations

import torch
import torch.distributed as dist


def frame_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced split of `total` frames: (first frame, count) of
    `rank`; the first total % world ranks get one frame more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def balanced_ranges(costs, world: int) -> list[tuple[int, int]]:
    """Contiguous split of frames with per-frame `costs` into `world` ranges
    of near-equal total cost (mixed SF balanced by
    sum(66 N log2 N)); returns (first, count) per rank."""
    import numpy as np
    c = np.cumsum(np.asarray(costs, dtype=np.float64))
    total = float(c[-1]) if c.size else 0.0
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(c, total * r / world, side="left")) + 1 if c.size else 0)
    cuts.append(len(c))
    cuts = [min(max(x, 0), len(c)) for x in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1] - cuts[r]) for r in range(world)]


def gather_payloads(local: torch.Tensor, frames: int, payload: int, total: int,
                    group=None) -> torch.Tensor:
    """All ranks' decoded payloads (uint8, frames*payload each, frame_range
    order) concatenated on every rank.  Uneven shards are padded to the
    largest shard for the collective and trimmed after."""
    world = dist.get_world_size(group)
    counts = [frame_range(total, world, r)[1] for r in range(world)]
    assert frames == counts[dist.get_rank(group)]
    cap = max(counts) * payload
    buf = local.reshape(-1)
    if buf.numel() != cap:
        pad = torch.zeros(cap, dtype=torch.uint8, device=local.device)
        pad[: buf.numel()] = buf
        buf = pad
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        out = torch.cat(parts)
    else:
        out = torch.empty(world * cap, dtype=torch.uint8, device=local.device)
        dist.all_gather_into_tensor(out, buf, group=group)
    if all(c * payload == cap for c in counts):
        return out
    return torch.cat([out[r * cap: r * cap + counts[r] * payload] for r in range(world)])


def gather_varlen(local: torch.Tensor, group=None) -> list[torch.Tensor]:
    """All ranks' uint8 buffers of possibly different lengths (e.g. the
    payloads of one SF bucket of a mixed-SF batch), in rank order, on every
    rank: sizes first, then one padded all_gather."""
    world = dist.get_world_size(group)
    buf = local.reshape(-1)
    n = torch.tensor([buf.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    cap = max(sizes) if sizes else 0
    if buf.numel() != cap:
        pad = torch.zeros(cap, dtype=torch.uint8, device=local.device)
        pad[: buf.numel()] = buf
        buf = pad
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return [p[:k] for p, k in zip(parts, sizes)]


def mixed_plan(total: int, world: int, rank: int, seed: int = 0xC3, payload: int = 32,
               sf_lo: int = 7, sf_hi: int = 12):
    """The mixed-SF stream of BASELINE.json's C3 config, as every rank sees
    it: `total` frames with SF drawn uniformly from [sf_lo, sf_hi] (seeded),
    random payloads, the contiguous range of this rank cut by equal cost
    sum(66 N log2 N), and its frames bucketed by SF.  Returns
    (first, count, sfs of the range, payloads of the range, {sf: indices of
    the bucket's frames within the range, in order})."""
    import numpy as np
    rng = np.random.default_rng(seed)
    sfs = rng.integers(sf_lo, sf_hi + 1, total)
    cost = (1 << sfs) * sfs.astype(np.float64)
    first, count = balanced_ranges(cost, world)[rank]
    pays = np.random.default_rng(seed + 1).integers(0, 256, (total, payload), dtype=np.uint8)
    mine = sfs[first:first + count]
    buckets = {int(sf): np.nonzero(mine == sf)[0] for sf in range(sf_lo, sf_hi + 1)}
    return first, count, mine, pays[first:first + count], {k: v for k, v in buckets.items() if v.size}


def reassemble(buckets: dict, parts: dict, count: int, payload: int = 32):
    """Inverse of the SF bucketing: `parts[sf]` holds the decoded payloads
    of bucket sf (frames in bucket order, `payload` bytes each, numpy or
    torch); returns the range's payloads in frame order (numpy)."""
    import numpy as np
    out = np.zeros((count, payload), np.uint8)
    for sf, idx in buckets.items():
        p = parts[sf]
        p = p.cpu().numpy() if hasattr(p, "cpu") else np.asarray(p)
        out[idx] = p.reshape(-1, payload)[: idx.size]
    return out
