"""Multi-GPU layout of a demodulation batch: one process per GPU, frames
sharded by index, no collective on the data path; the only exchange is the
gather of each rank's results - symbols, decoded payloads and frame records,
one contiguous slab per rank - to rank 0 (RCCL over xGMI, gloo
on CPU in the tests).  Frames are independent, so scaling is weak: each rank
owns its frames' IQ in its own HBM."""
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


META_BYTES = 32  # lphy_frame_meta (include/lphy_hip.h)


def _al(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


def slab_layout(counts, syms_per_frame: int, payload: int):
    """Byte layout of one rank's results in a single buffer (the
    u16 symbols, the decoded payload bytes and the 32-byte frame record per
    frame): one part per entry of `counts` (a single-SF batch has one part,
    a mixed-SF rank one per SF bucket), each [symbols | payloads | records],
    every section 256-byte aligned.  Returns ([(frames, off_syms, off_pay,
    off_meta)], bytes used)."""
    parts, off = [], 0
    for n in counts:
        n = int(n)
        s = off
        off += _al(n * syms_per_frame * 2)
        p = off
        off += _al(n * payload)
        m = off
        off += _al(n * META_BYTES)
        parts.append((n, s, p, m))
    return parts, off


class ResultSlab:
    """A rank's demodulation outputs in one contiguous uint8 device buffer
    (slab_layout), so the gather to rank 0 is a single collective per step.
    `nbytes` pads the buffer to the largest rank's layout: every rank's
    buffer then has the same size, as the collective needs."""

    def __init__(self, counts, syms_per_frame: int, payload: int, device, nbytes: int = 0):
        self.spf, self.payload = syms_per_frame, payload
        self.parts, self.used = slab_layout(counts, syms_per_frame, payload)
        self.nbytes = max(self.used, int(nbytes))
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)

    def views(self, i: int = 0):
        """(int16 symbols, uint8 payloads, uint8 frame records) of part i."""
        n, s, p, m = self.parts[i]
        b = self.buf
        return (b[s:s + n * self.spf * 2].view(torch.int16), b[p:p + n * self.payload],
                b[m:m + n * META_BYTES])


def unpack_slab(buf, counts, syms_per_frame: int, payload: int):
    """Host view of a gathered slab: per part (uint16 symbols [n, spf],
    uint8 payloads [n, payload], uint8 records [n, 32])."""
    import numpy as np
    a = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf, np.uint8)
    out = []
    for n, s, p, m in slab_layout(counts, syms_per_frame, payload)[0]:
        out.append((a[s:s + n * syms_per_frame * 2].view(np.uint16).reshape(n, syms_per_frame),
                    a[p:p + n * payload].reshape(n, payload),
                    a[m:m + n * META_BYTES].reshape(n, META_BYTES)))
    return out


def gather_slab(buf: torch.Tensor, dst: int = 0, group=None, async_op: bool = False):
    """Every rank's slab (equal sizes) to rank `dst`: RCCL gather over xGMI
    (ncclSend/ncclRecv in one group; gloo on CPU).  Returns (list of world
    buffers on dst, None elsewhere; the work handle when async_op)."""
    world = dist.get_world_size(group)
    out = ([torch.empty_like(buf) for _ in range(world)]
           if dist.get_rank(group) == dst else None)
    work = dist.gather(buf, out, dst=dst, group=group, async_op=async_op)
    return out, work


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


def reassemble(buckets: dict, parts: dict, count: int, payload: int = 32, dtype=None):
    """Inverse of the SF bucketing: `parts[sf]` holds bucket sf's rows
    (frames in bucket order, `payload` elements each - decoded payload
    bytes, u16 symbols or 32-byte records; numpy or torch); returns the
    range's rows in frame order (numpy, dtype of the parts or `dtype`)."""
    import numpy as np
    out = None
    for sf, idx in buckets.items():
        p = parts[sf]
        p = p.cpu().numpy() if hasattr(p, "cpu") else np.asarray(p)
        if out is None:
            out = np.zeros((count, payload), dtype or p.dtype)
        out[idx] = p.reshape(-1, payload)[: idx.size]
    return out if out is not None else np.zeros((count, payload), dtype or np.uint8)


def mixed_slab_bytes(total: int, world: int, syms_per_frame: int, payload: int, **plan_kw) -> int:
    """C3 (mixed SF): the size every rank's result slab is padded to - the
    largest rank's layout of one part per SF bucket - computed by every rank
    from the seeded plan, so no size exchange precedes the gather.  plan_kw:
    mixed_plan's seed / sf_lo / sf_hi (its payload is `payload`)."""
    best = 0
    for r in range(world):
        plan = mixed_plan(total, world, r, payload=payload, **plan_kw)[4]
        best = max(best, slab_layout([plan[sf].size for sf in sorted(plan)], syms_per_frame, payload)[1])
    return best


def gather_mixed(parts, total: int, world: int, syms_per_frame: int, payload: int, **plan_kw):
    """Rank 0 after the C3 gather: every rank's slab (one part per SF bucket,
    buckets in SF order) unpacked and put back in stream order.  Returns
    (symbols [total, spf] u16, payloads [total, payload] u8, records
    [total, 32] u8) of the whole stream."""
    import numpy as np
    syms, pays, recs = [], [], []
    for r in range(world):
        _, c_r, _, _, plan = mixed_plan(total, world, r, payload=payload, **plan_kw)
        order = sorted(plan)
        unp = unpack_slab(parts[r], [plan[sf].size for sf in order], syms_per_frame, payload)
        syms.append(reassemble(plan, {sf: u[0] for sf, u in zip(order, unp)}, c_r, syms_per_frame, np.uint16))
        pays.append(reassemble(plan, {sf: u[1] for sf, u in zip(order, unp)}, c_r, payload, np.uint8))
        recs.append(reassemble(plan, {sf: u[2] for sf, u in zip(order, unp)}, c_r, META_BYTES, np.uint8))
    return np.concatenate(syms), np.concatenate(pays), np.concatenate(recs)
