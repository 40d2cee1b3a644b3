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
