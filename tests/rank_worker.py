"""One rank of the CPU rehearsal of bench.py's N > 1 path (test helper, not
a test module): started by bench.launch_ranks with the rank environment it
sets (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), it joins a gloo group,
demodulates its frame_range of a seeded batch, writes the results into a
shard.ResultSlab (u16 symbols, payload bytes, 32-byte frame records) and
gathers the slabs to rank 0 with shard.gather_slab - the same layout and
collective as bench.py's RCCL gather.  The CPU oracle stands in for the
per-rank HIP launch (test infrastructure only).  Rank 0 unpacks every rank's
slab and compares it with the oracle run over the whole batch; the verdict
goes to the JSON file named by argv[1]."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"), str(ROOT / "tests")]

import lphy  # noqa: E402  (META_DTYPE only: no library load)
import shard  # noqa: E402
from checkers import Oracle  # noqa: E402

SF, PLEN = 7, 8
SPF = 2 * PLEN


def frame_results(o, iq, sf=SF):
    """Oracle stand-in for one frame: symbols, payload, frame record."""
    r, syms, sync, met = o.lora_demodulate(o.dechirp(iq, sf), sf)
    rec = np.zeros(1, lphy.META_DTYPE)
    rec["cfo"], rec["time_offset"], rec["sync_word"] = met[0], met[1], sync
    rec["have_sync"] = 1
    return syms.astype(np.uint16), o.lora_decode(syms)[1], rec.view(np.uint8)


def main(out_path: str, total: int) -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert int(os.environ["LOCAL_RANK"]) == rank
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = Oracle()
        rng = np.random.default_rng(99)
        pays = rng.integers(0, 256, (total, PLEN), dtype=np.uint8)
        iqs = [o.modulate(o.encode(p.tobytes()), SF) for p in pays]
        first, count = shard.frame_range(total, world, rank)
        counts = [shard.frame_range(total, world, r)[1] for r in range(world)]
        cap = max(shard.slab_layout([c], SPF, PLEN)[1] for c in counts)
        slab = shard.ResultSlab([count], SPF, PLEN, torch.device("cpu"), cap)
        sv, pv, mv = slab.views(0)
        for i in range(count):
            s, p, m = frame_results(o, iqs[first + i])
            sv[i * SPF:(i + 1) * SPF] = torch.from_numpy(s.view(np.int16).copy())
            pv[i * PLEN:(i + 1) * PLEN] = torch.from_numpy(p.copy())
            mv[i * 32:(i + 1) * 32] = torch.from_numpy(m.copy())
        parts, work = shard.gather_slab(slab.buf, async_op=True)
        work.wait()
        if rank == 0:
            ok, bad = 0, []
            for r in range(world):
                f_r, c_r = shard.frame_range(total, world, r)
                (gs, gp, gm), = shard.unpack_slab(parts[r], [c_r], SPF, PLEN)
                for i in range(c_r):
                    s, p, m = frame_results(o, iqs[f_r + i])
                    if (np.array_equal(gs[i], s) and np.array_equal(gp[i], p) and np.array_equal(gp[i], pays[f_r + i])
                            and np.array_equal(gm[i], m)):
                        ok += 1
                    else:
                        bad.append(f_r + i)
            Path(out_path).write_text(json.dumps({"world": world, "frames": total, "ok": ok, "bad": bad,
                                                  "all_ok": ok == total and not bad}))
    finally:
        dist.destroy_process_group()


def main_c3(out_path: str, total: int) -> None:
    """bench.py run_c3's N > 1 path: the seeded mixed-SF stream
    (shard.mixed_plan, SF 7-9 here to keep the oracle quick) cut into
    cost-balanced contiguous ranges, each rank's frames bucketed by SF, one
    slab per rank with a [symbols | payloads | records] part per bucket,
    padded to the largest rank's layout (shard.mixed_slab_bytes), ONE gather
    to rank 0, which puts every rank's buckets back in stream order
    (shard.gather_mixed) and checks each frame against the oracle run on the
    whole stream."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kw = dict(sf_lo=7, sf_hi=9)
    try:
        o = Oracle()
        first, count, sfs, pays, plan = shard.mixed_plan(total, world, rank, payload=PLEN, **kw)
        order = sorted(plan)
        cap = shard.mixed_slab_bytes(total, world, SPF, PLEN, **kw)
        slab = shard.ResultSlab([plan[sf].size for sf in order], SPF, PLEN, torch.device("cpu"), cap)
        for i, sf in enumerate(order):
            sv, pv, mv = slab.views(i)
            for j, fi in enumerate(plan[sf]):
                iq = o.modulate(o.encode(pays[fi].tobytes()), sf)
                s, p, m = frame_results(o, iq, sf)
                sv[j * SPF:(j + 1) * SPF] = torch.from_numpy(s.view(np.int16).copy())
                pv[j * PLEN:(j + 1) * PLEN] = torch.from_numpy(p.copy())
                mv[j * 32:(j + 1) * 32] = torch.from_numpy(m.copy())
        parts, work = shard.gather_slab(slab.buf, async_op=True)
        work.wait()
        if rank == 0:
            gs, gp, gm = shard.gather_mixed(parts, total, world, SPF, PLEN, **kw)
            _, _, all_sfs, all_pays, _ = shard.mixed_plan(total, 1, 0, payload=PLEN, **kw)
            ok, bad = 0, []
            for f in range(total):
                iq = o.modulate(o.encode(all_pays[f].tobytes()), int(all_sfs[f]))
                s, p, m = frame_results(o, iq, int(all_sfs[f]))
                if (np.array_equal(gs[f], s) and np.array_equal(gp[f], p) and np.array_equal(gp[f], all_pays[f])
                        and np.array_equal(gm[f], m)):
                    ok += 1
                else:
                    bad.append(f)
            counts = [shard.mixed_plan(total, world, r, payload=PLEN, **kw)[1] for r in range(world)]
            buckets = [len(shard.mixed_plan(total, world, r, payload=PLEN, **kw)[4]) for r in range(world)]
            Path(out_path).write_text(json.dumps({"world": world, "frames": total, "ok": ok, "bad": bad,
                                                  "counts": counts, "buckets": buckets,
                                                  "all_ok": ok == total and not bad}))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "c3":
        main_c3(sys.argv[1], int(sys.argv[2]))
    else:
        main(sys.argv[1], int(sys.argv[2]))
