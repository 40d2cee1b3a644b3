"""BASELINE.json's GPU configurations at their own sizes, through the same
code bench.py times (bench.Workload: device-generated lora_modulate IQ of
random 32-byte payloads, 66 symbols per frame, resident in HBM):

  C1  SF7  x 65,536 frames (4.43 GB of IQ)
  C2  SF12 x  4,096 frames (8.86 GB)
  C3  mixed SF7-12 stream, cost-balanced rank ranges, one launch per SF
      bucket (shard.mixed_plan), payloads reassembled in frame order

Size-independent properties over every frame (each payload recovered,
status 0, sync word 0x12) plus bit-exactness with the CPU oracle (symbols,
sync word, cfo / time_offset bits, CRC flag) on frames at the start, middle
and end of each batch: the frame offsets past 2^32 bytes of
IQ (C1, C2) are covered.  The oracle is the reference's algorithm restated
in C (oracle/lphy_oracle.c), pinned to the reference build."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import bench  # noqa: E402  (repo root on sys.path via conftest)
import shard  # noqa: E402


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def _oracle_frames(oracle, lphy, wl, mode, idx):
    syms = wl.syms.cpu().numpy().view(np.uint16).reshape(wl.frames, bench.DATA_SYMS)
    meta = wl.meta.cpu().numpy().view(lphy.META_DTYPE)
    for f in idx:
        x = wl.iq[f * wl.fs * 2:(f + 1) * wl.fs * 2].cpu().numpy().view(np.complex64)
        if mode == lphy.MODE_DEMODULATE:
            r, osyms, osync, omet = oracle.demodulate(x, wl.sf, bw_hz=wl.bw)
        else:
            r, osyms, osync, omet = oracle.lora_demodulate(oracle.dechirp(x, wl.sf, wl.bw), wl.sf)
        ctx = f"SF{wl.sf} mode {mode} frame {f}"
        np.testing.assert_array_equal(syms[f], osyms, err_msg=ctx)
        assert meta["sync_word"][f] == osync, ctx
        assert _bits(meta["cfo"][f]) == _bits(omet[0]), ctx
        assert _bits(meta["time_offset"][f]) == _bits(omet[1]), ctx
        if mode != lphy.MODE_DEMODULATE:  # decode + CRC flag of the frame (phy.cpp:245-261)
            assert meta["crc_ok"][f] == oracle.decode(osyms)[2], ctx


def _all_recovered(lphy, wl):
    torch.cuda.synchronize()
    pay = wl.pay.cpu().numpy().reshape(wl.frames, bench.PAYLOAD)
    meta = wl.meta.cpu().numpy().view(lphy.META_DTYPE)
    ok = (pay == wl.payloads).all(axis=1)
    assert ok.all(), f"SF{wl.sf}: {int((~ok).sum())} of {wl.frames} payloads not recovered, first {np.nonzero(~ok)[0][:8]}"
    assert (meta["status"] == 0).all()
    assert (meta["sync_word"] == 0x12).all()


@pytest.mark.parametrize("sf,frames", [(7, 65536), (10, 8192), (12, 4096)])
def test_full_size_config(oracle, lphy, sf, frames):
    """C1 / C2 at full size: mode 2 (the bench's) and mode 0 (lora_phy::
    demodulate) over the whole resident batch."""
    dev = torch.device("cuda", 0)
    wl = bench.Workload(sf, 125000, frames, 0, dev)
    assert wl.frames * wl.fs * 8 > 2 ** 32  # frame offsets past 4 GiB
    idx = [0, 1, frames // 2, frames - 2, frames - 1]
    wl.run(lphy.MODE_DECHIRP_LORA_DEMODULATE)
    _all_recovered(lphy, wl)
    _oracle_frames(oracle, lphy, wl, lphy.MODE_DECHIRP_LORA_DEMODULATE, idx)
    # mode 0 does not round-trip payloads in the reference:
    # bit-exactness with the oracle is the property
    wl.run(lphy.MODE_DEMODULATE)
    torch.cuda.synchronize()
    _oracle_frames(oracle, lphy, wl, lphy.MODE_DEMODULATE, idx)
    del wl
    torch.cuda.empty_cache()


@pytest.mark.parametrize("total,world", [(1500, 1), (1500, 3)])
def test_c3_mixed_stream(oracle, lphy, total, world):
    """C3 scaled down: the same plan bench.py --config c3 runs (shard.
    mixed_plan: seeded SF draw, cost-balanced contiguous rank ranges, SF
    buckets), every rank's range on this one GPU in turn.  Every bucket's
    payloads are recovered, the reassembled range equals the stream's
    payloads in frame order, the ranges tile the stream, and each bucket's
    first / middle / last frames are bit-exact with the oracle."""
    dev = torch.device("cuda", 0)
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    covered = 0
    for rank in range(world):
        first, count, mine, pays, buckets = shard.mixed_plan(total, world, rank)
        assert first == covered
        covered += count
        assert sum(v.size for v in buckets.values()) == count
        parts = {}
        for sf, idx in buckets.items():
            assert (mine[idx] == sf).all()
            wl = bench.Workload(sf, 125000, int(idx.size), rank, dev, payloads=pays[idx])
            wl.run(mode)
            _all_recovered(lphy, wl)
            n = wl.frames
            _oracle_frames(oracle, lphy, wl, mode, sorted({0, n // 2, n - 1}))
            parts[sf] = wl.pay.clone()
            del wl
        got = shard.reassemble(buckets, parts, count)
        np.testing.assert_array_equal(got, pays)
    assert covered == total
    torch.cuda.empty_cache()
