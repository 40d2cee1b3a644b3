#!/usr/bin/env python3
"""Throughput bench for the MI355X LoRa demodulation path (BASELINE.json).

Workload (BASELINE.json configs[1], "C1"): SF7 BW125, 65,536 synthetic frames
per GPU, each a 32-byte random payload -> lora_encode -> lora_modulate
(66 symbols: 2 sync + 64 data, 8,448 complex float32 samples = 67.6 KB).
The IQ is generated on the device (bit-exact lora_modulate kernel) and stays
resident in HBM; the timed step is one pass of the hot path over the batch:

    fused dechirp -> lora_demodulate (max-abs normalise, offset estimate,
    per-symbol rotate + KISS-identical FFT + argmax) -> lora_decode + CRC

(LPHY_MODE_DECHIRP_LORA_DEMODULATE + LPHY_F_DECODE through the C ABI), plus,
for N > 1 ranks, the gather of every rank's results (symbols, payloads,
32-byte frame records) to rank 0 (RCCL over xGMI, overlapped with the next
step).  `value` = data symbols demodulated by all ranks / max-over-ranks time.
`--gpus N` without WORLD_SIZE starts the N ranks itself (one process per
GPU); under torch.distributed.run it checks WORLD_SIZE == N.

Also reported: the high-level lora_phy::demodulate path (mode A), the
dominant kernel's roofline fraction (HIP events on the launch stream), and
the reference CPU path timed on this host's cores (rank 0, N = 1).

Run: python bench.py [--gpus N --steps K --warmup W --sf 7 --frames F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT / "tests"))

import lphy  # noqa: E402
import shard  # noqa: E402

# LPHY_BENCH_REHEARSE=1 rehearses the N > 1 path on a one-GPU box: every
# rank on cuda:0, gloo instead of RCCL, the slabs staged through host memory
# for the gather.  Its lines say "rehearsal" and are never a scaling result.
REHEARSE = os.environ.get("LPHY_BENCH_REHEARSE") == "1"
HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
PAYLOAD = 32                  # bytes per frame (performance_test.cpp:67)
DATA_SYMS = 2 * PAYLOAD       # 64 data symbols
TOTAL_SYMS = DATA_SYMS + 2    # + 2 sync symbols
DEFAULT_FRAMES = {7: 65536, 8: 32768, 9: 16384, 10: 8192, 11: 4096, 12: 4096}


def bytes_per_data_symbol(N: int) -> float:
    """IQ read (sync share included) + u16 symbol + 1/2 byte."""
    return 8.0 * N * TOTAL_SYMS / DATA_SYMS + 2.0 + 0.5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without WORLD_SIZE spawns the ranks itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--sf", type=int, default=7)
    ap.add_argument("--bw", type=int, default=125000)
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (0 = config default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-mode-a", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="also time SF8..SF12 BW125 (extra field)")
    ap.add_argument("--csv", default="", help="write the perf CSV (reference schema + hbm_gbps, "
                                             "roofline_frac) for the reference's profiles and SF9-12 BW125")
    ap.add_argument("--run-id", default=os.environ.get("RUN_ID", "run"))
    ap.add_argument("--config", default="c1", choices=["c1", "c2", "c3", "c4"],
                    help="BASELINE.json config: c1 SF7 x 65,536 (headline, default), c2 SF12 x "
                         "4,096, c3 mixed SF7-12 (1M frames over the ranks), c4 SF9 AWGN BER")
    ap.add_argument("--total-frames", type=int, default=0,
                    help="c3: frames over all ranks (default 131072 per rank: the 1 M frames of "
                         "C3 on 8 GPUs, ~93 GB of IQ resident per GPU)")
    return ap.parse_args()


class Workload:
    """One SF configuration resident on this rank's GPU."""

    def __init__(self, sf: int, bw: int, frames: int, rank: int, dev: torch.device, payloads=None,
                 outs=None):
        self.sf, self.N, self.bw, self.frames = sf, 1 << sf, bw, frames
        self.fs = TOTAL_SYMS * self.N
        self.dem = lphy.Demodulator(sf, bw, 1, lphy.WINDOW_NONE, device=dev.index)
        rng = np.random.default_rng(0x5EED + 7919 * rank + sf)
        self.payloads = (payloads if payloads is not None
                         else rng.integers(0, 256, (frames, PAYLOAD), dtype=np.uint8))
        syms = lphy.encode_payloads(self.payloads)
        stream = torch.cuda.current_stream().cuda_stream
        t_in = torch.from_numpy(syms.view(np.int16).reshape(-1).copy()).to(dev)
        self.iq = torch.empty(frames * self.fs * 2, dtype=torch.float32, device=dev)
        self.dem.modulate_batch(t_in, frames, DATA_SYMS, self.iq, 1.0, 0x12, stream)
        del t_in
        # output sets (symbols, payloads, frame records): one of its own, or
        # views into the rank's result slabs (N > 1: two, double-buffered
        # against the gather of the previous step)
        self.outs = outs or [(torch.zeros(frames * DATA_SYMS, dtype=torch.int16, device=dev),
                              torch.zeros(frames * PAYLOAD, dtype=torch.uint8, device=dev),
                              torch.zeros(frames * 32, dtype=torch.uint8, device=dev))]
        self.syms, self.pay, self.meta = self.outs[0]
        torch.cuda.synchronize()

    def run(self, mode: int, flags: int = lphy.F_DECODE, slot: int = 0):
        syms, pay, meta = self.outs[slot]
        self.dem.demod_batch(self.iq, self.frames, self.fs, syms, meta, mode,
                             flags, payload=pay,
                             stream=torch.cuda.current_stream().cuda_stream)

    def _event_ms(self, mode: int, flags: int, reps: int, warmup: int = 20) -> float:
        """Average device time of one demod_batch call with `flags` (HIP
        events recorded on the stream the kernels are launched on), after
        `warmup` untimed calls (the clocks settle after a change of load)."""
        for _ in range(warmup):
            self.run(mode, flags)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            self.run(mode, flags)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    def stage_times(self, mode: int, reps: int = 20) -> dict:
        """Device time per launch of each kernel of the product path: the
        fused prologue+symbols kernel (k_wave / k_frames, PROLOGUE|SYMBOLS selects it
        alone) and k_finalize; plus the separate-launch path's stages
        (LPHY_F_UNFUSED) for comparison."""
        D = lphy.F_DECODE
        both = lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
        return {
            "fused": self._event_ms(mode, D | both, reps),
            "final": self._event_ms(mode, D | lphy.F_STAGE_FINAL, reps),
            "unfused_prologue": self._event_ms(mode, D | lphy.F_UNFUSED | lphy.F_STAGE_PROLOGUE, reps),
            "unfused_symbols": self._event_ms(mode, D | lphy.F_UNFUSED | lphy.F_STAGE_SYMBOLS, reps),
        }

    def check(self, mode: int) -> dict:
        """Size-independent property over the whole batch (every payload
        recovered, CRC field consistent) + bit-exact oracle comparison on a
        sample of frames."""
        torch.cuda.synchronize()
        pay = self.pay.cpu().numpy().reshape(self.frames, PAYLOAD)
        res = {"payloads_recovered": int((pay == self.payloads).all(axis=1).sum()),
               "frames": self.frames}
        try:
            from checkers import Oracle
            o = Oracle()
            syms = self.syms.cpu().numpy().view(np.uint16).reshape(self.frames, DATA_SYMS)
            idx = np.unique(np.linspace(0, self.frames - 1, 8).astype(int))
            ok = 0
            for f in idx:
                x = self.iq[f * self.fs * 2:(f + 1) * self.fs * 2].cpu().numpy().view(np.complex64)
                if mode == lphy.MODE_DEMODULATE:
                    r, osyms, _, _ = o.demodulate(x, self.sf, bw_hz=self.bw)
                else:
                    r, osyms, _, _ = o.lora_demodulate(o.dechirp(x, self.sf, self.bw), self.sf)
                ok += int(np.array_equal(osyms, syms[f]))
            res["oracle_frames_bit_exact"] = f"{ok}/{len(idx)}"
        except Exception as e:  # checker unavailable: say so, never fall back
            res["oracle_frames_bit_exact"] = f"unavailable: {e}"
        return res


SETTLE_S = 0.15  # untimed settle before the warmup steps (see timed)


class Gatherer:
    """The §8e exchange of an N > 1 step: the rank's result slab (symbols,
    payloads, frame records of all its frames) gathered to rank 0 in one
    RCCL collective.  Two slabs alternate: step k's gather is issued async
    right after its launch, so it runs while step k+1 demodulates into the
    other slab; before step k+2 reuses slab k % 2 the stream waits for that
    gather.  `finish` drains both and returns rank 0's last gathered slabs."""

    def __init__(self, slabs):
        self.slabs = slabs
        self.work = [None] * len(slabs)
        self.out = [None] * len(slabs)
        self.last = 0

    def before(self, k: int) -> int:
        slot = k % len(self.slabs)
        if self.work[slot] is not None:
            self.work[slot].wait()  # the stream waits for the gather that reads this slab
            self.work[slot] = None
        return slot

    def after(self, slot: int) -> None:
        if REHEARSE:  # gloo: host copies, synchronous
            self.out[slot], _ = shard.gather_slab(self.slabs[slot].buf.cpu())
        else:
            self.out[slot], self.work[slot] = shard.gather_slab(self.slabs[slot].buf, async_op=True)
        self.last = slot

    def finish(self):
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None
        return self.out[self.last]


def timed(wl: Workload, mode: int, steps: int, warmup: int, world: int, events: list | None = None,
          settle_s: float = 0.0, gat: Gatherer | None = None):
    """Wall time of `steps` steps between barriers.  With `events`, each
    step issues the demodulation as two calls on the same stream - prologue
    + symbols (the fused launch and its fix-up), then the per-frame
    finalisation - and HIP events bracket the first, so the dominant
    kernel's duration is measured inside the timed region; the per-step
    (start, end) event pairs are appended to `events`.  With `gat` (N > 1)
    each step also gathers its results to rank 0 (Gatherer)."""
    both = lphy.F_DECODE | lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
    k_step = [0]

    def step(ev=None):
        slot = gat.before(k_step[0]) if gat else 0
        k_step[0] += 1
        if ev is None:
            wl.run(mode, slot=slot)
        else:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            wl.run(mode, both, slot=slot)
            b.record()
            wl.run(mode, lphy.F_DECODE | lphy.F_STAGE_FINAL, slot=slot)
            ev.append((a, b))
        if gat:
            gat.after(slot)

    # The card's clocks dip for the first ~20 ms of a new sustained load
    # (after an idle gap: one fast launch, then launches up to 40 % slower
    # while the power controller settles; profiles/r2 kernel traces).  The
    # demodulation runs untimed for `settle_s` of wall time before the W
    # warmup steps, so the K timed steps measure the sustained rate (local
    # launches only: ranks may loop a different number of times, so no
    # collective here).
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < settle_s:
        for _ in range(8):
            wl.run(mode)
        torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    if gat:
        gat.finish()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(events)
    if gat:
        gat.finish()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cpu" if REHEARSE else wl.iq.device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def rank_payloads(sf: int, frames: int, rank: int) -> np.ndarray:
    """The payloads Workload draws for `rank` (so rank 0 can check every
    rank's gathered results)."""
    rng = np.random.default_rng(0x5EED + 7919 * rank + sf)
    return rng.integers(0, 256, (frames, PAYLOAD), dtype=np.uint8)


def check_gathered(parts, sf: int, frames: int, world: int) -> dict:
    """Rank 0's view of the whole job after the gather: every rank's
    symbols, payloads and frame records (sync word, status) against what
    that rank transmitted."""
    meta_dt = lphy.META_DTYPE
    ok_pay = ok_sym = ok_rec = 0
    for r in range(world):
        (syms, pay, rec), = shard.unpack_slab(parts[r], [frames], DATA_SYMS, PAYLOAD)
        want = rank_payloads(sf, frames, r)
        m = rec.reshape(-1).view(meta_dt)
        ok_pay += int((pay == want).all(axis=1).sum())
        # (the modulator sends codeword c as bin c mod N: below SF 8 the
        # demodulated symbol is the codeword's low SF bits)
        ok_sym += int((syms == (lphy.encode_payloads(want) & ((1 << sf) - 1))).all(axis=1).sum())
        ok_rec += int(((m["status"] == 0) & (m["sync_word"] == 0x12) & (m["have_sync"] == 1)).sum())
    total = world * frames
    return {"frames": total, "payloads_recovered": ok_pay, "symbols_exact": ok_sym,
            "records_ok": ok_rec, "all_ok": ok_pay == ok_sym == ok_rec == total}


def usable_cpus() -> dict:
    """Host CPUs as the process sees them: os.cpu_count() (the machine),
    the affinity mask, and the cgroup CPU quota when one is set (a GPU box
    gives each job a share of a larger host)."""
    out = {"host_cpus": os.cpu_count() or 1}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        out["affinity_cpus"] = out["host_cpus"]
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    out["cgroup_cpu_quota"] = quota
    return out


def effective_cpus(c: dict | None = None) -> int:
    """CPUs this process can actually use: min(affinity mask, cgroup CPU
    quota rounded up).  A GPU box reports the whole host in os.cpu_count()
    (256) but grants a 16-CPU quota."""
    import math
    c = c or usable_cpus()
    n = c["affinity_cpus"]
    if c.get("cgroup_cpu_quota"):
        n = min(n, max(1, math.ceil(c["cgroup_cpu_quota"])))
    return max(1, n)


def cpu_baseline(wl: Workload, seconds: float, runs: int = 5) -> dict:
    """The reference CPU path on this host:
    one thread per effective CPU (effective_cpus), one workspace per thread,
    on a bounded sample of the same resident frames; each of `runs` runs
    repeats the sample until seconds / (2 runs) have passed, and the median
    rate is reported for mode B (dechirp + lora_demodulate + lora_decode,
    the bench's path) and mode A (demodulate + decode, phy.cpp).  A shorter
    mode-B run with os.cpu_count() threads is kept as an extra field."""
    import checkers
    cpus = usable_cpus()
    threads = effective_cpus(cpus)
    if checkers.reference_available():
        ck, kind = checkers.Reference(), "reference"
    else:
        ck, kind = checkers.Oracle(), "port"
    nf = min(wl.frames, max(2048, 8 * threads))
    x = wl.iq[: nf * wl.fs * 2].cpu().numpy().view(np.complex64)
    per_run = seconds / (2 * runs)
    res = {}
    for name, mode in (("mode_B", 1), ("mode_A", 0)):
        rates, out, total = [], None, 0
        for _ in range(runs):
            done, el = 0, 0.0
            while el < per_run or done == 0:
                t, out = ck.bench(mode, wl.sf, x, nf, wl.fs, threads, wl.bw)
                el += t
                done += nf
            rates.append(done * DATA_SYMS / el)
            total += done
        ok = bool((out.reshape(nf, PAYLOAD) == wl.payloads[:nf]).all())
        res[name] = {"value": float(np.median(rates)), "runs": [float(r) for r in rates],
                     "frames": total, "payloads_ok": ok}
    b = res["mode_B"]
    host = cpus["host_cpus"]
    if host != threads:  # oversubscribed: os.cpu_count() threads on the quota
        rates = []
        for _ in range(3):
            t, _ = ck.bench(1, wl.sf, x, nf, wl.fs, host, wl.bw)
            rates.append(nf * DATA_SYMS / t)
        res["mode_B_os_cpu_count_threads"] = {"value": float(np.median(rates)), "threads": host,
                                              "runs": [float(r) for r in rates]}
    return {"value": b["value"], "unit": "data symbols/s", "cores": threads, "kind": kind,
            "runs": len(b["runs"]), "modes": res, "cpus": cpus,
            "sample": f"SF{wl.sf} BW{wl.bw // 1000}: {nf}-frame batches of the bench's resident frames, "
                      f"{threads} threads (effective CPUs: min(affinity {cpus['affinity_cpus']}, cgroup quota "
                      f"{cpus['cgroup_cpu_quota']}); os.cpu_count() = {host}), median of {runs} runs of "
                      f"~{per_run:.1f} s per "
                      "mode; value = mode B (dechirp+lora_demodulate+lora_decode, payloads ok="
                      f"{b['payloads_ok']}); mode A = demodulate+decode (phy.cpp, does not round-trip, "
                      "SURVEY §0.3)"}


# tests/profiles.yaml of the reference (name, sf, bw): the rows of its
# performance CSV (performance_test.cpp:69-75)
REF_PROFILES = [("sf7_bw125_cr45", 7, 125000), ("sf7_bw125_cr47", 7, 125000), ("sf8_bw125_cr45", 8, 125000),
                ("sf9_bw250_cr48", 9, 250000), ("sf10_bw250_cr47", 10, 250000),
                ("sf11_bw500_cr45", 11, 500000), ("sf12_bw500_cr45", 12, 500000)]
CLOCK_HZ = 2.4e9  # MI355X max engine clock (MI355X_MICROARCH.md), for cycles_per_symbol


def profile_row(wl: Workload, ms_step: float, steps: int) -> dict:
    """One configuration's whole-step figures: frames (packets) per second,
    device clock cycles per data symbol at the 2.4 GHz engine clock (the
    whole chip's wall time per symbol, the analog of the reference's rdtsc
    cycles per symbol), the step's algorithmic HBM GB/s (SURVEY §8d bytes
    per data symbol) and its fraction of the 8 TB/s roofline; payloads
    recovered as the correctness check."""
    syms = wl.frames * DATA_SYMS
    gbps = syms * bytes_per_data_symbol(wl.N) / (ms_step * 1e-3) / 1e9
    chk = wl.check(lphy.MODE_DECHIRP_LORA_DEMODULATE)
    return {"sf": wl.sf, "N": wl.N, "bw_hz": wl.bw, "frames": wl.frames, "steps": steps,
            "ms_per_step": ms_step, "symbols_per_s": syms / (ms_step * 1e-3),
            "pps": wl.frames / (ms_step * 1e-3),
            "cycles_per_symbol": ms_step * 1e-3 * CLOCK_HZ / syms,
            "hbm_gbps": gbps, "roofline_frac": gbps / HBM_PEAK_GBPS,
            "payloads_recovered": chk["payloads_recovered"]}


def write_perf_csv(path: str, run_id: str, rows: list) -> None:
    """The reference's performance CSV (run_id,profile,sf,N,pps,
    cycles_per_symbol; performance_test.cpp:69-75,144-148) plus hbm_gbps
    and roofline_frac; tools/compare_perf.py gates on it."""
    import csv
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["run_id", "profile", "sf", "N", "pps", "cycles_per_symbol", "hbm_gbps", "roofline_frac"])
        for r in rows:
            w.writerow([run_id, r["profile"], r["sf"], r["N"], f"{r['pps']:.6g}", f"{r['cycles_per_symbol']:.6g}",
                        f"{r['hbm_gbps']:.6g}", f"{r['roofline_frac']:.6g}"])


def frames_fused(sf: int) -> bool:
    """Whether the bench frame shape takes a fused launch: every SF (k_frames
    up to SF 6, k_wave at SF 7-12; lphy_hip.hip frames_fit /
    wave_fit: the bench's batches are far above the fused crossover)."""
    return True


def fused_kernel(sf: int) -> str:
    """Name of the fused launch's kernel, as the PMC summaries key it, by the
    library's own rule for the bench's frames (66 symbols, osr 1, no window;
    lphy_hip.hip wave_fit: k_wave from SF 7 when a frame holds at least one
    wave unit of symbols, 4096 / N - which the bench's 66 always do; below
    SF 7, k_frames)."""
    if sf <= 6:
        return f"k_frames<{sf}>"
    return f"k_wave<{sf}>"


def measured_traffic(kernel: str, frames: int):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_*.json written by tools/pmc_summary.py from rocprofv3 --pmc
    passes of this bench's configuration; FETCH_SIZE x2 on gfx950 +
    WRITE_SIZE, per the MI355X guide), or None when no summary matches.  Of
    several summaries of the same kernel and configuration the newest wins:
    by the "written" stamp pmc_summary.py records (summaries from before it
    had one rank below every stamped one, then by name)."""
    best, best_key = None, None
    for f in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        k = d.get("kernels", {}).get(kernel)
        # the bench's mode (2) only; summaries without the HBM passes skipped
        if k and "hbm_bytes_per_launch" in k and d.get("frames") == frames and d.get("mode", 2) == 2:
            key = (d.get("written", ""), f.name)
            if best_key is None or key > best_key:
                best_key = key
                best = {"bytes": k["hbm_bytes_per_launch"], "source": f"{f.name}",
                        "written": d.get("written")}
    return best


def _sync_time(fn, steps, warmup, world, dev, gat=None):
    for _ in range(warmup):
        fn()
    if gat:
        gat.finish()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if gat:
        gat.finish()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cpu" if REHEARSE else dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def run_c3(args, baseline, world, rank, dev) -> dict:
    """C3: mixed SF7-12 stream, `--total-frames` frames with SF drawn
    uniformly (seeded), split across ranks by cost-balanced contiguous
    ranges (sum of 66 N log2 N), bucketed by SF on each rank
    (one resident batch and one launch per SF); payloads gathered."""
    total = args.total_frames or (1 << 17) * world  # weak scaling: 1 M frames at 8 ranks
    first, count, mine, payloads, plan = shard.mixed_plan(total, world, rank, payload=PAYLOAD)
    order = sorted(plan)
    slabs = None
    if world > 1:
        # one slab per rank holds all its buckets; every rank's layout is
        # known from the seeded plan, so the slabs are padded to the largest
        cap = shard.mixed_slab_bytes(total, world, DATA_SYMS, PAYLOAD)
        slabs = [shard.ResultSlab([plan[sf].size for sf in order], DATA_SYMS, PAYLOAD, dev, cap)
                 for _ in range(2)]
    buckets = [Workload(sf, args.bw, int(plan[sf].size), rank, dev, payloads=payloads[plan[sf]],
                        outs=[sl.views(i) for sl in slabs] if slabs else None)
               for i, sf in enumerate(order)]
    mode_b = lphy.MODE_DECHIRP_LORA_DEMODULATE

    gat = Gatherer(slabs) if world > 1 else None
    k_step = [0]

    def step():
        slot = gat.before(k_step[0]) if gat else 0
        k_step[0] += 1
        for wl in buckets:
            wl.run(mode_b, slot=slot)
        if gat:  # the only exchange: every bucket's results in one gather
            gat.after(slot)
    steps = max(2, args.steps // 4)
    dt = _sync_time(step, steps, 1, world, dev, gat)
    syms = torch.tensor([sum(w.frames for w in buckets) * DATA_SYMS], dtype=torch.float64,
                        device="cpu" if REHEARSE else dev)
    if world > 1:
        torch.distributed.all_reduce(syms)
    gathered = None
    if world > 1:
        parts = gat.finish()
        if rank == 0:
            # the whole stream, every rank's buckets put back in frame order
            _, _, alls, allp, _ = shard.mixed_plan(total, 1, 0, payload=PAYLOAD)
            gs, got, gm = shard.gather_mixed(parts, total, world, DATA_SYMS, PAYLOAD)
            m = gm.reshape(-1).view(lphy.META_DTYPE)
            # (codeword c arrives as bin c mod N)
            want_s = lphy.encode_payloads(allp) & ((1 << alls.astype(np.int64)) - 1)[:, None].astype(np.uint16)
            gathered = {"frames": int(total), "stream_in_order": bool(np.array_equal(got, allp)),
                        "symbols_exact": bool(np.array_equal(gs, want_s)),
                        "records_ok": int(((m["status"] == 0) & (m["sync_word"] == 0x12)).sum())}
        for wl in buckets:
            wl.run(mode_b)  # slot 0 again for the local checks below
    ok = sum(w.check(mode_b)["payloads_recovered"] for w in buckets)
    # the buckets' payloads put back in frame order = this rank's stream
    ordered = shard.reassemble(plan, {w.sf: w.pay for w in buckets}, count, PAYLOAD)
    in_order = bool(np.array_equal(ordered, payloads))
    per_sf = {f"SF{w.sf}": w.frames for w in buckets}
    iq_gb = sum(w.frames * w.fs * 8 for w in buckets) / 1e9
    return {"metric": baseline["metric"], "value": float(syms.item()) * steps / dt,
            "unit": "data symbols/s", "n_gpus": world, "steps": steps, "warmup": 1,
            "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (device-generated lora_modulate IQ of random payloads)",
            "config": {"workload": f"C3 mixed SF7-12, {total} frames over {world} rank(s), "
                                   "cost-balanced shards, one launch per SF bucket",
                       "frames_this_rank": int(count), "frames_per_sf_rank0": per_sf,
                       "iq_gb_rank0": iq_gb, "parallelism": f"frames sharded x{world}"},
            "check": {"payloads_recovered": ok, "frames": int(count), "reassembled_in_order": in_order,
                      "gathered_rank0": gathered}}


def run_c4(args, baseline, world, rank, dev) -> dict:
    """C4: SF9 BW125 under AWGN (sigma = sqrt(10^(-SNR/10)/2) per component,
    unit-power signal; SNR -10 and -15 dB), symbol / bit error rates of the
    GPU path against the transmitted payloads, and bit-exactness with the
    CPU oracle / reference on a sample of the same noisy frames."""
    sf = 9
    frames = args.frames or DEFAULT_FRAMES[sf]
    out = {}
    value = None
    for snr in (-10.0, -15.0):
        slabs = ([shard.ResultSlab([frames], DATA_SYMS, PAYLOAD, dev) for _ in range(2)]
                 if world > 1 else None)
        wl = Workload(sf, args.bw, frames, rank, dev, outs=[sl.views(0) for sl in slabs] if slabs else None)
        g = torch.Generator(device=dev)
        g.manual_seed(0xC4 + int(-snr) + 7919 * rank)
        sig = float(np.sqrt(10 ** (-snr / 10) / 2))
        wl.iq.add_(torch.randn(wl.iq.shape, generator=g, device=dev) * sig)
        mode_b = lphy.MODE_DECHIRP_LORA_DEMODULATE
        steps = max(3, args.steps // 4)
        gat = Gatherer(slabs) if slabs else None
        k_step = [0]

        def step():
            slot = gat.before(k_step[0]) if gat else 0
            k_step[0] += 1
            wl.run(mode_b, slot=slot)
            if gat:
                gat.after(slot)
        dt = _sync_time(step, steps, 1, world, dev, gat)
        if value is None:
            value = world * frames * DATA_SYMS * steps / dt
        torch.cuda.synchronize()
        # error rates over the whole job: rank 0 holds every rank's gathered
        # symbols and payloads (N > 1), and regenerates what each rank sent
        if gat:
            parts = gat.finish()
            res = [shard.unpack_slab(parts[r], [frames], DATA_SYMS, PAYLOAD)[0] for r in range(world)] \
                if rank == 0 else []
            sent_pay = [rank_payloads(sf, frames, r) for r in range(world)] if rank == 0 else []
        else:
            res = [(wl.syms.cpu().numpy().view(np.uint16).reshape(frames, DATA_SYMS),
                    wl.pay.cpu().numpy().reshape(frames, PAYLOAD), None)]
            sent_pay = [wl.payloads]
        wl.run(mode_b)  # slot 0 for the local oracle sample
        chk = wl.check(mode_b)
        if rank == 0:
            got = np.concatenate([r[0] for r in res])
            pay = np.concatenate([r[1] for r in res])
            sp = np.concatenate(sent_pay)
            ser = float((got != lphy.encode_payloads(sp)).mean())
            ber = float(np.unpackbits(pay ^ sp).mean())
            out[f"snr_{int(snr)}dB"] = {"ser": ser, "ber": ber, "frames": int(sp.shape[0]),
                                        "frame_error_rate": float((pay != sp).any(axis=1).mean()),
                                        "oracle_frames_bit_exact": chk["oracle_frames_bit_exact"]}
        del wl
        torch.cuda.empty_cache()
    return {"metric": baseline["metric"], "value": value, "unit": "data symbols/s",
            "n_gpus": world, "steps": max(3, args.steps // 4), "warmup": 1,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: device lora_modulate IQ + torch AWGN",
            "config": {"workload": f"C4 SF9 BW125 AWGN, {frames} frames/GPU", "sf": sf,
                       "parallelism": f"frames sharded x{world}"},
            "awgn": out}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int) -> dict:
    """The torch.distributed environment of one rank on this node (what
    torch.distributed.run sets): one process per GPU, rank r on GPU r."""
    return {"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
            "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
            "MASTER_PORT": str(port)}


def node_gpu_count(sysfs: str = "/sys/class/kfd/kfd/topology/nodes", env=None) -> int:
    """GPUs on this node without touching HIP: the KFD topology nodes with
    SIMDs (CPU nodes have simd_count 0), capped by the visible-device list
    (HIP_VISIBLE_DEVICES, ROCR_VISIBLE_DEVICES or CUDA_VISIBLE_DEVICES, as
    the runtime honours them).  0 when the topology is unreadable."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in sorted(Path(sysfs).iterdir()):
            props = {}
            for line in (node / "properties").read_text().splitlines():
                parts = line.split()
                if len(parts) == 2:
                    props[parts[0]] = parts[1]
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except (OSError, ValueError):
        return 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(cmd: list, world: int, devices: int | None = None) -> int:
    """Run `cmd` as `world` ranks, one child process per GPU, and return
    the first failing rank's exit code (0 when all succeed).  The parent
    never touches HIP: it counts the node's GPUs from the KFD topology in
    sysfs (node_gpu_count) and refuses when there are fewer than ranks.  A
    rank that fails ends the others (their own PIDs)."""
    import subprocess
    if devices is None:
        devices = world if REHEARSE else node_gpu_count()
    if devices < world:
        print(f"bench.py: --gpus {world} needs {world} GPUs, this node has {devices}", file=sys.stderr)
        return 3
    port = _free_port()
    procs = [subprocess.Popen(cmd, env={**os.environ, **rank_env(r, world, port)}) for r in range(world)]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in live:
                        q.terminate()
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        n = args.gpus or 1
        if n > 1:  # spawn the ranks ourselves (driver-style `bench.py --gpus N`)
            sys.exit(launch_ranks([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], n))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(3)
    if torch.cuda.device_count() < world and not REHEARSE:
        print(f"bench.py: {world} ranks, {torch.cuda.device_count()} GPUs", file=sys.stderr)
        sys.exit(3)
    if REHEARSE:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if REHEARSE:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=dev)
    baseline = json.loads((ROOT / "BASELINE.json").read_text())
    if args.config == "c2":
        args.sf = 12
        args.frames = args.frames or 4096
    elif args.config in ("c3", "c4"):
        line = (run_c3 if args.config == "c3" else run_c4)(args, baseline, world, rank, dev)
        if rank == 0:
            if REHEARSE:
                line["rehearsal"] = "all ranks on cuda:0 over gloo (LPHY_BENCH_REHEARSE): not a scaling result"
            print(json.dumps(line))
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    frames = args.frames or DEFAULT_FRAMES.get(args.sf, 4096)
    slabs = ([shard.ResultSlab([frames], DATA_SYMS, PAYLOAD, dev) for _ in range(2)]
             if world > 1 else None)
    wl = Workload(args.sf, args.bw, frames, rank, dev, outs=[sl.views(0) for sl in slabs] if slabs else None)
    gat = Gatherer(slabs) if slabs else None
    mode_b = lphy.MODE_DECHIRP_LORA_DEMODULATE
    live_ev: list = []
    dt = timed(wl, mode_b, args.steps, args.warmup, world, events=live_ev, settle_s=SETTLE_S, gat=gat)
    gathered = None
    if gat:
        parts = gat.finish()
        if rank == 0:
            gathered = check_gathered(parts, args.sf, frames, world)
        wl.run(mode_b)  # slot 0 holds the results the local checks read
    ms = dt / args.steps * 1e3
    live_kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in live_ev]))
    data_syms = world * frames * DATA_SYMS
    value = data_syms * args.steps / dt
    check_b = wl.check(mode_b)
    st = wl.stage_times(mode_b)

    N = wl.N
    # dominant kernel = the fused launch (k_wave from SF 7, k_frames below):
    # algorithmic bytes = every IQ sample once + one u16 per data
    # symbol + the 32-B frame record (the two-symbol scans and the
    # settled frames' estimate re-reads are extra traffic, which the PMC
    # summary below shows)
    fused = frames_fused(args.sf)
    kern_bytes = frames * (wl.fs * 8 + DATA_SYMS * 2 + (32 if fused else 0))
    # the fused launch timed live in the timed region (k_wave + its fix-up
    # launch, which is empty unless a frame needs the exact re-run)
    kern_ms = live_kernel_ms if fused else st["unfused_symbols"]
    achieved = kern_bytes / (kern_ms * 1e-3) / 1e9
    step_gbps = frames * DATA_SYMS * bytes_per_data_symbol(N) / (ms * 1e-3) / 1e9
    traffic = measured_traffic(fused_kernel(args.sf) if fused else f"k_demod<{args.sf}>", frames)

    extra = {}
    if not args.no_mode_a:
        # (the same warmup as the headline's W steps: mode A's kernels are
        # other code objects, and the first launches after a change of
        # kernel run at the transient clocks §4.3 of DESIGN describes)
        dta = timed(wl, lphy.MODE_DEMODULATE, max(3, args.steps // 2), args.warmup, world)
        extra["demodulate_mode_A"] = {
            "value": data_syms * max(3, args.steps // 2) / dta, "unit": "data symbols/s",
            "check": wl.check(lphy.MODE_DEMODULATE)}
        wl.run(mode_b)  # leave mode-B results in place
    if (args.sweep or args.csv) and world == 1:
        rows = []
        profiles = [(f"sf{sf}_bw125", sf, 125000) for sf in range(8, 13)]
        if args.csv:
            profiles = REF_PROFILES + [p for p in profiles if p[1] >= 9]
        head = {"profile": f"sf{args.sf}_bw{args.bw // 1000}", **profile_row(wl, ms, args.steps)}
        for name, sf, bw in profiles:
            w2 = Workload(sf, bw, DEFAULT_FRAMES[sf], rank, dev)
            k = max(5, args.steps // 10)
            d2 = timed(w2, mode_b, k, 2, 1, settle_s=0.05)
            rows.append({"profile": name, **profile_row(w2, d2 / k * 1e3, k)})
            del w2
            torch.cuda.empty_cache()
        extra["sweep"] = {r["profile"]: r for r in [head] + rows}
        if args.csv:
            write_perf_csv(args.csv, args.run_id, [head] + rows)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(wl, args.cpu_seconds)
        except Exception as e:
            cpu = {"value": None, "unit": "data symbols/s", "cores": 0, "kind": "port",
                   "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": baseline["metric"],
            "value": value,
            "unit": "data symbols/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_s": SETTLE_S,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated lora_modulate IQ of random payloads)",
            "config": {
                "workload": f"SF{args.sf} BW{args.bw // 1000} CR4/5, {frames} frames/GPU x "
                            f"{PAYLOAD} B payload ({TOTAL_SYMS} symbols), fused dechirp -> "
                            "lora_demodulate -> lora_decode+CRC" +
                            (", gather of symbols + payloads + frame records to rank 0" if world > 1 else ""),
                "sf": args.sf, "bw_hz": args.bw, "frames_per_gpu": frames,
                "symbols_per_frame": TOTAL_SYMS, "parallelism": f"frames sharded x{world}",
            },
            "hbm_gbps_step": step_gbps,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": fused_kernel(args.sf) if fused else f"k_demod<{args.sf}>",
                         "bytes_per_launch": kern_bytes,
                         "avg_launch_ms": kern_ms,
                         "timing": "HIP events around each timed step's fused launch (+ its fix-up)"
                                   if fused else "HIP events, separate symbol-stage launches"},
            "stage_ms": st,
            "check": check_b,
            "gathered_rank0": gathered,
            "cpu_baseline": cpu,
        }
        line.update(extra)
        if REHEARSE:
            line["rehearsal"] = "all ranks on cuda:0 over gloo (LPHY_BENCH_REHEARSE): not a scaling result"
        print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
