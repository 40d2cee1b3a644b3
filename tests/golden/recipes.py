"""Input recipes for the golden fixtures (TEST INFRASTRUCTURE ONLY).

A fixture input is either stored verbatim (complex64 in golden_v1.npz) or
described by a recipe that is regenerated here and checked against the
SHA-256 recorded by make_golden.py, so a drift in regeneration fails loudly
instead of silently comparing different inputs.

Recipe = {"payload_hex", "sf", "bw", "sync", "delay", "snr_db", "seed",
          "noise_only", "nsyms"}:
  payload -> lora_encode -> lora_modulate (the CPU oracle, itself pinned
  bit-for-bit to the reference's LoRaMod.cpp / ChirpGenerator.hpp), then an
  optional integer sample delay (zeros in front, same length) and optional
  AWGN from numpy's PCG64 default_rng(seed), sigma = sqrt(10^(-snr/10)/2)
  per component.
"""
from __future__ import annotations

import hashlib

import numpy as np


def sha256(iq: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(iq, np.complex64).tobytes()).hexdigest()


def make_iq(oracle, r: dict) -> np.ndarray:
    sf, bw = r["sf"], r["bw"]
    N = 1 << sf
    if r.get("noise_only"):
        n = r["nsyms"] * N
        rng = np.random.default_rng(r["seed"])
        iq = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * r.get("sigma", 1.0)
        return iq.astype(np.complex64)
    payload = bytes.fromhex(r["payload_hex"])
    syms = oracle.encode(payload)
    iq = oracle.modulate(syms, sf, bw_hz=bw, sync=r.get("sync", 0x12))
    d = r.get("delay", 0)
    if d:
        iq = np.concatenate([np.zeros(d, np.complex64), iq[:-d]]).astype(np.complex64)
    if r.get("snr_db") is not None:
        rng = np.random.default_rng(r["seed"])
        sig = np.sqrt(10 ** (-r["snr_db"] / 10) / 2)
        noise = sig * (rng.standard_normal(iq.size) + 1j * rng.standard_normal(iq.size))
        iq = (iq + noise).astype(np.complex64)
    return np.ascontiguousarray(iq, np.complex64)
