"""Iterate the committed golden fixtures (TEST INFRASTRUCTURE ONLY).

Each case yields its input IQ (stored in golden_v1.npz or regenerated from
its recipe and checked against the recorded SHA-256) and the reference's
recorded outputs for lora_phy::demodulate/decode and lora_demodulate/
lora_decode (tests/golden/make_golden.py wrote them from the reference
library built from /root/reference's sources)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from recipes import make_iq, sha256

HERE = Path(__file__).resolve().parent
MANIFEST = json.loads((HERE / "manifest.json").read_text())
_ARR = None


def arrays():
    global _ARR
    if _ARR is None:
        _ARR = dict(np.load(HERE / "golden_v1.npz", allow_pickle=False))
    return _ARR


def case_names():
    return [c["name"] for c in MANIFEST["cases"]]


def case(name: str) -> dict:
    return next(c for c in MANIFEST["cases"] if c["name"] == name)


def case_iq(oracle, c: dict) -> np.ndarray:
    if c["stored"]:
        iq = arrays()[f"{c['name']}__iq"]
    else:
        iq = make_iq(oracle, c["recipe"])
    assert iq.size == c["samples"], c["name"]
    assert sha256(iq) == c["sha256"], f"{c['name']}: regenerated input drifted"
    return iq


def expected_syms(c: dict, api: str) -> np.ndarray:
    return arrays()[f"{c['name']}__{api}__syms"]


def lora_input(oracle, c: dict, iq: np.ndarray) -> np.ndarray:
    """lora_demodulate's input: the externally dechirped buffer when the
    reference run dechirped (whole symbols), else the raw samples."""
    if c["results"]["lora_demodulate"]["input"] == "dechirped":
        return oracle.dechirp(iq, c["sf"], c["bw"])
    return iq


def fbits(x) -> str:
    return f"{int(np.asarray(x, np.float32).view(np.uint32)):08x}"
