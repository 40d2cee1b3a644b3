"""include/lora_phy/LoRaCodes.hpp (this tree's codec helpers) against the
reference's header of the same name: tests/cpp/codes_probe.cpp compiled
against each prints a transcript of every helper over exhaustive 8/16-bit
inputs, seeded buffers and the interleaver geometries; they must be equal.
The reference half needs /root/reference (skipped elsewhere); the whitening
known answer of the reference's own whitening_test.cpp:30-31 is checked on
this tree's header everywhere."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PROBE = ROOT / "tests" / "cpp" / "codes_probe.cpp"
REF_INC = Path("/root/reference/include/lora_phy")


def _transcript(tmp_path, inc: Path, name: str) -> list[str]:
    exe = tmp_path / name
    subprocess.run(["g++", "-O2", "-std=gnu++17", f"-I{inc}", "-o", str(exe), str(PROBE)], check=True)
    return subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines()


def test_whitening_known_answer(tmp_path):
    out = _transcript(tmp_path, ROOT / "include" / "lora_phy", "probe_ours")
    kat = [int(l.split()[1], 16) for l in out if l.startswith("wkat ")]
    assert kat == [0x21, 0x52, 0x90, 0x10, 0x2C, 0xF2]  # whitening_test.cpp:30-31


@pytest.mark.skipif(not (REF_INC / "LoRaCodes.hpp").exists(), reason="needs /root/reference")
def test_codes_match_reference(tmp_path):
    ours = _transcript(tmp_path, ROOT / "include" / "lora_phy", "probe_ours")
    ref = _transcript(tmp_path, REF_INC, "probe_ref")
    assert len(ours) == len(ref) > 100000
    bad = [(i, a, b) for i, (a, b) in enumerate(zip(ours, ref)) if a != b]
    assert not bad, bad[:10]
