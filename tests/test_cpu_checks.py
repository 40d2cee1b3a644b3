"""Host-side checks of the device code's building blocks (no GPU):
* csrc/libm_exact.h (the glibc-exact sincosf / atan2f / cabsf the kernels
  evaluate) against the host glibc, bit for bit, over float ranges that
  cover the fast path, the > 120 rad large-argument path, negatives,
  subnormals, infinities and NaN;
* csrc/lphy_fft.h's index algebra (LDS address bijection, lane/element bit
  split, every position touched once per pass) for SF 1-12."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CPP = ROOT / "tests" / "cpp"


@pytest.fixture(scope="module")
def bins(tmp_path_factory):
    d = tmp_path_factory.mktemp("cpu_checks")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o",
                    str(d / "libm_check"), str(CPP / "libm_exact_check.cpp")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "-o", str(d / "fft_layout"),
                    str(CPP / "fft_layout_check.hip")], check=True)
    return d


RANGES = {
    "tiny_and_subnormal": (0x00000000, 0x00400000),
    "around_pi_over_4": (0x3f400000, 0x3f800000),
    "one_to_eight": (0x3f800000, 0x41000000),
    "up_to_120": (0x42e00000, 0x42f00000),
    "large_path": (0x42f00000, 0x43300000),
    "huge": (0x4e000000, 0x4e200000),
    "negative": (0xbf800000, 0xc0400000),
    "inf_nan": (0x7f7ffff0, 0x7fc00010),
}


@pytest.mark.parametrize("name", sorted(RANGES))
def test_sincosf_exact_ranges(bins, name):
    lo, hi = RANGES[name]
    r = subprocess.run([str(bins / "libm_check"), "sincos", str(lo), str(hi), "8"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout


def test_payne_hanek_windows_without_memory(bins):
    """The device's memory-free Payne-Hanek windows (libm_exact.h
    inv_pio4_shift: shifts of the 2/pi bit string) equal glibc's table for
    every index, so the large-argument sincos path is unchanged bit for bit."""
    r = subprocess.run([str(bins / "libm_check"), "pio4", "0", "0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "mismatches=0 checked=24" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("what,seed", [("atan2", 1), ("atan2", 2), ("cabs", 3)])
def test_atan2f_cabsf_exact(bins, what, seed):
    r = subprocess.run([str(bins / "libm_check"), what, "2000000", str(seed), "8"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout


def test_fft_layout_algebra(bins):
    r = subprocess.run([str(bins / "fft_layout")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == 12, r.stdout


@pytest.mark.parametrize("what", ["logf", "log10"])
def test_log10f_exact_all_floats(bins, what):
    """log10f drives the osr>1 estimator's detector power (LoRaDetector.hpp:64);
    the restatement is checked against glibc for every float bit pattern."""
    for lo, hi in ((0x00000000, 0x7f800000), (0x7f800001, 0xffffffff)):
        r = subprocess.run([str(bins / "libm_check"), what, str(lo), str(hi), "8"],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "mismatches=0" in r.stdout
