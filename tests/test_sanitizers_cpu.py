"""Host sanitizer coverage (an ASan/UBSan build of the CPU side).

* oracle/_build/oracle_san: the CPU oracle under ASan + UBSan driven over
  exact-size heap buffers (oracle/san_driver.c: round trips SF 5-12, osr 1/2,
  Hann, ragged / truncated counts, capacity and scratch errors, garbage
  symbols, codec and LoRaWAN helpers).
* lib/san/: the C ABI's host code and the lora_phy:: / lorawan:: shims under
  ASan + UBSan (`make san`), driven here through the API probes without a GPU
  (argument validation and the no-device error paths); tests/test_gpu_sanitizers.py
  runs the same probes on the GPU against the reference transcripts."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"
SAN_LIB = PKG / "lib" / "san"
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"
SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:protect_shadow_gap=0:abort_on_error=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer")


def _clean(proc):
    text = proc.stdout + proc.stderr
    return [ln for ln in text.splitlines() if any(r in ln for r in REPORTS)]


def build_probe(src: Path, out: Path) -> None:
    subprocess.run([CLANGXX, "-O1", "-std=gnu++17", "-ffp-contract=off", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", f"-I{ROOT / 'include'}",
                    "-o", str(out), str(src), f"-L{SAN_LIB}", "-llora_phy_amd", f"-Wl,-rpath,{SAN_LIB}"],
                   check=True)


def run_san(args, **kw):
    env = dict(os.environ, **SAN_ENV)
    return subprocess.run(args, capture_output=True, text=True, env=env, **kw)


def test_oracle_under_asan_ubsan():
    exe = ROOT / "oracle" / "_build" / "oracle_san"
    if not exe.exists():
        if shutil.which("gcc") is None:
            pytest.skip("no gcc to build oracle/_build/oracle_san")
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "san"], check=True, capture_output=True)
    p = run_san([str(exe)], timeout=300)
    assert not _clean(p), "\n".join(_clean(p))
    assert p.returncode == 0, p.stderr[-2000:]
    assert "all checks held" in p.stdout


@pytest.mark.parametrize("probe", ["lora_phy_api_probe", "lorawan_api_probe"])
def test_api_host_code_under_asan_ubsan_without_gpu(tmp_path, probe):
    """The drop-in's host code (argument checks, workspace side effects, the
    no-device error returns) under ASan + UBSan, with no GPU: every call that
    needs the device fails with its error code and nothing is touched out of
    bounds."""
    if not (SAN_LIB / "liblora_phy_amd.so").exists() or not Path(CLANGXX).exists():
        pytest.skip("lib/san not built (make -C <pkg> san)")
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: tests/test_gpu_sanitizers.py covers this")
    except ImportError:
        pass
    exe = tmp_path / probe
    build_probe(ROOT / "tests" / "cpp" / f"{probe}.cpp", exe)
    p = run_san([str(exe), str(ROOT / "tests" / "golden")], timeout=300)
    assert not _clean(p), "\n".join(_clean(p)[:20])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(p.stdout.splitlines()) >= 10
