"""The drop-in's host code under ASan + UBSan on the GPU (lib/san/, built by
`make san`: csrc/lphy_hip.hip's host side and the lora_phy:: / lorawan::
shims instrumented, the kernels unchanged).  The API probes run the
reference-test scenarios through it with no sanitizer report, and print the
same transcript as the same probe source, built by the same compiler without
sanitizers, against the product libraries (lib/).  (The probe's impairment
generator rounds differently under clang and g++, so the reference
comparison itself stays with the g++ builds of tests/test_gpu_cxx_api.py.)"""
import subprocess
from pathlib import Path

import pytest

from test_sanitizers_cpu import CLANGXX, PKG, ROOT, SAN_LIB, _clean, build_probe, run_san

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("probe,min_lines", [("lora_phy_api_probe", 25), ("lorawan_api_probe", 400)])
def test_api_probe_under_asan_ubsan(tmp_path, probe, min_lines):
    if not (SAN_LIB / "liblora_phy_amd.so").exists():
        pytest.fail("lib/san not built: __graft_entry__.build() runs `make san`")
    if not Path(CLANGXX).exists():
        pytest.skip("no clang++ for the sanitizer runtime")
    src = ROOT / "tests" / "cpp" / f"{probe}.cpp"
    exe = tmp_path / f"{probe}_san"
    build_probe(src, exe)
    plain = tmp_path / f"{probe}_plain"
    lib = PKG / "lib"
    subprocess.run([CLANGXX, "-O1", "-std=gnu++17", "-ffp-contract=off", f"-I{ROOT / 'include'}", "-o", str(plain),
                    str(src), f"-L{lib}", "-llora_phy_amd", f"-Wl,-rpath,{lib}"], check=True)
    golden = str(ROOT / "tests" / "golden")
    ours = run_san([str(exe), golden], timeout=300)
    assert not _clean(ours), "\n".join(_clean(ours)[:20])
    assert ours.returncode == 0, ours.stderr[:6000]  # the report's head names the fault
    ref = subprocess.run([str(plain), golden], capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr
    a, b = ours.stdout.splitlines(), ref.stdout.splitlines()
    assert len(a) == len(b) and len(b) >= min_lines
    bad = [(x, y) for x, y in zip(a, b) if x != y]
    assert not bad, "\n".join(f"san:   {x[:300]}\nplain: {y[:300]}" for x, y in bad[:5])
