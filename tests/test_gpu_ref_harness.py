"""The reference's own test harness and runners against the drop-in
(VERDICT r4 missing 2).  oracle/Makefile `harness` compiles the UNMODIFIED
reference sources - tests/*.cpp with -Dmain=<name>_main and test_main.cpp,
as its CMakeLists.txt:37-64 does, and runners/{rx,tx}_runner.cpp
(CMakeLists.txt:28-33) - twice: against include/ + liblora_phy_amd.so (the
GPU drop-in) and against the reference's own sources (the CPU library), plus
one executable per test so that sync_word_test's heap overflow
aborts only itself.  Both run here from one working directory holding copies
of the data files the tests open (tests/golden/ref_harness: the reference's
tests/profiles.yaml and vectors/golden/*.b64, and the committed
modulation_tests.bin, which the reference tree lacks).

Asserted: every test's exit status is the reference build's, and equals
SURVEY §0.8's pattern with bit_exact now passing on the committed
modulation_tests.bin (its BW250/500 records hold the reference's own decode,
tests/golden/make_golden.py); the deterministic tests print the same lines;
tx_runner | rx_runner prints the reference's payload hex."""
import shutil
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
H = ROOT / "oracle" / "_ref" / "harness"
DATA = ROOT / "tests" / "golden" / "ref_harness"

# SURVEY §0.8 (reference, measured), bit_exact with the file present
EXPECTED = {
    "bit_exact_test": 0,
    "e2e_chain_test": 1,          # the 4 BW250/500 profiles do not round-trip
    "no_alloc_test": 0,
    "performance_test": 0,
    "roundtrip_test": 0,
    "whitening_test": 0,
    "equal_power_bin_test": 0,
    "sync_word_test": None,       # overflows its heap buffer: aborts (non-zero)
    "error_code_test": 1,         # error_code_test.cpp:101, :159
    "odd_symbol_count_test": 0,
    "scratch_buffer_error_test": 0,
    "lorawan_mic_test": 0,
}


def _need():
    for side in ("amd", "ref"):
        if not (H / side / "lora_phy_tests").exists():
            pytest.skip("reference harness not built (make -C oracle harness, needs /root/reference)")


@pytest.fixture
def workdir(tmp_path):
    _need()
    shutil.copytree(DATA, tmp_path, dirs_exist_ok=True)
    shutil.copy(ROOT / "tests" / "golden" / "modulation_tests.bin", tmp_path / "vectors" / "golden")
    return tmp_path


def _run(exe, cwd, timeout=300, **kw):
    return subprocess.run([str(exe)], cwd=cwd, capture_output=True, text=True, timeout=timeout, **kw)


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_reference_test_against_drop_in(workdir, name):
    ours = _run(H / "amd" / name, workdir)
    ref = _run(H / "ref" / name, workdir)
    want = EXPECTED[name]
    ctx = f"{name}: ours rc {ours.returncode}\n{ours.stdout[-2000:]}{ours.stderr[-2000:]}\n" \
          f"ref rc {ref.returncode}\n{ref.stdout[-1000:]}{ref.stderr[-1000:]}"
    if want is None:
        assert ours.returncode != 0 and ref.returncode != 0, ctx
        return
    assert ref.returncode == want, ctx
    assert ours.returncode == want, ctx
    if name != "performance_test":  # (timing lines)
        assert ours.stdout.splitlines() == ref.stdout.splitlines(), ctx
        assert ours.stderr.splitlines() == ref.stderr.splitlines(), ctx
    else:
        lines = [l for l in ours.stdout.splitlines() if " pps, " in l]
        assert len(lines) == 7, ctx  # one per profile of tests/profiles.yaml


def test_lora_phy_tests_binary(workdir):
    """The reference's single test executable (test_main.cpp runs every
    test in turn; the sync_word abort ends it in both builds)."""
    ours = _run(H / "amd" / "lora_phy_tests", workdir)
    ref = _run(H / "ref" / "lora_phy_tests", workdir)
    # sync_word_test.cpp:27-29 writes 256 samples into 255: undefined
    # behaviour that glibc reports as "malloc(): corrupted top size" (abort)
    # under the reference build and that may surface as a segfault instead
    # under another heap layout; either way the process dies by a signal in
    # both builds, and the output buffered before it is lost
    assert ours.returncode < 0 and ref.returncode < 0, (ours.returncode, ref.returncode, ours.stderr[-2000:])
    # the tests before sync_word report on stderr (unbuffered): the same lines
    strip = lambda s: [l for l in s.splitlines() if "corrupted" not in l]
    assert strip(ours.stderr) == strip(ref.stderr), (ours.stderr[-3000:], ref.stderr[-3000:])


@pytest.mark.parametrize("payload,sf", [("48656c6c6f", 7), ("48656c6c6f", 9), ("deadbeef00112233", 8),
                                        ("00", 12), ("0123456789abcdef0123456789abcdef", 10)])
def test_tx_rx_runner_pipe(workdir, payload, sf):
    out = {}
    for side in ("amd", "ref"):
        tx = subprocess.run([str(H / side / "tx_runner"), f"--payload={payload}", f"--sf={sf}", "--stdout"],
                            cwd=workdir, capture_output=True, timeout=120)
        assert tx.returncode == 0, tx.stderr
        rx = subprocess.run([str(H / side / "rx_runner"), f"--sf={sf}", "--report-offsets"], input=tx.stdout,
                            cwd=workdir, capture_output=True, timeout=120)
        assert rx.returncode == 0, rx.stderr
        out[side] = (tx.stdout, rx.stdout.decode())
    assert out["amd"][0] == out["ref"][0]  # the IQ, byte for byte
    assert out["amd"][1] == out["ref"][1], out
    if payload == "48656c6c6f" and sf == 7:
        assert out["ref"][1].splitlines()[0] == "Payload: 0ca9a0a0a3"
