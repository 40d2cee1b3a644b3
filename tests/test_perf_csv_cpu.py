"""The perf CSV (bench.py --csv) and its regression gate (tools/compare_perf.py),
on CPU: the schema is the reference's (performance_test.cpp:69-75) plus
hbm_gbps / roofline_frac, and the gate flags what scripts/compare_perf.py:
18-43 flags (pps down, cycles per symbol up) and a roofline drop."""
import csv
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import compare_perf  # noqa: E402


def _write(path, rows):
    import bench
    bench.write_perf_csv(str(path), "t", rows)


def _row(profile, pps, cps, gbps):
    return {"profile": profile, "sf": 7, "N": 128, "pps": pps, "cycles_per_symbol": cps,
            "hbm_gbps": gbps, "roofline_frac": gbps / 8000.0}


def test_csv_schema_and_gate(tmp_path):
    a, b = tmp_path / "a.csv", tmp_path / "b.csv"
    _write(a, [_row("sf7_bw125_cr45", 6.0e7, 0.6, 4400.0), _row("sf12_bw500_cr45", 1.0e6, 170.0, 2000.0)])
    with open(a, newline="") as f:
        r = list(csv.reader(f))
    assert r[0] == ["run_id", "profile", "sf", "N", "pps", "cycles_per_symbol", "hbm_gbps", "roofline_frac"]
    assert len(r) == 3 and r[1][1] == "sf7_bw125_cr45"
    _write(b, [_row("sf7_bw125_cr45", 6.1e7, 0.59, 4450.0), _row("sf12_bw500_cr45", 1.0e6, 170.0, 1900.0)])
    reg = compare_perf.compare(compare_perf.load(str(a)), compare_perf.load(str(b)))
    assert [(p, k) for p, k, _, _ in reg] == [("sf12_bw500_cr45", "hbm_gbps"), ("sf12_bw500_cr45", "roofline_frac")]
    assert compare_perf.compare(compare_perf.load(str(a)), compare_perf.load(str(b)), tol=0.06) == []
    p = subprocess.run([sys.executable, str(ROOT / "tools" / "compare_perf.py"), str(a), str(b)],
                       capture_output=True, text=True)
    assert p.returncode == 2 and "REGRESSION" in p.stdout
    p = subprocess.run([sys.executable, str(ROOT / "tools" / "compare_perf.py"), str(a), str(a)],
                       capture_output=True, text=True)
    assert p.returncode == 0
