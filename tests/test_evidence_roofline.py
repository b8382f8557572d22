"""The kept round evidence is self-consistent: every roofline `frac` in the
committed bench line is recomputable from the committed one-stream rocprof kernel-stats CSV
(tools/recompute_roofline.py) to within the HIP-event overhead, and the PMC traffic files carry
the source digests bench.py checks."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "profiles", "r05", "bench_final.json")
STATS = os.path.join(REPO, "profiles", "r05", "kernel_stats_bench_final.csv")


@pytest.mark.skipif(not (os.path.exists(BENCH) and os.path.exists(STATS)), reason="no kept evidence")
def test_every_frac_recomputes_from_the_kept_csv():
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "recompute_roofline.py"), BENCH, STATS],
                         capture_output=True, text=True, check=True).stdout.strip().splitlines()
    rows = [ln.split() for ln in out[1:]]
    assert len(rows) >= 3
    for r in rows:
        frac_bench, frac_csv = float(r[-2]), float(r[-1])
        assert frac_csv == pytest.approx(frac_bench, rel=0.05), r     # events add 1-3 % per launch


def test_traffic_files_name_their_kernels_and_digests():
    for name in ("traffic_latest.json", "traffic_kernels.json"):
        d = json.load(open(os.path.join(REPO, "profiles", name)))
        entries = [d] if name == "traffic_latest.json" else list(d.values())
        assert entries
        for e in entries:
            assert e["hbm_bytes_per_launch"] > 0 and len(e["source_digest"]) == 64 and "FETCH_SIZE" in e["method"]
