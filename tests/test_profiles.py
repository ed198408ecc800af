"""The committed per-round evidence (rounds 3 and 4) is self-consistent: tools/roofline_table.py recomputes every
workload line's roofline fraction from profiles/rNN_workloads.jsonl (bytes per launch over the
line's own time basis) and its HBM traffic ratio from the committed rocprofv3 PMC summaries
(profiles/rNN_<tag>_pmc.json).  CPU only: reads committed files."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("rnd", ["r03", "r04"])
def test_roofline_table_reproduces_lines(tmp_path, rnd):
    if not os.path.exists(os.path.join(ROOT, "profiles", f"{rnd}_workloads.jsonl")):
        pytest.skip(f"no {rnd} workload lines")
    out = tmp_path / "roof"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_table.py"), rnd, "--out", str(out)],
                   check=True, capture_output=True, timeout=120)
    rows = json.load(open(str(out) + ".json"))
    assert len(rows) >= 13
    for r in rows:
        if r["frac_line"] is not None and r["frac_recomputed"] is not None:
            assert abs(r["frac_recomputed"] - r["frac_line"]) <= 0.01 * max(r["frac_line"], 1e-9) + 0.002, r
    # every line with a committed PMC summary has its traffic ratio; streaming lines read each
    # byte about once
    covered = {r["workload"]: r["traffic_ratio"] for r in rows if r["pmc"]}
    assert len(covered) >= 10
    for w, ratio in covered.items():
        assert ratio is not None and 0.9 <= ratio <= 5.0, (w, ratio)
    for w in ("knn_k50_r0.5_10Mpts_per_gpu_grid500x500", "range_pp_r0.5_10Mpts_grid100",
              "sliding_knn_k100_r0.5_100Mpts_grid1000"):
        assert covered[w] <= 1.05, (w, covered[w])
