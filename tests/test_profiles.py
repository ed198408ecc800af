"""The committed per-round evidence (rounds 3 to 5) is self-consistent: tools/roofline_table.py recomputes every
workload line's roofline fraction from profiles/rNN_workloads.jsonl (bytes per launch over the
line's own time basis) and its HBM traffic ratio from the committed rocprofv3 PMC summaries
(profiles/rNN_<tag>_pmc.json).  CPU only: reads committed files."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("rnd", ["r03", "r04", "r05", "r06"])
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
            # (ms_per_step is printed to 4 decimals: a 3.3 us window carries 1.5 % of rounding)
            rel = 0.01 + 0.00005 / max(r["ms_per_step"], 1e-9)
            assert abs(r["frac_recomputed"] - r["frac_line"]) <= rel * max(r["frac_line"], 1e-9) + 0.002, r
    # every line with a committed PMC summary has its traffic ratio; streaming lines read each
    # byte about once
    covered = {r["workload"]: r["traffic_ratio"] for r in rows if r["pmc"]}
    assert len(covered) >= 10
    for w, ratio in covered.items():
        assert ratio is not None and 0.9 <= ratio <= 5.0, (w, ratio)
    for w in ("knn_k50_r0.5_10Mpts_per_gpu_grid500x500", "range_pp_r0.5_10Mpts_grid100",
              "sliding_knn_k100_r0.5_100Mpts_grid1000"):
        assert covered[w] <= 1.05, (w, covered[w])


@pytest.mark.parametrize("rnd", ["r05", "r06"])
def test_occupancy_measured(tmp_path, rnd):
    """from r05 on, every committed PMC summary carries a measured occupancy
    (mean resident waves per SIMD from SQ_WAVE_CYCLES, never the all-zero SQ_LEVEL_WAVES), and the
    roofline table reports it for every line with PMC next to the compiler's register bound."""
    pm = [f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.startswith(rnd + "_") and f.endswith("_pmc.json")]
    if not pm:
        pytest.skip(f"no {rnd} PMC summaries")
    for f in pm:
        d = json.load(open(os.path.join(ROOT, "profiles", f)))["pmc"]
        for k, v in d.items():
            assert v.get("mean_waves_per_simd", 0) > 0, (f, k)
            assert v["median"].get("SQ_WAVE_CYCLES", 0) > 0, (f, k)
    if not os.path.exists(os.path.join(ROOT, "profiles", f"{rnd}_workloads.jsonl")):
        pytest.skip(f"no {rnd} workload lines")
    out = tmp_path / "roof"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_table.py"), rnd, "--out", str(out)],
                   check=True, capture_output=True, timeout=120)
    for r in json.load(open(str(out) + ".json")):
        if r["pmc"]:
            assert r["occupancy"] and all(o["mean_waves_per_simd"] > 0 and o["reg_bound_waves_per_simd"]
                                          for o in r["occupancy"]), r["workload"]
