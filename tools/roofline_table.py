"""Recompute every workload line's roofline fraction and HBM traffic ratio from profiles/.

Inputs (all committed under profiles/):
  rNN_workloads.jsonl     the bench lines (tools/gpu_workloads.sh: bench.py --workload ...)
  rNN_<tag>_pmc.json      tools/pmc_table.py summaries of the rocprofv3 --pmc passes of the same
                          commands (tools/gpu_pmc_round.sh): per kernel the median FETCH_SIZE /
                          WRITE_SIZE per dispatch and the dispatch counts

Per line:  frac      = roofline.bytes_per_launch / time / peak, time = the line's own basis:
                       the window interval (ms_per_step) when it keeps windows in flight
                       ("interval" in achieved_basis), else the kernel's average launch
           traffic   = sum over the workload's kernels of (2 x FETCH_SIZE + WRITE_SIZE) per
                       dispatch x dispatches per main-kernel launch, / windows per launch
                       (config.windows_per_launch: batched range windows);
                       FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half of wide
                       streaming reads; other access widths are uncalibrated -- an upper bound)
           ratio     = traffic / algorithmic bytes

usage: roofline_table.py ROUND [--out profiles/ROUND_roofline]   (writes .json and .md)
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0  # GB/s (MI355X_MICROARCH.md)

# workload name prefix -> (PMC tag, regex of the main kernel, regex of the window's kernels)
TAGS = [
    ("knn_k50_r0.5_10Mpts_per_gpu_grid500x500_clustered", None, None, None),
    ("knn_k50", "knn", r"knn_fused", r"knn_"),
    ("knn_ppoly", "polyknn", r"knn_poly_scan|knn_poly_fused", r"knn_"),
    ("range_pp_r0.5_1Mpts", "range1m", r"range_batch|range_kernel", r"range_|expand"),
    ("range_pp_r0.5_10Mpts", "range10m", r"range_kernel", r"range_|expand"),
    ("ppoly_", "ppoly", r"range_kernel", r"range_|expand"),
    ("join_pp_10Mx1M_r0.001_grid1000_clustered", "joinc", r"join_band_probe", r"join_band"),
    ("join_pp_", "join", r"join_band_probe|join_row_probe", r"join_|scan1"),
    ("join_ppoly", "pjoin", r"join_ppoly_count", r"range_|join_ppoly"),
    ("sliding_", "sliding", r"knn_fused", r"knn_|pane"),
    # (the main-kernel regex sets the per-window normalisation: a kernel launched ONCE per window --
    # K2 runs two scatter passes per window, so the scatter would halve the traffic)
    ("bucket_", "bucket", r"radix_hist", r"radix|scan1|assign"),
    ("csv_", "csv", r"csv_parse", r"csv_|range_|expand|objid"),
    ("geojson_", "geojson", r"csv_parse", r"csv_|geo|range_|expand|objid"),
]


def tag_of(workload):
    for pre, tag, main, allk in TAGS:
        if workload.startswith(pre):
            return tag, main, allk
    return None, None, None


def traffic_of(pmc, main, allk):
    ks = {k: v for k, v in pmc.items() if re.search(allk, k)}
    mains = [v["dispatches"] for k, v in ks.items() if re.search(main, k)]
    if not mains:
        return None, None
    ref = max(mains)
    tot, rows = 0.0, []
    for k, v in sorted(ks.items()):
        if "hbm_read_bytes_corrected" not in v or "hbm_write_bytes" not in v:
            continue
        per = v["dispatches"] / ref
        b = (v["hbm_read_bytes_corrected"] + v["hbm_write_bytes"]) * per
        tot += b
        rows.append({"kernel": k, "launches_per_window": round(per, 3),
                     "read_MB": round(v["hbm_read_bytes_corrected"] / 1e6, 2),
                     "write_MB": round(v["hbm_write_bytes"] / 1e6, 2)})
    return tot, rows


def _short(k):
    """'void gf::knn_fused_kernel<0, 1>(gf::KnnScanArgs, ...) [clone .kd]' -> 'knn_fused_kernel<0, 1>'"""
    k = re.sub(r"^void ", "", k.split("(")[0])
    return k.replace("gf::", "")


def occupancy_of(pmc, main, rnd):
    """The main kernel's measured mean resident waves per SIMD (tools/pmc_table.py: SQ_WAVE_CYCLES over
    the busy cycles) and the compiler's register bound (profiles/<rnd>_resource_usage.json)."""
    meas = [(k, v["mean_waves_per_simd"]) for k, v in pmc.items() if re.search(main, k) and "mean_waves_per_simd" in v]
    ru = os.path.join(ROOT, "profiles", f"{rnd}_resource_usage.json")
    regs = {}
    if os.path.exists(ru):
        with open(ru) as fh:
            regs = {_short(k): v for k, v in json.load(fh)["kernels"].items()}
    out = []
    for k, w in meas:
        r = regs.get(_short(k), {})
        out.append({"kernel": _short(k), "mean_waves_per_simd": round(w, 2),
                    "vgpr": r.get("vgpr"), "reg_bound_waves_per_simd": r.get("waves_per_simd_regs")})
    return out or None


def main():
    rnd = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(ROOT, "profiles", f"{rnd}_roofline")
    res = []
    with open(os.path.join(ROOT, "profiles", f"{rnd}_workloads.jsonl")) as f:
        lines = [json.loads(x) for x in f if x.strip().startswith("{")]
    for d in lines:
        w = d["config"]["workload"]
        r = d["roofline"]
        bpl, us = r.get("bytes_per_launch"), r.get("avg_launch_us")
        basis = (r.get("achieved_basis") or (d.get("breakdown") or {}).get("achieved_basis") or "")
        if "interval" in basis:  # windows in flight: bytes of a window over the window interval
            us = 1000.0 * d["ms_per_step"]
        frac = bpl / (us * 1e-6) / 1e9 / PEAK if bpl and us else None
        wpl = d["config"].get("windows_per_launch", 1) or 1  # batched launches carry several windows
        row = {"workload": w, "ms_per_step": d["ms_per_step"], "algorithmic_MB": round(bpl / 1e6, 1) if bpl else None,
               "frac_line": r.get("frac"), "frac_recomputed": round(frac, 4) if frac else None,
               "traffic_MB": None, "traffic_ratio": None, "pmc": None, "kernels": None, "occupancy": None}
        tag, main, allk = tag_of(w)
        p = os.path.join(ROOT, "profiles", f"{rnd}_{tag}_pmc.json") if tag else None
        if p and os.path.exists(p):
            with open(p) as fh:
                pm = json.load(fh)["pmc"]
            row["occupancy"] = occupancy_of(pm, main, rnd)
            t, rows = traffic_of(pm, main, allk)
            if t:
                t /= wpl
                row.update(traffic_MB=round(t / 1e6, 1), traffic_ratio=round(t / bpl, 3) if bpl else None,
                           pmc=os.path.relpath(p, ROOT), kernels=rows)
        res.append(row)
    with open(out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    with open(out + ".md", "w") as f:
        f.write(f"# {rnd} roofline table (tools/roofline_table.py {rnd})\n\n")
        f.write("| workload | ms / window | algorithmic MB | frac (line) | frac (recomputed) | PMC traffic MB | "
                "traffic / algorithmic | main kernel: measured mean waves/SIMD (register bound) |\n")
        f.write("|---|---|---|---|---|---|---|---|\n")
        for r in res:
            occ = "; ".join(f"{o['kernel']}: {o['mean_waves_per_simd']} ({o['reg_bound_waves_per_simd']})"
                            for o in (r["occupancy"] or [])) or "n/a"
            f.write(f"| {r['workload']} | {r['ms_per_step']} | {r['algorithmic_MB']} | {r['frac_line']} | "
                    f"{r['frac_recomputed']} | {r['traffic_MB'] if r['traffic_MB'] is not None else 'n/a'} | "
                    f"{r['traffic_ratio'] if r['traffic_ratio'] is not None else 'n/a'} | {occ} |\n")
        f.write("\nOccupancy: mean resident waves per SIMD over the kernel's lifetime = 4 x SQ_WAVE_CYCLES / "
                "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) from the occ PMC pass (ramp-up and tail included); in "
                "parentheses the compiler's register bound (-Rpass-analysis=kernel-resource-usage, "
                f"profiles/{rnd}_resource_usage.json) -- LDS and block size can bound a launch lower.\n")
    print(open(out + ".md").read())


if __name__ == "__main__":
    main()
