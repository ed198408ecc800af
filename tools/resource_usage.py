"""Per-kernel register / LDS budget of the product's gfx950 code objects, from the compiler's
`-Rpass-analysis=kernel-resource-usage` remarks (VGPRs, AGPRs, SGPRs, scratch, static LDS, and the
compiler's waves-per-SIMD bound from registers alone).  The bound a LAUNCH gets is the minimum of
that and what its LDS (static + the dynamic LDS the host passes) and block size admit:
    waves/SIMD <= floor(160 KiB / LDS per block) * (threads per block / 64) / 4.
tools/pmc_table.py puts the MEASURED mean resident waves next to it (SQ_WAVE_CYCLES over the
kernel's busy cycles); tools/roofline_table.py prints both.

usage: python tools/resource_usage.py OUT.json   (compiles each .hip once, ~1 min)
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "spatialflink_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
         "-c", "-Rpass-analysis=kernel-resource-usage", "-o", os.devnull]
FIELDS = {"TotalSGPRs": "sgpr", "VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch_bytes",
          "Occupancy [waves/SIMD]": "waves_per_simd_regs", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "LDS Size [bytes/block]": "lds_static_bytes"}


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except Exception:  # noqa: BLE001
        return names


def usage(path):
    p = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, path], capture_output=True, text=True, cwd="/tmp")
    kernels, cur = {}, None
    for line in p.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+) \[", line)
        if m:
            cur = kernels.setdefault(m.group(1), {"file": os.path.basename(path)})
            continue
        m = re.search(r"remark:\s+([^:]+(?:\[[^\]]*\])?): (\S+) \[-Rpass", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            v = m.group(2)
            cur[FIELDS[m.group(1).strip()]] = int(v) if v.lstrip("-").isdigit() else v
    return kernels


def main():
    out = sys.argv[1]
    allk = {}
    for f in sorted(os.listdir(SRC)):
        if f.endswith(".hip"):
            allk.update(usage(os.path.join(SRC, f)))
    names = list(allk)
    res = {}
    for mangled, pretty in zip(names, demangle(names)):
        d = allk[mangled]
        d["mangled"] = mangled
        res[pretty] = d
    with open(out, "w") as fh:
        json.dump({"note": "hipcc -Rpass-analysis=kernel-resource-usage, gfx950; waves_per_simd_regs = the "
                           "compiler's register bound (dynamic LDS and block size not included)",
                   "kernels": res}, fh, indent=1, sort_keys=True)
    print(f"{len(res)} kernels -> {out}")


if __name__ == "__main__":
    main()
