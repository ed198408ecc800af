"""CPU: the inter-workgroup hand-offs of the join band probe and of the range scan's count
finalisation follow the write-through form of cdna_hip_programming.md Guideline 16 (R1), checked
in the gfx950 ISA the product is built from ("correct on gfx950 only by the
hardware's store-ack semantics, pinned by no dedicated test"):
  (1) every handed-off word is stored write-through (`global_store_* ... sc1`: agent-scope atomic
      stores),
  (2) the storing lane drains its stores (`s_waitcnt vmcnt(0)`) before the counter add that
      signals them,
  (3) the counter is an atomic (`global_atomic_add*`),
  (4) the last arriver reads the handed-off words with `sc1` loads (agent-scope atomic loads:
      they bypass this CU's L1, so no acquire fence is needed).
join_band_probe_kernel: the per-block pair counts / slice sizes -> the ticket -> join_region_prep;
range_kernel: the per-block partial counts -> the ticket -> finalize_counts."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


def device_asm(src, tmp_path):
    out = str(tmp_path / (os.path.basename(src) + ".s"))
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-x", "hip", "-S",
                    "--cuda-device-only", os.path.join(ROOT, "spatialflink_amd", "csrc", src), "-o", out], check=True,
                   capture_output=True)
    return open(out).read()


def function_body(asm, mangled_prefix):
    m = re.search(r"^(" + re.escape(mangled_prefix) + r"\S*):\s*;", asm, re.M)
    assert m, mangled_prefix
    end = asm.index(".Lfunc_end", m.end())
    return [ln.strip() for ln in asm[m.end():end].splitlines()]


def check_handoff(body, n_payload):
    """The signalling atomic add preceded by vmcnt(0) and n_payload sc1 stores; sc1 loads after it."""
    ticket = None
    for k, ln in enumerate(body):
        if not ln.startswith("global_atomic_add"):
            continue
        back = [b for b in body[max(0, k - 40):k] if b and not b.startswith((";", "v_readlane", "v_mov", "s_mov",
                                                                                "v_mbcnt", "v_cmp", "s_and_saveexec",
                                                                                "s_cbranch", "s_bcnt", "s_nop"))]
        if "s_waitcnt vmcnt(0)" not in back:
            continue
        w = len(back) - 1 - back[::-1].index("s_waitcnt vmcnt(0)")
        stores = [b for b in back[:w] if b.startswith("global_store")]
        if len(stores) >= n_payload and all(" sc1" in s_ for s_ in stores[-n_payload:]):
            # no store between the drain and the atomic
            assert not any(b.startswith("global_store") for b in back[w + 1:])
            ticket = k
            break
    assert ticket is not None, "no sc1 stores -> vmcnt(0) -> atomic add hand-off found"
    loads = [ln for ln in body[ticket:] if ln.startswith("global_load")][:2 * n_payload + 2]
    assert sum(" sc1" in ln for ln in loads) >= n_payload, loads
    return ticket


def static_lds(asm, mangled_prefix):
    m = re.search(r"^\s*\.amdhsa_kernel (" + re.escape(mangled_prefix) + r"\S*)$", asm, re.M)
    assert m, mangled_prefix
    f = re.search(r"\.amdhsa_group_segment_fixed_size (\d+)", asm[m.end():])
    return int(f.group(1))


@pytest.mark.timeout(600)
def test_join_band_probe_handoff_is_write_through(tmp_path):
    asm = device_asm("k_join.hip", tmp_path)
    for mode in (0, 1):
        body = function_body(asm, f"_ZN2gf22join_band_probe_kernelILi{mode}E")
        check_handoff(body, 2)  # bcount, bslice
        # the probe takes the whole 160 KB as dynamic LDS: any static LDS (e.g. the scratch word
        # of a __syncthreads_or) makes every dispatch invalid (HSA_STATUS_ERROR_INVALID_ALLOCATION)
        assert static_lds(asm, f"_ZN2gf22join_band_probe_kernelILi{mode}E") == 0


@pytest.mark.timeout(600)
def test_range_finalize_handoff_is_write_through(tmp_path):
    asm = device_asm("k_range.hip", tmp_path)
    body = function_body(asm, "_ZN2gf12range_kernelILi1ELi1ELi3ELi2E")
    check_handoff(body, 2)  # the block's two partial counts
