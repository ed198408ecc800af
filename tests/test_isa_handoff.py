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


def _after_barrier(body, k):
    """index of the first s_barrier at or after k whose preceding non-comment lines (within 12)
    hold s_waitcnt vmcnt(0)"""
    for j in range(k, len(body)):
        if body[j].startswith("s_barrier"):
            prev = [b for b in body[max(0, j - 12):j] if b and not b.startswith(";")]
            if any(b.startswith("s_waitcnt") and "vmcnt(0)" in b for b in prev):
                return j
    return None


@pytest.mark.timeout(600)
def test_range_drain_and_wave_queue_handoffs(tmp_path):
    """VERDICT r05 item 2.  (a) drain_own_queue's hand-off is the block queue in GLOBAL memory:
    s_waitcnt vmcnt(0) -> s_barrier, then the LDS cursor's atomic (ds_add_rtn, the active lanes'
    points), and only then the queue's global loads -- in the C3 kernel (DEFER 3) and in the
    deferred-test kernel (DEFER 1).  (b) Every intra-wave LDS hand-off of the C3 stream (the span
    queue read by other lanes, the bitmap-word ring) carries a wave barrier (wave_lds_sync): the
    compiler may not move a lane's read of a slot another lane wrote above that write."""
    asm = device_asm("k_range.hip", tmp_path)
    for name, min_wb in (("_ZN2gf12range_kernelILi1ELi1ELi3ELi2E", 3), ("_ZN2gf12range_kernelILi1ELi1ELi1E", 0)):
        body = function_body(asm, name)
        # the drain: the LAST vmcnt(0) + s_barrier pair followed by the cursor atomic
        found = False
        for k in range(len(body)):
            j = _after_barrier(body, k)
            if j is None:
                break
            rest = body[j + 1:]
            cur = next((i for i, b in enumerate(rest) if b.startswith("ds_add_rtn_u32")), None)
            if cur is not None and not any(b.startswith("global_load") for b in rest[:cur]):
                glb = next((i for i, b in enumerate(rest) if b.startswith("global_load")), None)
                assert glb is not None and glb > cur
                found = True
                break
            k = j + 1
        assert found, f"{name}: no vmcnt(0) -> s_barrier -> cursor atomic -> queue loads drain"
        assert sum(ln == "; wave barrier" for ln in body) >= min_wb, name


@pytest.mark.timeout(600)
def test_join_pair_buffers_carry_wave_barriers(tmp_path):
    """The join probes' per-wave pair buffers (written at ballot ranks, read by other lanes at the
    flush) and the windowed band's point queue are intra-wave LDS hand-offs: wave barriers in
    the band probe (both modes) and the row probe."""
    asm = device_asm("k_join.hip", tmp_path)
    for mode in (0, 1):
        body = function_body(asm, f"_ZN2gf22join_band_probe_kernelILi{mode}E")
        assert sum(ln == "; wave barrier" for ln in body) >= 3, mode
    body = function_body(asm, "_ZN2gf21join_row_probe_kernelILi0ELi1E")
    assert any(ln == "; wave barrier" for ln in body)
