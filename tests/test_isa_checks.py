"""Static checks on the built gfx950 code objects (no GPU needed).

The LDS-staged gradient kernels (grad_dense_staged, grad_staged_mfma) wait for their own LDS-DMA
loads with a hand-counted ``s_waitcnt vmcnt(n)`` (csrc/kernels/lds_dma.h): the count is only right
if the compiler issues no vector-memory LOAD of its own once the stage pipeline has started.  This
disassembles every instantiation from the built library and checks exactly that, so a compiler
change that breaks the assumption fails here instead of racing intermittently on the GPU

"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
VMEM_LOAD = re.compile(r"^(global_load|buffer_load|flat_load|global_atomic|flat_atomic|buffer_atomic)")


def _code_objects(tmp_path):
    from erasurehead_amd._ext import check_fresh

    so = check_fresh()["so"]
    dst = tmp_path / "c.so"
    shutil.copy(so, dst)
    subprocess.run([OBJDUMP, "--offloading", str(dst)], cwd=str(tmp_path), capture_output=True, check=True)
    return sorted(glob.glob(str(tmp_path / "c.so.*gfx950")))


def _functions(path):
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", path], capture_output=True, text=True, check=True).stdout
    for chunk in re.split(r"\n(?=[0-9a-f]+ <)", out):
        m = re.match(r"[0-9a-f]+ <([^>]+)>", chunk)
        if m:
            yield m.group(1), [l.strip() for l in chunk.splitlines()[1:] if l.strip()]


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not installed")
def test_staged_kernels_issue_no_compiler_loads_inside_the_stage_pipeline(tmp_path):
    checked = 0
    for co in _code_objects(tmp_path):
        for name, body in _functions(co):
            if "grad_dense_staged" not in name and "grad_staged_mfma" not in name:
                continue
            checked += 1
            first = next((i for i, l in enumerate(body) if "global_load_lds" in l.split()[0]), None)
            assert first is not None, f"{name}: no LDS-DMA loads found"
            bad = []
            for i in range(first, len(body)):
                op = body[i].split()[0]
                if not VMEM_LOAD.match(op) or "_lds" in op:
                    continue
                # allowed only if it is drained (vmcnt(0)) before the next LDS-DMA load
                nxt = next((l for l in body[i + 1:] if "global_load_lds" in l.split()[0]
                            or (l.split()[0] == "s_waitcnt" and "vmcnt(0)" in l)), "")
                if "vmcnt(0)" not in nxt:
                    bad.append(body[i])
            assert not bad, f"{name}: compiler-emitted vector loads inside the counted stage loop: {bad[:4]}"
    assert checked >= 48, f"only {checked} staged kernel instantiations found"


READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _kernel_regs(path):
    """{mangled kernel name: (vgpr_count, vgpr_spill_count)} from the code object's metadata notes."""
    out = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, check=True).stdout
    regs, cur = {}, {}
    for line in out.splitlines():
        m = re.match(r"\s*-?\s*\.(name|vgpr_count|vgpr_spill_count):\s+(\S+)", line)
        if not m:
            continue
        cur[m.group(1)] = m.group(2)
        if {"name", "vgpr_count", "vgpr_spill_count"} <= cur.keys():
            regs[cur["name"]] = (int(cur["vgpr_count"]), int(cur["vgpr_spill_count"]))
            cur = {}
    return regs


@pytest.mark.skipif(not os.path.exists(READELF), reason="llvm-readelf not installed")
def test_default_staged_kernels_keep_their_occupancy(tmp_path):
    """Register budgets of the headline kernels (d <= 1024: 16 columns per lane).  Waves per SIMD =
    512 // VGPRs rounded up to 8: fp32 pair bundles need <= 80 for 6 waves (93 -> 5 cost 10 % at the
    fp32 headline, docs/PERF_NOTES.md round 3), fp64 <= 168 for 3.  No default instantiation for
    d <= 1024 spills."""
    regs = {}
    for co in _code_objects(tmp_path):
        regs.update(_kernel_regs(co))
    staged = {n: r for n, r in regs.items() if "grad_dense_staged" in n}
    assert staged, "no default staged instantiations found"
    for n, (v, spill) in staged.items():  # d <= 1024; fp64 at 32 columns per lane (d <= 2048) spills 4
        if re.search(r"Li(2|4|8|16)ELi", n):
            assert spill == 0, f"{n} spills {spill} VGPRs"
    budget = {"IffLi16ELi0ELb1EEEv": 80, "IddLi16ELi0ELb0EEEv": 168, "IddLi16ELi0ELb1EEEv": 168}
    for key, limit in budget.items():
        hit = [(n, r) for n, r in staged.items() if key in n]
        assert hit, f"instantiation {key} not found"
        for n, (v, _) in hit:
            assert v <= limit, f"{n}: {v} VGPRs > {limit} (fewer waves per SIMD)"
    # one-wave bundles (the fp64 default): 3 replicas' accumulators + two row buffers must stay
    # within 256 VGPRs (2 waves per SIMD) without spilling
    multi = {n: r for n, r in regs.items() if "grad_dense_multi" in n}
    assert any("IddLi16ELi0ELi3E" in n for n in multi), "fp64 3-replica one-wave bundle not found"
    for n, (v, spill) in multi.items():
        assert spill == 0 and v <= 256, f"{n}: {v} VGPRs, {spill} spilled"
    mfma = [(n, r) for n, r in regs.items() if "grad_staged_mfma" in n]
    assert mfma and all(s == 0 for _, (_, s) in mfma), mfma


@pytest.mark.skipif(not os.path.exists(READELF), reason="llvm-readelf not installed")
def test_wide_row_bundles_do_not_spill(tmp_path):
    """grad_dense_wide with R replicas (one row load feeds R dot products and R gradients) keeps
    its accumulators in registers at every width and precision."""
    regs = {}
    for co in _code_objects(tmp_path):
        regs.update(_kernel_regs(co))
    wide = {n: r for n, r in regs.items() if "grad_dense_wide" in n}
    assert len(wide) >= 24, sorted(wide)  # 3 storage types x 2 losses x (256 threads x R in 1..3, 512 x R = 1)
    bad = {n: r for n, r in wide.items() if r[1] > 0}
    assert not bad, bad


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not installed")
def test_vgpr_ring_waits_only_for_its_oldest_register_set(tmp_path):
    """grad_vring_mfma (the bf16 packed bundles' VGPR-staged ring, an A/B) counts its own stage loads (inline asm,
    9 per stage and wave): once the pipeline has started, the only vector-memory loads are those 9-load
    groups, every copy into the ring waits vmcnt((NSET - 1) * 9) -- the other sets stay in flight --
    and no vmcnt(0) appears before the loop ends."""
    checked = 0
    for co in _code_objects(tmp_path):
        for name, body in _functions(co):
            if "grad_vring_mfma" not in name:
                continue
            nset = int(re.search(r"grad_vring_mfmaILi\d+ELi(\d+)E", name).group(1))
            checked += 1
            body = [l.split("//")[0].strip() for l in body]
            first = next(i for i, l in enumerate(body) if l.startswith("global_load_dwordx4") and l.endswith(" nt"))
            # the loop: from the first ring copy to the last barrier
            last = max(i for i, l in enumerate(body) if l.startswith("s_barrier"))
            waits = [l for l in body[first:last] if l.startswith("s_waitcnt") and "vmcnt" in l]
            assert waits, name
            want = f"vmcnt({(nset - 1) * 9})"
            assert all(want in w for w in waits), (name, waits)
            loads = [l.split()[0] for l in body[first:last] if VMEM_LOAD.match(l.split()[0])]
            assert loads.count("global_load_dwordx4") == 8 * loads.count("global_load_dword"), (name, loads[:12])
    assert checked >= 4, f"only {checked} grad_vring_mfma instantiations found"
