"""The scheduled replay kernels never read memory through the scalar cache except their kernel arguments.

Round 4's fault (DESIGN.md §4 "Round 4"): with `DocState* __restrict__` the compiler read a document's state with
scalar loads; a ticket hand-over's agent-scope acquire does not invalidate the scalar cache, so a workgroup
could resume a document from its previous chunk's stale state.  This compiles the observer kernels' translation
unit for gfx950 (hipcc -S, no GPU needed) and checks that every scalar load in the kernels that hand documents
over between workgroups within one launch (`mtb_replay_tick_kernel`) or that could (`mtb_replay_pass_kernel`)
reads the kernel-argument segment (s[0:1]).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "fluidframework_amd", "csrc", "mtb_replay.hip")


def _kernel_body(asm, name):
    m = re.search(rf"^{name}:.*?^\.Lfunc_end", asm, re.S | re.M)
    assert m, f"{name} not found in the assembly"
    return m.group(0)


@pytest.mark.timeout(600)
def test_scheduled_kernels_read_only_kernel_arguments_through_the_scalar_cache(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path / "tu1.s"
    subprocess.check_call([hipcc, "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DMTB_TU=1",
                           "--cuda-device-only", "-S", SRC, "-o", str(out)], stderr=subprocess.DEVNULL)
    asm = out.read_text()
    for kernel in ("mtb_replay_tick_kernel", "mtb_replay_pass_kernel"):
        body = _kernel_body(asm, kernel)
        loads = re.findall(r"^\s*(s_(?:buffer_)?load_\w+)\s+([^\n]*)$", body, re.M)
        bad = [f"{op} {args}" for op, args in loads if not re.match(r"(?:s\d+|s\[\d+:\d+\]),\s*s\[0:1\],", args)]
        assert loads, f"{kernel}: no scalar loads at all (the assembly format changed?)"
        assert not bad, f"{kernel}: scalar loads off a pointer other than the kernel arguments: {bad[:5]}"


@pytest.mark.timeout(600)
def test_observer_kernels_do_not_spill(tmp_path):
    """The observer kernels hold 4 waves per SIMD at 128 VGPRs with no spill code: rarely used
    machinery (irregular-key matchProperties, phantom tables, marker ids) is compiled into the marker variant
    only, which the host picks for the batches that need it."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path / "tu1.s"
    subprocess.check_call([hipcc, "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DMTB_TU=1",
                           "--cuda-device-only", "-S", SRC, "-o", str(out)], stderr=subprocess.DEVNULL)
    asm = out.read_text()
    meta = asm[asm.index("amdhsa.kernels:"):]
    seen = {}
    for blk in meta.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        seen[name] = (int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)),
                      int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1)))
    for kernel in ("mtb_replay_tick_kernel", "mtb_replay_pass_kernel", "mtb_replay_kernel"):
        assert kernel in seen, f"{kernel} not in the translation unit"
        vgprs, spills = seen[kernel]
        assert vgprs <= 128 and spills == 0, f"{kernel}: {vgprs} VGPRs, {spills} spilled"
