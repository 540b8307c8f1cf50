"""Code-generation guards for the scheduled replay kernels (compiled to gfx950 assembly with hipcc -S; no GPU).

* Round 4's fault (DESIGN.md §4 "Round 4"): with `DocState* __restrict__` the compiler read a document's state with
  scalar loads; a ticket hand-over's agent-scope acquire does not invalidate the scalar cache, so a workgroup could
  resume a document from its previous chunk's stale state.  Every scalar load in the kernels that hand documents
  over between workgroups within one launch (`mtb_replay_tick_kernel`) or that could (`mtb_replay_pass_kernel`)
  must read the kernel-argument segment (s[0:1]).
* The observer kernels hold 4 waves per SIMD at 128 VGPRs with no spill code.
* Round 6 (DESIGN.md §4 "Round 6"): the MTB_PROFILE_PACK build faulted deterministically in the ticket kernel, with
  or without hand-overs, and ran clean once the kernel made no calls: a kernel must not both use scratch and call
  functions.  The product ticket kernel uses no scratch at all; the profiling builds (which spill) make no calls.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "fluidframework_amd", "csrc", "mtb_replay.hip")
SCHEDULED = ("mtb_replay_tick_kernel", "mtb_replay_pass_kernel")


def _compile(tmp_path_factory, defines):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "tu1.s"
    subprocess.check_call([hipcc, "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DMTB_TU=1"] +
                          [f"-D{d}" for d in defines] + ["--cuda-device-only", "-S", SRC, "-o", str(out)],
                          stderr=subprocess.DEVNULL)
    return out.read_text()


@pytest.fixture(scope="module")
def product_asm(tmp_path_factory):
    return _compile(tmp_path_factory, [])


@pytest.fixture(scope="module")
def profpack_asm(tmp_path_factory):
    return _compile(tmp_path_factory, ["MTB_PROFILE", "MTB_PROFILE_PACK"])


def _kernel_body(asm, name):
    m = re.search(rf"^{name}:.*?^\.Lfunc_end", asm, re.S | re.M)
    assert m, f"{name} not found in the assembly"
    return m.group(0)


def _meta(asm):
    meta = asm[asm.index("amdhsa.kernels:"):]
    seen = {}
    for blk in meta.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        seen[name] = {f: int(re.search(rf"\.{f}:\s+(\d+)", blk).group(1))
                      for f in ("vgpr_count", "vgpr_spill_count", "private_segment_fixed_size")}
    return seen


@pytest.mark.timeout(600)
def test_scheduled_kernels_read_only_kernel_arguments_through_the_scalar_cache(product_asm):
    for kernel in SCHEDULED:
        body = _kernel_body(product_asm, kernel)
        loads = re.findall(r"^\s*(s_(?:buffer_)?load_\w+)\s+([^\n]*)$", body, re.M)
        bad = [f"{op} {args}" for op, args in loads if not re.match(r"(?:s\d+|s\[\d+:\d+\]),\s*s\[0:1\],", args)]
        assert loads, f"{kernel}: no scalar loads at all (the assembly format changed?)"
        assert not bad, f"{kernel}: scalar loads off a pointer other than the kernel arguments: {bad[:5]}"


@pytest.mark.timeout(600)
def test_observer_kernels_do_not_spill(product_asm):
    """The observer kernels hold 4 waves per SIMD at 128 VGPRs with no spill code: rarely used
    machinery (irregular-key matchProperties, phantom tables, marker ids) is compiled into the marker variant
    only, which the host picks for the batches that need it."""
    seen = _meta(product_asm)
    for kernel in SCHEDULED + ("mtb_replay_kernel",):
        assert kernel in seen, f"{kernel} not in the translation unit"
        m = seen[kernel]
        assert m["vgpr_count"] <= 128 and m["vgpr_spill_count"] == 0, f"{kernel}: {m}"
        assert m["private_segment_fixed_size"] == 0, f"{kernel} uses scratch: {m}"


@pytest.mark.timeout(600)
def test_no_kernel_both_spills_and_calls(product_asm, profpack_asm):
    for asm in (product_asm, profpack_asm):
        seen = _meta(asm)
        for kernel in SCHEDULED + ("mtb_replay_kernel", "mtb_replay_finish_kernel"):
            calls = len(re.findall(r"^\s*s_swappc_b64", _kernel_body(asm, kernel), re.M))
            assert not (calls and seen[kernel]["private_segment_fixed_size"]), \
                f"{kernel}: {calls} call(s) in a kernel with {seen[kernel]['private_segment_fixed_size']} B of scratch"
