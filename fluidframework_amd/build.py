"""Build the engine in-tree: `python -m fluidframework_amd.build`.

* fluidframework_amd/libmtb.so          HIP engine (hipcc, gfx950) exporting the C ABI of include/mtb.h
* fluidframework_amd/js/mtb_napi.node   Node N-API addon over that C ABI (gcc + node's headers), used by
                                        the JS drop-in package fluidframework_amd/js (index.js)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "mtb_replay.hip"), os.path.join(HERE, "csrc", "mtb_host.cpp"),
        os.path.join(HERE, "csrc", "mtb_multi.cpp")]
OUT = os.path.join(HERE, "libmtb.so")
NAPI_SRC = os.path.join(HERE, "js", "src", "mtb_napi.c")
NAPI_OUT = os.path.join(HERE, "js", "mtb_napi.node")
NODE_INCLUDE = "/usr/include/node"


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in deps)


def needs_build():
    deps = SRCS + [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))] + \
        [os.path.join(ROOT, "include", "mtb.h")]
    return _stale(OUT, deps)


# the kernel file is compiled once per kernel group (mtb_replay.hip MTB_TU_*), in parallel with the host
# sources; objects are kept under build/ and rebuilt when a source or header is newer
KERNEL_GROUPS = (1, 2, 3, 4, 5)
OBJ_DIR = os.path.join(ROOT, "build", "obj")


def _headers():
    return [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith((".h", ".hpp"))] + \
        [os.path.join(ROOT, "include", "mtb.h")]


def build(force=False, arch="gfx950", out=OUT, defines=(), extra=()):
    if not force and out == OUT and not needs_build():
        return OUT
    from concurrent.futures import ThreadPoolExecutor
    tag = "_".join([d.replace("=", "") for d in defines] + [x.strip("-").replace("-", "") for x in extra]) or "base"
    odir = os.path.join(OBJ_DIR, f"{arch}_{tag}")
    os.makedirs(odir, exist_ok=True)
    base = ["hipcc", "-x", "hip", f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"] + \
        [f"-D{d}" for d in defines] + list(extra)
    jobs = []  # (object, command, sources it depends on)
    hip = SRCS[0]
    for g in KERNEL_GROUPS:
        o = os.path.join(odir, f"mtb_replay_tu{g}.o")
        jobs.append((o, base + [f"-DMTB_TU={g}", "-c", hip, "-o", o], [hip]))
    for src in SRCS[1:]:
        o = os.path.join(odir, os.path.basename(src) + ".o")
        jobs.append((o, base + ["-c", src, "-o", o], [src]))
    hdrs = _headers()

    def run(job):
        o, cmd, deps = job
        if force or _stale(o, deps + hdrs):
            subprocess.check_call(cmd)
        return o

    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(run, jobs))
    subprocess.check_call(["hipcc", f"--offload-arch={arch}", "-shared", "-fPIC", "-o", out] + objs)
    return out


def build_napi(force=False):
    """The N-API addon links libmtb.so (rpath $ORIGIN/..); node resolves the napi_* symbols at load."""
    if not os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")):
        print("build_napi: node headers not found, JS addon not built", file=sys.stderr)
        return None
    if not force and not _stale(NAPI_OUT, [NAPI_SRC, OUT, os.path.join(ROOT, "include", "mtb.h")]):
        return NAPI_OUT
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-fPIC", "-shared", "-DNODE_GYP_MODULE_NAME=mtb_napi",
           f"-I{NODE_INCLUDE}", NAPI_SRC, f"-L{HERE}", "-lmtb", "-Wl,-rpath,$ORIGIN/..", "-o", NAPI_OUT]
    subprocess.check_call(cmd)
    return NAPI_OUT


if __name__ == "__main__":
    if "--variants" in sys.argv:  # occupancy variants for tuning runs (MTB_LIB=...)
        for w in (4, 5, 6):
            print(build(force=True, out=os.path.join(HERE, f"libmtb_w{w}.so"), defines=[f"MTB_WAVES_PER_SIMD={w}"]))
    print(build(force="--force" in sys.argv))
    print(build_napi(force="--force" in sys.argv))
