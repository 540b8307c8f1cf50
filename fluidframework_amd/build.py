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


# The engine is rebuilt by CONTENT, not by mtime: build() hashes every source and header that goes into
# libmtb.so together with the compile flags, embeds that hash in the library (a generated translation unit
# holding BUILD_ID_TAG + hex), and rebuilds whenever the hash found in an existing libmtb.so differs -- a
# prebuilt library that came with a tree (newer by mtime, or not) is never trusted.  Objects under build/obj
# carry the hash of their own inputs in a sidecar file in the same way.
BUILD_ID_TAG = b"MTB_SOURCE_SHA256="

# the kernel file is compiled once per kernel group (mtb_replay.hip MTB_TU_*), in parallel with the host
# sources
KERNEL_GROUPS = (1, 2, 3, 4, 5, 6)
# per-group code-generation flags: the few-document kernel (group 6: one wave per document, nothing to hide
# its latency) schedules for ILP (cfg4 +2.8 % in a same-box A/B; the batch kernels lose 0.3 % with it)
GROUP_FLAGS = {6: ["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"]}
OBJ_DIR = os.path.join(ROOT, "build", "obj")


def _headers():
    return sorted([os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))
                   if f.endswith((".h", ".hpp"))]) + [os.path.join(ROOT, "include", f) for f in ("mtb.h", "mtb_testing.h")]


def _digest(paths, flags):
    import hashlib
    h = hashlib.sha256()
    for f in flags:
        h.update(f.encode() + b"\0")
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def _base_flags(arch, defines, extra):
    return ["hipcc", "-x", "hip", f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"] + \
        [f"-D{d}" for d in defines] + list(extra)


def source_id(arch="gfx950", defines=(), extra=(), group_flags=None):
    """The hash build() embeds in the library it makes from the current sources and flags."""
    gf = GROUP_FLAGS if group_flags is None else group_flags
    flags = _base_flags(arch, defines, extra) + [f"{g}:{' '.join(f)}" for g, f in sorted(gf.items())]
    return _digest(SRCS + _headers(), flags)


def embedded_id(path=OUT):
    """The source hash embedded in a built library, or None (missing, or built without one)."""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_TAG)
    if i < 0:
        return None
    j = i + len(BUILD_ID_TAG)
    return data[j:j + 64].decode("ascii", "replace")


def needs_build(out=OUT, arch="gfx950", defines=(), extra=()):
    return embedded_id(out) != source_id(arch, defines, extra)


def build(force=False, arch="gfx950", out=OUT, defines=(), extra=(), group_flags=None):
    """group_flags: per-kernel-group flags instead of GROUP_FLAGS (measurement variants)."""
    gf = GROUP_FLAGS if group_flags is None else group_flags
    sid = source_id(arch, defines, extra, gf)
    if not force and embedded_id(out) == sid:
        return out
    from concurrent.futures import ThreadPoolExecutor
    tag = "_".join([d.replace("=", "") for d in defines] + [x.strip("-").replace("-", "") for x in extra]) or "base"
    if group_flags is not None:
        tag += "_g" + "_".join(f"{g}" + "".join(c for c in " ".join(f) if c.isalnum()) for g, f in sorted(gf.items()))
    odir = os.path.join(OBJ_DIR, f"{arch}_{tag}")
    os.makedirs(odir, exist_ok=True)
    base = _base_flags(arch, defines, extra)
    hdrs = _headers()
    jobs = []  # (object, command, sources it depends on)
    hip = SRCS[0]
    for g in KERNEL_GROUPS:
        o = os.path.join(odir, f"mtb_replay_tu{g}.o")
        jobs.append((o, base + gf.get(g, []) + [f"-DMTB_TU={g}", "-c", hip, "-o", o], [hip]))
    for src in SRCS[1:]:
        o = os.path.join(odir, os.path.basename(src) + ".o")
        jobs.append((o, base + ["-c", src, "-o", o], [src]))
    idsrc = os.path.join(odir, "mtb_build_id.c")
    with open(idsrc, "w") as fh:  # the embedded source hash (found by embedded_id, also mtb_build_id())
        fh.write('const char mtb_build_id_str[] = "%s%s";\n'
                 'const char* mtb_build_id(void) { return mtb_build_id_str + %d; }\n'
                 % (BUILD_ID_TAG.decode(), sid, len(BUILD_ID_TAG)))
    ido = idsrc[:-2] + ".o"
    jobs.append((ido, ["gcc", "-O2", "-fPIC", "-c", idsrc, "-o", ido], None))

    def run(job):
        o, cmd, deps = job
        if deps is None:
            subprocess.check_call(cmd)
            return o
        key = _digest(deps + hdrs, cmd)
        stamp = o + ".sha256"
        old = open(stamp).read() if os.path.exists(stamp) and os.path.exists(o) else None
        if force or old != key:
            subprocess.check_call(cmd)
            with open(stamp, "w") as fh:
                fh.write(key)
        return o

    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(run, jobs))
    tmp = out + ".tmp"
    subprocess.check_call(["hipcc", f"--offload-arch={arch}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, out)
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
    print(build(force="--force" in sys.argv))
    print(build_napi(force="--force" in sys.argv))
