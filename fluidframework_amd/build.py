"""Build the engine's shared library in-tree (hipcc, gfx950).  `python -m fluidframework_amd.build`."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "mtb_replay.hip"), os.path.join(HERE, "csrc", "mtb_host.cpp")]
OUT = os.path.join(HERE, "libmtb.so")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SRCS + [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))] + \
        [os.path.join(ROOT, "include", "mtb.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, arch="gfx950"):
    if not force and not needs_build():
        return OUT
    cmd = ["hipcc", "-x", "hip", f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-o", OUT] + SRCS
    subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
