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


def build(force=False, arch="gfx950", out=OUT, defines=()):
    if not force and out == OUT and not needs_build():
        return OUT
    cmd = ["hipcc", "-x", "hip", f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result"] + [f"-D{d}" for d in defines] + ["-o", out] + SRCS
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    if "--variants" in sys.argv:  # occupancy variants for tuning runs (MTB_LIB=...)
        for w in (2, 3, 4):
            print(build(force=True, out=os.path.join(HERE, f"libmtb_w{w}.so"), defines=[f"MTB_WAVES_PER_SIMD={w}"]))
    print(build(force="--force" in sys.argv))
