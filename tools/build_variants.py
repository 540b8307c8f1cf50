"""Build the engine's measurement variants into tools/lib/ (MTB_LIB=tools/lib/libmtb_<name>.so selects one;
they are profiling builds, not part of the package):

  prof      MTB_PROFILE                      per-phase cycle counters (mtb_profile lines on stderr)
  profpack  + MTB_PROFILE_PACK               packParent / zamboni sub-phase counters
  check     + MTB_CHECK                      bounds-checked slices (mtb_check lines on stderr)
  ppcrumbs  profpack + MTB_CRUMBS            ticket breadcrumbs in host memory (fault triage, mtb_crumbs lines)
  ppinline  profpack + MTB_TICK_INLINE       the ticket kernel's hand-over helpers inlined (no calls; fault triage)
  tabcheck  profpack + MTB_TABCHECK          the LDS copy of the batch tables checked against the kernel argument
                                             before every op (fault triage; a mismatch fails the document)

usage: python3 tools/build_variants.py [name ...]   (default: all)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd import build as b  # noqa: E402

LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
VARIANTS = {
    "prof": ["MTB_PROFILE"],
    "profpack": ["MTB_PROFILE", "MTB_PROFILE_PACK"],
    "check": ["MTB_PROFILE", "MTB_PROFILE_PACK", "MTB_CHECK"],
    "ppcrumbs": ["MTB_PROFILE", "MTB_PROFILE_PACK", "MTB_CRUMBS"],
    "ppinline": ["MTB_PROFILE", "MTB_PROFILE_PACK", "MTB_TICK_INLINE"],
    "tabcheck": ["MTB_PROFILE", "MTB_PROFILE_PACK", "MTB_TABCHECK"],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    print(b.build())
    for n in names:
        os.makedirs(LIBDIR, exist_ok=True)
        print(b.build(out=os.path.join(LIBDIR, f"libmtb_{n}.so"), defines=VARIANTS[n]))
