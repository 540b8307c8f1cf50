"""Debug: the snapshot.spec body case on the engine with per-replay slice use (MTB_SLICE_TRACE)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import snapshot_spec as sp  # noqa: E402

inc = sys.argv[1] == "1" if len(sys.argv) > 1 else True
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10010
s = sp.TestString(sp.EngineSide(False, "", "fakeId"))
for i in range(n):
    if i % 500 == 0 or i > n - 3:
        os.environ["MTB_SLICE_TRACE"] = "1"
    else:
        os.environ.pop("MTB_SLICE_TRACE", None)
    try:
        s.append(str(i % 10), inc)
    except Exception as e:
        print("failed at", i, e, flush=True)
        raise
print("ok", s.client.length())
