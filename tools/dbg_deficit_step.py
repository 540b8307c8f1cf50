"""Triage: for the small constructed summaries named in CASES (tools/dbg_deficit_small.py numbering), the first
remote op of the tail after which the engine's dump differs from the oracle's (each prefix replayed as its own
document of one batch)."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from fluidframework_amd import MergeTreeBatch, MergeTreeError  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from helpers import first_diff  # noqa: E402
from test_gpu_phantom import _tail_summary  # noqa: E402
from test_gpu_load import _remote_tail  # noqa: E402

new_mode = bool(int(os.environ.get("NEW", 0)))
for k in [int(x) for x in os.environ["CASES"].split(",")]:
    nn, nc, ch = 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7
    blobs = _tail_summary(7000 + k, nn, nc, ch)
    g = OracleDoc(new_length_calc=new_mode)
    g.load_v1(blobs, "obs")
    tail = _remote_tail(g, k, 30, 40, 10, ["client-0", "client-1", "client-7"])
    B = MergeTreeBatch(len(tail) + 1, new_length_calc=new_mode)
    for j in range(len(tail) + 1):
        B[j].load(blobs, "loader")
        for m in tail[:j]:
            B[j].applyMsg(m)
    try:
        B.flush()
    except MergeTreeError:
        pass
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(blobs, "loader")
    prev = o.dump_segments()
    for j in range(len(tail) + 1):
        if j:
            o.apply_msg(tail[j - 1])
        od = o.dump_segments()
        try:
            gd = B.dump_segments(j)
        except MergeTreeError as e:
            gd = "ERR " + str(e)
        if gd != od:
            print("case", k, "first differing after op", j, json.dumps(tail[j - 1]) if j else "(load)")
            print("oracle before:\n" + prev)
            print("engine after:\n" + gd)
            print("oracle after:\n" + od)
            break
        prev = od
    else:
        print("case", k, "equal throughout")
