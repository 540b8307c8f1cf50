"""Triage: small constructed SnapshotV1 summaries (tests/test_gpu_phantom._tail_summary shapes) with deficits,
engine vs oracle after the load and after a remote tail; prints the differing cases, smallest first."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from fluidframework_amd import MergeTreeBatch, MergeTreeError  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from helpers import first_diff  # noqa: E402
from test_gpu_phantom import _rising_tail, _tail_summary  # noqa: E402
from test_gpu_load import _remote_tail  # noqa: E402


N = int(os.environ.get("N", 400))
new_mode = bool(int(os.environ.get("NEW", 0)))
docs = []
for k in range(N):
    nn, nc, ch = 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7
    blobs = _tail_summary(7000 + k, nn, nc, ch)
    o = OracleDoc(new_length_calc=new_mode)
    try:
        o.load_v1(blobs, "loader")
        od = o.dump_segments()
    except Exception:
        continue
    if not o.stale_deficits():
        continue
    g = OracleDoc(new_length_calc=new_mode)
    g.load_v1(blobs, "obs")
    try:
        tail = _rising_tail(g, k, 60, 40) if os.environ.get("RISE") else \
            _remote_tail(g, k, 30, 40, 10, ["client-0", "client-1", "client-7"])
    except Exception:
        tail = []
    docs.append((k, nn, nc, ch, blobs, o, od, tail))
B = MergeTreeBatch(len(docs), new_length_calc=new_mode)
for j, d in enumerate(docs):
    B[j].load(d[4], "loader")
bad = []
try:
    B.flush()
except MergeTreeError:
    pass
res = []
for j, (k, nn, nc, ch, blobs, o, od, tail) in enumerate(docs):
    try:
        gd = B.dump_segments(j)
    except MergeTreeError as e:
        res.append((nn + nc, k, "engine-failed " + str(e)[:60]))
        continue
    if gd != od:
        res.append((nn + nc, k, "load differs " + first_diff(gd, od)[:200].replace("\n", " | ")))
        continue
    res.append((nn + nc, k, "equal"))
# tails on the loads that agree
ok = [j for j, r in enumerate(res) if r[2] == "equal"]
C = MergeTreeBatch(len(ok), new_length_calc=new_mode)
for q, j in enumerate(ok):
    C[q].load(docs[j][4], "loader")
    for m in docs[j][7]:
        C[q].applyMsg(m)
try:
    C.flush()
except MergeTreeError:
    pass
for q, j in enumerate(ok):
    k, nn, nc, ch, blobs, o, od, tail = docs[j]
    for m in tail:
        o.apply_msg(m)
    try:
        gd = C.dump_segments(q)
    except MergeTreeError as e:
        res[j] = (nn + nc, k, "tail engine-failed " + str(e)[:60])
        continue
    if gd != o.dump_segments():
        res[j] = (nn + nc, k, "tail differs " + first_diff(gd, o.dump_segments())[:200].replace("\n", " | "))
print("cases with deficits:", len(docs), "equal:", sum(r[2] == "equal" for r in res))
for r in sorted(res):
    if r[2] != "equal":
        print(r)
