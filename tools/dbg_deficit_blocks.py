"""Triage: the partial lengths the engine walks next to the oracle's, per block (mtb_debug_blocks /
OracleDoc.debug_blocks), for a small constructed summary (tools/dbg_deficit_small.py numbering) after its load
and after the first PREFIX ops of its rising-MSN tail, in the (REF, CLIENT) view."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from fluidframework_amd import MergeTreeBatch  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from test_gpu_phantom import _rising_tail, _tail_summary  # noqa: E402

k = int(os.environ["CASE"])
prefix = int(os.environ.get("PREFIX", 0))
ref = int(os.environ.get("REF", -1))
cid = os.environ.get("CLIENT")
blobs = _tail_summary(7000 + k, 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7)
g = OracleDoc()
g.load_v1(blobs, "obs")
tail = []
try:
    _rising_tail(g, k, 60, 40, out=tail)
except Exception:
    pass
o = OracleDoc()
o.load_v1(blobs, "loader")
B = MergeTreeBatch(1)
B[0].load(blobs, "loader")
for m in tail[:prefix]:
    o.apply_msg(m)
    B[0].applyMsg(m)
B.flush()
eb = B.debug_blocks(0, ref, cid)
ob = o.debug_blocks(ref, cid)
for e, q in zip(eb, ob):
    flag = "" if e["kids"] == q["kids"] else "   <<< differs"
    print("path", e["path"], "engine", e["kids"], "oracle", q["kids"], flag)
    print("    table", e["table"])
    print("    oracle minLength", q.get("minLength"), "main", q.get("main"), "cli", q.get("cli"))
print("next op:", json.dumps(tail[prefix]) if prefix < len(tail) else None)
