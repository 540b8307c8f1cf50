"""Triage: the small constructed summaries whose rising-MSN tail the reference fails ("MergeTree insert failed"):
does the engine fail the same op?  For each that it does not, the engine's and the oracle's block lengths in the
failing op's view just before it."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from fluidframework_amd import MergeTreeBatch, MergeTreeError  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from test_gpu_phantom import _rising_tail, _tail_summary  # noqa: E402

new_mode = bool(int(os.environ.get("NEW", 0)))
fails = []
for k in range(0, 300, 2):
    blobs = _tail_summary(7000 + k, 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7)
    o = OracleDoc(new_length_calc=new_mode)
    try:
        o.load_v1(blobs, "loader")
    except Exception:
        continue
    if not o.stale_deficits():
        continue
    g = OracleDoc(new_length_calc=new_mode)
    g.load_v1(blobs, "obs")
    tail = []
    try:
        _rising_tail(g, k, 60, 40, out=tail)
    except Exception:
        fails.append((k, blobs, tail))
B = MergeTreeBatch(2 * len(fails), new_length_calc=new_mode)
for j, (k, blobs, tail) in enumerate(fails):
    B[2 * j].load(blobs, "loader")
    B[2 * j + 1].load(blobs, "loader")
    for m in tail[:-1]:
        B[2 * j].applyMsg(m)
        B[2 * j + 1].applyMsg(m)
    B[2 * j + 1].applyMsg(tail[-1])
try:
    B.flush()
except MergeTreeError:
    pass
for j, (k, blobs, tail) in enumerate(fails):
    try:
        B.map_range(2 * j + 1, 0, 1)
        raised = False
    except MergeTreeError as e:
        raised = "MergeTree insert failed" in str(e)
    print("case", k, "ops", len(tail), "engine fails the op:", raised, json.dumps(tail[-1]["contents"]))
    if raised:
        continue
    m = tail[-1]
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(blobs, "loader")
    for x in tail[:-1]:
        o.apply_msg(x)
    eb = B.debug_blocks(2 * j, m["referenceSequenceNumber"], m["clientId"])
    ob = o.debug_blocks(m["referenceSequenceNumber"], m["clientId"])
    for e, q in zip(eb, ob):
        flag = "" if e["kids"] == q["kids"] else "   <<< differs"
        print("  path", e["path"], "engine", e["kids"], "oracle", q["kids"], flag)
        if flag:
            print("      table", e["table"])
            print("      oracle minLength", q.get("minLength"), "main", q.get("main"), "cli", q.get("cli"))
