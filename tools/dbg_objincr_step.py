"""Triage: replay one generated object-incr log message by message on the engine and the oracle; print the first
message after which their canonical dumps differ, with the message and the differing lines."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from helpers import first_diff, make_incr_log  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402

s = int(os.environ.get("DOC", 1))
n = int(os.environ.get("N_MSGS", 750))
init, msgs = make_incr_log(850 + s, n, n_clients=3 + s % 3, lag=4 + 5 * s, new_mode=False, p_incr=0.3,
                           string_incr=True, object_incr=True, objs=[{"x": 1}, {"y": 2}, {}])
B = MergeTreeBatch(1)
B[0].insertTextLocal(0, init)
B[0].startOrUpdateCollaboration("obs")
o = OracleDoc()
o.insert_text_local(0, init)
o.start_collab("obs")
prev = None
for j, m in enumerate(msgs):
    B[0].applyMsg(m)
    o.apply_msg(m)
    B.replay()
    g, w = B.dump_segments(0), o.dump_segments()
    if g != w:
        print("first difference after message", j, json.dumps(m))
        print(first_diff(g, w))
        print("--- oracle before:")
        print(prev)
        print("--- oracle after:")
        print(w)
        print("--- gpu after:")
        print(g)
        break
    prev = w
else:
    print("equal")
