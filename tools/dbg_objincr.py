"""Triage: which object-value shapes under an incr-annotated key make the engine's tree differ from the oracle's
(one line per variant: variant, first differing log or "equal")."""
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from helpers import make_incr_log  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402

VARIANTS = {
    "mixed-no-incr": dict(objs=[{"x": 1}, "str1", {"y": 2}, "[object Object]undefined"], incr_objects=False),
    "strings-no-incr": dict(objs=["a", "b", "c"], incr_objects=False),
    "strings-incr": dict(objs=["a", "b", "c"]),
    "objects-only": dict(objs=[{"x": 1}, {"y": 2}, {}]),
}
ONLY = os.environ.get("ONLY")
for name, kw in VARIANTS.items():
    if ONLY and name != ONLY:
        continue
    for new_mode in (False,):
        logs = [make_incr_log(850 + s, int(os.environ.get("N_MSGS", 900)), n_clients=3 + s % 3, lag=4 + 5 * s, new_mode=new_mode, p_incr=0.3,
                              string_incr=True, object_incr=True, **kw) for s in range(8)]
        B = MergeTreeBatch(len(logs), new_length_calc=new_mode)
        orc = []
        for i, (init, msgs) in enumerate(logs):
            B[i].insertTextLocal(0, init)
            B[i].startOrUpdateCollaboration("obs")
            o = OracleDoc(new_length_calc=new_mode)
            o.insert_text_local(0, init)
            o.start_collab("obs")
            for m in msgs:
                B[i].applyMsg(m)
                o.apply_msg(m)
            orc.append(o)
        B.replay()
        bad = [i for i, o in enumerate(orc) if B.dump_segments(i) != o.dump_segments()]
        print(name, new_mode, "equal" if not bad else f"differ {bad}", flush=True)
        if bad and os.environ.get("DUMP"):
            from helpers import first_diff
            print(first_diff(B.dump_segments(bad[0]), orc[bad[0]].dump_segments()))
