"""Triage: outcome of every constructed summary / long document of tests/test_gpu_phantom.py on the engine vs the
oracle after the load (one JSON line per case: case, mode, oracle deficits, outcome, first differing line)."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from fluidframework_amd import MergeTreeBatch, MergeTreeError  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from helpers import first_diff, make_tail_log  # noqa: E402
from test_gpu_phantom import _tail_summary  # noqa: E402


def cases():
    for new_mode in (False, True):
        for i in range(24):
            yield ("constructed", i, new_mode, 0, _tail_summary(500 + i, 120 + 20 * i, 60 + 5 * i, 100 + 10 * (i % 5)))
    if os.environ.get("LONG"):
        for new_mode in (False, True):
            for chunk in (0, 300):
                for i in list(range(16)) + [40, 47, 48, 59]:
                    text, msgs = make_tail_log(900 + i + 50 * int(new_mode), 1600, lag=24 + 8 * (i % 8), initial_len=9990,
                                               lo=9990, new_mode=new_mode, inserters=[0])
                    cut = len(msgs) // 2 + 37 * (i % 8)
                    a = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
                    a.insert_text_local(0, text)
                    a.start_collab("obs")
                    for m in msgs[:cut]:
                        a.apply_msg(m)
                    yield ("long%d" % chunk, i, new_mode, chunk, [list(x) for x in a.summarize_v1()["blobs"]])


out = open(os.environ.get("OUT", "gpurun_out/dbg_deficit.jsonl"), "w")
for kind, i, new_mode, chunk, blobs in cases():
    o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
    rec = {"case": kind, "i": i, "new_mode": new_mode}
    try:
        o.load_v1(blobs, "loader")
        od = o.dump_segments()
    except Exception as e:
        od = None
        rec["oracle"] = str(e)[:80]
    rec["deficits"] = o.stale_deficits()
    B = MergeTreeBatch(1, new_length_calc=new_mode, chunk_size=chunk)
    B[0].load(blobs, "loader")
    try:
        B.flush()
        gd = B.dump_segments(0)
        rec["outcome"] = "equal" if gd == od else "differs"
        if od is not None and gd != od:
            rec["diff"] = first_diff(gd, od)
    except MergeTreeError as e:
        rec["outcome"] = "failed" if od is None else "engine-failed"
        rec["engine"] = str(e)[:80]
    out.write(json.dumps(rec) + "\n")
    out.flush()
    print(json.dumps(rec)[:200], flush=True)
