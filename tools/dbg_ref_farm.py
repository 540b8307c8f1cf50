"""Debug helper (tests infrastructure): replay a reference-shaped reconnect farm on the engine and name the
first failing event (round, client, event index)."""
import json, sys
sys.path.insert(0, "."); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from helpers import run_ref_reconnect_farm
from fluidframework_amd import MergeTreeBatch
seed, nc = int(sys.argv[1]), int(sys.argv[2])
rec = {}
run_ref_reconnect_farm(seed, nc, record=rec)
ids = rec["ids"]
B = MergeTreeBatch(nc, new_length_calc=True)
for k, cid in enumerate(ids):
    B[k].startOrUpdateCollaboration(cid)
for r, rnd in enumerate(rec["rounds"]):
    for k, (events, _, _) in enumerate(rnd):
        nl = sum(1 for kind, _ in events if kind == "local")
        for i, (kind, x) in enumerate(events):
            try:
                if kind == "local":
                    B[k].applyLocalOp(x)
                elif kind == "regen":
                    got = B[k].regeneratePendingOp(x[0])
                    if got != x[1]:
                        print("diff", r, k, i, json.dumps(got), json.dumps(x[1])); sys.exit(1)
                else:
                    B[k].applyMsg(x)
            except Exception as e:
                print("fail round", r, "client", k, "event", i, kind, "locals", nl, e)
                print(json.dumps(x)[:500])
                sys.exit(1)
    B.replay()
    print("round", r, "ok", [B.text(k) == rnd[k][2] for k in range(nc)], flush=True)
