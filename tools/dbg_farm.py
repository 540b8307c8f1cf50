"""Debug helper (tests infrastructure): replay one local/reconnect farm on the engine and print the first
per-client divergence from the oracle clients (dump diff and the round's events)."""
import json
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
from helpers import run_local_farm, first_diff  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402


def main(seed, n_clients, n_rounds, new_mode, reconnect):
    from fluidframework_amd import MergeTreeBatch
    rec = {}
    run_local_farm(seed, n_clients=n_clients, n_rounds=n_rounds, new_mode=new_mode, annotate=True, record=rec,
                   reconnect=reconnect)
    ids = rec["ids"]
    B = MergeTreeBatch(n_clients, new_length_calc=new_mode)
    orc = []
    for k, cid in enumerate(ids):
        B[k].insertTextLocal(0, "hello world")
        B[k].startOrUpdateCollaboration(cid)
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, "hello world")
        o.start_collab(cid)
        orc.append(o)
    for r, rnd in enumerate(rec["rounds"]):
        for k, (events, _, _) in enumerate(rnd):
            for kind, x in events:
                if kind == "local":
                    B[k].applyLocalOp(x)
                    if x["type"] == 0:
                        orc[k].insert_local_op(x["pos1"], x["seg"])
                    elif x["type"] == 1:
                        orc[k].remove_local_op(x["pos1"], x["pos2"])
                    else:
                        orc[k].annotate_local_op(x["pos1"], x["pos2"], x["props"])
                elif kind == "regen":
                    got = B[k].regeneratePendingOp(x[0])
                    orc[k].regenerate_pending_op(x[0])
                    if json.dumps(got) != json.dumps(x[1]):
                        print("round", r, "client", k, "regen differs:", json.dumps(got), "want", json.dumps(x[1]))
                else:
                    B[k].applyMsg(x)
                    orc[k].apply_msg(x)
        B.replay()
        dig = B.digests()
        for k, (events, odig, otext) in enumerate(rnd):
            if dig[k] != odig or B.text(k) != otext:
                print("round", r, "client", k, "differs; events:")
                for e in events:
                    print("  ", json.dumps(e)[:300])
                gd, od = B.dump_segments(k), orc[k].dump_segments()
                print("oracle digest matches record:", orc[k].digest() == odig)
                print(first_diff(gd, od))
                print("--- engine dump"); print(gd[:3000]); print("--- oracle dump"); print(od[:3000])
                return k, r
    print("no divergence")


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1", float(sys.argv[5]))
