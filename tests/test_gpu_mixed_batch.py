"""One batch mixing every document kind the engine routes differently: marker-relative logs (reused ids
too), incr / rewrite logs (string incr), property logs with irregular matchProperties keys and remote
consensus, and documents loaded from mid-log SnapshotV1 summaries (phantom partial lengths) that then continue
with the same kinds of log.  A batch with any irregular key runs on the marker variant (mtb_host.cpp
launch_main); this checks that every other kind of document replays the same there as on its own.

Bar: bit-exact against the oracle (canonical dump, text, state digest, SnapshotV1 blobs) after each of two
replays, both length modes."""
import pytest

from helpers import first_diff, make_incr_log, make_marker_log, make_props_log

pytestmark = pytest.mark.gpu


def _logs(new_mode):
    b = 31 * int(new_mode)
    return ([("marker", make_marker_log(1300 + b + s, 700, n_clients=3 + s % 3, lag=10 + 8 * s, new_mode=new_mode,
                                        dup_ids=4 * (s % 2))) for s in range(3)]
            + [("incr", make_incr_log(1400 + b + s, 700, n_clients=4, lag=12, new_mode=new_mode, p_rewrite=0.2 * (s % 2),
                                      string_incr=True)) for s in range(3)]
            + [("props", make_props_log(1500 + b + s, 700, n_clients=3, lag=6 + 6 * s, new_mode=new_mode))
               for s in range(3)])


@pytest.mark.parametrize("new_mode", [False, True])
def test_mixed_kinds_in_one_batch(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    logs = _logs(new_mode)
    # incr and property logs again, loaded from a summary taken a third of the way in (not the marker logs: a
    # marker a zamboni unlinked before the summary is absent from the loaded document's id map, so a later op
    # relative to it is refused)
    loaded = [(k + "/loaded", (init, msgs)) for k, (init, msgs) in logs[3::2]]
    docs = logs + loaded
    B = MergeTreeBatch(len(docs), new_length_calc=new_mode)
    orc, rest = [], []
    for i, (kind, (init, msgs)) in enumerate(docs):
        o = OracleDoc(new_length_calc=new_mode)
        if kind.endswith("/loaded"):
            g = OracleDoc(new_length_calc=new_mode)
            g.insert_text_local(0, init)
            g.start_collab("obs")
            cut = len(msgs) // 3
            for m in msgs[:cut]:
                g.apply_msg(m)
            blobs = g.summarize_v1()["blobs"]
            g.close()
            B[i].load(blobs, "loader")
            o.load_v1(blobs, "loader")
            rest.append(msgs[cut:])
        else:
            B[i].insertTextLocal(0, init)
            B[i].startOrUpdateCollaboration("obs")
            o.insert_text_local(0, init)
            o.start_collab("obs")
            rest.append(msgs)
        orc.append(o)
    for half in (0, 1):
        for i, msgs in enumerate(rest):
            mid = len(msgs) // 2
            for m in (msgs[:mid] if half == 0 else msgs[mid:]):
                B[i].applyMsg(m)
                orc[i].apply_msg(m)
        st = B.replay()
        assert st["errors"] == 0, st
        for i, o in enumerate(orc):
            what = f"{docs[i][0]} doc {i} half {half}"
            gd, od = B.dump_segments(i), o.dump_segments()
            assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
            assert B.text(i) == o.get_text(), f"{what}: text differs"
            assert B.digests(i, 1)[0] == o.digest(), f"{what}: digest differs"
    for i, o in enumerate(orc):
        gb, _ = B.summarize_v1(i)
        assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"{docs[i][0]} doc {i}: SnapshotV1 differs"
        o.close()


def test_marker_documents_beside_a_ticket_scheduled_batch():
    """The kernel is chosen per document (mtb_host.cpp mark_variant_docs): 4,200 plain generated documents replay on
    the ticket-scheduled observer kernel while the batch's marker-id documents (and a property log with irregular
    keys) replay on the marker variant, in one mtb_replay; every document equals the oracle, also after a rewind
    and resident replay."""
    from fluidframework_amd import MergeTreeBatch
    from pyloggen import LogBatch, make_cfg
    from pyoracle import OracleDoc
    from helpers import load_logbatch
    lb = LogBatch(make_cfg(seed=1607, n_ops=150), 0, 4200)
    extra = [make_marker_log(1600 + s, 400, n_clients=3, lag=8, dup_ids=2 * s) for s in range(2)] + \
            [make_props_log(1650, 400, n_clients=3, lag=6)]
    B = MergeTreeBatch(lb.n + len(extra))
    load_logbatch(B, lb)
    orc = []
    for j, (init, msgs) in enumerate(extra):
        i = lb.n + j
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc()
        o.insert_text_local(0, init)
        o.start_collab("obs")
        for m in msgs:
            B[i].applyMsg(m)
            o.apply_msg(m)
        orc.append(o)
    for rep in range(2):
        st = B.replay() if rep == 0 else (B.rewind(), B.replay_resident())[1]
        assert st["errors"] == 0, st
        assert B.launch_info()["kernel"] == "mtb_replay_tick_kernel"
        dg = B.digests()
        bad = [j for j in range(lb.n) if dg[j] != lb.docs[j].digest]
        assert not bad, f"{len(bad)} plain documents differ (first {bad[:5]})"
        for j, o in enumerate(orc):
            i = lb.n + j
            gd, od = B.dump_segments(i), o.dump_segments()
            assert gd == od, f"extra doc {j} pass {rep}: segment dump differs: {first_diff(gd, od)}"
            assert dg[i] == o.digest()
