"""Live clients on the GPU engine: local inserts / removes /
annotates with pending segment groups, acks, remote ops overtaking pending removes, remote annotates
leaving pending local keys alone (segmentPropertiesManager.ts:60-157) and theUnfinishedNode.

Parity: the conflict farm of tests/helpers.run_local_farm (client.conflictFarm.spec.ts with
TestClientLogger) runs on the oracle; every client's event stream -- its local ops and the sequenced
messages as it received them -- is replayed on the engine, one document per client, and after every farm
round each document's state digest and text equal its oracle client's (pending segments included: an
unacked seq is UnassignedSequenceNumber in both).  Farms run without and with local annotates.
"""
import pytest

from helpers import run_local_farm

pytestmark = pytest.mark.gpu


def _replay_farm(seed, n_clients, n_rounds, new_mode, rounds_per_replay=1, annotate=False, reconnect=0.0, rewrite=0.0):
    rec = {}
    run_local_farm(seed, n_clients=n_clients, n_rounds=n_rounds, new_mode=new_mode, annotate=annotate, record=rec,
                   reconnect=reconnect, rewrite=rewrite)
    return _replay_record(rec, seed, new_mode, rounds_per_replay, "hello world")


def _replay_record(rec, seed, new_mode, rounds_per_replay, initial, observer=None, summary=None):
    """observer: an OracleDoc that applied rec["obs_log"]; it becomes one more document of the (live) batch,
    fed its messages in four parts across the replays, and is compared at the end.  summary: SnapshotV1 blobs
    every client (and the observer) loads first, as in run_local_farm(summary=...)."""
    import json
    from fluidframework_amd import MergeTreeBatch
    ids = rec["ids"]
    n_clients = len(ids)
    B = MergeTreeBatch(n_clients + (observer is not None), new_length_calc=new_mode)
    for k, cid in enumerate(ids):
        if summary is not None:
            B[k].load(summary, cid)
            continue
        if initial:
            B[k].insertTextLocal(0, initial)
        B[k].startOrUpdateCollaboration(cid)
    if observer is not None:
        if summary is not None:
            B[n_clients].load(summary, "obs")
        else:
            if initial:
                B[n_clients].insertTextLocal(0, initial)
            B[n_clients].startOrUpdateCollaboration("obs")
        obs_log = rec["obs_log"]
        obs_parts = [obs_log[len(obs_log) * q // 4: len(obs_log) * (q + 1) // 4] for q in range(4)]
    checked = 0
    for r, rnd in enumerate(rec["rounds"]):
        for k, (events, _, _) in enumerate(rnd):
            for kind, x in events:
                if kind == "local":
                    B[k].applyLocalOp(x)
                elif kind == "regen":  # the engine regenerates the same op(s), key order included
                    op, want = x
                    got = B[k].regeneratePendingOp(op)
                    assert json.dumps(got) == json.dumps(want), f"seed {seed} round {r} client {k}: regenerated op"
                else:
                    B[k].applyMsg(x)
        if (r + 1) % rounds_per_replay and r + 1 < len(rec["rounds"]):
            continue
        if observer is not None and obs_parts and (r + 1) * 4 >= len(rec["rounds"]) * (5 - len(obs_parts)):
            for m in obs_parts.pop(0):
                B[n_clients].applyMsg(m)
        B.replay()
        dig = B.digests()
        for k, (_, odig, otext) in enumerate(rnd):
            assert B.text(k) == otext, f"seed {seed} round {r} client {k}: text"
            assert dig[k] == odig, f"seed {seed} round {r} client {k}: digest"
            checked += 1
    if observer is not None:
        for part in obs_parts:
            for m in part:
                B[n_clients].applyMsg(m)
        B.replay()
        assert B.text(n_clients) == observer.get_text(), f"seed {seed}: observer text"
        assert B.digests(n_clients, 1)[0] == observer.digest(), f"seed {seed}: observer digest"
        assert B.dump_segments(n_clients) == observer.dump_segments(), f"seed {seed}: observer dump"
    return checked


@pytest.mark.parametrize("seed", list(range(1, 17)))
def test_local_farm_every_round(seed):
    """Replay after every round: pending groups, acks and remote ops interleave across replays."""
    assert _replay_farm(seed, n_clients=4, n_rounds=40, new_mode=False) > 0


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_local_farm_new_length_calc(seed):
    assert _replay_farm(seed, n_clients=4, n_rounds=40, new_mode=True) > 0


@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_local_farm_batched_rounds(seed):
    """Many rounds per replay (local ops, acks and remote messages in one launch), more clients."""
    assert _replay_farm(seed, n_clients=8, n_rounds=150, new_mode=seed % 2 == 0, rounds_per_replay=10) > 0


@pytest.mark.parametrize("seed", list(range(31, 47)))
def test_local_annotate_farm_every_round(seed):
    """Local annotates: pending keys on the annotated segments (and on split-off halves), remote annotates
    skipping them, zamboni holding the segments until the ack."""
    assert _replay_farm(seed, n_clients=4, n_rounds=40, new_mode=False, annotate=True) > 0


@pytest.mark.parametrize("seed", [51, 52, 53, 54])
def test_local_annotate_farm_new_length_calc(seed):
    assert _replay_farm(seed, n_clients=4, n_rounds=40, new_mode=True, annotate=True) > 0


@pytest.mark.parametrize("seed", [61, 62, 63, 64])
def test_local_annotate_farm_batched_rounds(seed):
    assert _replay_farm(seed, n_clients=8, n_rounds=120, new_mode=seed % 2 == 0, rounds_per_replay=10,
                        annotate=True) > 0


REWRITE_SEEDS = list(range(131, 147))


@pytest.mark.parametrize("seed", REWRITE_SEEDS)
def test_local_rewrite_farm(seed):
    """Local rewrite annotates (combiningOp "rewrite", segmentPropertiesManager.ts:60-157): pendingRewriteCount
    makes a remote annotate leave the segment alone until the ack, a rewrite's null keys are not pending, the
    count follows split-off halves (copyTo) and survives a reconnect (orphaned groups) -- half of the local
    annotates are rewrites, some farms reconnect; states equal the oracle clients' after every round and
    regenerated ops (combiningOp first, as createAnnotateRangeOp writes it) equal op for op."""
    assert _replay_farm(seed, n_clients=3 + seed % 4, n_rounds=40, new_mode=seed % 2 == 0, annotate=True,
                        reconnect=0.3 if seed % 3 == 0 else 0.0, rewrite=0.5) > 0


@pytest.mark.parametrize("seed", list(range(71, 87)))
def test_reconnect_farm(seed):
    """Reconnects (client.reconnectFarm.spec.ts): a client's unsequenced ops are dropped, it catches up, and
    regeneratePendingOp on the engine gives the oracle's ops (normalizeSegmentsOnRebase, positions at each
    group's localSeq, new pending groups); states stay equal to the oracle clients' after every round."""
    assert _replay_farm(seed, n_clients=3 + seed % 4, n_rounds=50, new_mode=seed % 2 == 0, annotate=True,
                        reconnect=0.35) > 0


@pytest.mark.parametrize("seed", [92, 93, 94, 95])
def test_reconnect_farm_batched_rounds(seed):
    assert _replay_farm(seed, n_clients=6, n_rounds=100, new_mode=seed % 2 == 0, rounds_per_replay=5, annotate=True,
                        reconnect=0.25) > 0


@pytest.mark.parametrize("n_clients", [2, 4, 8])
@pytest.mark.parametrize("seed", [0, 1])
def test_reference_shaped_reconnect_farm(seed, n_clients):
    """client.reconnectFarm.spec.ts's own shape (helpers.run_ref_reconnect_farm: empty start, 40..320 ops per
    round against the round-start view, clients 1 (and 2) reconnecting every round): every client's local
    ops, regenerations and received messages replayed on the engine give the oracle's ops, digests and
    texts after every round."""
    from helpers import run_ref_reconnect_farm
    rec = {}
    run_ref_reconnect_farm(seed, n_clients, record=rec)
    assert _replay_record(rec, seed, True, 1, "") > 0


@pytest.mark.parametrize("n_clients", [2, 4, 8])
@pytest.mark.parametrize("min_length", [1, 16, 512])
def test_reference_shaped_conflict_farm(min_length, n_clients):
    """client.conflictFarm.spec.ts's shape (helpers.run_ref_conflict_farm: 1..128 ops per round, 8 rounds
    each, lock step, inserts at segment starts): the engine gives the oracle's digests and texts after
    every round."""
    from helpers import run_ref_conflict_farm
    rec = {}
    run_ref_conflict_farm(0, n_clients, min_length, record=rec)
    assert _replay_record(rec, 0, True, 1, "") > 0


def test_pending_local_key_survives_a_remote_annotate():
    """annotateRangeLocal then a remote annotate of the same key before the ack: the local value stays
    (shouldModifyKey); after the ack a remote annotate applies again."""
    from fluidframework_amd import MergeTreeBatch
    B = MergeTreeBatch(1)
    c = B[0]
    c.insertTextLocal(0, "abcdef")
    c.startOrUpdateCollaboration("me")
    op = c.annotateRangeLocal(1, 4, {"color": "red", "size": 1})
    c.applyMsg({"clientId": "x", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                "type": "op", "contents": {"type": 2, "pos1": 0, "pos2": 6, "props": {"color": "blue", "w": 2}}})
    B.replay()
    segs = [(e["segment"].get("text"), e["segment"].get("properties")) for e in B.map_range(0)]
    assert segs == [("a", {"color": "blue", "w": 2}), ("bcd", {"color": "red", "size": 1, "w": 2}),
                    ("ef", {"color": "blue", "w": 2})], segs
    c.applyMsg({"clientId": "me", "sequenceNumber": 2, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                "type": "op", "contents": op})
    c.applyMsg({"clientId": "x", "sequenceNumber": 3, "referenceSequenceNumber": 2, "minimumSequenceNumber": 0,
                "type": "op", "contents": {"type": 2, "pos1": 2, "pos2": 3, "props": {"color": "green"}}})
    B.replay()
    segs = [(e["segment"].get("text"), e["segment"].get("properties")) for e in B.map_range(0)]
    assert segs[1:4] == [("b", {"color": "red", "size": 1, "w": 2}), ("c", {"color": "green", "size": 1, "w": 2}),
                         ("d", {"color": "red", "size": 1, "w": 2})], segs


def test_local_insert_then_ack_api():
    """Client-level calls: insertTextLocal / removeRangeLocal while collaborating return the ops to send;
    the sequenced messages ack them (client.ts:196-247, 641-662)."""
    from fluidframework_amd import MergeTreeBatch
    B = MergeTreeBatch(1)
    c = B[0]
    c.insertTextLocal(0, "hello")
    c.startOrUpdateCollaboration("me")
    op1 = c.insertTextLocal(5, " world")
    op2 = c.removeRangeLocal(0, 1)
    B.replay()
    assert c.getText() == "ello world"
    for seq, op in ((1, op1), (2, op2)):
        c.applyMsg({"clientId": "me", "sequenceNumber": seq, "referenceSequenceNumber": 0,
                    "minimumSequenceNumber": 0, "type": "op", "contents": op})
    c.applyMsg({"clientId": "other", "sequenceNumber": 3, "referenceSequenceNumber": 2, "minimumSequenceNumber": 2,
                "type": "op", "contents": {"type": 0, "pos1": 0, "seg": "H"}})
    B.replay()
    assert c.getText() == "Hello world"


def test_local_op_out_of_range_fails_at_replay():
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.client import MergeTreeError
    B = MergeTreeBatch(1)
    B[0].insertTextLocal(0, "abc")
    B[0].startOrUpdateCollaboration("me")
    B[0].removeRangeLocal(1, 9)  # getValidOpRange does not check the end against the length
    B.replay()
    assert B.text(0) == "a"
    B[0].removeRangeLocal(1, 2)  # start at the length: RangeOutOfBounds
    with pytest.raises(MergeTreeError):
        B.replay()


@pytest.mark.parametrize("seed,n_clients", [(36, 2), (9, 6)])
def test_reconnect_farm_reference_divergence(seed, n_clients):
    """General reconnect farms whose clients end up diverged by the reference's own normalizeAdjacentSegments
    (tests/test_reference_kats.py::test_reconnect_normalization_reorders_sequenced_segments): the engine
    still equals each oracle client after every round, diverged state included."""
    assert _replay_farm(seed, n_clients=n_clients, n_rounds=60, new_mode=True, annotate=True, reconnect=0.2) > 0


@pytest.mark.parametrize("seed", list(range(301, 317)))
def test_live_farm_reused_marker_ids(seed):
    """Live clients inserting markers whose ids come from a pool of 2-5 (reused: blockUpdate's re-mapping,
    mergeTree.ts:2392 -> addNodeReferences :296-306, decides what an id names) and sending marker-relative
    inserts / annotateMarker ops; acks (ackPendingSegment's nodesToUpdate, :1283-1322) and reconnects
    (normalizeAdjacentSegments, :2320-2331) re-map too.  Every client's digest and text equal its oracle
    client's after every round, and an observer document in the same live batch (relative positions naming
    reused ids, replayed by the live kernel) equals the oracle observer."""
    rec = {}
    _, obs, _ = run_local_farm(seed, n_clients=3 + seed % 3, n_rounds=40, new_mode=seed % 2 == 0, annotate=True,
                               record=rec, marker_ids=2 + seed % 4, reconnect=0.25 if seed % 3 == 0 else 0.0)
    assert _replay_record(rec, seed, seed % 2 == 0, 1, "hello world", observer=obs) > 0


@pytest.mark.parametrize("seed,reconnect", [(101, 0.0), (102, 0.0), (103, 0.3), (104, 0.3)])
def test_live_client_summaries_match_oracle(seed, reconnect):
    """SnapshotV1 of live clients with pending local ops (Client.summarize, snapshotV1.ts:180-312): unacked
    inserts are elided and so are segments whose removal is still unacked (removedSeq ===
    UnassignedSequenceNumber = -1 <= minSeq); engine summaries equal the oracle clients' after every round."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    rec = {}
    run_local_farm(seed, n_clients=4, n_rounds=30, new_mode=seed % 2 == 0, annotate=True, record=rec,
                   reconnect=reconnect)
    ids = rec["ids"]
    B = MergeTreeBatch(len(ids), new_length_calc=seed % 2 == 0)
    orc = []
    for k, cid in enumerate(ids):
        B[k].insertTextLocal(0, "hello world")
        B[k].startOrUpdateCollaboration(cid)
        o = OracleDoc(new_length_calc=seed % 2 == 0)
        o.insert_text_local(0, "hello world")
        o.start_collab(cid)
        orc.append(o)
    pending_seen = 0
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
                    B[k].regeneratePendingOp(x[0])
                    orc[k].regenerate_pending_op(x[0])
                else:
                    B[k].applyMsg(x)
                    orc[k].apply_msg(x)
        B.replay()
        for k in range(len(ids)):
            pending_seen += orc[k].pending_groups() > 0
            gb, gs = B.summarize_v1(k)
            osum = orc[k].summarize_v1()
            assert [list(b) for b in gb] == osum["blobs"], f"seed {seed} round {r} client {k}: summary blobs"
            assert gs == osum["summary"], f"seed {seed} round {r} client {k}: summary tree"
    assert pending_seen > 0


@pytest.mark.parametrize("new_mode", [False, True])
def test_live_farm_on_summaries_with_deficits(new_mode):
    """Live clients that each load a constructed summary whose body leaves the reference with partial-length
    deficits (tests/test_gpu_phantom._tail_summary; DESIGN.md section 7 "Deficits"), then run a conflict farm:
    local ops in their own views, acks (update() of the acked segments' blocks: copyDown of deficits), remote ops
    in deficit-shortened views, zamboni.  Every client's digest and text equal its oracle client's after every
    round, and the observer's dump at the end."""
    from pyoracle import OracleDoc, OracleError
    from test_gpu_phantom import _tail_summary
    done = 0
    for k in range(0, 400, 7):
        blobs = _tail_summary(7000 + k, 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7)
        o = OracleDoc(new_length_calc=new_mode)
        try:
            o.load_v1(blobs, "c0")
        except OracleError:
            continue
        if not o.stale_deficits():
            continue
        rec = {}
        try:
            _, obs, _ = run_local_farm(k, n_clients=3, n_rounds=25, new_mode=new_mode, annotate=True, record=rec,
                                       summary=blobs)
        except OracleError as e:  # (a deficit put a local op's position past a block: the reference throws)
            assert "MergeTree insert failed" in str(e)
            continue
        assert _replay_record(rec, k, new_mode, 1, None, observer=obs, summary=blobs) > 0
        done += 1
        if done >= 8:
            break
    assert done >= 4
