"""Known-answer tests restated from the reference's merge-tree unit tests, run on the
CPU oracle (test infrastructure).  Each test names the reference test it restates; the reference drives
MergeTree / TestClient directly, these drive the oracle's Client-level API with the same sequence of ops
(local ops as pending local ops acked by their sequenced message, remote ops as sequenced messages).

* mergeTree.markRangeRemoved.spec.ts:114-154 (all-remote remove/insert races) and :156-227 (a passive
  observer and client 1's own view agree);
* mergeTree.zamboni.spec.ts:22-80 (cached lengths and child counts after zamboniSegments / packParent);
* partialLength.spec.ts:39-330 ((seq, len) tables of getPartialLength, cross-checked against the leaf
  sum on every query: PartialSequenceLengths.options.verifier = verify, :20);
* mergeTree.annotate.spec.ts:26-48 + :529-575 (a remote annotate, and splitAt copying its properties);
* mergeTree.insertingWalk.spec.ts:285-356 (placement across a leaf-block boundary, trap T1).
The all-remote cases run on the GPU engine too (tests/test_gpu_kats.py).
"""
import json

import pytest


def _oracle(**kw):
    from pyoracle import OracleDoc
    return OracleDoc(**kw)


def msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def segments(doc):
    """(text, removed) per segment in tree order from the canonical dump (markers as "")."""
    out = []
    for line in doc.dump_segments().splitlines()[1:]:
        row = json.loads(line)
        path, kind, text, _seq, _client, rseq, rcs, props = row
        out.append({"path": path, "text": text if kind == "T" else "", "removed": rseq != -1 or len(rcs) > 0,
                    "props": props})
    return out


def root_child_count(doc):
    return len({tuple(s["path"][:1]) for s in segments(doc)}) if segments(doc) else 0


def hello_world_observer(observer="A", writer="local"):
    """markRangeRemoved.spec.ts:15-27: "hello world" inserted one character at a time by `writer`, each
    insert sequenced at currentSeq + 1 (here seen by an observer as remote ops)."""
    o = _oracle()
    o.start_collab(observer)
    for i, ch in enumerate("hello world"):
        o.apply_msg(msg(writer, i + 1, i, {"type": 0, "pos1": i, "seg": ch}))
    assert o.get_text() == "hello world"
    return o


# ------------------------------------------------------------------ markRangeRemoved.spec.ts

def test_remote_remove_followed_by_remote_insert():
    """markRangeRemoved.spec.ts:114-133."""
    o = hello_world_observer()
    cur = o.current_seq
    o.apply_msg(msg("remote2", cur + 1, cur, {"type": 1, "pos1": 0, "pos2": 11}))
    o.apply_msg(msg("remote", cur + 2, cur, {"type": 0, "pos1": 0, "seg": "text"}))
    assert o.get_text() == "text"


def test_remote_insert_followed_by_remote_remove():
    """markRangeRemoved.spec.ts:135-154."""
    o = hello_world_observer()
    cur = o.current_seq
    o.apply_msg(msg("remote", cur + 1, cur, {"type": 0, "pos1": 0, "seg": "text"}))
    o.apply_msg(msg("remote2", cur + 2, cur, {"type": 1, "pos1": 0, "pos2": 11}))
    assert o.get_text() == "text"


def passive_observer_race_msgs():
    """markRangeRemoved.spec.ts:160-187: the sequenced ops of the race, as a passive observer sees them."""
    return [msg("1", 1, 0, {"type": 0, "pos1": 0, "seg": "a"}),
            msg("1", 2, 0, {"type": 1, "pos1": 0, "pos2": 1}),
            msg("2", 3, 0, {"type": 0, "pos1": 0, "seg": "X"}),
            msg("1", 4, 2, {"type": 0, "pos1": 0, "seg": "c"})]


@pytest.mark.parametrize("new_mode", [False, True])
def test_local_and_remote_race_at_removed_segment(new_mode):
    """markRangeRemoved.spec.ts:156-227: a passive observer (all ops remote) and client 1 (its own ops
    local, acked) end with the same text."""
    expected = _oracle(new_length_calc=new_mode, verify=True)
    expected.start_collab("3")
    for m in passive_observer_race_msgs():
        expected.apply_msg(m)
    actual = _oracle(new_length_calc=new_mode, verify=True)
    actual.start_collab("1")
    op1 = actual.insert_local_op(0, "a")
    op2 = actual.remove_local_op(0, 1)
    actual.apply_msg(msg("1", 1, 0, op1))
    actual.apply_msg(msg("1", 2, 0, op2))
    ref_at2 = actual.current_seq
    op4 = actual.insert_local_op(0, "c")
    actual.apply_msg(msg("2", 3, 0, {"type": 0, "pos1": 0, "seg": "X"}))
    actual.apply_msg(msg("1", 4, ref_at2, op4))
    assert actual.get_text() == expected.get_text()
    assert expected.get_text() == "cX"


# ------------------------------------------------------------------ mergeTree.zamboni.spec.ts

def zamboni_client():
    """mergeTree.zamboni.spec.ts:15-21: "hello world" inserted locally one character at a time before
    collaboration starts, then startOrUpdateCollaboration("localUser")."""
    o = _oracle()
    for ch in "hello world":
        o.insert_text_local(o.get_length(), ch)
    o.start_collab("localUser")
    return o


def test_zamboni_pack_parent_with_no_children_segments():
    """mergeTree.zamboni.spec.ts:22-43."""
    o = zamboni_client()
    o.apply_msg(msg("localUser", 1, 0, o.remove_local_op(0, o.get_length() - 1)))
    o.pack_parent_root()
    assert o.get_length() == 1
    cur = o.current_seq
    o.apply_msg(msg("localUser", cur, cur, o.remove_local_op(0, o.get_length()), msn=cur))
    assert o.get_length() == 0
    o.pack_parent_root()
    assert root_child_count(o) == 0


def test_zamboni_with_no_segments_to_scour():
    """mergeTree.zamboni.spec.ts:44-52."""
    o = zamboni_client()
    n, cc = o.get_length(), root_child_count(o)
    o.zamboni()
    assert (o.get_length(), root_child_count(o)) == (n, cc)


def test_zamboni_with_one_segment_to_scour():
    """mergeTree.zamboni.spec.ts:53-66: root.children[0] keeps its child count."""
    o = zamboni_client()
    first = sum(1 for s in segments(o) if s["path"][0] == 0)
    n = o.get_length()
    o.remove_local_op(0, 1)
    o.zamboni()
    assert o.get_length() == n - 1
    assert sum(1 for s in segments(o) if s["path"][0] == 0) == first


def test_zamboni_with_many_segments_to_scour():
    """mergeTree.zamboni.spec.ts:67-79: the first block's length drops to 0 and packParent leaves one child."""
    o = zamboni_client()
    o.remove_local_op(0, 6)
    assert all(s["removed"] for s in segments(o) if s["path"][0] == 0)
    o.zamboni()
    o.pack_parent_root()
    assert root_child_count(o) == 1


# ------------------------------------------------------------------ partialLength.spec.ts

def partial_doc():
    """partialLength.spec.ts:19-33: "hello world!" at seq 0, collaboration from seq 0.  Clients 17, 18 and
    19 of the reference are remote clients c17, c18, c19 of an observer; getPartialLength(seq, client) is
    the remote length of the root in that client's view (the oracle checks every query against the sum of
    the leaves' visibilities, the reference's validatePartialLengths)."""
    o = _oracle(verify=True)
    o.insert_text_local(0, "hello world!")
    o.start_collab("obs")
    for c in ("c17", "c18", "c19"):
        o.add_client(c)
    return o


def plen(o, seq, client):
    return o.remote_length(seq, o.client_ids().index(client))


def test_partial_lengths_no_ops():
    """partialLength.spec.ts:39-41."""
    assert plen(partial_doc(), 0, "c17") == 12


@pytest.mark.parametrize("writer", ["c17", "c18"])
def test_partial_lengths_single_insert(writer):
    """partialLength.spec.ts:43-96: a single insert of "more " at 0 is in both views at seq 1."""
    o = partial_doc()
    o.apply_msg(msg(writer, 1, 0, {"type": 0, "pos1": 0, "seg": "more "}))
    assert plen(o, 1, "c17") == 17 and plen(o, 1, "c18") == 17


@pytest.mark.parametrize("writer", ["c17", "c18"])
def test_partial_lengths_single_remove(writer):
    """partialLength.spec.ts:98-152: removing all 12 characters leaves 0 in both views at seq 1."""
    o = partial_doc()
    o.apply_msg(msg(writer, 1, 0, {"type": 1, "pos1": 0, "pos2": 12}))
    assert plen(o, 1, "c17") == 0 and plen(o, 1, "c18") == 0


def test_partial_lengths_aggregation():
    """partialLength.spec.ts:155-196."""
    o = partial_doc()
    for k, (w, t) in enumerate([("c17", "1"), ("c18", "2"), ("c17", "3"), ("c18", "4")]):
        o.apply_msg(msg(w, k + 1, k, {"type": 0, "pos1": 0, "seg": t}))
    assert plen(o, 4, "c17") == 16 and plen(o, 4, "c18") == 16


def test_partial_lengths_different_heights():
    """partialLength.spec.ts:198-215: 100 inserts deepen the tree; every prefix length stays right."""
    o = partial_doc()
    for i in range(100):
        o.apply_msg(msg("c17", i + 1, i, {"type": 0, "pos1": 0, "seg": "a"}))
        for c in ("c17", "c18"):
            for s in range(1, i + 2):  # validatePartialLengths: every seq in (minSeq, currentSeq] against
                plen(o, s, c)           # the leaf sum (verify mode raises on a mismatch)
            assert plen(o, i + 1, c) == i + 13
    assert plen(o, 100, "c17") == 112 and plen(o, 100, "c18") == 112


def test_partial_lengths_concurrent_overlapping_remote_deletes():
    """partialLength.spec.ts:218-243."""
    o = partial_doc()
    o.apply_msg(msg("c18", 1, 0, {"type": 1, "pos1": 0, "pos2": 10}))
    o.apply_msg(msg("c19", 2, 0, {"type": 1, "pos1": 0, "pos2": 10}))
    assert plen(o, 1, "c17") == 2


def test_partial_lengths_concurrent_local_and_remote_deletes():
    """partialLength.spec.ts:244-270."""
    o = partial_doc()
    o.apply_msg(msg("c17", 1, 0, {"type": 1, "pos1": 0, "pos2": 10}))
    o.apply_msg(msg("c18", 2, 0, {"type": 1, "pos1": 0, "pos2": 10}))
    assert plen(o, 1, "c17") == 2 and plen(o, 1, "c18") == 2


def test_partial_lengths_remote_and_unsequenced_local_deletes():
    """partialLength.spec.ts:271-297: client 17's own remove still pending when client 18's arrives."""
    o = _oracle(verify=True)
    o.insert_text_local(0, "hello world!")
    o.start_collab("c17")
    o.add_client("c18")
    op = o.remove_local_op(0, 10)
    o.apply_msg(msg("c18", 1, 0, {"type": 1, "pos1": 0, "pos2": 10}))
    assert o.remote_length(1, o.client_ids().index("c18")) == 2
    assert o.get_length() == 2
    o.apply_msg(msg("c17", 2, 0, op))
    assert o.get_length() == 2


# ------------------------------------------------------------------ mergeTree.annotate.spec.ts

def annotate_doc():
    """mergeTree.annotate.spec.ts:28-48: "hello world!" at seq 0, then a remote client inserts a Tile marker
    (refType 1) at position 3 with seq 1."""
    o = _oracle()
    o.insert_text_local(0, "hello world!")
    o.start_collab("local")
    o.apply_msg(msg("remote", 1, 0, {"type": 0, "pos1": 3, "seg": {"marker": {"refType": 1}}}))
    return o


def test_annotate_remote_first_sets_props_and_split_copies_them():
    """mergeTree.annotate.spec.ts:529-575 (remote first: remote only / split remote): a remote annotate of
    [1, 5) sets its properties; splitting an annotated segment copies them to both halves."""
    o = annotate_doc()
    o.apply_msg(msg("remote", 2, 1, {"type": 2, "pos1": 1, "pos2": 5,
                                     "props": {"propertySource": "remote", "remoteProperty": 1}}))
    segs = segments(o)
    pos, hit = 0, None
    for s in segs:
        ln = len(s["text"]) if s["text"] else 1
        if pos <= 1 < pos + ln:
            hit = s
        pos += ln
    assert hit["props"] == {"propertySource": "remote", "remoteProperty": 1}
    # splitAt(1) of the segment holding position 1: a remote insert at position 2 splits "el"
    o.apply_msg(msg("other", 3, 2, {"type": 0, "pos1": 2, "seg": "Z"}))
    texts = [(s["text"], s["props"]) for s in segments(o)]
    assert ("e", {"propertySource": "remote", "remoteProperty": 1}) in texts
    assert ("l", {"propertySource": "remote", "remoteProperty": 1}) in texts
    assert o.get_text() == "heZllo world!"


# ------------------------------------------------------------------ mergeTree.insertingWalk.spec.ts

@pytest.mark.parametrize("new_mode", [False, True])
def test_inserting_walk_conflict_across_block_boundary(new_mode):
    """mergeTree.insertingWalk.spec.ts:285-356: seven unacked local inserts at 0 split the root into two
    blocks; with "DCBA" removed locally, a concurrent remote insert at 0 lands directly before "0"."""
    o = _oracle(new_length_calc=new_mode, verify=True)
    o.insert_text_local(0, "0")
    o.start_collab("local")
    for i in range(1, 8):
        o.insert_local_op(0, chr(i + 64))
    assert root_child_count(o) == 2
    assert o.get_text() == "GFEDCBA0"
    o.remove_local_op(3, 7)
    assert o.get_text() == "GFE0"
    o.apply_msg(msg("remote", 1, 0, {"type": 0, "pos1": 0, "seg": "x"}))
    got = [f"({s['text']})" if s["removed"] else s["text"] for s in segments(o)]
    assert got == ["G", "F", "E", "(D)", "(C)", "(B)", "(A)", "x", "0"]


def test_normalize_segments_on_rebase_docstring_example():
    """mergeTree.ts:2337-2356 (normalizeSegmentsOnRebase's example, new length calculations): client 1 inserts
    "good " into "hi my friend" while client 2's removal of "my " is sequenced; client 1 reconnects at seq 1:
    its segments ["hi ", Removed"my ", Local"good ", "friend"] become ["hi ", Local"good ", Removed"my ",
    "friend"] -- client 2's order once the regenerated insert (at 3) lands -- and regeneratePendingOp
    (client.ts:917-960) gives that insert."""
    import json
    from pyoracle import OracleDoc
    c1, c2 = OracleDoc(new_length_calc=True), OracleDoc(new_length_calc=True)  # c2: a third client observing both
    for c, cid in ((c1, "c1"), (c2, "c3")):
        c.insert_text_local(0, "hi my friend")
        c.start_collab(cid)
    op = c1.insert_local_op(6, "good ")
    assert c1.get_text() == "hi my good friend"
    rm = {"clientId": "c2", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
          "type": "op", "contents": {"pos1": 3, "pos2": 6, "type": 1}}
    c1.apply_msg(rm)
    c2.apply_msg(rm)
    order = lambda c: [json.loads(l)[2] for l in c.dump_segments().splitlines()[1:]]  # noqa: E731
    assert order(c1) == ["hi ", "my ", "good ", "friend"]
    new = c1.regenerate_pending_op(op)
    assert new == {"pos1": 3, "seg": "good ", "type": 0}
    assert order(c1) == ["hi ", "good ", "my ", "friend"]
    ack = {"clientId": "c1", "sequenceNumber": 2, "referenceSequenceNumber": 1, "minimumSequenceNumber": 0,
           "type": "op", "contents": new}
    c1.apply_msg(ack)
    c2.apply_msg(ack)
    assert order(c1) == order(c2) == ["hi ", "good ", "my ", "friend"]
    assert c1.get_text() == c2.get_text() == "hi good friend"


@pytest.mark.parametrize("seed", list(range(1, 13)))
def test_reconnect_farm_converges(seed):
    """client.reconnectFarm.spec.ts-style farms (new length calculations): clients drop their in-flight ops,
    catch up and resubmit regeneratePendingOp's output; every client ends with the observer's text and
    per-character properties (partial lengths cross-checked against leaf sums on every query).  A small
    fraction of such farms (about 1 in 100 with 2 or 6+ clients) does not converge on the oracle -- lagging
    clients with other clients' ops in flight, which the reference's own farm shape never creates (that shape,
    test_reference_shaped_reconnect_farm below, converged in 600 of 600 farms); DESIGN.md section 10."""
    from helpers import chars_with_props, run_local_farm
    clients, obs, _ = run_local_farm(seed, n_clients=3 + seed % 4, n_rounds=50, new_mode=True, annotate=True,
                                     verify=True, reconnect=0.3)
    want = chars_with_props(obs)
    for c in clients:
        assert c.get_text() == obs.get_text()
        assert chars_with_props(c) == want


@pytest.mark.parametrize("n_clients", [2, 4, 8])
@pytest.mark.parametrize("seed", [0, 1])
def test_reference_shaped_reconnect_farm(seed, n_clients):
    """client.reconnectFarm.spec.ts's own shape (clients 2/4/8, 40..320 ops per round, 3 rounds each, client 1
    -- and on a coin flip client 2 -- reconnecting every round, everyone else in lock step): all clients agree
    on text and per-character properties after every round.  200 seeds x 3 client counts of this shape ran
    green on the oracle (helpers.run_ref_reconnect_farm)."""
    from helpers import run_ref_reconnect_farm
    clients = run_ref_reconnect_farm(seed, n_clients)
    assert len({c.get_text() for c in clients}) == 1


@pytest.mark.parametrize("n_clients", [2, 4, 8])
@pytest.mark.parametrize("min_length", [1, 16, 512])
def test_reference_shaped_conflict_farm(min_length, n_clients):
    """client.conflictFarm.spec.ts's shape (defaultOptions: 1..128 ops per round, 8 rounds each, lock step,
    minLength 1..512): all clients agree on text and per-character properties after every round."""
    from helpers import run_ref_conflict_farm
    clients = run_ref_conflict_farm(0, n_clients, min_length)
    assert len({c.get_text() for c in clients}) == 1


def _acked_order(doc):
    """Text of every sequenced segment (removed ones included) in tree order, from the canonical dump."""
    import json as _json
    out = []
    for line in doc.dump_segments().split("\n")[1:]:
        if line.strip():
            _, _, text, seq, *_ = _json.loads(line)
            if seq != -1:
                out.append(text)
    return "".join(out).encode("utf-16-le", "surrogatepass").decode("utf-16-le", "surrogatepass")


def test_reconnect_normalization_reorders_sequenced_segments():
    """Why ~1 in 100 general reconnect farms (helpers.run_local_farm, reconnect > 0) diverge: the reference's
    normalizeAdjacentSegments (mergeTree.ts:2234-2336), run by regeneratePendingOp (client.ts:917-960), slides
    remotely removed (acked) segments after the run's last segment that is not removed-and-acked -- and that
    segment may be an acked insert that is only *locally* removed.  The reconnecting client then holds two
    sequenced segments in an order no other client has.  Farm (seed 36, 2 clients, new length calculation),
    client c1, regeneration at currentSeq 51: the run [f (local insert, local remove), "\\n", "x" (removed at
    49), "xyzx" (removed at 50), "yzxy", "z" (seq 45, local remove)] becomes [f, "yzxy", "z", "\\n", "x",
    "xyzx"], while every receiver of the regenerated ops keeps [f, "\\n", "x", "xyzx", "yzxy", "z"]
    (insertingWalk places f before the zero-length tombstones; removes move nothing).  c0's insert at seq 58
    (refSeq 47: "xyzx" and "yzxy" both still visible to it) then resolves pos 23 at different places on c1
    and on the rest, and the texts diverge.  The reference's own reconnect farm
    (client.reconnectFarm.spec.ts:25-121) never sends an op whose refSeq predates the overlapped removes, so
    it cannot see this; the oracle follows mergeTree.ts step for step here, and the engine matches the oracle
    client for client on this farm (tests/test_gpu_local.py::test_reconnect_farm_reference_divergence)."""
    from helpers import run_local_farm
    from pyoracle import OracleDoc
    rec = {}
    clients, obs, _ = run_local_farm(36, n_clients=2, n_rounds=60, new_mode=True, annotate=True, reconnect=0.2,
                                     record=rec)
    c1 = OracleDoc(new_length_calc=True)
    c1.insert_text_local(0, "hello world")
    c1.start_collab(rec["ids"][1])
    o = OracleDoc(new_length_calc=True)
    o.insert_text_local(0, "hello world")
    o.start_collab("obs")
    stop = False
    for rnd in rec["rounds"]:
        for kind, x in rnd[1][0]:
            if kind == "msg" and x["sequenceNumber"] == 58:
                stop = True
                break
            if kind == "local":
                if x["type"] == 0:
                    c1.insert_local_op(x["pos1"], x["seg"])
                elif x["type"] == 1:
                    c1.remove_local_op(x["pos1"], x["pos2"])
                else:
                    c1.annotate_local_op(x["pos1"], x["pos2"], x["props"])
            elif kind == "regen":
                c1.regenerate_pending_op(x[0])
            else:
                c1.apply_msg(x)
                o.apply_msg(x)
        if stop:
            break
    assert c1.current_seq == o.current_seq == 57
    mine, theirs = _acked_order(c1), _acked_order(o)
    assert "\U0001F600def" + "yzxyz" + "\nx" + "xyzx" + "yzxy" in mine
    assert "\U0001F600def" + "\nx" + "xyzx" + "yzxyz" + "yzxy" in theirs
    assert clients[0].get_text() == obs.get_text() and clients[1].get_text() != obs.get_text()
