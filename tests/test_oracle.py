"""CPU oracle vs the reference's own golden data (no GPU).

* 30 committed conflict-farm replay logs (packages/dds/merge-tree/src/test/results, replayed by
  client.replay.spec.ts:16-72): the text after each of the 1,920 groups.
* the same logs with the partial-length verifier on: every remote-perspective block length returned by
  the PartialSequenceLengths restatement equals the sum of its leaves' visibilities (the identity the
  GPU's window lists rely on).
* the 6 committed SnapshotV1 summaries (packages/dds/sequence/src/test/snapshots/v1), byte-exact, from
  the generateSharedStrings.ts:47-146 recipes.
* known-answer tests restated from client.applyMsg.spec.ts on the observer path.
"""
import pytest
from pyoracle import OracleDoc, OracleError

from helpers import msg_from_compact, replay_fixtures, snapshot_fixture

FIXTURES = replay_fixtures()


@pytest.mark.parametrize("name,d", FIXTURES, ids=[n for n, _ in FIXTURES])
def test_replay_log_text_after_every_group(name, d):
    o = OracleDoc()
    o.insert_text_local(0, d["initialText"])
    o.start_collab("A")
    for gi, g in enumerate(d["groups"]):
        for m in g["msgs"]:
            o.apply_msg(msg_from_compact(m))
        assert o.get_text() == g["resultText"], f"{name}: group {gi}"


@pytest.mark.parametrize("idx", [0, 7, 15, 22, 29])
def test_partial_lengths_equal_leaf_sums(idx):
    name, d = FIXTURES[idx]
    o = OracleDoc(verify=True)
    o.insert_text_local(0, d["initialText"])
    o.start_collab("A")
    for g in d["groups"]:
        for m in g["msgs"]:
            o.apply_msg(msg_from_compact(m))
    assert o.get_text() == d["groups"][-1]["resultText"]


SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk


def _build_detached(name):
    """generateSharedStrings.ts:47-146 on a detached (non-collaborating) string."""
    d = OracleDoc()
    t = "text"
    if name in ("headerOnly", "withIntervals"):
        for i in range(int(SIZE_OF_FIRST_CHUNK / len(t) / 2)):
            d.insert_text_local(0, f"{t}{i}")
    elif name == "headerAndBody":
        for i in range(int(SIZE_OF_FIRST_CHUNK / len(t) * 2)):
            d.insert_text_local(0, f"{t}{i}")
    elif name == "largeBody":
        for i in range(SIZE_OF_FIRST_CHUNK):
            d.insert_text_local(0, f"{t}-{i}")
    elif name == "withMarkers":
        for i in range(int(SIZE_OF_FIRST_CHUNK / len(t) * 2)):
            d.insert_text_local(0, f"{t}{i}")
        i = 0
        while i < d.get_length():
            d.insert_marker_local(i, 1, {"ItemType": "Paragraph", "Properties": {"Bold": False},
                                         "markerId": f"marker{i}", "referenceTileLabels": ["Eop"]})
            i += 70
    elif name == "withAnnotations":
        for i in range(int(SIZE_OF_FIRST_CHUNK / len(t) * 2)):
            d.insert_text_local(0, f"{t}{i}")
        i = 0
        while i < d.get_length():
            d.annotate_local(i, i + 10, {"bold": True})
            i += 70
    return d


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations",
                                  "withIntervals"])
def test_snapshot_v1_fixture_bytes(name):
    expected = [b for b in snapshot_fixture(name)]
    got = _build_detached(name).summarize_v1(0, 0)
    assert [list(b) for b in got["blobs"]] == expected
    stats = got["summary"]["stats"]
    assert stats["blobNodeCount"] == len(expected)
    assert stats["treeNodeCount"] == 1


def _msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def _initial(state, new_mode=False):
    """createClientsAtInitialState (testClientLogger.ts:51): '-' become detached tombstones."""
    o = OracleDoc(new_length_calc=new_mode)
    o.insert_text_local(0, state)
    while "-" in o.get_text():
        i = o.get_text().index("-")
        o.remove_local(i, i + 1)
    o.start_collab("A")
    return o


def test_kat_conflicting_inserts_at_deleted_segment_position():
    # client.applyMsg.spec.ts:440-462 -> "ab"
    o = _initial("a----bcd-ef")
    o.apply_msg(_msg("B", 1, 0, {"type": 0, "pos1": 4, "seg": "B"}))
    o.apply_msg(_msg("C", 2, 0, {"type": 0, "pos1": 4, "seg": "CC"}))
    o.apply_msg(_msg("C", 3, 0, {"type": 1, "pos1": 2, "pos2": 8}))
    o.apply_msg(_msg("B", 4, 2, {"type": 1, "pos1": 5, "pos2": 8}))
    assert o.get_text() == "ab"


def test_kat_9703_new_length_calculations():
    # client.applyMsg.spec.ts:464-493 (mergeTreeUseNewLengthCalculations: true) -> "ayzXd"
    o = _initial("abcd", new_mode=True)
    o.apply_msg(_msg("B", 1, 0, {"type": 1, "pos1": 1, "pos2": 3}))
    o.apply_msg(_msg("B", 2, 1, {"type": 0, "pos1": 1, "seg": "yz"}))
    o.apply_msg(_msg("C", 3, 0, {"type": 0, "pos1": 2, "seg": "X"}))
    assert o.get_text() == "ayzXd"


def test_kat_remote_remove_before_conflicting_insert():
    # client.applyMsg.spec.ts:415-438 -> "CB"
    o = _initial("Z")
    o.apply_msg(_msg("B", 1, 0, {"type": 1, "pos1": 0, "pos2": 1}))
    o.apply_msg(_msg("B", 2, 0, {"type": 0, "pos1": 0, "seg": "B"}))
    o.apply_msg(_msg("C", 3, 1, {"type": 0, "pos1": 0, "seg": "C"}))
    assert o.get_text() == "CB"


def test_assert_codes():
    o = _initial("abc")
    o.apply_msg(_msg("B", 5, 0, {"type": 0, "pos1": 0, "seg": "x"}))
    with pytest.raises(Exception, match="0x038"):
        o.apply_msg(_msg("B", 4, 0, {"type": 0, "pos1": 0, "seg": "y"}))


def test_group_op_members_share_seq():
    o = _initial("hello")
    o.apply_msg(_msg("B", 1, 0, {"type": 3, "ops": [{"type": 0, "pos1": 5, "seg": " world"},
                                                     {"type": 2, "pos1": 0, "pos2": 5, "props": {"bold": True}}]}))
    assert o.get_text() == "hello world"
    dump = o.dump_segments().splitlines()
    assert any('"bold":true' in line for line in dump)


# ---- SnapshotV1 load (snapshotLoader.ts:41-220) ----

@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations",
                                  "withIntervals"])
def test_snapshot_v1_load_roundtrip(name):
    """Loading a committed reference summary and summarizing it again reproduces the same bytes."""
    blobs = snapshot_fixture(name)
    o = OracleDoc()
    o.load_v1(blobs, "snapshot")
    got = o.summarize_v1(0, 0)
    assert [list(b) for b in got["blobs"]] == blobs


@pytest.mark.parametrize("idx", [0, 4, 11, 18, 25, 29])
@pytest.mark.parametrize("cut", [16, 40])
def test_snapshot_v1_load_mid_stream_then_continue(idx, cut):
    """Summarize an observer after `cut` groups, load the summary into a fresh client, keep replaying:
    the loaded client matches the reference's golden text after every later group."""
    name, d = FIXTURES[idx]
    a = OracleDoc()
    a.insert_text_local(0, d["initialText"])
    a.start_collab("A")
    groups = d["groups"]
    for g in groups[:cut]:
        for m in g["msgs"]:
            a.apply_msg(msg_from_compact(m))
    blobs = a.summarize_v1()["blobs"]
    b = OracleDoc()
    b.load_v1([list(x) for x in blobs], "A")
    assert b.get_text() == groups[cut - 1]["resultText"]
    for gi in range(cut, len(groups)):
        for m in groups[gi]["msgs"]:
            b.apply_msg(msg_from_compact(m))
        assert b.get_text() == groups[gi]["resultText"], f"{name}: group {gi}"


# ---- SharedMatrix PermutationVectors (matrix/src/permutationvector.ts, handletable.ts) ----

@pytest.mark.parametrize("seed", [1, 2, 3])
def test_matrix_oracle_handle_table_invariants(seed):
    """Allocated handles are distinct and marked 0 in the table; the free list threads every other slot
    and ends at the table's length (handletable.ts:36-58)."""
    import json
    from helpers import make_matrix_log
    from pyoracle import OracleMatrix
    msgs = make_matrix_log(seed, 600, n_clients=4, lag=12)
    o = OracleMatrix()
    o.start_collab("obs")
    for m in msgs:
        o.apply_msg(m)
    for vec in (o.rows, o.cols):
        lines = vec.dump_segments().splitlines()
        table = json.loads(lines[0])["handles"]
        owned = []
        for ln in lines[1:]:
            row = json.loads(ln)
            length, start = row[2]
            if start >= 1:
                owned += range(start, start + length)
        assert len(owned) == len(set(owned))
        assert all(table[h] == 0 for h in owned)
        free, h = [], table[0]
        while h < len(table):
            free.append(h)
            h = table[h]
        assert h == len(table)
        assert not set(free) & set(owned)
        # removed-but-not-yet-unlinked segments may still own handles
        assert len(free) + len(owned) == len(table) - 1


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations",
                                  "withIntervals"])
def test_snapshot_legacy_fixture_bytes(name):
    """SnapshotLegacy (snapshotlegacy.ts:122-259) of the generateSharedStrings.ts recipes, byte-exact against
    the reference's committed snapshots/legacy files (the interval-collection blob aside)."""
    expected = snapshot_fixture(name, "legacy")
    got = _build_detached(name).summarize_legacy(0, 0)
    assert [list(b) for b in got["blobs"]] == expected


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations",
                                  "withIntervals"])
def test_snapshot_legacy_fixture_loads_and_resummarizes(name):
    """Client.load of the reference's snapshots/legacy files (legacy chunks through toLatestVersion,
    snapshotChunks.ts:151-199; header, then the "body" chunk when chunkLengthChars < totalLengthChars,
    snapshotLoader.ts:133-220): the generating recipe's text, and SnapshotLegacy of the loaded string gives the
    fixture's bytes again."""
    blobs = snapshot_fixture(name, "legacy")
    o = OracleDoc()
    assert o.load_v1(blobs, "loader") == []  # no catch-up blob
    assert o.get_text() == _build_detached(name).get_text()
    assert [list(b) for b in o.summarize_legacy(0, 0)["blobs"]] == blobs


def _legacy_midstream(d, g, chunk=0):
    """Replay groups [0, g) with catch-up tracking, then SnapshotLegacy at the MSN (with the catch-up blob)."""
    o = OracleDoc(chunk_size=chunk)
    o.insert_text_local(0, d["initialText"])
    o.start_collab("A")
    o.enable_catch_up()
    for grp in d["groups"][:g]:
        for m in grp["msgs"]:
            o.apply_msg(msg_from_compact(m))
    return o, o.summarize_legacy()["blobs"]


@pytest.mark.parametrize("idx", [0, 5, 11, 17, 23, 29])
@pytest.mark.parametrize("g", [16, 40])
def test_legacy_load_with_catch_up_continues_the_reference_logs(idx, g):
    """SharedSegmentSequence.loadCore over a SnapshotLegacy summary taken mid-log (sequence.ts:568-610): load
    the MSN state, replay the catch-up blob with the collab-window validation (lagging messages were rewritten
    to refSeq = seq - 1, sequence.ts:697-748), then the rest of the log: the golden text after every later
    group, and a legacy summary of the loaded string at the end equal to the never-stopped one's text."""
    name, d = FIXTURES[idx]
    o, blobs = _legacy_midstream(d, g, chunk=300 if idx % 2 else 0)
    r = OracleDoc(chunk_size=300 if idx % 2 else 0)
    msgs = r.load_v1(blobs, "loader")
    assert msgs and all(m["minimumSequenceNumber"] == r.min_seq for m in msgs)
    r.apply_catch_up(msgs)
    assert r.get_text() == o.get_text() and r.current_seq == o.current_seq
    for grp in d["groups"][g:]:
        for m in grp["msgs"]:
            r.apply_msg(msg_from_compact(m))
        assert r.get_text() == grp["resultText"], name


def test_catch_up_validation_rejects_stale_messages():
    """sequence.ts:580-596: a catch-up message at or below the loaded collab window throws."""
    name, d = FIXTURES[3]
    _, blobs = _legacy_midstream(d, 20)
    r = OracleDoc()
    msgs = r.load_v1(blobs, "loader")
    with pytest.raises(OracleError, match="Invalid catchup"):
        r.apply_catch_up([dict(msgs[0], sequenceNumber=r.current_seq)])


def _msn_backwards(msgs):
    """The catch-up list with one message's MSN raised to its refSeq, above the next message's MSN: that next
    message then lies below the window the raised one moved (setMinSeq), which sequence.ts:578-585 rejects."""
    i = next(i for i in range(len(msgs) - 1)
             if msgs[i]["referenceSequenceNumber"] > msgs[i + 1]["minimumSequenceNumber"])
    out = [dict(m) for m in msgs]
    out[i]["minimumSequenceNumber"] = out[i]["referenceSequenceNumber"]
    return out


def test_catch_up_validation_follows_the_moving_window():
    """getCollabWindow() is read again for every catch-up message (sequence.ts:578-585): a message whose MSN
    is below an earlier message's MSN is rejected, not only one below the header's window."""
    name, d = FIXTURES[3]
    _, blobs = _legacy_midstream(d, 20)
    r = OracleDoc()
    msgs = r.load_v1(blobs, "loader")
    assert len(msgs) >= 2
    with pytest.raises(OracleError, match="Invalid catchup"):
        r.apply_catch_up(_msn_backwards(msgs))


@pytest.mark.parametrize("idx", [0, 3, 9, 17, 26])
def test_catch_up_messages_replay_to_the_final_text(idx):
    """SnapshotLegacy + catch-up (sequence.ts:680-748): the header/body text at the MSN, then the stored
    catch-up messages (lagging ones rewritten from their deltas to refSeq = seq - 1) replayed in order,
    reproduce the reference's golden final text."""
    import json
    name, d = FIXTURES[idx]
    o = OracleDoc()
    o.insert_text_local(0, d["initialText"])
    o.start_collab("A")
    o.enable_catch_up()
    for g in d["groups"]:
        for m in g["msgs"]:
            o.apply_msg(msg_from_compact(m))
    blobs = dict(o.summarize_legacy()["blobs"])
    header = json.loads(blobs["header"])
    texts = header["segmentTexts"] + (json.loads(blobs["body"])["segmentTexts"] if "body" in blobs else [])
    msgs = json.loads(blobs.get("catchupOps", "[]"))
    assert msgs, "the logs end with lagging messages above the MSN"
    msn = header["chunkSequenceNumber"]
    r = OracleDoc()
    r.insert_text_local(0, "".join(t if isinstance(t, str) else t["text"] for t in texts))
    r.start_collab("loader", msn, msn)
    for m in msgs:
        assert m["referenceSequenceNumber"] == m["sequenceNumber"] - 1
        r.apply_msg(m)
    assert r.get_text() == d["groups"][-1]["resultText"], name


def _catch_up_kat_doc():
    """"abcdef" {s: "x", m: 0}; seq 1 inserts "zz" at 0; seq 2 (refSeq 0) rewrites [2, 4) of its view with
    {n: 1, m: 0}; seq 3 (another client, refSeq 0) incrs m over [0, 4) of its view (two segments, "ab" and "cd")."""
    o = OracleDoc()
    o.insert_text_local(0, "abcdef")
    o.annotate_local(0, 6, {"s": "x", "m": 0})
    o.start_collab("A")
    o.enable_catch_up()
    msg = dict(type="op", minimumSequenceNumber=0, referenceSequenceNumber=0)
    o.apply_msg(dict(msg, clientId="c1", sequenceNumber=1, contents={"type": 0, "pos1": 0, "seg": "zz"}))
    o.apply_msg(dict(msg, clientId="c2", sequenceNumber=2, contents={
        "type": 2, "pos1": 2, "pos2": 4, "props": {"n": 1, "m": 0}, "combiningOp": {"name": "rewrite"}}))
    o.apply_msg(dict(msg, clientId="c3", sequenceNumber=3, contents={
        "type": 2, "pos1": 0, "pos2": 4, "props": {"m": 1}, "combiningOp": {"name": "incr"}}))
    return o


def test_catch_up_rewriting_kat():
    """Hand-derived known answer for createOpsFromDelta over propertyDeltas (segmentPropertiesManager.ts:107-154):
    the lagging rewrite's props are its deleted keys in their old order (s: gone -> null; m: falsy in the
    rewrite -> deleted, then re-set to 0) followed by its own key n; the lagging incr's NaN values (JSON null)
    never matchProperties-equal, so its two adjacent segments stay two ops of a GROUP."""
    import json
    o = _catch_up_kat_doc()
    cu = json.loads(dict(o.summarize_legacy()["blobs"])["catchupOps"])
    assert [m["contents"] for m in cu] == [
        {"type": 0, "pos1": 0, "seg": "zz"},
        {"pos1": 4, "pos2": 6, "props": {"s": None, "m": 0, "n": 1}, "type": 2},
        {"ops": [{"pos1": 2, "pos2": 4, "props": {"m": None}, "type": 2},
                 {"pos1": 4, "pos2": 6, "props": {"m": None}, "type": 2}], "type": 3}]
    assert [list(m["contents"].get("props", {})) for m in cu[1:2]] == [["s", "m", "n"]]
    assert all(m["referenceSequenceNumber"] == m["sequenceNumber"] - 1 for m in cu[1:])


def _char_props(o):
    """Each visible character's property set (map_range segments), NaN/null-valued keys dropped."""
    out = []
    for r in o.map_range():
        seg = r["segment"]
        props = {k: v for k, v in (seg.get("properties") or {}).items() if v is not None}
        out += [props] * seg["cachedLength"]
    return out


@pytest.mark.parametrize("seed,p_incr", [(1, 0.0), (2, 0.0), (3, 0.15), (4, 0.15)])
@pytest.mark.parametrize("new_mode", [False, True])
def test_catch_up_rewriting_of_rewrite_and_incr_annotates(seed, p_incr, new_mode):
    """createOpsFromDelta (sequence.ts:120-172) over a lagging rewrite annotate's propertyDeltas -- the keys it
    deleted, in their old order, then its own (segmentPropertiesManager.ts:107-154) -- and over an incr's NaN
    values (never matchProperties-equal, JSON null): a legacy summary taken mid-log with its catch-up blob,
    loaded and caught up, equals the never-stopped document in text and, for rewrite-only logs, in every
    character's properties; both then continue to the same text (and properties)."""
    import json
    from helpers import make_incr_log
    init, msgs = make_incr_log(seed, 700, lag=24, new_mode=new_mode, p_incr=p_incr, p_rewrite=0.2)
    cut = 450
    src = OracleDoc(new_length_calc=new_mode)
    src.insert_text_local(0, init)
    src.start_collab("A")
    src.enable_catch_up()
    for m in msgs[:cut]:
        src.apply_msg(m)
    blobs = src.summarize_legacy()["blobs"]
    msn = src.min_seq
    lagging = [m for m in msgs[:cut] if m["sequenceNumber"] > msn and
               m["referenceSequenceNumber"] != m["sequenceNumber"] - 1 and "combiningOp" in m["contents"]]
    assert any(m["contents"]["combiningOp"]["name"] == "rewrite" for m in lagging)
    if p_incr:
        assert any(m["contents"]["combiningOp"]["name"] == "incr" for m in lagging)
    cu = json.loads(dict(blobs)["catchupOps"])
    assert all(m["referenceSequenceNumber"] == m["sequenceNumber"] - 1 for m in cu)
    assert not any("combiningOp" in json.dumps(m["contents"]) for m in cu
                   if m["sequenceNumber"] in {x["sequenceNumber"] for x in lagging})
    r = OracleDoc(new_length_calc=new_mode)
    r.apply_catch_up(r.load_v1(blobs, "loader"))
    assert r.get_text() == src.get_text()
    if not p_incr:
        assert _char_props(r) == _char_props(src)
    for m in msgs[cut:]:
        src.apply_msg(m)
        r.apply_msg(m)
    assert r.get_text() == src.get_text()
    if not p_incr:
        assert _char_props(r) == _char_props(src)


# ---------------------------------------------------------------- SharedMatrix cells (SparseArray2D)
def _sa2d_fill(a, r0, c0, nr, nc):  # matrix/src/test/utils.ts fill: value = row * rowCount + col
    for r in range(r0, r0 + nr):
        for c in range(c0, c0 + nc):
            a.set_cell(r, c, str(r * nr + c))


def _sa2d_extract(a, r0, c0, nr, nc):
    return [[a.get_cell(r, c) for c in range(c0, c0 + nc)] for r in range(r0, r0 + nr)]


def test_sparse_array_2d_read_write_corners():
    """sparsearray2d.spec.ts "read/write top-left / bottom-right 256x256" (64x64 here: same tiles)."""
    from pyoracle import OracleSparseArray2D
    a = OracleSparseArray2D()
    for r0 in (0, 0xFFFFFF00):
        _sa2d_fill(a, r0, r0, 64, 64)
        assert _sa2d_extract(a, r0, r0, 64, 64) == [[str(r * 64 + c) for c in range(r0, r0 + 64)]
                                                    for r in range(r0, r0 + 64)]
    assert a.get_cell(0, 0xFFFFFF00) is None and a.get_cell(5, 300) is None


def _clear_cases():
    cases = [(0, 0, 1, 1, 0, 1), (0, 0, 256, 256, 127, 2)]
    cases += [(0, 0, 16, 16, i, 1) for i in range(16)]
    s = 0xFFFFFFF0
    cases += [(s, s, 16, 16, i, 1) for i in range(s, s + 16)]
    return cases


@pytest.mark.parametrize("rows", [True, False])
def test_sparse_array_2d_clear_rows_cols(rows):
    """sparsearray2d.spec.ts "clear row/cols": clearing equals setting the cleared cells to undefined."""
    from pyoracle import OracleSparseArray2D
    for (r0, c0, nr, nc, cs, cn) in _clear_cases():
        if nr == 256:
            nr = nc = 160  # straddles the 127/128 discontinuity, fewer cells
        actual, expected = OracleSparseArray2D(), OracleSparseArray2D()
        _sa2d_fill(actual, r0, c0, nr, nc)
        _sa2d_fill(expected, r0, c0, nr, nc)
        if rows:
            actual.clear_rows(cs, cn)
            for r in range(cs, cs + cn):
                for c in range(c0, c0 + nc):
                    expected.set_cell(r, c, None)
        else:
            actual.clear_cols(cs, cn)
            for r in range(r0, r0 + nr):
                for c in range(cs, cs + cn):
                    expected.set_cell(r, c, None)
        assert _sa2d_extract(actual, r0, c0, nr, nc) == _sa2d_extract(expected, r0, c0, nr, nc)


def test_sparse_array_2d_snapshot_layout():
    """snapshot() is the root array itself: JSON.stringify turns holes and undefined into null; levels are
    256-entry arrays created on first write and never removed (clears only reset leaves)."""
    import json
    from pyoracle import OracleSparseArray2D
    a = OracleSparseArray2D()
    assert a.snapshot() == "[null]"
    a.set_cell(1, 2, '"x"')  # keyLo = row bits odd, col bits even = 0b110 -> leaf index 6
    snap = json.loads(a.snapshot())
    assert len(snap) == 1 and len(snap[0]) == 256 and snap[0][0][0][0][6] == "x"
    a.clear_rows(1, 1)
    assert json.loads(a.snapshot())[0][0][0][0] == [None] * 256
    a.set_cell(0x10000, 0, "1")  # keyHi = morton(1, 0) = 2: the root grows to length 3 with a hole
    snap = json.loads(a.snapshot())
    assert len(snap) == 3 and snap[1] is None and snap[2][0][0][0][0] == 1


def test_matrix_cells_follow_handles():
    """SharedMatrix observer cells (matrix.ts:668-690): set at (rowHandle, colHandle) when both positions
    survive; recycled handles clear their row/col before reuse (matrix.ts:721-733)."""
    import json
    from helpers import make_matrix_log
    from pyoracle import OracleMatrix
    o = OracleMatrix()
    o.start_collab("obs")
    for m in make_matrix_log(11, 600, n_clients=3, lag=8):
        o.apply_msg(m)
    s = o.summarize()
    paths = [p for p, _ in s["blobs"]]
    assert paths[-1] == "cells" and "rows/handleTable" in paths and "cols/handleTable" in paths
    cells, pending = json.loads(s["blobs"][-1][1])
    assert pending == [None]
    st = s["summary"]["stats"]
    assert st["treeNodeCount"] == 5 and st["blobNodeCount"] == len(paths)
    assert st["totalBlobSize"] == sum(len(c.encode()) for _, c in s["blobs"])
    assert list(s["summary"]["summary"]["tree"]) == ["rows", "cols", "cells"]


@pytest.mark.parametrize("new_mode", [False, True])
def test_matrix_summary_load_round_trip(new_mode):
    """SharedMatrix.loadCore (matrix.ts:611-634) of summarizeCore's output, mid-stream: the loaded matrix
    continues with the rest of the log to the same summary and cells as the one that never stopped."""
    from helpers import make_matrix_log
    from pyoracle import OracleMatrix
    msgs = make_matrix_log(31 + int(new_mode), 900, n_clients=4, lag=12, new_mode=new_mode)
    a = OracleMatrix(new_length_calc=new_mode)
    a.start_collab("obs")
    half = 500
    for m in msgs[:half]:
        a.apply_msg(m)
    s = a.summarize()
    b = OracleMatrix(new_length_calc=new_mode)
    b.load(s["blobs"], "obs")
    assert b.summarize()["blobs"] == s["blobs"]
    for m in msgs[half:]:
        a.apply_msg(m)
        b.apply_msg(m)
    # the loaded tree is rebuilt 7 segments per block with an empty zamboni heap, so later segment
    # boundaries, handle recycling and so the blobs may differ (tree shape and the zamboni schedule are
    # observable, mergeTree.ts:1816-1829, zamboni.ts:19-60); the matrix as read by position may not
    assert (b.rows.get_length(), b.cols.get_length()) == (a.rows.get_length(), a.cols.get_length())
    nr, nc = a.rows.get_length(), a.cols.get_length()
    assert [b.get_cell(r, c) for r in range(nr) for c in range(nc)] == [a.get_cell(r, c) for r in range(nr) for c in range(nc)]


# ---------------------------------------------------------------- a live client's local ops
@pytest.mark.parametrize("new_mode", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_local_op_farm_converges(seed, new_mode):
    """Local insert / remove / annotate with pending segment groups and acks (mergeTree.ts:1283-1357,
    mergeTreeNodes.ts:439-480, segmentPropertiesManager.ts:60-157): every client, each with its own
    local ops and lag, converges to the observer's text and properties once all ops are acked."""
    from helpers import chars_with_props, run_local_farm
    # verify: every length query cross-checks the block partial lengths against the leaf sum
    clients, obs, log = run_local_farm(seed, n_clients=4, n_rounds=80, new_mode=new_mode, verify=True)
    want = obs.get_text()
    wp = chars_with_props(obs)
    assert len(log) > 100
    for k, c in enumerate(clients):
        assert c.pending_groups() == 0, f"client {k} still has pending ops"
        assert c.get_text() == want, f"client {k} text diverged"
        assert chars_with_props(c) == wp, f"client {k} properties diverged"


def test_state_digest_is_path_independent_and_sensitive():
    """The oracle's state digest (DESIGN.md "State digest") is the same whether the log is replayed by
    the generator or through the record path, and distinguishes documents."""
    from pyloggen import LogBatch, make_cfg
    from pyoracle import OracleDoc
    cfg = make_cfg(seed=77, n_ops=400, n_clients=4)
    lb = LogBatch(cfg, 0, 6)
    props = lb.props_json()
    seen = set()
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        o = OracleDoc()
        if il:
            o.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        o.start_collab("obs")
        for cid in lb.client_ids(i)[1:]:
            o.add_client(cid)
        o.apply_records(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props)
        assert o.digest() == lb.docs[i].digest
        seen.add(o.digest())
    assert len(seen) == lb.n
    a, b = OracleDoc(), OracleDoc()
    a.insert_text_local(0, "abc")
    b.insert_text_local(0, "abd")
    assert a.digest() != b.digest()
