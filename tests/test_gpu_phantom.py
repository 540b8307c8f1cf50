"""GPU parity of SnapshotV1 loads whose body holds removed segments inserted by collaborating clients: the
reference's phantom partial lengths (tests/phantom_cases.py; mtb_replay.hip "phantom partial lengths").
Bar: the engine equals the oracle -- dump, text, summary -- after the load and after later remote ops:
* the hand-derived known answer (text "h1234567ZY", not the exact-lengths "h1234567YZ");
* constructed summaries with client-inserted segments, removed or not, in header and body chunks;
* synthetic documents of more than 10,000 characters summarized mid-collaboration (SnapshotV1's default
  chunk size, so the removed collaborator-inserted segments past char 10,000 are body segments) and a small
  chunk size, loaded, then the rest of each log replayed."""
import json

import pytest

import phantom_cases as pc
from helpers import first_diff, make_v1_summary, records_to_msgs

pytestmark = pytest.mark.gpu


def _same(B, i, o, what):
    gd, od = B.dump_segments(i), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(i) == o.get_text(), f"{what}: text differs"
    gb, gs = B.summarize_v1(i)
    assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"{what}: SnapshotV1 blobs differ"


def _phantoms(blobs):
    n = 0
    for path, content in blobs[1:]:
        for s in json.loads(content)["segments"]:
            n += isinstance(s, dict) and "client" in s and "removedSeq" in s
    return n


@pytest.mark.parametrize("new_mode", [False, True])
def test_phantom_kat_on_the_engine(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(pc.kat_summary(), "L")
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    B[0].load(pc.kat_summary(), "L")
    B.flush()
    _same(B, 0, o, "after load")
    for m in pc.kat_msgs():
        B[0].applyMsg(m)
        o.apply_msg(m)
    B.flush()
    assert B.text(0) == pc.KAT_TEXT
    _same(B, 0, o, "after the two inserts")


@pytest.mark.parametrize("new_mode", [False, True])
def test_constructed_summaries_with_removed_client_segments_in_the_body(new_mode):
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc
    from test_gpu_load import _remote_tail
    n = 24
    sums = [make_v1_summary(500 + i, 200 + 30 * i, 120, 10, 40, p_removed=0.2, p_client=0.3, client_body=True,
                            client_removed=True) for i in range(n)]
    assert sum(_phantoms(s) for s in sums) > 20
    B = MergeTreeBatch(n, new_length_calc=new_mode)
    oracles = {}
    for i, blobs in enumerate(sums):
        o = OracleDoc(new_length_calc=new_mode)
        try:
            o.load_v1(blobs, "obs")
            o.get_text()
        except Exception as e:  # the reference's "MergeTree insert failed" for body appends outside the view
            assert "MergeTree insert failed" in str(e), str(e)
            continue
        oracles[i] = o
        B[i].load(blobs, "obs")
    assert len(oracles) >= n // 3
    B.flush()
    tails = {}
    for i, o in oracles.items():
        _same(B, i, o, f"constructed summary {i}")
        tails[i] = _remote_tail(o, 11 * i, 150, 40, 10, ["client-0", "client-1", "client-7"])
        for m in tails[i]:
            B[i].applyMsg(m)
    B.flush()
    for i, o in oracles.items():
        _same(B, i, o, f"constructed summary {i} + 150 remote ops")


@pytest.mark.parametrize("new_mode", [False, True])
@pytest.mark.parametrize("chunk", [0, 300])
def test_long_documents_summarized_mid_collaboration(new_mode, chunk):
    """One client inserts past char 9,990 of a long text, every client removes and annotates there
    (tests/helpers.make_tail_log); a SnapshotV1 summary mid-log holds that client's segments removed above the
    MSN in its body.  Each document: the reference's outcome on the oracle -- load fails, a later op fails
    ("MergeTree insert failed": the (refSeq 0, client) view the body is appended in can leave segments out),
    or the whole log applies -- and the engine's must be the same, with equal state before the failing step."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from helpers import make_tail_log
    from pyoracle import OracleDoc
    done_with_phantoms = 0
    for i in range(16):
        text, msgs = make_tail_log(900 + i + 50 * int(new_mode), 1600, lag=24 + 8 * (i % 8), initial_len=9990, lo=9990,
                                   new_mode=new_mode, inserters=[0])
        cut = len(msgs) // 2 + 37 * (i % 8)
        a = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
        a.insert_text_local(0, text)
        a.start_collab("obs")
        for m in msgs[:cut]:
            a.apply_msg(m)
        blobs = [list(x) for x in a.summarize_v1()["blobs"]]
        nph = _phantoms(blobs)
        o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
        B = MergeTreeBatch(1, new_length_calc=new_mode, chunk_size=chunk)
        B[0].load(blobs, "loader")
        try:
            o.load_v1(blobs, "loader")
            o.get_text()
        except Exception as e:
            assert "MergeTree insert failed" in str(e)
            with pytest.raises(MergeTreeError, match="MergeTree insert failed"):
                B.flush()
            continue
        B.flush()
        _same(B, 0, o, f"doc {i} after load")
        failed = False
        for k, m in enumerate(msgs[cut:]):
            try:
                o.apply_msg(m)
            except Exception as e:
                assert "MergeTree insert failed" in str(e)
                B.flush()
                B[0].applyMsg(m)
                with pytest.raises(MergeTreeError, match="MergeTree insert failed"):
                    B.flush()
                failed = True
                break
            B[0].applyMsg(m)
        if failed:
            continue
        B.flush()
        _same(B, 0, o, f"doc {i} after load + tail")
        done_with_phantoms += nph > 0
    assert done_with_phantoms >= 2
