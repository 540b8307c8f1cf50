"""mtb_summarize_v1_many when the device extraction must refuse a document's tree: the count pass
of mtb_extract_v1_kernel reports MTB_NONE for it and the host gives it no room in the outputs, so the emit pass
must write nothing for it -- the next document's output (or the end of the buffers, for the last document)
would take the writes.  The tree is broken with a test hook (include/mtb_testing.h): valid input never makes one."""
import ctypes

import pytest

from helpers import ROOT  # noqa: F401  (sys.path)

pytestmark = pytest.mark.gpu


def _batch(n=4, ops=600):
    from fluidframework_amd import MergeTreeBatch
    from pyloggen import LogBatch, make_cfg
    lb = LogBatch(make_cfg(seed=11, n_ops=ops, n_clients=4), 0, n)
    B = MergeTreeBatch(n)
    for p in lb.props_json()[1:]:
        B.intern_props(p)
    for i in range(n):
        tb = lb.doc_text_bytes(i)
        B.init_doc(i, tb[: lb.docs[i].initial_len * 2].decode("utf-16-le"), "obs")
        for cid in lb.client_ids(i)[1:]:
            B.add_client(i, cid)
        B.append_records(i, lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb)
    assert B.replay()["errors"] == 0
    return B, lb


def _set_root_child(B, doc, value):
    L = B._L
    L.mtb_test_set_root_child.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint32)]
    old = ctypes.c_uint32()
    assert L.mtb_test_set_root_child(B._h, doc, value, ctypes.byref(old)) == 0
    return old.value


@pytest.mark.parametrize("bad_doc", [1, 3])  # a middle document, and the last one (its writes would run off the end)
@pytest.mark.parametrize("kind", ["out_of_slice", "cycle"])
def test_refused_tree_does_not_touch_other_summaries(bad_doc, kind):
    from fluidframework_amd import MergeTreeError
    B, lb = _batch()
    want = B.summarize_v1_many(list(range(4)), threads=2, fingerprints=True)
    assert all(want[i] == lb.docs[i].summary_fnv for i in range(4))
    # a huge id points outside the slice; 0xFFFFFFFE asks the hook for the root's own id (a cycle)
    old = _set_root_child(B, bad_doc, 0x7FFFFFF0 if kind == "out_of_slice" else 0xFFFFFFFE)
    assert not (old & 0x80000000), "the root must hold block children (a two-level tree)"
    with pytest.raises(MergeTreeError, match=f"document {bad_doc}: corrupt tree"):
        B.summarize_v1_many(list(range(4)), threads=2, fingerprints=True)
    others = [i for i in range(4) if i != bad_doc]
    got = B.summarize_v1_many(others, threads=2, fingerprints=True)
    assert [got[k] for k in range(len(others))] == [want[i] for i in others]
    _set_root_child(B, bad_doc, old)
    assert B.summarize_v1_many(list(range(4)), threads=2, fingerprints=True) == want
