"""The reference's two-client SharedMatrix conflict KATs (matrix.spec.ts:349-607) on the oracle.

The cases are restated as sequenced op logs in `matrix_kats.py` (the MockContainerRuntimeFactory order) and
replayed by an observer `OracleMatrix`; its `extract()` grid must equal the spec's literal, in both length
modes.  The same logs run on the GPU in `test_gpu_matrix.py::test_reference_conflict_kats_gpu`.
"""
import json

import pytest

from matrix_kats import CASES, case_messages, grid


def oracle_grid(msgs, new_mode):
    from pyoracle import OracleMatrix
    o = OracleMatrix(new_length_calc=new_mode)
    o.start_collab("observer")
    for m in msgs:
        o.apply_msg(m)

    def cell(r, c):
        v = o.get_cell(r, c)
        return None if v is None else json.loads(v)
    return grid(o.rows.get_length(), o.cols.get_length(), cell), o


@pytest.mark.parametrize("new_mode", [False, True])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_reference_conflict_kat(case, new_mode):
    name, line, steps, expected = case
    g, _ = oracle_grid(case_messages(steps), new_mode)
    if expected is not None:
        assert g == expected, f"matrix.spec.ts:{line} {name!r}"


def test_case_messages_shape():
    # "insert col conflict": A's col insert + setCell, then B's, all at refSeq 1 after the first expect()
    msgs = case_messages(CASES[4][2])
    assert [m["sequenceNumber"] for m in msgs] == [1, 2, 3, 4, 5]
    assert [m["referenceSequenceNumber"] for m in msgs] == [0, 1, 1, 1, 1]
    assert [m["minimumSequenceNumber"] for m in msgs] == [0, 1, 1, 1, 1]
    assert msgs[3]["contents"] == {"pos1": 0, "seg": [1, -2147483648], "type": 0, "target": "cols"}
