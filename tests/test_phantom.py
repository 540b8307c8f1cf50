"""Phantom partial lengths after a SnapshotV1 load (tests/phantom_cases.py), on the oracle: the hand-derived
known answer, in both length-calculation modes."""
import json

import pytest

import phantom_cases as pc


@pytest.mark.parametrize("new_mode", [False, True])
def test_phantom_kat_on_the_oracle(new_mode):
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(pc.kat_summary(), "L")
    assert o.get_text() == "h1234567"
    rows = [json.loads(r) for r in o.dump_segments().splitlines()[1:]]
    # root [ L1 [h 1 2 3], L2 [4 5 6 7 pp], L3 [a b c d] ]
    assert [(r[0], r[2]) for r in rows] == [([0, 0], "h"), ([0, 1], "1"), ([0, 2], "2"), ([0, 3], "3"),
                                           ([1, 0], "4"), ([1, 1], "5"), ([1, 2], "6"), ([1, 3], "7"),
                                           ([1, 4], "pp"), ([2, 0], "a"), ([2, 1], "b"), ([2, 2], "c"), ([2, 3], "d")]
    for m in pc.kat_msgs():
        o.apply_msg(m)
    assert o.get_text() == pc.KAT_TEXT != pc.EXACT_TEXT
    assert [r[2] for r in (json.loads(x) for x in o.dump_segments().splitlines()[1:])][9:] == \
        ["a", "Z", "b", "Y", "c", "d"]


@pytest.mark.parametrize("new_mode", [False, True])
def test_deficit_kat_on_the_oracle(new_mode):
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(pc.def_summary(), "L")
    assert o.get_text() == "h1234567ABCDEF"
    assert o.stale_deficits() == 1
    rows = [json.loads(r) for r in o.dump_segments().splitlines()[1:]]
    # root [ L1 [h 1 2 3], L2 [4 5 6 7 AB CD EF], L3 [a b c d] ]
    assert [(r[0], r[2]) for r in rows] == [([0, 0], "h"), ([0, 1], "1"), ([0, 2], "2"), ([0, 3], "3"),
                                           ([1, 0], "4"), ([1, 1], "5"), ([1, 2], "6"), ([1, 3], "7"),
                                           ([1, 4], "AB"), ([1, 5], "CD"), ([1, 6], "EF"),
                                           ([2, 0], "a"), ([2, 1], "b"), ([2, 2], "c"), ([2, 3], "d")]
    msgs = pc.def_msgs()
    o.apply_msg(msgs[0])
    assert o.get_text() == "h1234567ABCDEFY"  # the client term: Y passes L2
    o.apply_msg(msgs[1])
    assert o.get_text() == pc.DEF_TEXT != pc.DEF_EXACT_TEXT
    assert [r[2] for r in (json.loads(x) for x in o.dump_segments().splitlines()[1:])][11:] == \
        ["a", "Z", "Y", "b", "c", "d"]


_DEFCHECK = r"""
import sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
from test_gpu_phantom import _rising_tail, _tail_summary
from pyoracle import OracleDoc
n = d = 0
for new_mode in (False, True):
    for k in range(0, 300, 2):
        blobs = _tail_summary(7000 + k, 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7)
        o = OracleDoc(new_length_calc=new_mode)
        try:
            o.load_v1(blobs, "loader")
            d += o.stale_deficits() > 0
            _rising_tail(o, k, 60, 40)
        except Exception as e:
            assert "deficit model" not in str(e), str(e)
            continue
        n += 1
print(n, d)
"""


def test_deficit_model_restated_on_the_oracle():
    """The engine's deficit model (DESIGN.md section 7 "Deficits": main-set deficits from t1, client-set deficits
    below t1c, moved when their first entry is recomputed, copied down into minLength, kept by recombination only
    once copied down) checked against the oracle's own partial-length sets after every update, copyDown and
    combine (MTO_DEFCHECK: the shortfall of every entry and of minLength equals the model's), over small
    constructed summaries loaded and continued with a rising MSN, both length modes."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MTO_DEFCHECK="1")
    r = subprocess.run([sys.executable, "-c", _DEFCHECK, here, os.path.join(os.path.dirname(here), "oracle")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    n, d = map(int, r.stdout.split())
    assert n >= 200 and d >= 100
