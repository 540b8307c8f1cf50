"""snapshot.spec.ts:15-124 (the reference's only checks of collaborative SnapshotV1 merge info) on the oracle
(CPU) and on the engine (-m gpu, every summary byte-equal to the oracle's), both length modes.  The cases and
the TestString harness are restated in tests/snapshot_spec.py."""
import pytest

import snapshot_spec as sp

MODES = [False, True]
IDS = ["legacy", "new"]


@pytest.mark.parametrize("new_mode", MODES, ids=IDS)
@pytest.mark.parametrize("case", sp.EMPTY_CASES, ids=[c.__name__ for c in sp.EMPTY_CASES])
def test_spec_case_on_the_oracle(case, new_mode):
    sp.run_case(case, lambda init, cid: sp.OracleSide(new_mode, init, cid))


@pytest.mark.parametrize("new_mode", MODES, ids=IDS)
def test_spec_non_empty_initial_state_on_the_oracle(new_mode):
    sp.run_non_empty(lambda init, cid: sp.OracleSide(new_mode, init, cid))


def _engine_equals_oracle(run, new_mode):
    o = run(lambda init, cid: sp.OracleSide(new_mode, init, cid))
    g = run(lambda init, cid: sp.EngineSide(new_mode, init, cid))
    assert len(g.summaries) == len(o.summaries)
    for k, (a, b) in enumerate(zip(g.summaries, o.summaries)):
        assert a == b, f"summary {k} differs"
    assert g.client.text() == o.client.text() and g.client.length() == o.client.length()


@pytest.mark.gpu
@pytest.mark.parametrize("new_mode", MODES, ids=IDS)
@pytest.mark.parametrize("case", sp.EMPTY_CASES, ids=[c.__name__ for c in sp.EMPTY_CASES])
def test_spec_case_on_the_engine(case, new_mode):
    _engine_equals_oracle(lambda mk: sp.run_case(case, mk), new_mode)


@pytest.mark.gpu
@pytest.mark.parametrize("new_mode", MODES, ids=IDS)
def test_spec_non_empty_initial_state_on_the_engine(new_mode):
    _engine_equals_oracle(sp.run_non_empty, new_mode)
