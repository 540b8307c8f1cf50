"""Local rewrite annotates of a live client on the oracle (segmentPropertiesManager.ts:60-157,
pendingRewriteCount): a remote annotate sequenced while the client's own rewrite is pending leaves the
segment alone, so the client converges with everyone else once its rewrite is sequenced.  The engine's
parity on farms with local rewrites is tests/test_gpu_local.py::test_local_rewrite_farm."""
from helpers import run_local_farm


def _msg(cid, seq, ref, msn, op):
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "type": "op", "contents": op}


def _props(doc):
    """The properties of every visible position (segment boundaries differ between clients)."""
    out = []
    for e in doc.map_range():
        seg = e["segment"]
        pr = seg.get("properties") or None  # (key order is not convergent in the reference either)
        out += [sorted(pr.items()) if pr else None] * seg.get("cachedLength", 0)
    return out


def test_pending_local_rewrite_blocks_remote_annotates():
    from pyoracle import OracleDoc
    a, obs = OracleDoc(), OracleDoc()
    for d, cid in ((a, "A"), (obs, "obs")):
        d.insert_text_local(0, "hello")
        d.start_collab(cid)
    rw = a.local_op_json({"combiningOp": {"name": "rewrite"}, "pos1": 0, "pos2": 5, "props": {"x": 1}, "type": 2})
    assert list(rw) == ["combiningOp", "pos1", "pos2", "props", "type"]  # createAnnotateRangeOp's key order
    remote = _msg("B", 1, 0, 0, {"type": 2, "pos1": 0, "pos2": 5, "props": {"y": 2}})
    mine = _msg("A", 2, 0, 0, rw)
    for m in (remote, mine):
        a.apply_msg(m)
        obs.apply_msg(m)
    # the rewrite (sequenced last) leaves only its own keys: {"x": 1} everywhere; without the pending count
    # the live client would have kept "y"
    assert _props(a) == _props(obs) == [[("x", 1)]] * 5


def test_local_rewrite_farms_converge_in_the_new_length_calculation():
    for seed in range(300, 316):
        clients, obs, log = run_local_farm(seed, n_clients=3 + seed % 3, n_rounds=30, new_mode=True, annotate=True,
                                           rewrite=0.6, reconnect=0.25 if seed % 2 else 0.0, verify=True)
        assert any(m["contents"].get("combiningOp") for m in log)
        texts = {c.get_text() for c in clients} | {obs.get_text()}
        assert len(texts) == 1, seed
        props = {str(_props(c)) for c in clients} | {str(_props(obs))}
        assert len(props) == 1, seed
