"""Shared helpers for the parity tests (test infrastructure)."""
import glob
import gzip
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def replay_fixtures():
    """The 30 reference conflict-farm replay logs (compact form, tests/golden/replay)."""
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "replay", "*.json.gz"))):
        with gzip.open(f, "rt") as fh:
            out.append((os.path.basename(f).replace(".json.gz", ""), json.load(fh)))
    return out


def snapshot_fixture(name, version="v1"):
    with gzip.open(os.path.join(GOLDEN, f"snapshots_{version}", f"{name}.json.gz"), "rt") as fh:
        return json.load(fh)["blobs"]


def msg_from_compact(m):
    cid, seq, ref, msn, contents = m
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def first_diff(a, b):
    la, lb = a.splitlines(), b.splitlines()
    for i, (x, y) in enumerate(zip(la, lb)):
        if x != y:
            return f"line {i}:\n  gpu   : {x[:300]}\n  oracle: {y[:300]}"
    return f"length differs: {len(la)} vs {len(lb)} lines"


def records_to_msgs(ops_bytes, n, text_bytes, props_json, long_ids):
    """Turn packed 32-byte records (mtb_op layout) back into ISequencedDocumentMessages: records sharing a
    seq up to the one flagged LAST form one message (a GROUP op when there are several)."""
    import struct
    text = text_bytes.decode("utf-16-le", "surrogatepass")
    msgs, cur = [], []
    for k in range(n):
        t, fl, c, seq, ref, msn, p1, p2, pay, pr = struct.unpack_from("<BBHIIIIIII", ops_bytes, 32 * k)
        if t == 0:
            if fl & 0x02:
                seg = {"marker": {"refType": p2} if p2 != 0xFFFFFFFF else {}}
                if pr:
                    seg["props"] = json.loads(props_json[pr])
            else:
                seg = text[pay:pay + p2]
                if pr or fl & 0x08:
                    seg = {"text": seg}
                    if pr:
                        seg["props"] = json.loads(props_json[pr])
            op = {"type": 0, "pos1": p1, "seg": seg}
        elif t in (1, 2):
            op = {"type": t, "pos1": p1, "pos2": p2}
            if t == 2:
                op["props"] = json.loads(props_json[pr])
                if fl & 0x04:
                    op["combiningOp"] = {"name": "rewrite"}
        else:
            raise ValueError(f"record type {t} has no message form here")
        cur.append(op)
        if fl & 0x01:
            contents = cur[0] if len(cur) == 1 else {"type": 3, "ops": cur}
            msgs.append({"clientId": long_ids[c], "sequenceNumber": seq, "referenceSequenceNumber": ref,
                         "minimumSequenceNumber": msn, "type": "op", "contents": contents})
            cur = []
    assert not cur, "trailing records without a LAST flag"
    return msgs


def make_v1_summary(seed, n_segments, chunk_len, msn, seq, n_clients=4, p_removed=0.25, p_client=0.0,
                    client_body=False, client_removed=False, inserters=None):
    """A constructed SnapshotV1 summary (snapshotV1.ts layout) for load tests: text / marker / props
    segments; NonCollab segments removed above the MSN by 1-3 clients; optionally segments inserted above
    the MSN by clients (header only unless `client_body`).  Returns [(path, content), ...]."""
    import random
    rng = random.Random(seed)
    clients = [f"client-{k}" for k in range(n_clients)]
    segs = []
    for i in range(n_segments):
        r = rng.random()
        if r < 0.1:
            spec = {"marker": {"refType": rng.choice([0, 1, 2])}, "props": {"markerId": f"m{i}"}}
            ln = 1
        else:
            t = "".join(rng.choice("abcdefgh \n") for _ in range(rng.randint(1, 12)))
            spec = t if r < 0.75 else {"text": t, "props": rng.choice([{"bold": True}, {"color": "red"}, {"bold": True, "k": 1}])}
            ln = len(t)
        segs.append([spec, ln])
    out = []
    for i, (spec, ln) in enumerate(segs):
        u = rng.random()
        if u < p_removed:
            rs = rng.randint(msn + 1, seq)
            rcs = rng.sample(clients, rng.randint(1, 3))
            out.append(({"json": spec, "removedSeq": rs, "removedClientIds": rcs}, ln))
        elif u < p_removed + p_client:
            s = rng.randint(msn + 1, seq)
            m = {"json": spec, "client": rng.choice(clients if inserters is None else [clients[k] for k in inserters]),
                 "seq": s}
            if client_removed and rng.random() < 0.3 and s < seq:
                m["removedSeq"] = rng.randint(s + 1, seq)
                m["removedClientIds"] = [rng.choice(clients)]
            out.append((m, ln))
        else:
            out.append((spec, ln))
    chunks, cur, cur_len = [], [], 0
    for spec, ln in out:
        cur.append(spec)
        cur_len += ln
        if cur_len >= chunk_len:
            chunks.append(cur)
            cur, cur_len = [], 0
    if cur or not chunks:
        chunks.append(cur)
    if not client_body:  # keep client-inserted segments in the header chunk
        for c in chunks[1:]:
            for k, spec in enumerate(c):
                if isinstance(spec, dict) and "client" in spec:
                    c[k] = spec["json"]
    ids = ["header"] + [f"body_{k}" for k in range(len(chunks) - 1)]
    blobs = []
    start = 0
    for k, c in enumerate(chunks):
        o = {"version": "1", "segmentCount": len(c), "length": 0, "segments": c, "startIndex": start}
        if k == 0:
            o["headerMetadata"] = {"minSequenceNumber": msn, "sequenceNumber": seq,
                                   "orderedChunkMetadata": [{"id": x} for x in ids],
                                   "totalLength": 0, "totalSegmentCount": len(out)}
        start += len(c)
        blobs.append([ids[k], json.dumps(o, separators=(",", ":"))])
    return blobs


UNALLOCATED = -2147483648  # Handle.unallocated (matrix/src/handletable.ts:11)


def make_matrix_log(seed, n_msgs, n_clients=4, lag=16, p_set=0.45, max_count=8, new_mode=False, start=None):
    """A SharedMatrix op stream (matrix.ts message shapes) valid in each author's (refSeq, client) view:
    row/col inserts and removes of 1..max_count, and setCell at a row/col inside the author's view.
    Generated by driving the oracle as the observer; returns the messages.  start=(oracle, seq0): continue
    from that observer's state (e.g. a loaded summary) with every client caught up at seq0."""
    import random
    from pyoracle import OracleMatrix
    rng = random.Random(seed)
    if start is None:
        m = OracleMatrix(new_length_calc=new_mode)
        m.start_collab("obs")
        seq0 = 0
    else:
        m, seq0 = start
    clients = [f"w{k}" for k in range(n_clients)]
    ref = {c: seq0 for c in clients}
    msgs, seq = [], seq0

    def vlen(doc, w, r):
        doc.add_client(w)
        return doc.remote_length(r, doc.client_ids().index(w))

    for _ in range(n_msgs):
        w = rng.choice(clients)
        ref[w] = max(ref[w], seq - rng.randint(0, lag))
        r = ref[w]
        seq += 1
        rl, cl = vlen(m.rows, w, r), vlen(m.cols, w, r)
        if rng.random() < p_set and rl > 0 and cl > 0:
            contents = {"type": 2, "row": rng.randrange(rl), "col": rng.randrange(cl), "value": rng.randint(0, 99)}
        else:
            target = rng.choice(["rows", "cols"])
            ln = rl if target == "rows" else cl
            if ln == 0 or rng.random() < 0.6:
                contents = {"type": 0, "pos1": rng.randint(0, ln), "seg": [rng.randint(1, max_count), UNALLOCATED],
                            "target": target}
            else:
                p1 = rng.randrange(ln)
                contents = {"type": 1, "pos1": p1, "pos2": min(ln, p1 + rng.randint(1, max_count)), "target": target}
        msg = {"clientId": w, "sequenceNumber": seq, "referenceSequenceNumber": r,
               "minimumSequenceNumber": min(ref.values()), "type": "op", "contents": contents}
        m.apply_msg(msg)
        msgs.append(msg)
    return msgs


def run_local_farm(seed, n_clients=4, n_rounds=60, new_mode=False, annotate=True, initial="hello world", verify=False,
                   record=None, reconnect=0.0, rewrite=0.0, marker_ids=0, incr=0.0, summary=None):
    """A conflict farm in the style of the reference's (client.conflictFarm.spec.ts with TestClientLogger):
    `n_clients` live clients make local ops against their own view, a sequencer orders them (refSeq = the
    client's currentSeq at submission, MSN = the lowest refSeq any client can still send), and every client
    receives the sequenced stream with its own lag (its own ops come back as acks).  An observer receives
    everything.  With `reconnect` > 0 a client disconnects (probability per round) in the style of
    client.reconnectFarm.spec.ts: its ops still in the sequencer's queue are dropped, it catches up on the
    sequenced stream, then regenerates each dropped op (Client.regeneratePendingOp, client.ts:917-960) and
    resubmits the result at its current seq.  With `rewrite` > 0 that fraction of the local annotates are
    `rewrite` annotates (combiningOp {"name": "rewrite"}: pendingRewriteCount, segmentPropertiesManager.ts).
    With `marker_ids` > 0 clients also insert markers whose `markerId` comes from a pool of that many (ids are
    reused, so blockUpdate's re-mapping decides what an id names, mergeTree.ts:2392 -> :296-306) and send
    marker-relative inserts and annotateMarker ops (relativePos1 {id, before}, relativePos2 {id}) for ids
    their own view resolves.  With `incr` > 0 that fraction of the local annotates are combiningOp "incr"
    annotates (their numeric keys become NaN; a remote incr modifies pending keys too, shouldModifyKey).
    With `summary` (SnapshotV1 blobs) every client and the observer start by loading it (Client.load with their
    own ids) instead of from `initial`, and the sequence numbers continue from the summary's.
    Returns (clients, observer, sequenced messages)."""
    import random
    from pyoracle import OracleDoc, OracleError
    rng = random.Random(seed)
    ids = [f"c{k}" for k in range(n_clients)]
    clients = []
    seq0 = 0
    if summary is not None:
        import json as _json
        seq0 = _json.loads(summary[0][1])["headerMetadata"]["sequenceNumber"]

    def start(o, cid):
        if summary is not None:
            o.load_v1(summary, cid)
        else:
            o.insert_text_local(0, initial)
            o.start_collab(cid)
    for cid in ids:
        o = OracleDoc(new_length_calc=new_mode, verify=verify)
        start(o, cid)
        clients.append(o)
    obs = OracleDoc(new_length_calc=new_mode, verify=verify)
    start(obs, "obs")
    queue, log, seen = [], [], [0] * n_clients
    words = ["a", "bc", "def", "\n", "xyz" * 3, "\U0001F600"]

    def local_op(c):
        n = c.get_length()
        r = rng.random()
        if marker_ids:
            mid = f"d{rng.randrange(marker_ids)}"
            if r < 0.12:
                return c.insert_local_op(rng.randint(0, n), {"marker": {"refType": 1}, "props": {"markerId": mid}})
            if r < 0.26 and n > 0:
                p = c.pos_from_relative({"id": mid, "before": True}, c.current_seq, 0)
                if 0 <= p < n:
                    if rng.random() < 0.5:
                        return c.local_op_json({"type": 0, "relativePos1": {"id": mid, "before": True},
                                                "seg": rng.choice(words)})
                    return c.local_op_json({"type": 2, "relativePos1": {"id": mid, "before": True},
                                            "relativePos2": {"id": mid}, "props": {"seen": rng.randint(0, 3)}})
            r = rng.random()
        if n == 0 or r < 0.5:
            t = rng.choice(words)
            seg = {"text": t, "props": {"k": rng.randint(0, 2)}} if rng.random() < 0.2 else t
            return c.insert_local_op(rng.randint(0, n), seg)
        a = rng.randrange(n)
        b = min(n, a + rng.randint(1, 6))
        if not annotate or r < 0.8:
            return c.remove_local_op(a, b)
        props = {"k": rng.choice([1, 2, None]), "w": rng.randint(0, 1)}
        if incr and rng.random() < incr:  # combiningOp incr: the numeric keys become NaN (properties.ts:24-69)
            return c.local_op_json({"combiningOp": {"name": "incr"}, "pos1": a, "pos2": b, "props": props, "type": 2})
        if rewrite and rng.random() < rewrite:
            return c.local_op_json({"combiningOp": {"name": "rewrite"}, "pos1": a, "pos2": b, "props": props, "type": 2})
        return c.annotate_local_op(a, b, props)

    def sequence(m):
        cid, ref, op = queue.pop(0)
        msn = min([c.current_seq for c in clients] + [q[1] for q in queue] + [ref])
        msg = {"clientId": cid, "sequenceNumber": seq0 + len(log) + 1, "referenceSequenceNumber": ref,
               "minimumSequenceNumber": msn, "type": "op", "contents": op}
        log.append(msg)

    def deliver(k, upto):
        while seen[k] < upto:
            clients[k].apply_msg(log[seen[k]])
            seen[k] += 1

    # record (a dict): per round, each client's events ("local", op) / ("msg", msg) and then its state
    # (digest, text), for replaying the same farm on the engine
    rounds = record.setdefault("rounds", []) if record is not None else None
    if record is not None:
        record["ids"] = ids
        _deliver = deliver

        def deliver(k, upto):  # noqa: F811
            while seen[k] < upto:
                rounds[-1][k].append(("msg", log[seen[k]]))
                _deliver(k, seen[k] + 1)

    def end_round():
        if rounds is not None:
            rounds[-1] = [(ev, clients[k].digest(), clients[k].get_text()) for k, ev in enumerate(rounds[-1])]

    try:
        _farm_rounds(n_rounds, rounds, reconnect, rng, queue, ids, clients, deliver, n_clients, local_op, sequence,
                     end_round, log, seen)
    except OracleError:
        # reused marker ids: clients' idToSegment maps diverge (the reference's own behaviour), so a later op
        # can be invalid on a receiver; the farm ends at the last complete round
        if not marker_ids:
            raise
        if rounds is not None:
            rounds.pop()
            record["stopped"] = True
        obs_log = []
        for m in log:
            try:
                obs.apply_msg(m)
            except OracleError:
                break
            obs_log.append(m)
        if record is not None:
            record["obs_log"] = obs_log
        return clients, obs, log
    for m in log:
        obs.apply_msg(m)
    if record is not None:
        record["obs_log"] = log
    return clients, obs, log


def _farm_rounds(n_rounds, rounds, reconnect, rng, queue, ids, clients, deliver, n_clients, local_op, sequence,
                 end_round, log, seen):
    for _ in range(n_rounds):
        if rounds is not None:
            rounds.append([[] for _ in range(n_clients)])
        if reconnect and rng.random() < reconnect:
            k = rng.randrange(n_clients)
            dropped = [q for q in queue if q[0] == ids[k]]
            queue[:] = [q for q in queue if q[0] != ids[k]]
            deliver(k, len(log))
            n_groups = sum(len(op["ops"]) if op.get("type") == 3 else 1 for (_, _, op) in dropped)
            assert clients[k].pending_groups() == n_groups, (clients[k].pending_groups(), n_groups)
            for (_, _, op) in dropped:
                new = clients[k].regenerate_pending_op(op)
                if rounds is not None:
                    rounds[-1][k].append(("regen", (op, new)))
                queue.append((ids[k], clients[k].current_seq, new))
        for k in rng.sample(range(n_clients), rng.randint(1, n_clients)):
            for _ in range(rng.randint(1, 3)):
                ref = clients[k].current_seq
                op = local_op(clients[k])
                if op is not None:
                    queue.append((ids[k], ref, op))
                    if rounds is not None:
                        rounds[-1][k].append(("local", op))
        for _ in range(rng.randint(0, len(queue))):
            sequence(None)
        for k in range(n_clients):
            deliver(k, seen[k] + rng.randint(0, len(log) - seen[k]))
        end_round()
    if rounds is not None:
        rounds.append([[] for _ in range(n_clients)])
    while queue:
        sequence(None)
    for k in range(n_clients):
        deliver(k, len(log))
    end_round()


def _doover(lo, hi, grow):
    """doOverRange (mergeTreeOperationRunner.ts:90-107): lo, grow(lo), ... up to hi; a non-growing step +1."""
    v, last = lo, None
    while v <= hi:
        if v == last:
            v += 1
        last = v
        yield v
        v = grow(v)


REF_CLIENT_NAMES = [chr(ord("A") + i) for i in range(26)] + [chr(ord("a") + i) for i in range(26)]


def run_ref_reconnect_farm(seed, n_clients, ops_range=(40, 320), rounds=3, record=None):
    """The reference's own reconnect farm shape (client.reconnectFarm.spec.ts:25-121 over
    mergeTreeOperationRunner.ts:200-307, new length calculations), on oracle clients: `n_clients` clients
    start empty; per round `ops` local ops (ops doubling over `ops_range`, `rounds` rounds each) are made by
    clients 1.. against the round-start view (insert while shorter than 16, else annotate / remove / insert
    of the client's name); client 1 (and, on a coin flip with more than two clients, client 2) has its ops of
    the round held back, catches up on everyone else's, and resubmits regeneratePendingOp's result at its
    current seq.  After every round all clients' characters and per-character properties must agree
    (TestClientLogger.validate) -- an AssertionError names the round otherwise.  `record` (a dict) gets the
    same per-round event format as run_local_farm's.  Returns the clients."""
    return run_ref_farm(seed, n_clients, 16, ops_range, rounds, True, record)


def run_ref_conflict_farm(seed, n_clients, min_length, ops_range=(1, 128), rounds=8, record=None):
    """The reference's conflict farm shape (client.conflictFarm.spec.ts, defaultOptions: ops per round
    1..128 doubling, 8 rounds each, clients made from one snapshot, everyone in lock step): inserts while
    the document is shorter than `min_length`, then remove / annotate / insert-at-a-segment-start
    (insertAtRefPos, mergeTreeOperationRunner.ts:32-69, places text at an existing segment's position; here
    at the start of a visible segment of the client's view, since local references are outside the path)."""
    return run_ref_farm(seed, n_clients, min_length, ops_range, rounds, False, record)


def run_ref_farm(seed, n_clients, min_length, ops_range, rounds, reconnect, record=None):
    import random
    from pyoracle import OracleDoc
    rng = random.Random(seed * 1000 + n_clients * 10 + (0 if reconnect else min_length))
    names = REF_CLIENT_NAMES[:n_clients]
    clients = []
    for cid in names:
        c = OracleDoc(new_length_calc=True)
        c.start_collab(cid)
        clients.append(c)
    log_rounds = record.setdefault("rounds", []) if record is not None else None
    if record is not None:
        record["ids"] = names
    seq = 0

    def send(cid, ref, msn, op):
        nonlocal seq
        seq += 1
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
             "minimumSequenceNumber": msn, "type": "op", "contents": op}
        for k, c in enumerate(clients):
            c.apply_msg(m)
            if log_rounds is not None:
                log_rounds[-1][k].append(("msg", m))

    def segment_start(c, a):
        """the start of the visible segment holding position a of c's view"""
        pos = 0
        for e in c.map_range():
            n = len(e["segment"].get("text", "x").encode("utf-16-le", "surrogatepass")) // 2
            if pos + n > a:
                return pos
            pos += n
        return pos

    for n_ops in _doover(ops_range[0], ops_range[1], lambda x: x * 2):
        for rnd in range(rounds):
            if log_rounds is not None:
                log_rounds.append([[] for _ in clients])
            msn, msgs = seq, []
            for _ in range(n_ops):
                k = rng.randint(1, n_clients - 1)
                c = clients[k]
                n = c.get_length()
                name = names[k] * rng.randint(1, 3)
                if n == 0 or n < min_length:
                    op = c.insert_local_op(rng.randint(0, n), name)
                else:
                    which, a = rng.randint(0, 2), rng.randint(0, n - 1)
                    b = rng.randint(a + 1, n)
                    if which == 0:
                        op = c.annotate_local_op(a, b, {"client": names[k]})
                    elif which == 1:
                        op = c.remove_local_op(a, b)
                    elif reconnect:
                        op = c.insert_local_op(rng.randint(0, n), name)
                    else:
                        op = c.insert_local_op(segment_start(c, a), name)
                msgs.append((k, c.current_seq, op))
                if log_rounds is not None:
                    log_rounds[-1][k].append(("local", op))
            recon = ([1, 2] if n_clients > 2 and rng.random() < 0.5 else [1]) if reconnect else []
            held = []
            for k, ref, op in msgs:
                if k in recon:
                    held.append((k, op))
                else:
                    send(names[k], ref, msn, op)
            again = []
            for k, op in held:
                new = clients[k].regenerate_pending_op(op)
                if log_rounds is not None:
                    log_rounds[-1][k].append(("regen", (op, new)))
                again.append((k, clients[k].current_seq, new))
            for k, ref, op in again:
                send(names[k], ref, msn, op)
            base = chars_with_props(clients[0])
            for k, c in enumerate(clients[1:], 1):
                assert chars_with_props(c) == base, f"seed {seed}: {n_ops} ops/round, round {rnd}, client {k}"
            if log_rounds is not None:
                log_rounds[-1] = [(ev, clients[k].digest(), clients[k].get_text())
                                  for k, ev in enumerate(log_rounds[-1])]
    return clients


def chars_with_props(doc):
    """(character, properties) per visible character of a document's local view (TestClientLogger.validate
    compares text and the properties at every position)."""
    out = []
    for e in doc.map_range():
        s = e["segment"]
        t = s.get("text", "￼").encode("utf-16-le", "surrogatepass")  # per UTF-16 code unit (a split may cut a pair)
        p = json.dumps(s.get("properties"), sort_keys=True)
        out.extend((t[i:i + 2], p) for i in range(0, len(t), 2))
    return out


def load_logbatch(B, lb, docs=None, props_interned=False):
    """Queue generated logs (oracle/loggen.cpp) into engine batch B: document j of B gets log docs[j]
    (default: log j).  The props table is interned first so its ids follow the generator's table."""
    docs = list(range(lb.n)) if docs is None else list(docs)
    if not props_interned:
        props = lb.props_json()
        ids = [B.intern_props(p) if p else 0 for p in props]
        assert ids == list(range(len(props))), "props ids must follow the generator table"
    for j, u in enumerate(docs):
        tb = lb.doc_text_bytes(u)
        il = lb.docs[u].initial_len
        B.init_doc(j, tb[: il * 2].decode("utf-16-le"), "obs")
        for cid in lb.client_ids(u)[1:]:
            B.add_client(j, cid)
        # payload offsets in the generated records index the doc's text arena (initial text first)
        B.append_records(j, lb.doc_ops_bytes(u), lb.docs[u].n_ops, tb)
    return docs


def _marker_ids_ok(gen, a, b, R, cid, mid):
    """Every marker in [a, b) of the (R, cid) view carries markerId `mid` (annotateRange's assert 0x5ad)."""
    for e in gen.map_range(a, b, R, cid):
        seg = e["segment"]
        if seg.get("type") == "Marker" and (seg.get("properties") or {}).get("markerId") != mid:
            return False
    return True


def make_marker_log(seed, n_msgs, n_clients=4, lag=24, new_mode=False, initial="hello marker world", p_rel=0.5,
                    dup_ids=0):
    """A sequenced op log with markers carrying unique `markerId`s and ops whose positions are marker-relative
    (IRelativePosition, ops.ts:77-92): `annotateMarker` ops (opBuilder.ts:25-43, {id, before: true} ..
    {id}) and inserts / removes / annotates with relativePos1/2 (before / offset), next to plain ones.  A
    generator oracle (every message applied as it is made) resolves each candidate relative position in the
    sender's (refSeq, client) view (posFromRelativePos) so that only in-range ops are emitted; markers that
    were removed, or unlinked by zamboni, stay eligible.  With `dup_ids` > 0 marker ids come from a pool of
    that many (so ids are reused and blockUpdate's re-mapping decides what they name), annotates may name
    markerId (the marker's own id, as assert 0x5ad requires; text ranges any id) and rewrite annotates drop
    markers' ids.  Returns (initial text, messages)."""
    import random
    from pyoracle import OracleDoc
    rng = random.Random(seed)
    ids = [f"client-{k}" for k in range(n_clients)]
    gen = OracleDoc(new_length_calc=new_mode)
    if initial:
        gen.insert_text_local(0, initial)
    gen.start_collab("gen-observer")
    short = {}
    for cid in ids:
        gen.add_client(cid)
        short[cid] = len(short) + 1
    ref = [0] * n_clients
    markers, msgs = [], []
    words = ["ab", "c", "xyz", "\n", "long-ish text "]

    def rel(pos_ok):
        for _ in range(4):
            if not markers:
                return None
            r = {"id": rng.choice(markers)}
            if rng.random() < 0.5:
                r["before"] = True
            if rng.random() < 0.4:
                r["offset"] = rng.randint(0, 3)
            return r
        return None

    for seq in range(1, n_msgs + 1):
        k = rng.randrange(n_clients)
        ref[k] = max(ref[k], seq - 1 - rng.randint(0, lag))
        R, C, cid = ref[k], short[ids[k]], ids[k]
        n = gen.remote_length(R, C)
        x = rng.random()
        op = None
        if x < 0.12 or n == 0:
            mid = f"d{rng.randrange(dup_ids)}" if dup_ids else f"m{seed}-{seq}"
            p = rng.randint(0, n)
            op = {"type": 0, "pos1": p, "seg": {"marker": {"refType": rng.choice([0, 1, 2])},
                                                 "props": {"markerId": mid, "kind": rng.randint(0, 2)}}}
            markers.append(mid)
        elif x < 0.25 and markers:  # annotateMarker
            mid = rng.choice(markers)
            p = gen.pos_from_relative({"id": mid, "before": True}, R, C)
            if 0 <= p and p + 1 <= n:
                op = {"type": 2, "relativePos1": {"id": mid, "before": True}, "relativePos2": {"id": mid},
                      "props": {"state": rng.choice(["open", "closed", None])}}
                if dup_ids and rng.random() < 0.5 and _marker_ids_ok(gen, p, p + 1, R, cid, mid):
                    op["props"]["markerId"] = mid  # the marker's own id: no assert
        elif dup_ids and x < 0.31 and n > 0:  # rewrite (drops markerId) or a markerId annotate over text
            a = rng.randrange(n)
            b = min(n, a + rng.randint(1, 4))
            if rng.random() < 0.5:
                op = {"type": 2, "pos1": a, "pos2": b, "props": {"state": "rw"}, "combiningOp": {"name": "rewrite"}}
            elif _marker_ids_ok(gen, a, b, R, cid, "t"):
                op = {"type": 2, "pos1": a, "pos2": b, "props": {"markerId": "t"}}
        if op is None:
            t = rng.choice([0, 0, 1, 2])
            if t == 0:
                op = {"type": 0, "seg": rng.choice(words)}
                r = rel(True) if rng.random() < p_rel else None
                p = gen.pos_from_relative(r, R, C) if r else -1
                if r and 0 <= p <= n:
                    op["relativePos1"] = r
                else:
                    op["pos1"] = rng.randint(0, n)
            elif n > 0:
                a = rng.randrange(n)
                b = min(n, a + rng.randint(1, 5))
                op = {"type": t}
                for key, val in (("1", a), ("2", b)):
                    r = rel(True) if rng.random() < p_rel else None
                    p = gen.pos_from_relative(r, R, C) if r else -1
                    if r and 0 <= p <= n and (key == "1" and p < b or key == "2" and p > op.get("_a", a)):
                        op["relativePos" + key] = r
                        if key == "1":
                            op["_a"] = p
                    else:
                        op["pos" + key] = val
                        if key == "1":
                            op["_a"] = val
                op.pop("_a")
                if t == 2:
                    op["props"] = {"client": cid, "n": rng.randint(0, 3)}
            else:
                op = {"type": 0, "pos1": 0, "seg": "seed"}
        msn = min(ref)
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": R, "minimumSequenceNumber": msn,
             "type": "op", "contents": op}
        gen.apply_msg(m)
        msgs.append(m)
    gen.close()
    return initial, msgs


def make_incr_log(seed, n_msgs, n_clients=4, lag=16, new_mode=False, initial="hello incr world", p_incr=0.15,
                  p_rewrite=0.0, string_incr=False, object_incr=False, objs=None, incr_objects=True):
    """A sequenced op log whose annotates are partly combiningOp "incr" annotates (segmentPropertiesManager.ts:
    145-147 -> combine(op, previous, undefined) of properties.ts:24-69): numeric keys "n" / "m" (incr makes
    them NaN, JSON null, never matchProperties-equal), a string key "s" that incr never names, null deletes,
    some incr ops with a numeric defaultValue / minValue; inserts with props, removes.  With `p_rewrite` that
    fraction of the annotates are combiningOp "rewrite" annotates (falsy values -- 0, "", null -- delete or
    re-append keys, :107-154).  Every message is applied to a generator oracle as it is made.  Returns
    (initial text, messages).  With `string_incr` incr annotates also name the string key "s" (string
    concatenation: s + "undefined", then a string minValue when larger) and take string defaultValues.  With
    `object_incr` a key "o" holds object / array values (inserted and annotated) that incr annotates name too
    (String(value) + "undefined"), with object / array defaultValues and minValues."""
    import random
    from pyoracle import OracleDoc
    rng = random.Random(seed)
    ids = [f"client-{k}" for k in range(n_clients)]
    gen = OracleDoc(new_length_calc=new_mode)
    if initial:
        gen.insert_text_local(0, initial)
    gen.start_collab("gen-observer")
    short = {}
    for cid in ids:
        gen.add_client(cid)
        short[cid] = len(short) + 1
    ref = [0] * n_clients
    msgs = []
    words = ["ab", "c", "xyz", "\n", "more text "]
    if objs is None:
        objs = [{"x": 1}, [1, 2], [], [None, "q", [3, [4]]], {"y": [1]}, ["[object Object]"]]
    for seq in range(1, n_msgs + 1):
        k = rng.randrange(n_clients)
        ref[k] = max(ref[k], seq - 1 - rng.randint(0, lag))
        R, C, cid = ref[k], short[ids[k]], ids[k]
        n = gen.remote_length(R, C)
        x = rng.random()
        if x < 0.4 or n == 0:
            seg = rng.choice(words)
            if rng.random() < 0.3:
                seg = {"text": seg, "props": {"n": rng.randint(0, 2)} if rng.random() < 0.7 else {"s": "v"}}
                if object_incr and rng.random() < 0.5:
                    seg["props"]["o"] = rng.choice(objs)
            op = {"type": 0, "pos1": rng.randint(0, n), "seg": seg}
        else:
            a = rng.randrange(n)
            b = min(n, a + rng.randint(1, 6))
            if x < 0.6:
                op = {"type": 1, "pos1": a, "pos2": b}
            elif x < 0.6 + p_rewrite:
                props = rng.choice([{"n": 1}, {"s": "a", "m": 0}, {"m": None}, {"n": 0, "s": "b"}, {"s": ""},
                                    {"m": 2, "n": 2}])
                op = {"type": 2, "pos1": a, "pos2": b, "props": props, "combiningOp": {"name": "rewrite"}}
            elif x < 0.6 + p_rewrite + p_incr:
                comb = {"name": "incr"}
                r = rng.random()
                if r < 0.2:
                    comb["defaultValue"] = rng.randint(0, 3)
                elif r < 0.3:
                    comb["minValue"] = 1
                elif string_incr and r < 0.45:
                    comb["defaultValue"] = rng.choice(["d", "zz", ""])
                elif string_incr and r < 0.6:
                    comb["minValue"] = rng.choice(["b", "bundefined", "zz"])
                elif object_incr and r < 0.75:
                    comb["defaultValue" if rng.random() < 0.5 else "minValue"] = rng.choice(objs)
                keys = ["n", "m", "s"] if string_incr else ["n", "m"]
                if object_incr and incr_objects:
                    keys = keys + ["o", "o"]
                op = {"type": 2, "pos1": a, "pos2": b, "props": {rng.choice(keys): rng.randint(1, 3)},
                      "combiningOp": comb}
            else:
                props = rng.choice([{"n": rng.randint(0, 2)}, {"m": rng.randint(0, 2), "s": "w"}, {"n": None},
                                    {"s": rng.choice(["a", "b"])}, {"m": None, "n": 1}])
                if object_incr and rng.random() < 0.4:
                    props = {"o": rng.choice(objs + [None])}
                op = {"type": 2, "pos1": a, "pos2": b, "props": props}
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": R, "minimumSequenceNumber": min(ref),
             "type": "op", "contents": op}
        gen.apply_msg(m)
        msgs.append(m)
    gen.close()
    return initial, msgs


def make_tail_log(seed, n_msgs, n_clients=4, lag=48, initial_len=12000, lo=10200, new_mode=False, inserters=None):
    """A multi-client log that edits only positions >= `lo` of a long initial text (remote views, lagging
    refSeqs, inserts / removes / annotates; MSN = the lowest refSeq); only the clients in `inserters` (indices,
    default all) insert.  With lo = initial_len and one inserter, a SnapshotV1 summary taken mid-log loads in
    the reference too (every body segment is visible in the (refSeq 0, inserter) view the loader appends it in,
    snapshotLoader.ts:201-254), and its body holds that client's segments removed above the MSN by any client:
    phantom partial lengths.  Returns (text, msgs)."""
    import random
    from pyoracle import OracleDoc
    rng = random.Random(seed)
    text = "".join(rng.choice("abcdefghij ") for _ in range(initial_len))
    ids = [f"client-{k}" for k in range(n_clients)]
    gen = OracleDoc(new_length_calc=new_mode)
    gen.insert_text_local(0, text)
    gen.start_collab("gen-observer")
    short = {}
    for cid in ids:
        gen.add_client(cid)
        short[cid] = len(short) + 1
    ref = [0] * n_clients
    msgs = []
    ins = list(range(n_clients)) if inserters is None else list(inserters)
    for seq in range(1, n_msgs + 1):
        k = rng.randrange(n_clients)
        ref[k] = max(ref[k], seq - 1 - rng.randint(0, lag))
        R, cid = ref[k], ids[k]
        n = gen.remote_length(R, short[cid])
        r = rng.random()
        if k not in ins and n <= lo + 2:
            k = ins[0]
            R, cid = ref[k], ids[k]
            n = gen.remote_length(R, short[cid])
        if k in ins and (r < 0.5 or n <= lo + 2):
            op = {"type": 0, "pos1": rng.randint(lo, n), "seg": "".join(rng.choice("XYZ\n") for _ in range(rng.randint(1, 5)))}
        else:
            a = rng.randint(lo, n - 1)
            b = min(n, a + rng.randint(1, 6))
            op = {"type": 1, "pos1": a, "pos2": b} if r < 0.8 else \
                {"type": 2, "pos1": a, "pos2": b, "props": {"k": rng.randint(0, 2)}}
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": R, "minimumSequenceNumber": min(ref),
             "type": "op", "contents": op}
        gen.apply_msg(m)
        msgs.append(m)
    gen.close()
    return text, msgs


PROP_PALETTE = [5, {}, "ab", {"0": "a", "1": "b"}, {"x": None}, {"x": 0}, [], 0, "", {"0": "a"}, "a", [1],
                {"x": {"y": None}}, {"x": {}}, 7, True]


def make_props_log(seed, n_msgs, n_clients=4, lag=16, new_mode=False, initial="hello props world", p_cons=0.15):
    """A sequenced op log whose property values are outside any equivalence of matchProperties
    (properties.ts:71-96): key "k" mixes primitives, objects, arrays, strings and index objects, nested nulls
    (PROP_PALETTE); key "j" holds small integers; null deletes.  A fraction `p_cons` of the annotates are remote
    combiningOp "consensus" annotates (properties.ts:46-62) without a defaultValue, with a primitive one, or with
    an object one whose seq is -1.  Inserts with props, removes; every message is applied to a generator oracle
    as it is made.  Returns (initial text, messages)."""
    import random
    from pyoracle import OracleDoc
    rng = random.Random(seed)
    ids = [f"client-{k}" for k in range(n_clients)]
    gen = OracleDoc(new_length_calc=new_mode)
    if initial:
        gen.insert_text_local(0, initial)
    gen.start_collab("gen-observer")
    short = {}
    for cid in ids:
        gen.add_client(cid)
        short[cid] = len(short) + 1
    ref = [0] * n_clients
    msgs = []
    words = ["ab", "c", "xyz", "\n", "more text "]

    def props():
        r = rng.random()
        if r < 0.45:
            return {"k": rng.choice(PROP_PALETTE)}
        if r < 0.65:
            return {"k": rng.choice(PROP_PALETTE), "j": rng.randint(0, 2)}
        if r < 0.8:
            return {"j": rng.randint(0, 2)}
        if r < 0.9:
            return {"k": None}
        return {"o": rng.choice([{"x": None}, {"x": 0}, 0, {}])}

    for seq in range(1, n_msgs + 1):
        k = rng.randrange(n_clients)
        ref[k] = max(ref[k], seq - 1 - rng.randint(0, lag))
        R, C, cid = ref[k], short[ids[k]], ids[k]
        n = gen.remote_length(R, C)
        x = rng.random()
        if x < 0.4 or n == 0:
            seg = rng.choice(words)
            if rng.random() < 0.5:
                seg = {"text": seg, "props": {kk: v for kk, v in props().items() if v is not None}}
            op = {"type": 0, "pos1": rng.randint(0, n), "seg": seg}
        else:
            a = rng.randrange(n)
            b = min(n, a + rng.randint(1, 8))
            if x < 0.55:
                op = {"type": 1, "pos1": a, "pos2": b}
            elif x < 0.55 + p_cons:
                comb = {"name": "consensus"}
                r = rng.random()
                if r < 0.25:
                    comb["defaultValue"] = rng.choice([3, "d", True])
                elif r < 0.4:
                    comb["defaultValue"] = {"seq": -1, "v": rng.randint(0, 1)}
                op = {"type": 2, "pos1": a, "pos2": b, "props": {rng.choice(["k", "c"]): 1}, "combiningOp": comb}
            else:
                op = {"type": 2, "pos1": a, "pos2": b, "props": props()}
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": R, "minimumSequenceNumber": min(ref),
             "type": "op", "contents": op}
        gen.apply_msg(m)
        msgs.append(m)
    return initial, msgs
