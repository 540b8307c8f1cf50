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


def snapshot_fixture(name):
    with gzip.open(os.path.join(GOLDEN, "snapshots_v1", f"{name}.json.gz"), "rt") as fh:
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
