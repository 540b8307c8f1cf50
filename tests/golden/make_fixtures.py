"""Generate compact golden fixtures from the reference's own committed test data.

Sources (read-only, /root/reference):
  packages/dds/merge-tree/src/test/results/*.json        -- 30 conflict-farm replay logs
      (ReplayGroup{msgs, initialText, resultText, seq}, mergeTreeOperationRunner.ts:191-196;
       replayed by client.replay.spec.ts:16-72 with default (legacy length) options)
  packages/dds/sequence/src/test/snapshots/v1/*.json      -- SnapshotV1 summaries of detached
      SharedStrings (generateSharedStrings.ts:47-146, compared by snapshotVersion.spec.ts:137-151)

Outputs (data only: inputs and expected outputs, no reference source):
  tests/golden/replay/<name>.json.gz   {"initialText", "groups":[{"msgs":[[clientId,seq,refSeq,msn,contents]...],
                                         "resultText"}]}
  tests/golden/snapshots_v1/<name>.json.gz  {"blobs": [[path, contents], ...]} of the "content" subtree
  packages/dds/sequence/src/test/snapshots/legacy/*.json  -- SnapshotLegacy summaries of the same strings
  tests/golden/snapshots_legacy/<name>.json.gz  (same layout)
"""
import gzip
import json
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def replay_fixtures():
    src = os.path.join(REF, "packages/dds/merge-tree/src/test/results")
    out_dir = os.path.join(HERE, "replay")
    os.makedirs(out_dir, exist_ok=True)
    for name in sorted(os.listdir(src)):
        with open(os.path.join(src, name)) as f:
            groups = json.load(f)
        out = {"source": f"packages/dds/merge-tree/src/test/results/{name}",
               "initialText": groups[0]["initialText"], "groups": []}
        prev = groups[0]["initialText"]
        for g in groups:
            assert g["initialText"] == prev, name
            msgs = []
            for m in g["msgs"]:
                assert m["type"] == "op"
                msgs.append([m["clientId"], m["sequenceNumber"], m["referenceSequenceNumber"],
                             m["minimumSequenceNumber"], m["contents"]])
            out["groups"].append({"msgs": msgs, "resultText": g["resultText"]})
            prev = g["resultText"]
        dst = os.path.join(out_dir, name.replace(".json", ".json.gz"))
        with gzip.open(dst, "wt", compresslevel=9) as f:
            json.dump(out, f, separators=(",", ":"))
        print("wrote", dst, os.path.getsize(dst))


def snapshot_fixtures(version="v1"):
    src = os.path.join(REF, f"packages/dds/sequence/src/test/snapshots/{version}")
    out_dir = os.path.join(HERE, f"snapshots_{version}")
    os.makedirs(out_dir, exist_ok=True)
    for name in sorted(os.listdir(src)):
        with open(os.path.join(src, name)) as f:
            tree = json.load(f)
        content = [e for e in tree["entries"] if e["path"] == "content"][0]["value"]["entries"]
        blobs = []
        for e in content:
            assert e["type"] == "Blob" and e["mode"] == "100644" and e["value"]["encoding"] == "utf-8"
            blobs.append([e["path"], e["value"]["contents"]])
        dst = os.path.join(out_dir, name.replace(".json", ".json.gz"))
        with gzip.open(dst, "wt", compresslevel=9) as f:
            json.dump({"source": f"packages/dds/sequence/src/test/snapshots/{version}/{name}", "blobs": blobs}, f)
        print("wrote", dst, os.path.getsize(dst))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference checkout not present; fixtures are already committed")
    replay_fixtures()
    snapshot_fixtures("v1")
    snapshot_fixtures("legacy")
