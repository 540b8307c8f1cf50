"""Known-answer case for the reference's phantom partial lengths (test infrastructure).

SnapshotLoader.loadBody appends a removed body segment inserted by a collaborating client on its own
(snapshotLoader.ts:242-254) through insertSegments -> blockUpdateLength's incremental path (mergeTree.ts:
2436-2453): PartialSequenceLengths.update adds the segment's cachedLength at its seq because
removedSeq !== seq (partialLengths.ts:636-686), and nothing records the removal, so every block that update
reaches keeps a surplus for perspectives that see the removal.

The constructed summary (header ["h"], body: "1".."7", four NonCollab tombstones a..d removed at seq 20 by
b, then "pp" inserted by a at seq 11 and removed by b at seq 12; MSN 5, seq 20) loads, by the reference's
rules (derived by hand in DESIGN.md section 7), to the tree

    root [ L1 [h 1 2 3] , L2 [4 5 6 7 pp] , L3 [a b c d] ]

("pp" is appended at root.cachedLength = 8 in the (refSeq 0, "a") view, where the tombstones are visible:
at the end of L2, whose length then carries pp's insert but not its removal).  Then:
* c inserts "Z" at 11 with refSeq 15: L2's partial length is 4 + 2 there (the removal at 12 <= 15 is not
  recorded), so pos 11 passes L1 (4) and L2 (6) and lands 1 into L3: [a Z b c d]; without the surplus it
  would land 3 into L3: [a b c Z d];
* d inserts "Y" at 12 with refSeq 11 (pp still visible, Z not yet): 4 + 6 = 10, 2 into L3 -> after b:
  [a Z b Y c d].
So the text is "h1234567ZY" (exact partial lengths would give "h1234567YZ").
"""
import json

KAT_TEXT = "h1234567ZY"
EXACT_TEXT = "h1234567YZ"


def kat_summary():
    vis = [str(i) for i in range(1, 8)]
    tomb = [{"json": t, "removedSeq": 20, "removedClient": "b", "removedClientIds": ["b"]} for t in "abcd"]
    pp = {"json": "pp", "seq": 11, "client": "a", "removedSeq": 12, "removedClient": "b", "removedClientIds": ["b"]}
    body = vis + tomb + [pp]
    hdr = {"version": "1", "segmentCount": 1, "length": 1, "segments": ["h"], "startIndex": 0,
           "headerMetadata": {"minSequenceNumber": 5, "sequenceNumber": 20,
                              "orderedChunkMetadata": [{"id": "header"}, {"id": "body_0"}],
                              "totalLength": 14, "totalSegmentCount": 1 + len(body)}}
    b0 = {"version": "1", "segmentCount": len(body), "length": 13, "segments": body, "startIndex": 1}
    return [["header", json.dumps(hdr)], ["body_0", json.dumps(b0)]]


def kat_msgs():
    def m(cid, seq, ref, op):
        return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": 5,
                "type": "op", "contents": op}
    return [m("c", 21, 15, {"type": 0, "pos1": 11, "seg": "Z"}), m("d", 22, 11, {"type": 0, "pos1": 12, "seg": "Y"})]
