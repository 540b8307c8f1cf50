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


# ---------------------------------------------------------------------------------------------------------------
# Known answer for the reference's partial-length DEFICITS (addSeq over an existing entry below newer ones).
#
# PartialSequenceLengths.update (partialLengths.ts:636-686) calls addSeq (:543-577) on the block's main set and on
# the updating client's set.  When the set already holds an entry AT the update's seq, addSeq replaces that
# entry's seglen with the recomputed total and its len with (entry before).len + seglen, but leaves every later
# entry's cumulative len as it was: from the first later entry on, lengths are short by the added segment.  In
# getPartialLength (:698-716) the main term latestLeq(refSeq).len is short for refSeq >= t1 (the main set's first
# entry above the seq); the client term cliLatest.len - latestLeq_client(refSeq).len is short for refSeq < t1c
# (that client's first entry above the seq).
#
# The constructed summary (header ["h"]; body "1".."7", four NonCollab tombstones a..d removed at seq 20 by b --
# one NonCollab batch, as in the phantom case -- then "AB" by a at seq 12, "CD" by a at seq 15, "EF" by a at
# seq 12; MSN 5, seq 20) loads to
#
#     root [ L1 [h 1 2 3] , L2 [4 5 6 7 AB CD EF] , L3 [a b c d] ]
#
# AB, CD and EF are appended one by one at root.cachedLength (8, 10, 12) in the (refSeq 0, "a") view: L1 is 4,
# L2 is 4 + a's own segments, so each lands at the end of L2 (pos == length descends into a block, breakTie
# mergeTree.ts:1719-1738).  AB adds L2 entry 12, CD entry 15; EF finds entry 12 with 15 above it: L2's main
# entry 15 keeps len 4 (exact 6) and a's client entry 15 too.  Then:
# * a inserts "Y" at 13 with refSeq 12: the main term is exact there (12 < 15), the client term is short by 2,
#   so L2 is 8 (exact 10) and pos 13 passes L1 (4) and L2 (8) and lands 1 into L3, where tombstone "a" (1) ends
#   at 1 (breakTie is false for a leaf at pos != 0): before "b" -> L3 [a Y b c d];
# * c inserts "Z" at 13 with refSeq 16: the main term latestLeq(16) = entry 15 is short by 2, so L2 is 8 again;
#   1 into L3 passes "a", and at pos 0 before Y (seq 21, invisible to c at 16, length 0) breakTie(22 > 21)
#   places Z before Y -> L3 [a Z Y b c d].
# The text is "h1234567ABCDEFZY"; exact partial lengths would split EF for both: "h1234567ABCDEZYF".
DEF_TEXT = "h1234567ABCDEFZY"
DEF_EXACT_TEXT = "h1234567ABCDEZYF"


def def_summary():
    vis = [str(i) for i in range(1, 8)]
    tomb = [{"json": t, "removedSeq": 20, "removedClient": "b", "removedClientIds": ["b"]} for t in "abcd"]
    xs = [{"json": "AB", "seq": 12, "client": "a"}, {"json": "CD", "seq": 15, "client": "a"},
          {"json": "EF", "seq": 12, "client": "a"}]
    body = vis + tomb + xs
    hdr = {"version": "1", "segmentCount": 1, "length": 1, "segments": ["h"], "startIndex": 0,
           "headerMetadata": {"minSequenceNumber": 5, "sequenceNumber": 20,
                              "orderedChunkMetadata": [{"id": "header"}, {"id": "body_0"}],
                              "totalLength": 18, "totalSegmentCount": 1 + len(body)}}
    b0 = {"version": "1", "segmentCount": len(body), "length": 17, "segments": body, "startIndex": 1}
    return [["header", json.dumps(hdr)], ["body_0", json.dumps(b0)]]


def def_msgs():
    def m(cid, seq, ref, op):
        return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": 5,
                "type": "op", "contents": op}
    return [m("a", 21, 12, {"type": 0, "pos1": 13, "seg": "Y"}), m("c", 22, 16, {"type": 0, "pos1": 13, "seg": "Z"})]
