// Client / TestClient call shapes of the JS drop-in on the GPU (tests/test_js_package.py): TestClient
// message helpers (testClient.ts:224-327), getText ranges counting markers (MergeTreeTextHelper.ts:20-81),
// Client.annotateMarker (client.ts:190) with its pending keys, its ack, and a remote marker-relative op.
// Prints one JSON line with the results the Python side compares with the oracle.
"use strict";
const { MergeTreeBatch } = require("..");

const batch = new MergeTreeBatch(1, { mergeTreeUseNewLengthCalculations: true });
const c = batch.client(0);
c.insertTextLocal(0, "hello world");
c.startOrUpdateCollaboration("me");
c.insertTextRemote(0, "ab", undefined, 1, 0, "a");
c.insertMarkerRemote(2, { refType: 1 }, { markerId: "m" }, 2, 1, "b");
const ranges = [c.getText(), c.getText(0, 3), c.getText(2, 5), c.getText(4)];
const op = c.annotateMarker("m", { color: "red" });
c.annotateRangeRemote(0, 4, { color: "blue", w: 1 }, 3, 2, "a");
c.applyMsg(c.makeOpMessage(op, 4, 2, "me"));
c.applyMsg(c.makeOpMessage({ relativePos1: { id: "m" }, seg: "!", type: 0 }, 5, 4, "b"));
console.log(JSON.stringify({ ranges, op, text: c.getText(), digest: batch.digests()[0] }));
