// A live-client conflict farm through the JS drop-in (tests/test_js_package.py): every client of the
// recorded farm is one Client slot; its local ops go through applyLocalOp, its received messages (acks
// included) through applyMsg.  Prints every client's text after each round as one JSON line.
"use strict";
const fs = require("fs");
const { MergeTreeBatch } = require("..");

const rec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const batch = new MergeTreeBatch(rec.ids.length, { mergeTreeUseNewLengthCalculations: !!rec.newMode });
const clients = rec.ids.map((id, k) => {
  const c = batch.client(k);
  c.insertTextLocal(0, rec.initial);
  c.startOrUpdateCollaboration(id);
  return c;
});
const texts = [];
for (const round of rec.rounds) {
  round.forEach((events, k) => {
    for (const [kind, x] of events) {
      if (kind === "local") clients[k].applyLocalOp(x);
      else clients[k].applyMsg(x);
    }
  });
  texts.push(clients.map((c) => c.getText()));
}
// batch-scale reads after the last round (all ops acked): digests and SnapshotV1 of every client
const digests = batch.digests();
const sums = batch.summarizeV1Many(clients.map((_, k) => k));
if (digests.length !== clients.length || sums.length !== clients.length) throw new Error("batch reads");
console.log(JSON.stringify({ texts, digests, summaries: sums.map((x) => x.summary) }));
