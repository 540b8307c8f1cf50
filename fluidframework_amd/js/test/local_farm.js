// A live-client conflict farm through the JS drop-in (tests/test_js_package.py): every client of the
// recorded farm is one Client slot; its local ops go through applyLocalOp, its received messages (acks
// included) through applyMsg, its reconnects through regeneratePendingOp.  Prints every client's text after each round as one JSON line.
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
      else if (kind === "regen") {
        // a reconnect: the regenerated op must equal the oracle's (x = [resetOp, expected]), key order included
        const got = JSON.stringify(clients[k].regeneratePendingOp(x[0]));
        if (got !== JSON.stringify(x[1])) throw new Error(`regeneratePendingOp: ${got} != ${JSON.stringify(x[1])}`);
      } else clients[k].applyMsg(x);
    }
  });
  texts.push(clients.map((c) => c.getText()));
}
// batch-scale reads after the last round (all ops acked): digests and SnapshotV1 of every client
const digests = batch.digests();
const sums = batch.summarizeV1Many(clients.map((_, k) => k));
if (digests.length !== clients.length || sums.length !== clients.length) throw new Error("batch reads");
console.log(JSON.stringify({ texts, digests, summaries: sums.map((x) => x.summary) }));
