"use strict";
/*
 * Parity test of the JS drop-in package, written like the reference's client.replay.spec.ts:16-72:
 * every committed conflict-farm replay log (tests/golden/replay, from
 * packages/dds/merge-tree/src/test/results) is applied message by message through
 * Client.applyMsg on an observer that started from `initialText`, and getText() must equal the
 * log's resultText after every group.  All 30 logs are documents of one batch (one GPU launch per
 * group).
 *
 *   node test/parity.js          GPU run (expects an MI355X)
 *   node test/parity.js --cpu    no GPU: package/addon load, message packing, loud NODEV failure
 */
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");

const { MergeTreeBatch, MatrixBatch, native } = require("..");

const GOLDEN = path.join(__dirname, "..", "..", "..", "tests", "golden", "replay");
const SNAPSHOTS = path.join(__dirname, "..", "..", "..", "tests", "golden", "snapshots_v1");

function snapshotBlobs(name) {
  return JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(SNAPSHOTS, `${name}.json.gz`))).toString("utf8")).blobs;
}
/** IChannelStorageService over [[path, content], ...] */
function storageOf(blobs) {
  const m = new Map(blobs);
  return { readBlob: async (p) => Buffer.from(m.get(p), "utf8"), contains: async (p) => m.has(p) };
}

function loadFixtures() {
  return fs.readdirSync(GOLDEN).filter((f) => f.endsWith(".json.gz")).sort().map((f) => ({
    name: f.replace(".json.gz", ""),
    log: JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(GOLDEN, f))).toString("utf8")),
  }));
}

function toMsg(m) {
  const [clientId, sequenceNumber, referenceSequenceNumber, minimumSequenceNumber, contents] = m;
  return { clientId, sequenceNumber, referenceSequenceNumber, minimumSequenceNumber, type: "op", contents };
}

function cpuChecks() {
  const names = ["create", "docInit", "applyMsg", "appendOps", "addClient", "internProps", "replay", "replayAsync",
    "getText", "getLength", "getSeq", "dumpSegments", "checksum", "summarizeV1", "rewind", "replayResident",
    "clientLongId", "loadV1", "matrixInit", "matrixApplyMsg", "matrixSummarize", "matrixGetCell", "mapRange", "matrixLoad", "summarizeLegacy"];
  for (const n of names) assert.strictEqual(typeof native[n], "function", n);
  const fx = loadFixtures();
  assert.strictEqual(fx.length, 30);
  const batch = new MergeTreeBatch(fx.length);
  fx.forEach(({ log }, i) => {
    const c = batch.client(i);
    c.insertTextLocal(0, log.initialText);
    c.startOrUpdateCollaboration("A");
    for (const g of log.groups) for (const m of g.msgs) c.applyMsg(toMsg(m));
  });
  // reference error text survives the boundary (client.ts:880 assert 0x038)
  const b2 = new MergeTreeBatch(1);
  b2.client(0).startOrUpdateCollaboration("A");
  b2.client(0).applyMsg(toMsg(["B", 5, 0, 0, { type: 0, pos1: 0, seg: "x" }]));
  assert.throws(() => b2.client(0).applyMsg(toMsg(["B", 4, 0, 0, { type: 0, pos1: 0, seg: "y" }])), /0x038/);
  // no CPU fallback
  assert.throws(() => batch.flush(), (e) => e.code === -2);
  // Client.load packs the summary on the host; the body append still needs the GPU
  const b3 = new MergeTreeBatch(1);
  b3.client(0).load(undefined, storageOf(snapshotBlobs("withMarkers"))).then(() => {
    assert.throws(() => b3.flush(), (e) => e.code === -2);
    console.log("js cpu checks ok: summary load packed, flush fails with MTB_E_NODEV");
  }).catch((e) => { console.error(e); process.exit(1); });
  console.log("js cpu checks ok: 30 logs packed, flush fails with MTB_E_NODEV");
}

async function gpuChecks() {
  const fx = loadFixtures();
  const batch = new MergeTreeBatch(fx.length);
  fx.forEach(({ log }, i) => {
    const c = batch.client(i);
    c.insertTextLocal(0, log.initialText);
    c.startOrUpdateCollaboration("A");
  });
  const ngroups = fx[0].log.groups.length;
  let checked = 0;
  const bad = [];
  for (let g = 0; g < ngroups; g++) {
    fx.forEach(({ log }, i) => { for (const m of log.groups[g].msgs) batch.client(i).applyMsg(toMsg(m)); });
    if (g % 2) await batch.flushAsync(); else batch.flush();
    fx.forEach(({ name, log }, i) => {
      checked++;
      if (batch.client(i).getText() !== log.groups[g].resultText) bad.push(`${name}#${g}`);
    });
  }
  assert.deepStrictEqual(bad, [], `mismatching checkpoints: ${bad.slice(0, 5)}`);
  // summary read-out and collab window through the drop-in surface
  const c0 = batch.client(0);
  const s = c0.summarize();
  assert.strictEqual(s.summary.type, 1);
  assert.ok(s.summary.tree.header);
  assert.strictEqual(c0.getLength(), c0.getText().length);
  assert.strictEqual(c0.getCurrentSeq(), fx[0].log.groups[ngroups - 1].msgs.slice(-1)[0][1]);
  // segment queries: walkSegments covers the text in order; getContainingSegment agrees with it
  fx.forEach((_, i) => {
    const c = batch.client(i);
    let text = "";
    const walked = [];
    c.walkSegments((seg, pos) => { text += seg.text || ""; walked.push([pos, seg]); });
    assert.strictEqual(text, c.getText());
    for (const [pos, seg] of walked.slice(0, 40)) {
      const hit = c.getContainingSegment(pos);
      assert.deepStrictEqual([hit.segment, hit.offset], [seg, 0]);
      assert.deepStrictEqual(c.getPropertiesAtPosition(pos), seg.properties);
    }
  });
  // SnapshotLegacy with tracked catch-up messages (newMergeTreeSnapshotFormat false), against the oracle
  const lexp = process.env.MTB_JS_LEGACY_EXPECT;
  if (lexp) {
    const e = JSON.parse(fs.readFileSync(lexp, "utf8"));
    const lb = new MergeTreeBatch(fx.length, { newMergeTreeSnapshotFormat: false });
    fx.forEach(({ log }, i) => {
      lb.client(i).insertTextLocal(0, log.initialText);
      lb.client(i).startOrUpdateCollaboration("A");
      for (const grp of log.groups) for (const m of grp.msgs) lb.client(i).applyMsg(toMsg(m));
    });
    lb.flush();
    fx.forEach(({ name }, i) => {
      const got = lb.summarizeLegacy(i);
      assert.deepStrictEqual(got.blobs, e[i].blobs, `${name}: legacy blobs`);
      assert.deepStrictEqual(got.summary, e[i].summary, `${name}: legacy summary`);
      assert.deepStrictEqual(lb.client(i).summarize(), e[i].summary, `${name}: Client.summarize`);
    });
    console.log("js gpu legacy ok");
  }
  console.log(`js gpu parity ok: ${checked} text checkpoints over ${fx.length} reference logs`);
  // Client.load: every document's summary loads into a fresh batch and summarizes back to the same bytes
  const loaded = new MergeTreeBatch(fx.length);
  const sums = fx.map((_, i) => batch.summarizeV1(i).blobs);
  for (let i = 0; i < fx.length; i++) await loaded.client(i).load({ clientId: "A" }, storageOf(sums[i]));
  await loaded.flushAsync();
  fx.forEach(({ name, log }, i) => {
    assert.strictEqual(loaded.client(i).getText(), log.groups[ngroups - 1].resultText, `${name}: text after load`);
    assert.deepStrictEqual(loaded.summarizeV1(i).blobs, sums[i], `${name}: summary after load`);
  });
  // SharedMatrix through the drop-in surface: a matrix log replayed twice, in one batch of two matrices
  const mlog = JSON.parse(fs.readFileSync(path.join(__dirname, "matrix_log.json"), "utf8"));
  const mb = new MatrixBatch(2);
  for (let m = 0; m < 2; m++) {
    mb.matrix(m).startOrUpdateCollaboration("obs");
    for (const msg of mlog) mb.matrix(m).applyMsg(msg);
  }
  mb.flush();
  const v0 = mb.matrix(0).summarizeVectors(), v1 = mb.matrix(1).summarizeVectors();
  assert.deepStrictEqual(v0, v1);
  assert.strictEqual(v0.rows.blobs[v0.rows.blobs.length - 1][0], "handleTable");
  // SharedMatrix.summarize (rows, cols, cells) against the oracle's, when the harness passes it
  const s0 = mb.matrix(0).summarize();
  assert.deepStrictEqual(s0, mb.matrix(1).summarize());
  assert.strictEqual(s0.blobs[s0.blobs.length - 1][0], "cells");
  const expect = process.env.MTB_JS_MATRIX_EXPECT;
  if (expect) {
    const e = JSON.parse(fs.readFileSync(expect, "utf8"));
    assert.deepStrictEqual(s0.blobs, e.blobs, "matrix summary blobs vs oracle");
    assert.deepStrictEqual(s0.summary, e.summary, "matrix summary tree vs oracle");
    for (const [r, c, v] of e.cells)
      assert.deepStrictEqual(mb.matrix(0).getCell(r, c), v === null ? undefined : JSON.parse(v), `getCell(${r}, ${c})`);
  }
  // SharedMatrix.load of that summary: the same summary back, the same cells by position
  const lm = new MatrixBatch(1);
  const store = new Map(s0.blobs);
  await lm.matrix(0).load({ clientId: "obs" }, { readBlob: async (p) => store.get(p) });
  assert.deepStrictEqual(lm.matrix(0).summarize().blobs, s0.blobs);
  assert.strictEqual(lm.matrix(0).rowCount, mb.matrix(0).rowCount);
  for (let r = 0; r < mb.matrix(0).rowCount; r += 3)
    for (let c = 0; c < mb.matrix(0).colCount; c += 3)
      assert.deepStrictEqual(lm.matrix(0).getCell(r, c), mb.matrix(0).getCell(r, c));
  console.log("js gpu matrix ok");
  const ref = new MergeTreeBatch(1);
  await ref.client(0).load(undefined, storageOf(snapshotBlobs("withMarkers")));
  assert.deepStrictEqual(ref.summarizeV1(0, 0, 0).blobs, snapshotBlobs("withMarkers"));
  console.log(`js gpu load ok: ${fx.length} summaries + the withMarkers reference summary round-trip`);
}

if (process.argv.includes("--cpu")) {
  cpuChecks();
} else {
  gpuChecks().catch((e) => {
    console.error(e);
    process.exit(1);
  });
}
