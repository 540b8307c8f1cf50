// Type declarations for @fluid-mi355x/merge-tree-batch (see index.js).
export interface ReplayStats {
  opsApplied: number;
  docs: number;
  segmentsFinal: number;
  textUnitsFinal: number;
  bytesAlg: number;
  errors: number;
  kernelMs: number;
  checksum: string;
}
export interface BatchOptions {
  mergeTreeUseNewLengthCalculations?: boolean;
  mergeTreeSnapshotChunkSize?: number;
  device?: number;
  /** GPU indices to spread the documents over (documents placed by hash, one engine + stream per device) */
  devices?: number[];
  /** false: SnapshotLegacy summaries with tracked catch-up messages (the reference default); default true here */
  newMergeTreeSnapshotFormat?: boolean;
}
export interface ISequencedDocumentMessage {
  clientId: string | null;
  sequenceNumber: number;
  referenceSequenceNumber: number;
  minimumSequenceNumber: number;
  type: string;
  contents: unknown;
}
export declare class MergeTreeBatch {
  constructor(ndocs: number, options?: BatchOptions);
  readonly ndocs: number;
  digests(first?: number, n?: number): string[];
  summarizeV1Many(docs: number[], msn?: number, seq?: number, threads?: number):
    { blobs: [string, string][]; summary: string }[];
  lastStats: ReplayStats | undefined;
  client(i: number): TestClient;
  flush(): ReplayStats;
  flushAsync(): Promise<ReplayStats>;
  internProps(props: object | string): number;
  appendOps(doc: number, records: Uint8Array, payload: Uint16Array): void;
  addClient(doc: number, longId: string): void;
  dumpSegments(doc: number): string;
  checksum(doc: number): string;
  summarizeV1(doc: number, msn?: number, seq?: number): { blobs: [string, string][]; summary: unknown };
  summarizeLegacy(doc: number, msn?: number, seq?: number, catchUpMsgs?: unknown[]): { blobs: [string, string][]; summary: unknown };
  rewind(): void;
  replayResident(): ReplayStats;
}
/** A segment as the read queries return it (short client ids). */
export interface SegmentInfo {
  type: "TextSegment" | "Marker" | "PermutationSegment";
  text?: string;
  refType?: number | null;
  start?: number;
  cachedLength: number;
  seq: number;
  clientId: number;
  removedSeq?: number;
  removedClientIds?: number[];
  properties?: Record<string, unknown>;
}
export declare class Client {
  insertTextLocal(pos: number, text: string, props?: Record<string, unknown>): unknown;
  applyLocalOp(op: Record<string, unknown> | string): unknown;
  insertSegmentLocal(pos: number, seg: unknown): Record<string, unknown>;
  removeRangeLocal(start: number, end: number): Record<string, unknown>;
  regeneratePendingOp(resetOp: Record<string, unknown> | string, segmentGroup?: unknown): Record<string, unknown>;
  annotateRangeLocal(start: number, end: number, props: Record<string, unknown>, combiningOp?: unknown): Record<string, unknown>;
  annotateMarker(markerId: string, props: Record<string, unknown>, combiningOp?: unknown): Record<string, unknown>;
  annotateMarkerNotifyConsensus(markerId: string, props: Record<string, unknown>): Record<string, unknown>;
  startOrUpdateCollaboration(longClientId: string, minSeq?: number, currentSeq?: number): void;
  load(runtime: { clientId?: string } | undefined,
       storage: { readBlob(path: string): Promise<ArrayBufferLike | Uint8Array | string> }): Promise<{ catchupOpsP: Promise<unknown[]> }>;
  applyMsg(msg: ISequencedDocumentMessage | string, local?: boolean): void;
  getText(start?: number, end?: number): string;
  getLength(): number;
  getCurrentSeq(): number;
  getCollabWindow(): { clientId: number; collaborating: boolean; minSeq: number; currentSeq: number };
  getLongClientId(shortClientId: number): string;
  getClientId(): number;
  getContainingSegment(pos: number, sequenceArgs?: { referenceSequenceNumber: number; clientId: string }):
    { segment: SegmentInfo | undefined; offset: number | undefined };
  getPropertiesAtPosition(pos: number): Record<string, unknown> | undefined;
  walkSegments<T>(handler: (segment: SegmentInfo, pos: number, refSeq: number, clientId: number, start: number,
                            end: number, accum?: T) => boolean | void, start?: number, end?: number, accum?: T): void;
  summarize(runtime?: { deltaManager?: { minimumSequenceNumber?: number; lastSequenceNumber?: number } }, handle?: unknown,
            serializer?: unknown, catchUpMsgs?: unknown[]): unknown;
}
export declare class TestClient extends Client {
  makeOpMessage(op: Record<string, unknown>, seq?: number, refSeq?: number, longClientId?: string, minSeqNumber?: number): Record<string, unknown>;
  insertTextRemote(pos: number, text: string, props: Record<string, unknown> | undefined, seq: number, refSeq: number, longClientId: string): void;
  removeRangeRemote(start: number, end: number, seq: number, refSeq: number, longClientId: string): void;
  annotateRangeRemote(start: number, end: number, props: Record<string, unknown>, seq: number, refSeq: number, longClientId: string): void;
  insertMarkerRemote(pos: number, markerDef: { refType?: number } | undefined, props: Record<string, unknown> | undefined, seq: number, refSeq: number, longClientId: string): void;
  insertMarkerLocal(pos: number, behaviors: number, props?: Record<string, unknown>): Record<string, unknown>;
}

/** A batch of SharedMatrix observers (rows / cols PermutationVectors replayed on the GPU). */
export declare class MatrixBatch extends MergeTreeBatch {
  constructor(nmatrices: number, options?: { mergeTreeUseNewLengthCalculations?: boolean; mergeTreeSnapshotChunkSize?: number; device?: number });
  matrix(m: number): SharedMatrix;
}
export declare class SharedMatrix {
  startOrUpdateCollaboration(longClientId: string, minSeq?: number, currentSeq?: number): void;
  applyMsg(msg: ISequencedDocumentMessage | string): void;
  /** SharedMatrix.loadCore (matrix.ts:611) of a summary written by summarize(). */
  load(runtime: { clientId?: string } | undefined,
       storage: { readBlob(path: string): Promise<ArrayBufferLike | Uint8Array | string> }): Promise<void>;
  /** SharedMatrix.summarizeCore (matrix.ts:449): rows / cols PermutationVector summaries and the cells blob. */
  summarize(): { blobs: [string, string][]; summary: unknown };
  /** SharedMatrix.getCell (matrix.ts:173) in the observer's view. */
  getCell(row: number, col: number): unknown;
  readonly rowCount: number;
  readonly colCount: number;
  summarizeVectors(): { rows: { blobs: [string, string][]; summary: unknown }; cols: { blobs: [string, string][]; summary: unknown } };
}
