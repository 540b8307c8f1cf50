"""The reference's two-client SharedMatrix conflict cases as sequenced op logs (test vectors, not source).

`packages/dds/matrix/src/test/matrix.spec.ts:349-607` ("Connected with two clients" / "conflict") drives two
live SharedMatrix clients through `MockContainerRuntimeFactory` and checks the final grid of both with
`extract()`.  Here each case is restated as the op messages that run produces, seen by a third client that
only observes (every message is remote to it), so the observer's grid must equal the spec's literal:

* submission: `MockContainerRuntime.submit` (`runtime/test-runtime-utils/src/mocks.ts:143-156`) stamps
  `referenceSequenceNumber = deltaManager.lastSequenceNumber` of the submitting client and queues the
  message; `pushMessage` (:238-248) records a client's first refSeq in the MSN table;
* `expect()` (matrix.spec.ts:315) = `processAllMessages` (:288-292): FIFO over both clients, each message
  gets `sequenceNumber = ++seq`, the sender's MSN entry = its refSeq, `minimumSequenceNumber` = the
  table's minimum (:256-268), and every client's lastSequenceNumber advances;
* message contents as SharedMatrix submits them: `insertCols/Rows` -> the PermutationVector insert op
  `{pos1, seg: [count, Handle.unallocated], type: 0, target}` (`permutationvector.ts:41-149`,
  `matrix.ts:311-369`), `removeCols/Rows` -> `{pos1, pos2, type: 1, target}`, `setCell(s)` -> one
  `{type: 2 (MatrixOp.set), row, col, value}` per cell in row-major order with the sender's local positions
  (`matrix.ts:216-308`); an undefined value is dropped by the wire's JSON round trip (mocks.ts:259).

Each case: (name, spec line, steps, expected grid or None).  A step is ("A" | "B", method, *args) on
matrix1 / matrix2, or ("expect",).  `None` marks a case whose spec checks only that both clients converge
(no literal grid): there the engine is compared with the oracle only.
"""

UNALLOCATED = -2147483648  # Handle.unallocated (matrix/src/handletable.ts:11)
U = None  # undefined cell

CASES = [
    ("setCell", 359, [
        ("A", "insertCols", 0, 1), ("A", "insertRows", 0, 1), ("expect",),
        ("A", "setCell", 0, 0, "1st"), ("B", "setCell", 0, 0, "2nd"), ("expect",)], [["2nd"]]),
    ("clear unallocated cell", 371, [
        ("A", "insertCols", 0, 1), ("A", "insertRows", 0, 1), ("expect",),
        ("A", "setCell", 0, 0, "x"), ("B", "setCell", 0, 0, U), ("expect",)], [[U]]),
    ("insert and set in new row", 381, [
        ("A", "insertCols", 0, 2), ("expect",), ("A", "insertRows", 0, 1),
        ("A", "setCells", 0, 1, 1, ["x"]), ("expect",)], [[U, "x"]]),
    ("insert and set in new col", 389, [
        ("A", "insertRows", 0, 2), ("expect",), ("A", "insertCols", 0, 1),
        ("A", "setCells", 1, 0, 1, ["x"]), ("expect",)], [[U], ["x"]]),
    ("insert col conflict", 397, [
        ("A", "insertRows", 0, 1), ("expect",),
        ("A", "insertCols", 0, 1), ("A", "setCell", 0, 0, "1st"),
        ("B", "insertCols", 0, 1), ("B", "setCell", 0, 0, "2nd"), ("expect",)], [["2nd", "1st"]]),
    ("insert row conflict", 410, [
        ("A", "insertCols", 0, 1), ("expect",),
        ("A", "insertRows", 0, 1), ("A", "setCell", 0, 0, "1st"),
        ("B", "insertRows", 0, 1), ("B", "setCell", 0, 0, "2nd"), ("expect",)], [["2nd"], ["1st"]]),
    ("overlapping remove col", 423, [
        ("A", "insertCols", 0, 3), ("A", "insertRows", 0, 1),
        ("A", "setCell", 0, 0, "A"), ("A", "setCell", 0, 1, "B"), ("A", "setCell", 0, 2, "C"), ("expect",),
        ("A", "removeCols", 1, 1), ("B", "removeCols", 1, 1), ("expect",)], [["A", "C"]]),
    ("overlapping remove row", 437, [
        ("A", "insertCols", 0, 1), ("A", "insertRows", 0, 3),
        ("A", "setCell", 0, 0, "A"), ("A", "setCell", 1, 0, "B"), ("A", "setCell", 2, 0, "C"), ("expect",),
        ("A", "removeRows", 1, 1), ("B", "removeRows", 1, 1), ("expect",)], [["A"], ["C"]]),
    ("insert col vs. remove row", 451, [
        ("A", "insertCols", 0, 2), ("A", "insertRows", 0, 3),
        ("A", "setCells", 0, 0, 2, ["A1", "C1", "A2", "C2", "A3", "C3"]), ("expect",),
        ("A", "insertCols", 1, 1), ("A", "setCells", 0, 1, 1, ["B1", "B2", "B3"]),
        ("B", "removeRows", 1, 1), ("expect",)], [["A1", "B1", "C1"], ["A3", "B3", "C3"]]),
    ("insert row vs. remove col", 480, [
        ("A", "insertRows", 0, 2), ("A", "insertCols", 0, 3),
        ("A", "setCells", 0, 0, 3, ["A1", "B1", "C1", "A3", "B3", "C3"]), ("expect",),
        ("A", "insertRows", 1, 1), ("A", "setCells", 1, 0, 3, ["A2", "B2", "C2"]),
        ("B", "removeCols", 1, 1), ("expect",)], [["A1", "C1"], ["A2", "C2"], ["A3", "C3"]]),
    ("insert col vs. insert & remove row", 539, [
        ("A", "insertRows", 0, 2), ("A", "insertCols", 0, 2),
        ("A", "setCells", 0, 0, 2, ["A1", "C1", "A2", "C2"]),
        ("A", "removeRows", 1, 1), ("A", "insertCols", 1, 1), ("expect",)], [["A1", U, "C1"]]),
    ("insert row & col vs. insert row and set", 556, [
        ("A", "insertRows", 0, 4), ("A", "insertCols", 0, 4), ("A", "setCells", 0, 0, 4, list(range(16))),
        ("expect",),
        ("A", "insertRows", 0, 1), ("B", "insertRows", 0, 2), ("B", "setCells", 0, 0, 4, ["A", "B", "C", "D"]),
        ("A", "insertCols", 1, 1), ("expect",)], None),
    ("remove rows vs. set cells", 578, [
        ("A", "insertRows", 0, 3), ("A", "insertCols", 0, 2), ("A", "setCells", 0, 0, 2, [0, 1, 2, 3]),
        ("B", "insertRows", 0, 1), ("expect",),
        ("A", "removeRows", 1, 1), ("B", "setCells", 0, 0, 1, ["A", "B", "C"]), ("expect",)], None),
    ("overlapping insert/set vs. remove/insert/set", 596, [
        ("A", "insertRows", 0, 1), ("A", "insertCols", 0, 4), ("A", "setCells", 0, 0, 4, [0, 1, 2, 3]),
        ("expect",),
        ("B", "insertCols", 1, 1), ("B", "setCells", 0, 1, 1, ["A"]),
        ("A", "removeCols", 0, 2), ("A", "insertCols", 0, 1), ("A", "setCells", 0, 0, 1, ["B"]),
        ("expect",)], [["B", "A", 2, 3]]),
]

CLIENT_IDS = {"A": "matrix1-client", "B": "matrix2-client"}


def case_messages(steps):
    """The sequenced messages of one case, in sequence order (see the module docstring)."""
    last = {"A": 0, "B": 0}  # each client's deltaManager.lastSequenceNumber
    msn_table = {}  # MockContainerRuntimeFactory.minSeq (insertion-ordered like a JS Map)
    queue, out = [], []
    seq = 0

    def submit(c, contents):
        ref = last[c]
        msn_table.setdefault(CLIENT_IDS[c], ref)
        queue.append((CLIENT_IDS[c], ref, contents))

    def vec(c, target, kind, pos, count):
        if kind == "insert":
            submit(c, {"pos1": pos, "seg": [count, UNALLOCATED], "type": 0, "target": target})
        else:
            submit(c, {"pos1": pos, "pos2": pos + count, "type": 1, "target": target})

    def set_cell(c, r, col, v):
        contents = {"type": 2, "row": r, "col": col}
        if v is not None:
            contents["value"] = v
        submit(c, contents)

    for st in steps:
        if st[0] == "expect":
            for cid, ref, contents in queue:
                msn_table[cid] = ref
                seq += 1
                out.append({"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                            "minimumSequenceNumber": min(msn_table.values()), "type": "op", "contents": contents})
            queue.clear()
            last = {k: seq for k in last}
            continue
        c, meth, *a = st
        if meth in ("insertCols", "insertRows", "removeCols", "removeRows"):
            vec(c, "cols" if meth.endswith("Cols") else "rows", "insert" if meth.startswith("insert") else "remove",
                a[0], a[1])
        elif meth == "setCell":
            set_cell(c, a[0], a[1], a[2])
        elif meth == "setCells":
            r0, c0, ncols, values = a
            for k, v in enumerate(values):
                set_cell(c, r0 + k // ncols, c0 + k % ncols, v)
        else:
            raise ValueError(meth)
    assert not queue, "a case must end with expect"
    return out


def grid(n_rows, n_cols, get_cell):
    """extract() (matrix/src/test/utils.ts): rows x cols of getCell values, None for undefined."""
    return [[get_cell(r, c) for c in range(n_cols)] for r in range(n_rows)]
