"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes binding of the synthetic op-log generator (oracle/loggen.cpp).

The generator drives the oracle as the observer so that every generated op is valid in its author's
(refSeq, client) perspective; the oracle's final state is the expected result.
"""
import ctypes
import os

from pyoracle import lib as _oracle_lib


class LoggenCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_clients", ctypes.c_int32), ("n_ops", ctypes.c_int32),
                ("lag", ctypes.c_int32), ("initial_len", ctypes.c_int32), ("pct_insert", ctypes.c_int32),
                ("pct_remove", ctypes.c_int32), ("pct_group", ctypes.c_int32),
                ("new_length_calc", ctypes.c_int32), ("min_length", ctypes.c_int32),
                ("annotate_keys", ctypes.c_int32), ("pct_set", ctypes.c_int32), ("max_count", ctypes.c_int32)]


class LoggenDoc(ctypes.Structure):
    _fields_ = [("ops", ctypes.c_void_p), ("n_ops", ctypes.c_uint32), ("n_msgs", ctypes.c_uint32),
                ("text", ctypes.c_void_p), ("n_text", ctypes.c_uint32), ("initial_len", ctypes.c_uint32),
                ("client_writer", ctypes.c_uint16 * 256), ("n_short", ctypes.c_uint32),
                ("checksum", ctypes.c_uint64), ("ops_applied", ctypes.c_uint64),
                ("segs_touched", ctypes.c_uint64), ("final_len", ctypes.c_uint32),
                ("final_segments", ctypes.c_uint32), ("error", ctypes.c_int32), ("digest", ctypes.c_uint64),
                ("summary_fnv", ctypes.c_uint64)]


class LoggenMatrix(ctypes.Structure):
    _fields_ = [("ops", ctypes.c_void_p * 2), ("n_ops", ctypes.c_uint32 * 2), ("n_msgs", ctypes.c_uint32),
                ("n_sets", ctypes.c_uint32), ("client_writer", (ctypes.c_uint16 * 256) * 2),
                ("n_short", ctypes.c_uint32 * 2), ("checksum", ctypes.c_uint64 * 2), ("error", ctypes.c_int32),
                ("digest", ctypes.c_uint64 * 2), ("summary_fnv", ctypes.c_uint64)]


def _lib():
    L = _oracle_lib()
    if not getattr(L, "_loggen_ready", False):
        L.loggen_matrix_generate_batch.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.c_int, ctypes.POINTER(LoggenMatrix)]
        L.loggen_matrix_free.argtypes = [ctypes.POINTER(LoggenMatrix)]
        L.loggen_matrix_cpu_replay.restype = ctypes.c_double
        L.loggen_matrix_cpu_replay.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.POINTER(LoggenMatrix), ctypes.c_uint32,
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]
        L.loggen_generate.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.c_uint32, ctypes.POINTER(LoggenDoc)]
        L.loggen_generate_batch.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_int, ctypes.POINTER(LoggenDoc)]
        L.loggen_free.argtypes = [ctypes.POINTER(LoggenDoc)]
        L.loggen_cpu_summarize.restype = ctypes.c_double
        L.loggen_cpu_summarize.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.POINTER(LoggenDoc), ctypes.c_uint32,
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]
        L.loggen_props_count.argtypes = [ctypes.c_int, ctypes.c_int]
        L.loggen_props_json.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.loggen_cpu_replay.restype = ctypes.c_double
        L.loggen_cpu_replay.argtypes = [ctypes.POINTER(LoggenCfg), ctypes.POINTER(LoggenDoc), ctypes.c_uint32,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int32)]
        L._loggen_ready = True
    return L


def make_cfg(seed=1, n_clients=8, n_ops=1000, lag=128, initial_len=64, pct_insert=50, pct_remove=30,
             pct_group=5, new_length_calc=False, min_length=1, annotate_keys=1, pct_set=40, max_count=8):
    return LoggenCfg(seed, n_clients, n_ops, lag, initial_len, pct_insert, pct_remove, pct_group,
                     int(new_length_calc), min_length, annotate_keys, pct_set, max_count)


class LogBatch:
    """Generated logs for docs [begin, end) (owned C buffers, freed on close)."""

    def __init__(self, cfg, begin, end, threads=None):
        self.cfg = cfg
        self.n = end - begin
        self.docs = (LoggenDoc * self.n)()
        L = _lib()
        threads = threads or min(16, os.cpu_count() or 1)
        rc = L.loggen_generate_batch(ctypes.byref(cfg), begin, end, threads, self.docs)
        if rc != 0:
            raise RuntimeError(f"loggen failed rc={rc}")

    def props_json(self):
        L = _lib()
        n = L.loggen_props_count(self.cfg.n_clients, self.cfg.annotate_keys)
        out = []
        buf = ctypes.create_string_buffer(256)
        for i in range(n):
            k = L.loggen_props_json(self.cfg.n_clients, self.cfg.annotate_keys, i, buf, 256)
            out.append(buf.value.decode() if k > 0 else None)
        return out

    def doc_ops_bytes(self, i):
        d = self.docs[i]
        return ctypes.string_at(d.ops, d.n_ops * 32)

    def doc_text_bytes(self, i):
        d = self.docs[i]
        return ctypes.string_at(d.text, d.n_text * 2)

    def client_ids(self, i):
        d = self.docs[i]
        return ["obs"] + [f"c{d.client_writer[s]}" for s in range(1, d.n_short)]

    def cpu_replay(self, n=None, threads=1):
        L = _lib()
        ck = ctypes.c_uint64()
        err = ctypes.c_int32()
        n = self.n if n is None else n
        secs = L.loggen_cpu_replay(ctypes.byref(self.cfg), self.docs, n, threads, ctypes.byref(ck), ctypes.byref(err))
        return secs, ck.value, err.value

    def cpu_summarize(self, n=None, threads=1):
        """(seconds, mismatches): the oracle's summarizeV1 of the first n documents (replayed beforehand, untimed)
        on `threads` threads, each fingerprint checked against the generator's."""
        bad = ctypes.c_int32()
        n = self.n if n is None else n
        secs = _lib().loggen_cpu_summarize(ctypes.byref(self.cfg), self.docs, n, threads, ctypes.byref(bad))
        return secs, bad.value

    def close(self):
        if self.docs is not None:
            L = _lib()
            for i in range(self.n):
                L.loggen_free(ctypes.byref(self.docs[i]))
            self.docs = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MatrixLogBatch:
    """Generated SharedMatrix logs for matrices [begin, end): per matrix the rows / cols record streams
    (setCell records in both), their client tables and the oracle's final checksums."""

    def __init__(self, cfg, begin, end, threads=None):
        self.cfg = cfg
        self.n = end - begin
        self.mats = (LoggenMatrix * self.n)()
        threads = threads or min(16, os.cpu_count() or 1)
        rc = _lib().loggen_matrix_generate_batch(ctypes.byref(cfg), begin, end, threads, self.mats)
        if rc != 0:
            raise RuntimeError(f"loggen matrix failed rc={rc}")

    def ops_bytes(self, i, v):
        m = self.mats[i]
        return ctypes.string_at(m.ops[v], m.n_ops[v] * 32)

    def intern_values(self, B):
        """A setCell record of message m carries value id m + 1, the id a MatrixBatch gives the JSON text "m"
        when "0", "1", ... are interned first (id 0 = undefined): intern them into B in that order."""
        for k in range(self.cfg.n_ops):
            if B.intern_value(str(k)) != k + 1:
                raise RuntimeError("the batch interned setCell values before the generator's table")

    def client_ids(self, i, v):
        m = self.mats[i]
        return ["obs"] + [f"c{m.client_writer[v][s]}" for s in range(1, m.n_short[v])]

    def cpu_replay(self, n=None, threads=1):
        bad = ctypes.c_int32()
        n = self.n if n is None else n
        secs = _lib().loggen_matrix_cpu_replay(ctypes.byref(self.cfg), self.mats, n, threads, ctypes.byref(bad))
        return secs, bad.value

    def close(self):
        if self.mats is not None:
            L = _lib()
            for i in range(self.n):
                L.loggen_matrix_free(ctypes.byref(self.mats[i]))
            self.mats = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _cache_key(cfg, begin, end):
    f = [getattr(cfg, n) for n, _ in LoggenCfg._fields_]
    return "logs_" + "_".join(str(int(x)) for x in f) + f"_{begin}_{end}.npz"


def cached_log_batch(cfg, begin, end, threads=None, cache_dir=None):
    """LogBatch for docs [begin, end), reused from `cache_dir` (env MTB_LOG_CACHE) when a run with the same
    config already generated it: profiling child runs of bench.py replay the same 10^8 ops without paying
    the generator again.  Without a cache dir this is LogBatch."""
    cache_dir = cache_dir if cache_dir is not None else os.environ.get("MTB_LOG_CACHE")
    if not cache_dir:
        return LogBatch(cfg, begin, end, threads)
    path = os.path.join(cache_dir, _cache_key(cfg, begin, end))
    if os.path.exists(path):
        return LoadedLogBatch(cfg, path)
    lb = LogBatch(cfg, begin, end, threads)
    os.makedirs(cache_dir, exist_ok=True)
    lb.save(path + ".tmp.npz")
    os.replace(path + ".tmp.npz", path)
    return lb


def _save(self, path):
    import numpy as np
    n = self.n
    meta = np.frombuffer(ctypes.string_at(ctypes.addressof(self.docs), ctypes.sizeof(self.docs)), dtype=np.uint8)
    ops = b"".join(self.doc_ops_bytes(i) for i in range(n))
    text = b"".join(self.doc_text_bytes(i) for i in range(n))
    np.savez(path, meta=meta, ops=np.frombuffer(ops, dtype=np.uint8), text=np.frombuffer(text, dtype=np.uint8))


LogBatch.save = _save


class LoadedLogBatch(LogBatch):
    """A LogBatch read back from LogBatch.save: the C records point into numpy buffers this object owns."""

    def __init__(self, cfg, path):
        import numpy as np
        self.cfg = cfg
        z = np.load(path)
        meta = z["meta"]
        self.n = meta.size // ctypes.sizeof(LoggenDoc)
        self.docs = (LoggenDoc * self.n).from_buffer_copy(meta.tobytes())
        self._ops = np.ascontiguousarray(z["ops"])
        self._text = np.ascontiguousarray(z["text"])
        po, pt = self._ops.ctypes.data, self._text.ctypes.data
        for i in range(self.n):
            d = self.docs[i]
            d.ops, d.text = po, pt
            po += d.n_ops * 32
            pt += d.n_text * 2

    def close(self):
        self.docs = None
