"""Debug: find the first body segment whose load makes the engine differ from the oracle (prefixes of a
summary's body), for the long-document phantom test's documents.  usage: dbg_phantom.py new_mode chunk i"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from helpers import make_tail_log  # noqa: E402
from pyoracle import OracleDoc  # noqa: E402
from fluidframework_amd import MergeTreeBatch  # noqa: E402

new_mode = sys.argv[1] == "1"
chunk = int(sys.argv[2])
i = int(sys.argv[3])
only_mismatch = len(sys.argv) > 4 and sys.argv[4] == "mismatch"
if len(sys.argv) > 4 and sys.argv[4] == "tail":  # test_gpu_phantom._tail_summary(500 + i, ...)
    from test_gpu_phantom import _tail_summary
    blobs = _tail_summary(500 + i, 120 + 20 * i, 60 + 5 * i, 100 + 10 * (i % 5))
else:
    text, msgs = make_tail_log(900 + i + 50 * int(new_mode), 1600, lag=24 + 8 * (i % 8), initial_len=9990, lo=9990,
                               new_mode=new_mode, inserters=[0])
    cut = len(msgs) // 2 + 37 * (i % 8)
    a = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
    a.insert_text_local(0, text)
    a.start_collab("obs")
    for m in msgs[:cut]:
        a.apply_msg(m)
    blobs = [list(x) for x in a.summarize_v1()["blobs"]]


def compact(dump):
    out = []
    for line in dump.splitlines():
        try:
            r = json.loads(line)
        except Exception:
            out.append(line[:200])
            continue
        if isinstance(r, list):
            r[2] = r[2][:8] if isinstance(r[2], str) else r[2]
            out.append(json.dumps(r))
        else:
            out.append(line[:200])
    return "\n".join(out)
hdr = json.loads(blobs[0][1])
body = [s for p, c in blobs[1:] for s in json.loads(c)["segments"]]
print("header segments", len(hdr["segments"]), "body segments", len(body), flush=True)


def seglen(s):
    j = s["json"] if isinstance(s, dict) and "json" in s else s
    if isinstance(j, str):
        return len(j)
    if "text" in j:
        return len(j["text"])
    return 1


def prefix(k):
    h = dict(hdr)
    md = dict(h["headerMetadata"])
    b = body[:k]
    md["orderedChunkMetadata"] = [{"id": "header"}] + ([{"id": "body_0"}] if b else [])
    md["totalLength"] = h["length"] + sum(seglen(s) for s in b)
    md["totalSegmentCount"] = len(h["segments"]) + len(b)
    h["headerMetadata"] = md
    out = [["header", json.dumps(h)]]
    if b:
        out.append(["body_0", json.dumps({"version": "1", "segmentCount": len(b), "length": sum(seglen(s) for s in b),
                                           "segments": b, "startIndex": len(hdr["segments"])})])
    return out


def outcome(bl):
    o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
    try:
        o.load_v1(bl, "loader")
        o.get_text()
        r = "ok"
    except Exception as e:
        r = "fail"
    oo = "stale" if o.stale_updates() else r
    B = MergeTreeBatch(1, new_length_calc=new_mode, chunk_size=chunk)
    try:
        B[0].load(bl, "loader")
        B.flush()
        g = "ok"
    except Exception as e:
        g = "stale" if "stale" in str(e) else "fail"
    return oo, g


if only_mismatch:
    oo, g = outcome(blobs)
    print("doc", i, "oracle", oo, "engine", g, flush=True)
    if oo == g:
        sys.exit(0)
    for k in range(0, len(body) + 1):
        oo, g = outcome(prefix(k))
        if oo != g:
            print("first outcome difference at body prefix", k, "oracle", oo, "engine", g)
            print("segment", json.dumps(body[k - 1]) if k else None)
            print("previous", [json.dumps(s)[:100] for s in body[max(0, k - 6):k - 1]])
            break
    sys.exit(0)

for k in range(0, len(body) + 1):
    bl = prefix(k)
    o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
    try:
        o.load_v1(bl, "loader")
        od = o.dump_segments()
    except Exception as e:
        od = "FAIL " + str(e)
    B = MergeTreeBatch(1, new_length_calc=new_mode, chunk_size=chunk)
    try:
        B[0].load(bl, "loader")
        B.flush()
        gd = B.dump_segments(0)
    except Exception as e:
        gd = "FAIL " + str(e)
    if od != gd:
        print("first difference at body prefix", k, "segment", json.dumps(body[k - 1]) if k else None)
        print("previous segments", [json.dumps(s)[:80] for s in body[max(0, k - 4):k - 1]])
        print("--- oracle\n" + compact(od))
        print("--- engine\n" + compact(gd))
        pk = prefix(k - 1)
        o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
        o.load_v1(pk, "loader")
        print("--- oracle at k-1\n" + compact(o.dump_segments()))
        break
else:
    print("no difference over", len(body), "prefixes")
