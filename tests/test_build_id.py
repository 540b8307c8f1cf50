"""build() trusts a prebuilt libmtb.so only when the source hash embedded in it equals the hash of the tree's
sources, headers and flags: a stale or foreign library is rebuilt whatever its mtime."""
import ctypes
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fluidframework_amd import build as b  # noqa: E402


def test_built_library_carries_the_tree_hash():
    assert b.embedded_id(b.OUT) == b.source_id(), "libmtb.so was not built from this tree (run build())"
    assert not b.needs_build()


def test_stale_or_foreign_library_needs_a_rebuild(tmp_path):
    stale = tmp_path / "libmtb.so"
    shutil.copy(b.OUT, stale)
    data = bytearray(stale.read_bytes())
    i = data.find(b.BUILD_ID_TAG) + len(b.BUILD_ID_TAG)
    data[i:i + 64] = b"0" * 64  # a library built from other sources
    stale.write_bytes(bytes(data))
    os.utime(stale, (2**31, 2**31))  # and newer than every source: mtime must not matter
    assert b.needs_build(out=str(stale))
    nohash = tmp_path / "old.so"
    nohash.write_bytes(b"\x7fELF prebuilt without a hash")
    assert b.needs_build(out=str(nohash))
    assert b.needs_build(out=str(tmp_path / "missing.so"))


def test_hash_follows_sources_and_flags():
    assert b.source_id() != b.source_id(defines=["MTB_PROFILE"])


def test_library_reports_its_build_id():
    L = ctypes.CDLL(b.OUT)
    L.mtb_build_id.restype = ctypes.c_char_p
    assert L.mtb_build_id().decode() == b.source_id()
