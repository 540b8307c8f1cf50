"""Host JSON quoting: the UTF-8 fast path of the summary serializers (hjson.hpp quote_utf8 / quote_u8) gives
the bytes JSON.stringify-style quote(from_utf8(u)) gives, for random well-formed and ill-formed inputs (lone
surrogates, controls, astral characters, invalid bytes).  Compiled with g++ from the header alone."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include <cstdio>
#include <random>
#include "hjson.hpp"
int main() {
  std::mt19937 rng(7);
  const char16_t pick[] = {u'a', u'"', u'\\', u'\n', 0x01, 0x1f, 0x7f, 0xe9, 0x20ac, 0xd83d, 0xde00, 0xdc00, 0xffff, u' '};
  int fast = 0;
  for (int t = 0; t < 20000; t++) {
    std::u16string s;
    const int n = rng() % 24;
    for (int k = 0; k < n; k++) s.push_back(pick[rng() % (sizeof pick / sizeof pick[0])]);
    std::string u = hj::to_utf8(s.data(), s.size());
    if (rng() % 8 == 0 && !u.empty()) u[rng() % u.size()] = (char)(0x80 + rng() % 0x80);  // ill-formed bytes
    std::string a, b;
    hj::quote(a, hj::from_utf8(u));
    fast += hj::quote_utf8(b, u);
    std::string c;
    hj::quote_u8(c, u);
    if (!(b.empty() || a == b) || a != c) { printf("mismatch at %d\n", t); return 1; }
  }
  printf("ok %d\n", fast);
  return 0;
}
'''


def test_quote_utf8_equals_the_utf16_round_trip(tmp_path):
    src = tmp_path / "q.cpp"
    src.write_text(SRC)
    exe = tmp_path / "q"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "fluidframework_amd", "csrc"),
                           str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert int(out.stdout.split()[1]) > 2000  # (the fast path took the well-formed inputs)
