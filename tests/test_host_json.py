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


# JSON.stringify quoting of a UTF-16 string, one code unit at a time: the straightforward form the pointer-writing
# hj::quote16 must reproduce byte for byte (and its ASCII flag: every unit below 0x80)
SRC16 = r'''
#include <cstdio>
#include <random>
#include "hjson.hpp"
static void ref_quote(std::string& o, const char16_t* s, size_t n) {
  static const char kHex[] = "0123456789abcdef";
  o += '"';
  for (size_t i = 0; i < n; i++) {
    const uint32_t c = s[i];
    if (c == 0x22) { o += "\\\""; continue; }
    if (c == 0x5C) { o += "\\\\"; continue; }
    if (c == 0x08) { o += "\\b"; continue; }
    if (c == 0x0C) { o += "\\f"; continue; }
    if (c == 0x0A) { o += "\\n"; continue; }
    if (c == 0x0D) { o += "\\r"; continue; }
    if (c == 0x09) { o += "\\t"; continue; }
    const bool lead = c >= 0xD800 && c < 0xDC00, trail = c >= 0xDC00 && c < 0xE000;
    if (lead && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
      hj::put_utf8(o, 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00));
      i++;
    } else if (c < 0x20 || lead || trail) {
      o += "\\u";
      o += kHex[(c >> 12) & 15]; o += kHex[(c >> 8) & 15]; o += kHex[(c >> 4) & 15]; o += kHex[c & 15];
    } else {
      hj::put_utf8(o, c);
    }
  }
  o += '"';
}
int main() {
  std::mt19937 rng(11);
  const char16_t pick[] = {u'a', u'"', u'\\', u'\n', u'\t', 0x01, 0x1f, 0x7f, 0xe9, 0x20ac, 0xd83d, 0xde00, 0xdc00, 0xffff, u' ', u'z'};
  for (int t = 0; t < 20000; t++) {
    std::u16string s;
    const int n = t % 50 == 0 ? 3000 + (int)(rng() % 3000) : (int)(rng() % 40);
    const int alphabet = t % 3 == 0 ? 2 : (int)(sizeof pick / sizeof pick[0]);
    for (int k = 0; k < n; k++) s.push_back(pick[rng() % alphabet]);
    std::string pre(rng() % 20, 'x');
    std::string a = pre, b = pre;
    ref_quote(a, s.data(), s.size());
    const bool ascii = hj::quote16(b, s.data(), s.size());
    bool want = true;
    for (char16_t c : s) want = want && c < 0x80;
    if (a != b || ascii != want) { printf("mismatch at %d\n", t); return 1; }
    std::string c = pre, d = pre;  // and the UTF-8 path against the round trip, with a prefix and long inputs
    const std::string u = hj::to_utf8(s.data(), s.size());
    hj::quote(c, hj::from_utf8(u));
    hj::quote_u8(d, u);
    if (c != d) { printf("u8 mismatch at %d\n", t); return 1; }
  }
  printf("ok\n");
  return 0;
}
'''


def test_quote16_equals_the_unit_by_unit_form(tmp_path):
    src = tmp_path / "q16.cpp"
    src.write_text(SRC16)
    exe = tmp_path / "q16"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "fluidframework_amd", "csrc"),
                           str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr


def test_quote_utf8_equals_the_utf16_round_trip(tmp_path):
    src = tmp_path / "q.cpp"
    src.write_text(SRC)
    exe = tmp_path / "q"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "fluidframework_amd", "csrc"),
                           str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert int(out.stdout.split()[1]) > 2000  # (the fast path took the well-formed inputs)
