// ORACLE / TEST INFRASTRUCTURE ONLY.
// JSON value model used by the CPU oracle (oracle/mt_oracle.cpp).  It restates the parts of
// V8's JSON.parse / JSON.stringify and of JS object-key ordering that the merge-tree reference
// relies on for properties and summaries:
//   - property enumeration order: array-index keys ascending, then string keys in insertion
//     order (packages/dds/merge-tree/src/properties.ts:165 createMap = Object.create(null));
//   - JSON.stringify string escaping (well-formed stringify, lone surrogates -> \udXXX);
//   - Number::toString for numbers;
//   - matchProperties (properties.ts:71-96).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use the oracle.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace orc {

using u16str = std::u16string;

struct JVal;
using JObj = std::vector<std::pair<u16str, JVal>>;

struct JVal {
  enum T : uint8_t { Undef, Null, False, True, Num, Str, Arr, Obj } t = Undef;
  double num = 0;
  u16str str;
  std::vector<JVal> arr;
  JObj obj;
  static JVal undef() { return JVal(); }
  static JVal null() { JVal v; v.t = Null; return v; }
  static JVal boolean(bool b) { JVal v; v.t = b ? True : False; return v; }
  static JVal number(double d) { JVal v; v.t = Num; v.num = d; return v; }
  static JVal string(u16str s) { JVal v; v.t = Str; v.str = std::move(s); return v; }
  bool isObjectLike() const { return t == Obj || t == Arr; }
  bool isUndef() const { return t == Undef; }
};

// ---------------------------------------------------------------- UTF helpers
inline u16str utf8_to_u16(const char* s, size_t n) {
  u16str out;
  out.reserve(n);
  size_t i = 0;
  while (i < n) {
    uint8_t c = (uint8_t)s[i];
    uint32_t cp;
    int extra;
    if (c < 0x80) { cp = c; extra = 0; }
    else if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; extra = 1; }
    else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; extra = 2; }
    else { cp = c & 0x07; extra = 3; }
    if (i + extra >= n + (extra ? 0 : 1)) { /* truncated */ }
    for (int k = 1; k <= extra && i + k < n; k++) cp = (cp << 6) | ((uint8_t)s[i + k] & 0x3F);
    i += 1 + extra;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back((char16_t)(0xD800 + (cp >> 10)));
      out.push_back((char16_t)(0xDC00 + (cp & 0x3FF)));
    } else {
      out.push_back((char16_t)cp);
    }
  }
  return out;
}
inline u16str utf8_to_u16(const std::string& s) { return utf8_to_u16(s.data(), s.size()); }

inline void append_utf8_cp(std::string& out, uint32_t cp) {
  if (cp < 0x80) out.push_back((char)cp);
  else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// UTF-16 -> UTF-8 (lone surrogates encoded as 3-byte sequences; callers that need valid UTF-8
// escape them first, as JSON.stringify does).
inline std::string u16_to_utf8(const u16str& s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); i++) {
    uint32_t c = s[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
      append_utf8_cp(out, cp);
      i++;
    } else {
      append_utf8_cp(out, c);
    }
  }
  return out;
}

// ---------------------------------------------------------------- JS key order
// ECMAScript array index: canonical uint32 string < 2^32-1.
inline bool is_array_index(const u16str& k, uint32_t* val = nullptr) {
  if (k.empty() || k.size() > 10) return false;
  if (k.size() > 1 && k[0] == u'0') return false;
  uint64_t v = 0;
  for (char16_t c : k) {
    if (c < u'0' || c > u'9') return false;
    v = v * 10 + (c - u'0');
  }
  if (v >= 4294967295ull) return false;
  if (val) *val = (uint32_t)v;
  return true;
}

// Set key in a JS-ordered property list (existing key keeps its slot).
inline void obj_set(JObj& o, const u16str& k, JVal v) {
  for (auto& kv : o) {
    if (kv.first == k) { kv.second = std::move(v); return; }
  }
  uint32_t idx;
  if (is_array_index(k, &idx)) {
    size_t pos = 0;
    for (; pos < o.size(); pos++) {
      uint32_t other;
      if (!is_array_index(o[pos].first, &other) || other > idx) break;
    }
    o.insert(o.begin() + pos, {k, std::move(v)});
  } else {
    o.push_back({k, std::move(v)});
  }
}
inline bool obj_del(JObj& o, const u16str& k) {
  for (size_t i = 0; i < o.size(); i++) {
    if (o[i].first == k) { o.erase(o.begin() + i); return true; }
  }
  return false;
}
inline const JVal* obj_get(const JObj& o, const u16str& k) {
  for (auto& kv : o)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

// ---------------------------------------------------------------- parser
struct JParser {
  const char* p;
  const char* e;
  explicit JParser(const char* s, size_t n) : p(s), e(s + n) {}
  [[noreturn]] void fail(const char* why) { throw std::runtime_error(std::string("JSON parse error: ") + why); }
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) >= n && memcmp(p, s, n) == 0) { p += n; return true; }
    return false;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  u16str str() {
    if (p >= e || *p != '"') fail("expected string");
    p++;
    u16str out;
    const char* runStart = p;
    auto flush = [&](const char* upto) {
      if (upto > runStart) {
        u16str t = utf8_to_u16(runStart, upto - runStart);
        out += t;
      }
    };
    while (true) {
      if (p >= e) fail("unterminated string");
      char c = *p;
      if (c == '"') { flush(p); p++; break; }
      if (c == '\\') {
        flush(p);
        p++;
        if (p >= e) fail("bad escape");
        char x = *p++;
        switch (x) {
          case '"': out.push_back(u'"'); break;
          case '\\': out.push_back(u'\\'); break;
          case '/': out.push_back(u'/'); break;
          case 'b': out.push_back(u'\b'); break;
          case 'f': out.push_back(u'\f'); break;
          case 'n': out.push_back(u'\n'); break;
          case 'r': out.push_back(u'\r'); break;
          case 't': out.push_back(u'\t'); break;
          case 'u': {
            if (e - p < 4) fail("bad \\u");
            int v = 0;
            for (int k = 0; k < 4; k++) {
              int h = hexv(p[k]);
              if (h < 0) fail("bad hex");
              v = v * 16 + h;
            }
            p += 4;
            out.push_back((char16_t)v);
            break;
          }
          default: fail("bad escape char");
        }
        runStart = p;
        continue;
      }
      p++;
    }
    return out;
  }
  JVal value() {
    ws();
    if (p >= e) fail("unexpected end");
    char c = *p;
    if (c == '{') {
      p++;
      JVal v; v.t = JVal::Obj;
      ws();
      if (p < e && *p == '}') { p++; return v; }
      while (true) {
        ws();
        u16str k = str();
        ws();
        if (p >= e || *p != ':') fail("expected :");
        p++;
        JVal x = value();
        obj_set(v.obj, k, std::move(x));  // duplicate keys: last wins, first position kept
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') { p++; break; }
        fail("expected , or }");
      }
      return v;
    }
    if (c == '[') {
      p++;
      JVal v; v.t = JVal::Arr;
      ws();
      if (p < e && *p == ']') { p++; return v; }
      while (true) {
        v.arr.push_back(value());
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; break; }
        fail("expected , or ]");
      }
      return v;
    }
    if (c == '"') return JVal::string(str());
    if (lit("true")) return JVal::boolean(true);
    if (lit("false")) return JVal::boolean(false);
    if (lit("null")) return JVal::null();
    // number
    const char* s = p;
    if (p < e && (*p == '-' || *p == '+')) p++;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) p++;
    if (p == s) fail("unexpected char");
    std::string num(s, p - s);
    return JVal::number(strtod(num.c_str(), nullptr));
  }
};

inline JVal json_parse(const char* s, size_t n) {
  JParser ps(s, n);
  JVal v = ps.value();
  ps.ws();
  if (ps.p != ps.e) ps.fail("trailing characters");
  return v;
}
inline JVal json_parse(const std::string& s) { return json_parse(s.data(), s.size()); }

// ---------------------------------------------------------------- stringify (V8 semantics)
inline std::string js_number_to_string(double x) {
  if (std::isnan(x)) return "NaN";
  if (x == 0) return "0";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  std::string sign;
  if (x < 0) { sign = "-"; x = -x; }
  char buf[64];
  int prec = 1;
  for (; prec <= 17; prec++) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, x);
    if (strtod(buf, nullptr) == x) break;
  }
  // buf = d[.ddd]e[+-]XX
  std::string digits;
  const char* q = buf;
  while (*q && *q != 'e') { if (*q != '.') digits.push_back(*q); q++; }
  int exp10 = atoi(q + 1);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  int k = (int)digits.size();
  int n = exp10 + 1;
  std::string out;
  if (k <= n && n <= 21) {
    out = digits + std::string(n - k, '0');
  } else if (0 < n && n <= 21) {
    out = digits.substr(0, n) + "." + digits.substr(n);
  } else if (-6 < n && n <= 0) {
    out = "0." + std::string(-n, '0') + digits;
  } else {
    int e = n - 1;
    std::string es = (e >= 0 ? "+" : "-") + std::to_string(std::abs(e));
    if (k == 1) out = digits + "e" + es;
    else out = digits.substr(0, 1) + "." + digits.substr(1) + "e" + es;
  }
  return sign + out;
}

inline void json_quote(std::string& out, const u16str& s) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  for (size_t i = 0; i < s.size(); i++) {
    uint32_t c = s[i];
    switch (c) {
      case '"': out += "\\\""; continue;
      case '\\': out += "\\\\"; continue;
      case '\b': out += "\\b"; continue;
      case '\f': out += "\\f"; continue;
      case '\n': out += "\\n"; continue;
      case '\r': out += "\\r"; continue;
      case '\t': out += "\\t"; continue;
      default: break;
    }
    if (c < 0x20) {
      out += "\\u00";
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    } else if (c >= 0xD800 && c <= 0xDBFF) {
      if (i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
        uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
        append_utf8_cp(out, cp);
        i++;
      } else {
        out += "\\u";
        for (int sh = 12; sh >= 0; sh -= 4) out.push_back(hex[(c >> sh) & 15]);
      }
    } else if (c >= 0xDC00 && c <= 0xDFFF) {
      out += "\\u";
      for (int sh = 12; sh >= 0; sh -= 4) out.push_back(hex[(c >> sh) & 15]);
    } else {
      append_utf8_cp(out, c);
    }
  }
  out.push_back('"');
}

inline void json_stringify_to(std::string& out, const JVal& v) {
  switch (v.t) {
    case JVal::Undef: out += "null"; break;  // only reached inside arrays
    case JVal::Null: out += "null"; break;
    case JVal::False: out += "false"; break;
    case JVal::True: out += "true"; break;
    case JVal::Num:
      if (!std::isfinite(v.num)) out += "null";
      else out += js_number_to_string(v.num);
      break;
    case JVal::Str: json_quote(out, v.str); break;
    case JVal::Arr: {
      out.push_back('[');
      for (size_t i = 0; i < v.arr.size(); i++) {
        if (i) out.push_back(',');
        json_stringify_to(out, v.arr[i]);
      }
      out.push_back(']');
      break;
    }
    case JVal::Obj: {
      out.push_back('{');
      bool first = true;
      for (auto& kv : v.obj) {
        if (kv.second.t == JVal::Undef) continue;
        if (!first) out.push_back(',');
        first = false;
        json_quote(out, kv.first);
        out.push_back(':');
        json_stringify_to(out, kv.second);
      }
      out.push_back('}');
      break;
    }
  }
}
inline std::string json_stringify(const JVal& v) {
  std::string s;
  json_stringify_to(s, v);
  return s;
}

// ---------------------------------------------------------------- matchProperties (properties.ts:71)
inline bool js_falsy(const JVal* v) {
  if (!v) return true;
  switch (v->t) {
    case JVal::Undef: case JVal::Null: case JVal::False: return true;
    case JVal::Num: return v->num == 0 || std::isnan(v->num);
    case JVal::Str: return v->str.empty();
    default: return false;
  }
}
// Object.keys(x) for a JSON value (strings expose their index keys).
inline std::vector<u16str> js_keys(const JVal* v) {
  std::vector<u16str> ks;
  if (!v) return ks;
  if (v->t == JVal::Obj) for (auto& kv : v->obj) ks.push_back(kv.first);
  else if (v->t == JVal::Arr) for (size_t i = 0; i < v->arr.size(); i++) { std::string s = std::to_string(i); ks.push_back(u16str(s.begin(), s.end())); }
  else if (v->t == JVal::Str) for (size_t i = 0; i < v->str.size(); i++) { std::string s = std::to_string(i); ks.push_back(u16str(s.begin(), s.end())); }
  return ks;
}
// x[key] for a JSON value; returns Undef holder when absent.  `tmp` stores a synthesized value.
inline const JVal* js_get(const JVal* v, const u16str& k, JVal& tmp) {
  if (!v) return nullptr;
  if (v->t == JVal::Obj) return obj_get(v->obj, k);
  uint32_t idx;
  if (v->t == JVal::Arr && is_array_index(k, &idx)) return idx < v->arr.size() ? &v->arr[idx] : nullptr;
  if (v->t == JVal::Str && is_array_index(k, &idx)) {
    if (idx < v->str.size()) { tmp = JVal::string(u16str(1, v->str[idx])); return &tmp; }
    return nullptr;
  }
  return nullptr;
}
inline bool js_strict_equal(const JVal* a, const JVal* b) {
  bool au = !a || a->t == JVal::Undef, bu = !b || b->t == JVal::Undef;
  if (au || bu) return au && bu;
  if (a->t == JVal::True || a->t == JVal::False || b->t == JVal::True || b->t == JVal::False) return a->t == b->t;
  if (a->t != b->t) return false;
  switch (a->t) {
    case JVal::Null: return true;
    case JVal::Num: return a->num == b->num;  // NaN != NaN, 0 === -0
    case JVal::Str: return a->str == b->str;
    default: return a == b;  // object identity
  }
}
inline bool match_properties(const JVal* a, const JVal* b) {
  if (js_falsy(a) && js_falsy(b)) return true;
  auto ka = js_keys(a);
  auto kb = js_keys(b);
  if (ka.size() != kb.size()) return false;
  for (auto& k : ka) {
    JVal tb, ta;
    const JVal* bv = js_get(b, k, tb);
    if (!bv || bv->t == JVal::Undef) return false;
    const JVal* av = js_get(a, k, ta);
    if (bv->t == JVal::Obj || bv->t == JVal::Arr || bv->t == JVal::Null) {
      if (!match_properties(av, bv)) return false;
    } else if (!js_strict_equal(bv, av)) {
      return false;
    }
  }
  return true;
}

}  // namespace orc
