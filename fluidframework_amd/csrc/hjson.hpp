// Host-side JSON for the replay engine: parse ISequencedDocumentMessage / props JSON into a small
// DOM with JavaScript property order, and serialize with V8 JSON.stringify semantics (needed for
// byte-identical SnapshotV1 blobs, snapshotV1.ts:122 -> serializer.stringify).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace hj {

using U16 = std::u16string;

struct Value {
  enum Kind : uint8_t { kUndef, kNull, kBool, kNum, kStr, kArr, kObj } kind = kUndef;
  bool b = false;
  double n = 0;
  U16 s;
  std::vector<Value> items;                      // array elements
  std::vector<std::pair<U16, Value>> members;    // object members in JS enumeration order
  const Value* find(const char16_t* k) const {
    for (auto& m : members)
      if (m.first == k) return &m.second;
    return nullptr;
  }
  bool truthy() const {
    switch (kind) {
      case kUndef: case kNull: return false;
      case kBool: return b;
      case kNum: return n != 0 && !std::isnan(n);
      case kStr: return !s.empty();
      default: return true;
    }
  }
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// canonical array index (ECMAScript): "0".."4294967294" without leading zeros
inline bool array_index(const U16& k, uint32_t* out) {
  if (k.empty() || k.size() > 10 || (k.size() > 1 && k[0] == u'0')) return false;
  uint64_t v = 0;
  for (char16_t c : k) {
    if (c < u'0' || c > u'9') return false;
    v = v * 10 + (uint64_t)(c - u'0');
  }
  if (v > 4294967294ull) return false;
  if (out) *out = (uint32_t)v;
  return true;
}

// [[Set]] on an ordinary object: existing keys keep their slot; new integer keys sort first.
inline void put(std::vector<std::pair<U16, Value>>& m, const U16& k, Value v) {
  for (auto& e : m)
    if (e.first == k) { e.second = std::move(v); return; }
  uint32_t ki;
  if (!array_index(k, &ki)) { m.emplace_back(k, std::move(v)); return; }
  size_t at = 0;
  uint32_t other;
  while (at < m.size() && array_index(m[at].first, &other) && other < ki) at++;
  m.insert(m.begin() + at, {k, std::move(v)});
}

class Reader {
 public:
  Reader(const char* p, size_t n) : p_(p), end_(p + n) {}
  Value document() {
    Value v = value();
    skip();
    if (p_ != end_) throw ParseError("trailing data");
    return v;
  }

 private:
  const char* p_;
  const char* end_;
  void skip() { while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_; }
  char peek() { if (p_ >= end_) throw ParseError("unexpected end"); return *p_; }
  void expect(char c) { if (peek() != c) throw ParseError(std::string("expected ") + c); ++p_; }
  static uint32_t decode_utf8(const char*& p, const char* end) {
    const uint8_t c0 = (uint8_t)*p++;
    if (c0 < 0x80) return c0;
    int n = c0 >= 0xF0 ? 3 : c0 >= 0xE0 ? 2 : 1;
    uint32_t cp = c0 & (0x3F >> n);
    while (n-- > 0 && p < end) cp = (cp << 6) | ((uint8_t)*p++ & 0x3F);
    return cp;
  }
  U16 string() {
    expect('"');
    U16 out;
    while (true) {
      if (p_ >= end_) throw ParseError("unterminated string");
      const char c = *p_;
      if (c == '"') { ++p_; return out; }
      if (c != '\\') {
        uint32_t cp = decode_utf8(p_, end_);
        if (cp >= 0x10000) {
          cp -= 0x10000;
          out.push_back((char16_t)(0xD800 | (cp >> 10)));
          out.push_back((char16_t)(0xDC00 | (cp & 0x3FF)));
        } else {
          out.push_back((char16_t)cp);
        }
        continue;
      }
      ++p_;
      const char e = peek();
      ++p_;
      switch (e) {
        case 'b': out.push_back(u'\b'); break;
        case 'f': out.push_back(u'\f'); break;
        case 'n': out.push_back(u'\n'); break;
        case 'r': out.push_back(u'\r'); break;
        case 't': out.push_back(u'\t'); break;
        case 'u': {
          if (end_ - p_ < 4) throw ParseError("short \\u escape");
          uint32_t v = 0;
          for (int i = 0; i < 4; i++) {
            const char h = *p_++;
            v <<= 4;
            if (h >= '0' && h <= '9') v |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') v |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') v |= (uint32_t)(h - 'A' + 10);
            else throw ParseError("bad hex digit");
          }
          out.push_back((char16_t)v);
          break;
        }
        default: out.push_back((char16_t)(uint8_t)e); break;  // \" \\ \/
      }
    }
  }
  Value value() {
    skip();
    Value v;
    const char c = peek();
    if (c == '{') {
      ++p_;
      v.kind = Value::kObj;
      skip();
      if (peek() == '}') { ++p_; return v; }
      while (true) {
        skip();
        U16 k = string();
        skip();
        expect(':');
        Value x = value();
        put(v.members, k, std::move(x));
        skip();
        if (peek() == ',') { ++p_; continue; }
        expect('}');
        return v;
      }
    }
    if (c == '[') {
      ++p_;
      v.kind = Value::kArr;
      skip();
      if (peek() == ']') { ++p_; return v; }
      while (true) {
        v.items.push_back(value());
        skip();
        if (peek() == ',') { ++p_; continue; }
        expect(']');
        return v;
      }
    }
    if (c == '"') { v.kind = Value::kStr; v.s = string(); return v; }
    auto word = [&](const char* w) {
      const size_t n = strlen(w);
      if ((size_t)(end_ - p_) < n || memcmp(p_, w, n) != 0) throw ParseError("bad literal");
      p_ += n;
    };
    if (c == 't') { word("true"); v.kind = Value::kBool; v.b = true; return v; }
    if (c == 'f') { word("false"); v.kind = Value::kBool; v.b = false; return v; }
    if (c == 'n') { word("null"); v.kind = Value::kNull; return v; }
    const char* s = p_;
    while (p_ < end_ && strchr("+-0123456789.eE", *p_)) ++p_;
    if (s == p_) throw ParseError("unexpected character");
    v.kind = Value::kNum;
    v.n = strtod(std::string(s, p_).c_str(), nullptr);
    return v;
  }
};

inline Value parse(const char* p, size_t n) { return Reader(p, n).document(); }

// ------------------------------------------------------------------ serialization
inline void put_utf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) { o += (char)cp; return; }
  if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); return; }
  if (cp < 0x10000) {
    o += (char)(0xE0 | (cp >> 12));
    o += (char)(0x80 | ((cp >> 6) & 0x3F));
    o += (char)(0x80 | (cp & 0x3F));
    return;
  }
  o += (char)(0xF0 | (cp >> 18));
  o += (char)(0x80 | ((cp >> 12) & 0x3F));
  o += (char)(0x80 | ((cp >> 6) & 0x3F));
  o += (char)(0x80 | (cp & 0x3F));
}

inline std::string to_utf8(const char16_t* s, size_t n) {
  std::string o;
  o.reserve(n);
  for (size_t i = 0; i < n; i++) {
    uint32_t c = s[i];
    if (c >= 0xD800 && c < 0xDC00 && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
      c = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
      i++;
    }
    put_utf8(o, c);
  }
  return o;
}

inline U16 from_utf8(const std::string& s) {
  U16 out;
  const char* p = s.data();
  const char* e = p + s.size();
  while (p < e) {
    const uint8_t c0 = (uint8_t)*p++;
    uint32_t cp = c0;
    if (c0 >= 0x80) {
      int n = c0 >= 0xF0 ? 3 : c0 >= 0xE0 ? 2 : 1;
      cp = c0 & (0x3F >> n);
      while (n-- > 0 && p < e) cp = (cp << 6) | ((uint8_t)*p++ & 0x3F);
    }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back((char16_t)(0xD800 | (cp >> 10)));
      out.push_back((char16_t)(0xDC00 | (cp & 0x3FF)));
    } else {
      out.push_back((char16_t)cp);
    }
  }
  return out;
}

// JSON.stringify string quoting (well-formed: lone surrogates escaped as \udXXX).  Writes through a pointer into
// room made up front: before unit i the string holds at least (n - i) + 1 unwritten bytes (one per remaining
// unit plus the closing quote), and an escape makes room for its own expansion.  Returns whether every unit was
// below 0x80 (the output is then ASCII).
inline bool quote16(std::string& o, const char16_t* s, size_t n) {
  static const char kHex[] = "0123456789abcdef";
  size_t at = o.size();
  o.resize(at + n + 18);
  char* w = &o[0];
  w[at++] = '"';
  bool ascii = true;
  for (size_t i = 0; i < n; i++) {
    const uint32_t c = s[i];
    if (c >= 0x20 && c < 0x80 && c != 0x22 && c != 0x5C) {  // (the common case first)
      w[at++] = (char)c;
      continue;
    }
    if (at + 14 + (n - i) > o.size()) {
      o.resize((at + 14 + (n - i)) * 5 / 4 + 16);
      w = &o[0];
    }
    char e2 = 0;
    switch (c) {
      case 0x22: e2 = '"'; break;
      case 0x5C: e2 = '\\'; break;
      case 0x08: e2 = 'b'; break;
      case 0x0C: e2 = 'f'; break;
      case 0x0A: e2 = 'n'; break;
      case 0x0D: e2 = 'r'; break;
      case 0x09: e2 = 't'; break;
      default: break;
    }
    if (e2) {
      w[at++] = '\\';
      w[at++] = e2;
      continue;
    }
    if (c >= 0x80) ascii = false;
    const bool lead = c >= 0xD800 && c < 0xDC00, trail = c >= 0xDC00 && c < 0xE000;
    uint32_t cp = c;
    if (lead && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
      cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
      i++;
    } else if (c < 0x20 || lead || trail) {
      w[at++] = '\\';
      w[at++] = 'u';
      w[at++] = kHex[(c >> 12) & 15];
      w[at++] = kHex[(c >> 8) & 15];
      w[at++] = kHex[(c >> 4) & 15];
      w[at++] = kHex[c & 15];
      continue;
    }
    if (cp < 0x800) {
      w[at++] = (char)(0xC0 | (cp >> 6));
      w[at++] = (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      w[at++] = (char)(0xE0 | (cp >> 12));
      w[at++] = (char)(0x80 | ((cp >> 6) & 0x3F));
      w[at++] = (char)(0x80 | (cp & 0x3F));
    } else {
      w[at++] = (char)(0xF0 | (cp >> 18));
      w[at++] = (char)(0x80 | ((cp >> 12) & 0x3F));
      w[at++] = (char)(0x80 | ((cp >> 6) & 0x3F));
      w[at++] = (char)(0x80 | (cp & 0x3F));
    }
  }
  w[at++] = '"';
  o.resize(at);
  return ascii;
}
inline void quote(std::string& o, const char16_t* s, size_t n) { quote16(o, s, n); }
inline void quote(std::string& o, const U16& s) { quote(o, s.data(), s.size()); }

// Length of the well-formed UTF-8 sequence at p (1-4 bytes), or 0 for an invalid one or an encoded surrogate.
inline size_t utf8_seq(const uint8_t* p, const uint8_t* e) {
  const uint8_t c = *p;
  if (c < 0x80) return 1;
  size_t n;
  uint32_t cp;
  if (c >= 0xC2 && c <= 0xDF) { n = 1; cp = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { n = 2; cp = c & 0x0F; }
  else if (c >= 0xF0 && c <= 0xF4) { n = 3; cp = c & 0x07; }
  else return 0;
  if ((size_t)(e - p) <= n) return 0;
  for (size_t k = 1; k <= n; k++) {
    if ((p[k] & 0xC0) != 0x80) return 0;
    cp = (cp << 6) | (p[k] & 0x3F);
  }
  if ((n == 2 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) || (n == 3 && (cp < 0x10000 || cp > 0x10FFFF))) return 0;
  return n + 1;
}
// quote(o, from_utf8(u)) without the UTF-16 round trip, for u well-formed UTF-8 without encoded surrogates (what
// these serializers produce): bytes pass through and only '"', '\\' and control characters are escaped, exactly
// as quote() escapes the same code points.  Returns false, leaving o as it was, for any other u.  The summary
// blobs it escapes are a quarter quotes, so an ASCII byte takes no branch: its replacement (1, 2 or 6 bytes)
// comes from a table as one 8-byte copy into a per-thread scratch with 8 bytes of slack, appended at the end.
struct JsonEscTab {
  char s[128][8];
  uint8_t n[128];
  JsonEscTab() {
    static const char kHex[] = "0123456789abcdef";
    for (int c = 0; c < 128; c++) {
      memset(s[c], 0, 8);
      const char* e = nullptr;
      switch (c) {
        case 0x22: e = "\\\""; break;
        case 0x5C: e = "\\\\"; break;
        case 0x08: e = "\\b"; break;
        case 0x0C: e = "\\f"; break;
        case 0x0A: e = "\\n"; break;
        case 0x0D: e = "\\r"; break;
        case 0x09: e = "\\t"; break;
        default: break;
      }
      if (e) {
        memcpy(s[c], e, 2);
        n[c] = 2;
      } else if (c < 0x20) {
        const char u[6] = {'\\', 'u', '0', '0', kHex[c >> 4], kHex[c & 15]};
        memcpy(s[c], u, 6);
        n[c] = 6;
      } else {
        s[c][0] = (char)c;
        n[c] = 1;
      }
    }
  }
};
inline bool quote_utf8(std::string& o, const std::string& u) {
  static const JsonEscTab T;
  thread_local std::vector<char> buf;
  const size_t need = 6 * u.size() + 16;
  if (buf.size() < need) buf.resize(need);
  char* w = buf.data();
  size_t at = 0;
  w[at++] = '"';
  const uint8_t* p = reinterpret_cast<const uint8_t*>(u.data());
  const uint8_t* const e = p + u.size();
  while (p < e) {
    const uint8_t c = *p;
    if (c < 0x80) {
      memcpy(w + at, T.s[c], 8);
      at += T.n[c];
      p++;
      continue;
    }
    const size_t n = utf8_seq(p, e);
    if (!n) return false;
    memcpy(w + at, p, n);
    at += n;
    p += n;
  }
  w[at++] = '"';
  o.append(w, at);
  return true;
}
// quote(o, from_utf8(u)) by the fast path when it applies
inline void quote_u8(std::string& o, const std::string& u) {
  if (!quote_utf8(o, u)) quote(o, from_utf8(u));
}

// Number::toString(10) (ECMA-262 7.1.12.1) for finite doubles
inline std::string number(double x) {
  if (std::isnan(x) || std::isinf(x)) return "null";
  if (x == 0) return "0";
  if (x == std::floor(x) && std::fabs(x) < 1e21) {
    char b[32];
    snprintf(b, sizeof b, "%.0f", x);
    return b;
  }
  std::string sign = x < 0 ? "-" : "";
  const double a = std::fabs(x);
  char b[40];
  int prec = 1;
  for (; prec < 17; prec++) {
    snprintf(b, sizeof b, "%.*e", prec - 1, a);
    if (strtod(b, nullptr) == a) break;
  }
  snprintf(b, sizeof b, "%.*e", prec - 1, a);
  std::string digits;
  const char* q = b;
  for (; *q && *q != 'e'; q++)
    if (*q != '.') digits += *q;
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int k = (int)digits.size();
  const int n = atoi(q + 1) + 1;
  std::string r;
  if (k <= n && n <= 21) r = digits + std::string(n - k, '0');
  else if (n > 0 && n <= 21) r = digits.substr(0, n) + "." + digits.substr(n);
  else if (n > -6 && n <= 0) r = "0." + std::string(-n, '0') + digits;
  else {
    const int e = n - 1;
    r = digits.substr(0, 1);
    if (k > 1) r += "." + digits.substr(1);
    r += e < 0 ? "e-" : "e+";
    r += std::to_string(e < 0 ? -e : e);
  }
  return sign + r;
}

inline void write(std::string& o, const Value& v) {
  switch (v.kind) {
    case Value::kUndef:
    case Value::kNull: o += "null"; return;
    case Value::kBool: o += v.b ? "true" : "false"; return;
    case Value::kNum: o += number(v.n); return;
    case Value::kStr: quote(o, v.s); return;
    case Value::kArr:
      o += '[';
      for (size_t i = 0; i < v.items.size(); i++) {
        if (i) o += ',';
        write(o, v.items[i]);
      }
      o += ']';
      return;
    case Value::kObj: {
      o += '{';
      bool first = true;
      for (auto& m : v.members) {
        if (m.second.kind == Value::kUndef) continue;
        if (!first) o += ',';
        first = false;
        quote(o, m.first);
        o += ':';
        write(o, m.second);
      }
      o += '}';
      return;
    }
  }
}
inline std::string dump(const Value& v) {
  std::string o;
  write(o, v);
  return o;
}

}  // namespace hj
