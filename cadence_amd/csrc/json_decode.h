// json_decode.h -- JSON-encoded history batches -> Events (private to libcadence_host.so).
//
// serializerImpl.deserialize (common/persistence/serializer.go:312-334) decodes a DataBlob whose
// encoding is json / unknown / empty ("for backward-compatibility") with json.Unmarshal into
// []*types.HistoryEvent.  This restates what that yields for the fields ApplyEvents reads: the
// common/types JSON tags (common/types/shared.go:3662-3710 HistoryEvent and the *EventAttributes
// structs), keys matched case-insensitively as encoding/json does, the last of duplicate keys
// winning, enum values as JSON strings only (EventType / TimeoutType / ContinueAsNewInitiator
// implement UnmarshalText alone: a name, case-insensitive, or strconv.ParseInt's decimal text; a bare
// number is encoding/json's UnmarshalTypeError), null as absent, unknown keys skipped, nesting deeper
// than encoding/json's scanner allows (maxNestingDepth = 10000) an error, and a malformed value or a
// type mismatch in a field the replay reads an error (json.Unmarshal fails the whole blob).
//
// Narrower than json.Unmarshal (documented, pinned by tests/test_decode_json.py): fields the replay
// never reads are checked for JSON syntax only, not against their Go types, and a duplicated
// attributes object replaces the earlier one instead of merging into it.
#pragma once

#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "host_flatten.h"

namespace crr_host {

struct JsonError {
  int code;
};

class JsonReader {
 public:
  JsonReader(const char* p, const char* end) : p_(p), end_(end) {}
  const char* pos() const { return p_; }
  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  char peek() {
    ws();
    if (p_ >= end_) fail();
    return *p_;
  }
  // '{' / '[' open a level, '}' / ']' close one (encoding/json's scanner: at most kMaxDepth levels)
  void expect(char c) {
    if (peek() != c) fail();
    ++p_;
    level(c);
  }
  bool consume(char c) {
    if (peek() != c) return false;
    ++p_;
    level(c);
    return true;
  }
  static constexpr int kMaxDepth = 10000;
  bool null() {  // a JSON null (Go: the pointer / field stays unset)
    if (peek() != 'n') return false;
    lit("null");
    return true;
  }
  void at_end() {
    ws();
    if (p_ != end_) fail();
  }
  [[noreturn]] void fail() const { throw JsonError{CRR_DECODE_BAD_JSON}; }

  std::string str() {
    expect('"');
    std::string s;
    for (;;) {
      if (p_ >= end_) fail();
      const char c = *p_++;
      if (c == '"') return s;
      if ((unsigned char)c < 0x20) fail();
      if (c != '\\') { s.push_back(c); continue; }
      if (p_ >= end_) fail();
      const char e = *p_++;
      switch (e) {
        case '"': s.push_back('"'); break;
        case '\\': s.push_back('\\'); break;
        case '/': s.push_back('/'); break;
        case 'b': s.push_back('\b'); break;
        case 'f': s.push_back('\f'); break;
        case 'n': s.push_back('\n'); break;
        case 'r': s.push_back('\r'); break;
        case 't': s.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            const char* save = p_;
            p_ += 2;
            const uint32_t lo = hex4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else { p_ = save; cp = 0xFFFD; }
          } else if (cp >= 0xD800 && cp < 0xE000) {
            cp = 0xFFFD;  // lone surrogate: encoding/json substitutes U+FFFD
          }
          utf8(s, cp);
          break;
        }
        default: fail();
      }
    }
  }
  // a JSON integer that fits T (encoding/json: fractions, exponents and overflow are type errors)
  template <class T>
  T integer() {
    ws();
    bool neg = false;
    if (p_ < end_ && *p_ == '-') { neg = true; ++p_; }
    if (p_ >= end_ || *p_ < '0' || *p_ > '9') fail();
    if (*p_ == '0' && p_ + 1 < end_ && p_[1] >= '0' && p_[1] <= '9') fail();
    unsigned __int128 v = 0;
    while (p_ < end_ && *p_ >= '0' && *p_ <= '9') {
      v = v * 10 + (unsigned)(*p_++ - '0');
      if (v > ((unsigned __int128)1 << 64)) fail();
    }
    if (p_ < end_ && (*p_ == '.' || *p_ == 'e' || *p_ == 'E')) fail();
    const __int128 sv = neg ? -(__int128)v : (__int128)v;
    if (sv < (__int128)std::numeric_limits<T>::min() || sv > (__int128)std::numeric_limits<T>::max()) fail();
    return (T)sv;
  }
  // an enum (UnmarshalText): a JSON string holding its name (case-insensitive, `names`) or a decimal
  // int32; any other token is an UnmarshalTypeError
  int enum_value(const char* const* names, int n) {
    if (peek() != '"') fail();
    const std::string s = str();
    for (int i = 0; i < n; ++i)
      if (iequal(s, names[i])) return i;
    // UnmarshalText's default: strconv.ParseInt(s, 10, 32) -- an optional sign, decimal digits
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    if (i == s.size()) fail();
    int64_t v = 0;
    for (; i < s.size(); ++i) {
      if (s[i] < '0' || s[i] > '9') fail();
      v = v * 10 + (s[i] - '0');
      if (v > (int64_t)1 << 31) fail();
    }
    if (neg) v = -v;
    if (v < std::numeric_limits<int32_t>::min() || v > std::numeric_limits<int32_t>::max()) fail();
    return (int)v;
  }
  void skip() {  // any value
    const char c = peek();
    if (c == '"') { (void)str(); return; }
    if (c == '{') {
      expect('{');
      if (consume('}')) return;
      do { (void)str(); expect(':'); skip(); } while (consume(','));
      expect('}');
      return;
    }
    if (c == '[') {
      expect('[');
      if (consume(']')) return;
      do { skip(); } while (consume(','));
      expect(']');
      return;
    }
    if (c == 't') { lit("true"); return; }
    if (c == 'f') { lit("false"); return; }
    if (c == 'n') { lit("null"); return; }
    number();
  }
  static bool iequal(const std::string& a, const char* b) {  // ASCII strings.EqualFold
    const size_t n = strlen(b);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; ++i) {
      char x = a[i], y = b[i];
      if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
      if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
      if (x != y) return false;
    }
    return true;
  }

 private:
  void lit(const char* w) {
    ws();
    const size_t n = strlen(w);
    if ((size_t)(end_ - p_) < n || strncmp(p_, w, n) != 0) fail();
    p_ += n;
  }
  void level(char c) {
    if (c == '{' || c == '[') {
      if (++depth_ > kMaxDepth) fail();
    } else if (c == '}' || c == ']') {
      --depth_;
    }
  }
  bool digit() const { return p_ < end_ && *p_ >= '0' && *p_ <= '9'; }
  // the JSON number grammar: -? (0 | [1-9][0-9]*) (. [0-9]+)? ([eE] [+-]? [0-9]+)?
  void number() {
    ws();
    if (p_ < end_ && *p_ == '-') ++p_;
    if (!digit()) fail();
    if (*p_ == '0') ++p_;
    else while (digit()) ++p_;
    if (p_ < end_ && *p_ == '.') {
      ++p_;
      if (!digit()) fail();
      while (digit()) ++p_;
    }
    if (p_ < end_ && (*p_ == 'e' || *p_ == 'E')) {
      ++p_;
      if (p_ < end_ && (*p_ == '+' || *p_ == '-')) ++p_;
      if (!digit()) fail();
      while (digit()) ++p_;
    }
    if (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == '+' || *p_ == '-' || *p_ == 'e' || *p_ == 'E'))
      fail();
  }
  uint32_t hex4() {
    if (end_ - p_ < 4) fail();
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail();
    }
    return v;
  }
  static void utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s.push_back((char)cp);
    else if (cp < 0x800) { s.push_back((char)(0xC0 | (cp >> 6))); s.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      s.push_back((char)(0xE0 | (cp >> 12)));
      s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      s.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      s.push_back((char)(0xF0 | (cp >> 18)));
      s.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      s.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  const char* p_;
  const char* end_;
  int depth_ = 0;
};

// Decode one JSON batch (a JSON array of HistoryEvent objects) into `out`.
void json_decode_batch(const char* p, const char* end, std::vector<Event>& out);

}  // namespace crr_host
