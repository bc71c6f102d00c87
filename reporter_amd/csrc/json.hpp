// json.hpp — small strict JSON reader for /report traces and Valhalla-style
// config files.  Only what the drop-in boundary needs: objects, arrays,
// strings, numbers (kept as double and, when integral, as int64), bools, null.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rm {
namespace json {

struct Value {
  enum Type { Null, Bool, Number, String, Array, Object } type = Null;
  bool b = false;
  double num = 0.0;
  bool is_int = false;
  int64_t i64 = 0;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  const Value* get(const char* key) const {
    if (type != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  bool is_num() const { return type == Number; }
};

class Parser {
 public:
  explicit Parser(const char* s) : p_(s), s0_(s) {}
  Value parse() {
    Value v = value(0);
    ws();
    if (*p_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* s0_;
  [[noreturn]] void fail(const char* m) {
    throw std::runtime_error(std::string("invalid JSON (") + m + ") at offset " + std::to_string(p_ - s0_));
  }
  void ws() { while (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r') ++p_; }
  Value value(int depth) {
    if (depth > 64) fail("nesting too deep");
    ws();
    Value v;
    switch (*p_) {
      case '{': {
        ++p_; v.type = Value::Object; ws();
        if (*p_ == '}') { ++p_; return v; }
        for (;;) {
          ws();
          if (*p_ != '"') fail("expected key");
          std::string k = string();
          ws();
          if (*p_ != ':') fail("expected ':'");
          ++p_;
          v.obj.emplace_back(std::move(k), value(depth + 1));
          ws();
          if (*p_ == ',') { ++p_; continue; }
          if (*p_ == '}') { ++p_; return v; }
          fail("expected ',' or '}'");
        }
      }
      case '[': {
        ++p_; v.type = Value::Array; ws();
        if (*p_ == ']') { ++p_; return v; }
        for (;;) {
          v.arr.push_back(value(depth + 1));
          ws();
          if (*p_ == ',') { ++p_; continue; }
          if (*p_ == ']') { ++p_; return v; }
          fail("expected ',' or ']'");
        }
      }
      case '"': v.type = Value::String; v.str = string(); return v;
      case 't': if (!std::strncmp(p_, "true", 4)) { p_ += 4; v.type = Value::Bool; v.b = true; return v; } fail("bad literal");
      case 'f': if (!std::strncmp(p_, "false", 5)) { p_ += 5; v.type = Value::Bool; v.b = false; return v; } fail("bad literal");
      case 'n': if (!std::strncmp(p_, "null", 4)) { p_ += 4; return v; } fail("bad literal");
      default: return number();
    }
  }
  Value number() {
    const char* st = p_;
    if (*p_ == '-') ++p_;
    if (!(*p_ >= '0' && *p_ <= '9')) fail("bad number");
    bool integral = true;
    while (*p_ >= '0' && *p_ <= '9') ++p_;
    if (*p_ == '.') { integral = false; ++p_; while (*p_ >= '0' && *p_ <= '9') ++p_; }
    if (*p_ == 'e' || *p_ == 'E') {
      integral = false; ++p_;
      if (*p_ == '+' || *p_ == '-') ++p_;
      if (!(*p_ >= '0' && *p_ <= '9')) fail("bad exponent");
      while (*p_ >= '0' && *p_ <= '9') ++p_;
    }
    Value v;
    v.type = Value::Number;
    std::string tok(st, p_);
    v.num = std::strtod(tok.c_str(), nullptr);
    if (integral && tok.size() < 19) { v.is_int = true; v.i64 = std::strtoll(tok.c_str(), nullptr, 10); }
    return v;
  }
  static void utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xc0 | (c >> 6)); o += (char)(0x80 | (c & 0x3f)); }
    else if (c < 0x10000) { o += (char)(0xe0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3f)); o += (char)(0x80 | (c & 0x3f)); }
    else { o += (char)(0xf0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3f)); o += (char)(0x80 | ((c >> 6) & 0x3f)); o += (char)(0x80 | (c & 0x3f)); }
  }
  uint32_t hex4() {
    uint32_t c = 0;
    for (int i = 0; i < 4; ++i) {
      const char h = *p_++;
      c <<= 4;
      if (h >= '0' && h <= '9') c |= h - '0';
      else if (h >= 'a' && h <= 'f') c |= h - 'a' + 10;
      else if (h >= 'A' && h <= 'F') c |= h - 'A' + 10;
      else fail("bad \\u escape");
    }
    return c;
  }
  std::string string() {
    ++p_;  // opening quote
    std::string o;
    for (;;) {
      const char c = *p_++;
      if (c == '"') return o;
      if (c == 0) fail("unterminated string");
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') { o += c; continue; }
      const char e = *p_++;
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xd800 && cp < 0xdc00 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            const uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xd800) << 10) + (lo - 0xdc00);
          }
          utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }
};

inline Value parse(const char* s) { return Parser(s).parse(); }

}  // namespace json
}  // namespace rm
