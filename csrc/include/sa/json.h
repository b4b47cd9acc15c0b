// Minimal JSON reader (objects, arrays, strings, numbers, true/false/null) for safetensors
// headers and engine plan/config files.  Header-only, no dependencies.
#pragma once
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace sa {
namespace json {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;  // insertion order kept
  bool is_object() const { return kind == Obj; }
  const Value& at(const std::string& k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return kv.second;
    throw std::runtime_error("json: missing key " + k);
  }
  bool has(const std::string& k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return true;
    return false;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != s_.size()) fail("trailing data");
    return v;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) ++i_;
  }
  char peek() {
    ws();
    if (i_ >= s_.size()) fail("unexpected end");
    return s_[i_];
  }
  void expect(char c) {
    if (peek() != c) fail("unexpected character");
    ++i_;
  }
  std::string string_() {
    expect('"');
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= s_.size()) fail("bad escape");
        char e = s_[i_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            if (i_ + 4 > s_.size()) fail("bad \\u escape");
            unsigned cp = (unsigned)std::strtoul(s_.substr(i_, 4).c_str(), nullptr, 16);
            i_ += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) {
              out += (char)(0xC0 | (cp >> 6));
              out += (char)(0x80 | (cp & 0x3F));
            } else {
              out += (char)(0xE0 | (cp >> 12));
              out += (char)(0x80 | ((cp >> 6) & 0x3F));
              out += (char)(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (i_ >= s_.size()) fail("unterminated string");
    ++i_;
    return out;
  }
  Value value() {
    char c = peek();
    Value v;
    if (c == '{') {
      ++i_;
      v.kind = Value::Obj;
      if (peek() == '}') {
        ++i_;
        return v;
      }
      for (;;) {
        std::string k = string_();
        expect(':');
        v.obj.emplace_back(k, value());
        char d = peek();
        ++i_;
        if (d == '}') break;
        if (d != ',') fail("expected , or }");
      }
    } else if (c == '[') {
      ++i_;
      v.kind = Value::Arr;
      if (peek() == ']') {
        ++i_;
        return v;
      }
      for (;;) {
        v.arr.push_back(value());
        char d = peek();
        ++i_;
        if (d == ']') break;
        if (d != ',') fail("expected , or ]");
      }
    } else if (c == '"') {
      v.kind = Value::Str;
      v.str = string_();
    } else if (s_.compare(i_, 4, "true") == 0) {
      v.kind = Value::Bool;
      v.b = true;
      i_ += 4;
    } else if (s_.compare(i_, 5, "false") == 0) {
      v.kind = Value::Bool;
      i_ += 5;
    } else if (s_.compare(i_, 4, "null") == 0) {
      i_ += 4;
    } else {
      v.kind = Value::Num;
      const char* b = s_.c_str() + i_;
      char* e = nullptr;
      v.num = std::strtod(b, &e);
      if (e == b) fail("bad number");
      i_ += (size_t)(e - b);
    }
    return v;
  }
};

inline Value parse(const std::string& s) { return Parser(s).parse(); }

}  // namespace json
}  // namespace sa
