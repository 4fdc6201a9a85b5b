// Minimal JSON value / parser / writer for the model architecture files (path.json) the C++ host
// API shares with the Python front end. Objects keep insertion order (the files are diffed and
// read by people).
#pragma once
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace dcnn {
namespace json {

class Value {
 public:
  enum class Kind { Null, Bool, Number, String, Array, Object };
  Value() = default;
  Value(std::nullptr_t) {}
  Value(bool b) : k_(Kind::Bool), b_(b) {}
  Value(int v) : k_(Kind::Number), n_(v), int_(true) {}
  Value(int64_t v) : k_(Kind::Number), n_((double)v), int_(true) {}
  Value(double v) : k_(Kind::Number), n_(v) {}
  Value(const char* s) : k_(Kind::String), s_(s) {}
  Value(std::string s) : k_(Kind::String), s_(std::move(s)) {}
  static Value array() { Value v; v.k_ = Kind::Array; return v; }
  static Value object() { Value v; v.k_ = Kind::Object; return v; }

  Kind kind() const { return k_; }
  bool is_object() const { return k_ == Kind::Object; }
  bool is_null() const { return k_ == Kind::Null; }
  bool as_bool() const {
    if (k_ == Kind::Number) return n_ != 0;
    check(Kind::Bool);
    return b_;
  }
  double as_number() const { check(Kind::Number); return n_; }
  int64_t as_int() const { check(Kind::Number); return (int64_t)n_; }
  const std::string& as_string() const { check(Kind::String); return s_; }
  const std::vector<Value>& items() const { check(Kind::Array); return a_; }
  const std::vector<std::pair<std::string, Value>>& members() const { check(Kind::Object); return o_; }

  void push(Value v) { check(Kind::Array); a_.push_back(std::move(v)); }
  Value& operator[](const std::string& k) {
    if (k_ == Kind::Null) k_ = Kind::Object;
    check(Kind::Object);
    for (auto& m : o_)
      if (m.first == k) return m.second;
    o_.emplace_back(k, Value());
    return o_.back().second;
  }
  const Value* find(const std::string& k) const {
    if (k_ != Kind::Object) return nullptr;
    for (auto& m : o_)
      if (m.first == k) return &m.second;
    return nullptr;
  }
  bool has(const std::string& k) const { return find(k) != nullptr; }
  const Value& at(const std::string& k) const {
    const Value* v = find(k);
    if (!v) throw std::out_of_range("json: missing key '" + k + "'");
    return *v;
  }
  int64_t get_int(const std::string& k, int64_t d) const { const Value* v = find(k); return v ? v->as_int() : d; }
  double get_number(const std::string& k, double d) const { const Value* v = find(k); return v ? v->as_number() : d; }
  bool get_bool(const std::string& k, bool d) const { const Value* v = find(k); return v ? v->as_bool() : d; }
  std::string get_string(const std::string& k, const std::string& d) const {
    const Value* v = find(k);
    return v ? v->as_string() : d;
  }

  std::string dump(int indent = 4) const {
    std::ostringstream o;
    write(o, indent, 0);
    return o.str();
  }
  static Value parse(const std::string& text) {
    size_t i = 0;
    Value v = parse_value(text, i);
    skip_ws(text, i);
    if (i != text.size()) throw std::runtime_error("json: trailing characters");
    return v;
  }

 private:
  void check(Kind k) const {
    if (k_ != k) throw std::runtime_error("json: wrong value kind");
  }
  static void write_string(std::ostream& o, const std::string& s) {
    o << '"';
    for (unsigned char c : s) {
      switch (c) {
        case '"': o << "\\\""; break;
        case '\\': o << "\\\\"; break;
        case '\n': o << "\\n"; break;
        case '\t': o << "\\t"; break;
        case '\r': o << "\\r"; break;
        default:
          if (c < 0x20) {
            char b[8];
            std::snprintf(b, sizeof b, "\\u%04x", c);
            o << b;
          } else {
            o << c;
          }
      }
    }
    o << '"';
  }
  void write(std::ostream& o, int ind, int lvl) const {
    auto nl = [&](int l) {
      if (ind > 0) o << '\n' << std::string((size_t)(ind * l), ' ');
    };
    switch (k_) {
      case Kind::Null: o << "null"; break;
      case Kind::Bool: o << (b_ ? "true" : "false"); break;
      case Kind::Number:
        if (int_ || (n_ == (double)(int64_t)n_ && std::abs(n_) < 1e15)) {
          o << (int64_t)n_;
        } else {
          char b[32];
          std::snprintf(b, sizeof b, "%.17g", n_);
          o << b;
        }
        break;
      case Kind::String: write_string(o, s_); break;
      case Kind::Array:
        o << '[';
        for (size_t i = 0; i < a_.size(); ++i) {
          if (i) o << ',';
          nl(lvl + 1);
          a_[i].write(o, ind, lvl + 1);
        }
        if (!a_.empty()) nl(lvl);
        o << ']';
        break;
      case Kind::Object:
        o << '{';
        for (size_t i = 0; i < o_.size(); ++i) {
          if (i) o << ',';
          nl(lvl + 1);
          write_string(o, o_[i].first);
          o << (ind > 0 ? ": " : ":");
          o_[i].second.write(o, ind, lvl + 1);
        }
        if (!o_.empty()) nl(lvl);
        o << '}';
        break;
    }
  }
  static void skip_ws(const std::string& t, size_t& i) {
    while (i < t.size() && std::isspace((unsigned char)t[i])) ++i;
  }
  static std::string parse_string(const std::string& t, size_t& i) {
    if (t[i] != '"') throw std::runtime_error("json: expected string");
    ++i;
    std::string s;
    while (i < t.size() && t[i] != '"') {
      char c = t[i++];
      if (c == '\\') {
        if (i >= t.size()) break;
        char e = t[i++];
        switch (e) {
          case 'n': s += '\n'; break;
          case 't': s += '\t'; break;
          case 'r': s += '\r'; break;
          case 'b': s += '\b'; break;
          case 'f': s += '\f'; break;
          case 'u': {
            const unsigned cp = (unsigned)std::stoul(t.substr(i, 4), nullptr, 16);
            i += 4;
            if (cp < 0x80) {
              s += (char)cp;
            } else if (cp < 0x800) {
              s += (char)(0xc0 | (cp >> 6));
              s += (char)(0x80 | (cp & 0x3f));
            } else {
              s += (char)(0xe0 | (cp >> 12));
              s += (char)(0x80 | ((cp >> 6) & 0x3f));
              s += (char)(0x80 | (cp & 0x3f));
            }
            break;
          }
          default: s += e;
        }
      } else {
        s += c;
      }
    }
    if (i >= t.size()) throw std::runtime_error("json: unterminated string");
    ++i;
    return s;
  }
  static Value parse_value(const std::string& t, size_t& i) {
    skip_ws(t, i);
    if (i >= t.size()) throw std::runtime_error("json: unexpected end");
    const char c = t[i];
    if (c == '{') {
      ++i;
      Value v = object();
      skip_ws(t, i);
      if (t[i] == '}') { ++i; return v; }
      while (true) {
        skip_ws(t, i);
        std::string k = parse_string(t, i);
        skip_ws(t, i);
        if (t[i] != ':') throw std::runtime_error("json: expected ':'");
        ++i;
        v.o_.emplace_back(std::move(k), parse_value(t, i));
        skip_ws(t, i);
        if (t[i] == ',') { ++i; continue; }
        if (t[i] == '}') { ++i; return v; }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Value v = array();
      skip_ws(t, i);
      if (t[i] == ']') { ++i; return v; }
      while (true) {
        v.a_.push_back(parse_value(t, i));
        skip_ws(t, i);
        if (t[i] == ',') { ++i; continue; }
        if (t[i] == ']') { ++i; return v; }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    }
    if (c == '"') return Value(parse_string(t, i));
    if (t.compare(i, 4, "true") == 0) { i += 4; return Value(true); }
    if (t.compare(i, 5, "false") == 0) { i += 5; return Value(false); }
    if (t.compare(i, 4, "null") == 0) { i += 4; return Value(); }
    size_t j = i;
    bool integral = true;
    while (j < t.size() && (std::isdigit((unsigned char)t[j]) || t[j] == '-' || t[j] == '+' || t[j] == '.' ||
                            t[j] == 'e' || t[j] == 'E')) {
      if (t[j] == '.' || t[j] == 'e' || t[j] == 'E') integral = false;
      ++j;
    }
    if (j == i) throw std::runtime_error("json: unexpected character");
    Value v(std::stod(t.substr(i, j - i)));
    v.int_ = integral;
    i = j;
    return v;
  }

  Kind k_ = Kind::Null;
  bool b_ = false;
  double n_ = 0;
  bool int_ = false;
  std::string s_;
  std::vector<Value> a_;
  std::vector<std::pair<std::string, Value>> o_;
};

}  // namespace json
}  // namespace dcnn
