// json.hpp — minimal JSON value + parser + writer for the SceneBuilder interchange format
// (serde_json 1.0 as used by scenes.rs:128-143).  Numbers are parsed with strtod (exact round
// trip) and written in shortest round-trip form with a ".0" suffix on integral values, as ryu /
// serde_json print f64.
#pragma once

#include <charconv>
#include <cstdlib>
#include <system_error>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace host {

struct Json {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;  // insertion order kept (serde field order)

  static Json number(double v) { Json j; j.kind = Number; j.num = v; return j; }
  static Json string(std::string s) { Json j; j.kind = String; j.str = std::move(s); return j; }
  static Json array() { Json j; j.kind = Array; return j; }
  static Json object() { Json j; j.kind = Object; return j; }

  Json& set(const std::string& k, Json v) {
    kind = Object;
    obj.emplace_back(k, std::move(v));
    return *this;
  }
  void push(Json v) { kind = Array; arr.push_back(std::move(v)); }
  const Json* find(const std::string& k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Json& at(const std::string& k) const {
    const Json* j = find(k);
    if (!j) throw std::runtime_error("missing field `" + k + "`");
    return *j;
  }
  double as_number() const {
    if (kind != Number) throw std::runtime_error("expected a number");
    return num;
  }
  const std::string& as_string() const {
    if (kind != String) throw std::runtime_error("expected a string");
    return str;
  }
};

class JsonParser {
 public:
  explicit JsonParser(const std::string& s) : s_(s) {}
  Json parse() {
    Json v = value();
    ws();
    if (i_ != s_.size()) err("trailing characters");
    return v;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  [[noreturn]] void err(const char* m) { throw std::runtime_error(std::string("json: ") + m + " at offset " + std::to_string(i_)); }
  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
  }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
    return false;
  }
  // serde_json's recursion limit: deeper nesting is an error, not a stack overflow
  static constexpr int kMaxDepth = 128;
  int depth_ = 0;
  struct Nest {
    JsonParser& p;
    explicit Nest(JsonParser& q) : p(q) {
      if (++p.depth_ > kMaxDepth) p.err("recursion limit exceeded");
    }
    ~Nest() { --p.depth_; }
  };
  Json value() {
    ws();
    if (i_ >= s_.size()) err("unexpected end");
    char c = s_[i_];
    if (c == '{') { Nest n(*this); return object(); }
    if (c == '[') { Nest n(*this); return array(); }
    if (c == '"') return Json::string(string());
    if (lit("true")) { Json j; j.kind = Json::Bool; j.b = true; return j; }
    if (lit("false")) { Json j; j.kind = Json::Bool; j.b = false; return j; }
    if (lit("null")) return Json();
    return number();
  }
  // JSON number grammar (RFC 8259 §6, as serde_json accepts it): -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
  // validated first, then converted with from_chars (locale-independent, correctly rounded); no
  // "inf", "nan", hex floats or a leading '+'.  Out-of-range magnitudes are errors, as in serde_json.
  Json number() {
    const size_t b = i_, n = s_.size();
    auto digit = [&](size_t k) { return k < n && s_[k] >= '0' && s_[k] <= '9'; };
    size_t k = b;
    if (k < n && s_[k] == '-') ++k;
    if (!digit(k)) err("bad value");
    if (s_[k] == '0') ++k; else while (digit(k)) ++k;
    if (k < n && s_[k] == '.') {
      ++k;
      if (!digit(k)) err("bad number");
      while (digit(k)) ++k;
    }
    if (k < n && (s_[k] == 'e' || s_[k] == 'E')) {
      ++k;
      if (k < n && (s_[k] == '+' || s_[k] == '-')) ++k;
      if (!digit(k)) err("bad number");
      while (digit(k)) ++k;
    }
    double v = 0.0;
    const auto r = std::from_chars(s_.data() + b, s_.data() + k, v);
    if (r.ec == std::errc::result_out_of_range) {
      // underflow to zero / denormal is fine (serde_json rounds), overflow is "number out of range"
      const std::string t(s_, b, k - b);
      v = std::strtod(t.c_str(), nullptr);
      if (std::isinf(v)) err("number out of range");
    } else if (r.ec != std::errc() || r.ptr != s_.data() + k) {
      err("bad number");
    }
    i_ = k;
    return Json::number(v);
  }
  unsigned hex4() {
    if (i_ + 4 > s_.size()) err("bad \\u escape");
    unsigned cp = 0;
    for (int q = 0; q < 4; ++q) {
      const char h = s_[i_++];
      cp <<= 4;
      if (h >= '0' && h <= '9') cp |= (unsigned)(h - '0');
      else if (h >= 'a' && h <= 'f') cp |= (unsigned)(h - 'a' + 10);
      else if (h >= 'A' && h <= 'F') cp |= (unsigned)(h - 'A' + 10);
      else err("bad \\u escape");
    }
    return cp;
  }
  std::string string() {
    ++i_;  // "
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= s_.size()) err("bad escape");
        char e = s_[i_++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {  // UTF-16 escape, surrogate pairs combined (lone surrogates are errors)
            unsigned cp = hex4();
            if (cp >= 0xDC00 && cp <= 0xDFFF) err("lone surrogate");
            if (cp >= 0xD800 && cp <= 0xDBFF) {
              if (!(i_ + 1 < s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u')) err("lone surrogate");
              i_ += 2;
              const unsigned lo = hex4();
              if (lo < 0xDC00 || lo > 0xDFFF) err("lone surrogate");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else if (cp < 0x10000) { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            else {
              out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
              out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: err("bad escape");
        }
      } else {
        if ((unsigned char)c < 0x20) err("control character in string");
        out += c;
      }
    }
    if (i_ >= s_.size()) err("unterminated string");
    ++i_;
    return out;
  }
  Json array() {
    ++i_;
    Json a = Json::array();
    ws();
    if (i_ < s_.size() && s_[i_] == ']') { ++i_; return a; }
    for (;;) {
      a.arr.push_back(value());
      ws();
      if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
      if (i_ < s_.size() && s_[i_] == ']') { ++i_; return a; }
      err("expected , or ]");
    }
  }
  Json object() {
    ++i_;
    Json o = Json::object();
    ws();
    if (i_ < s_.size() && s_[i_] == '}') { ++i_; return o; }
    for (;;) {
      ws();
      if (i_ >= s_.size() || s_[i_] != '"') err("expected key");
      std::string k = string();
      ws();
      if (i_ >= s_.size() || s_[i_] != ':') err("expected :");
      ++i_;
      o.obj.emplace_back(std::move(k), value());
      ws();
      if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
      if (i_ < s_.size() && s_[i_] == '}') { ++i_; return o; }
      err("expected , or }");
    }
  }
};

inline std::string json_number(double v) {
  if (std::isnan(v) || std::isinf(v)) return "null";  // serde_json writes non-finite floats as null
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v);
  std::string s(buf, r.ptr);
  if (s.find_first_of(".eE") == std::string::npos) s += ".0";
  return s;
}

inline void json_escape(const std::string& s, std::string& out) {
  out += '"';
  for (char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out += c;
        }
    }
  }
  out += '"';
}

// pretty printer in serde_json::to_writer_pretty style (2-space indent)
inline void json_write(const Json& j, std::string& out, int indent = 0, bool pretty = true) {
  auto nl = [&](int ind) {
    if (!pretty) return;
    out += '\n';
    out.append((size_t)ind * 2, ' ');
  };
  switch (j.kind) {
    case Json::Null: out += "null"; break;
    case Json::Bool: out += j.b ? "true" : "false"; break;
    case Json::Number: out += json_number(j.num); break;
    case Json::String: json_escape(j.str, out); break;
    case Json::Array:
      if (j.arr.empty()) { out += "[]"; break; }
      out += '[';
      for (size_t k = 0; k < j.arr.size(); ++k) {
        if (k) out += ',';
        nl(indent + 1);
        json_write(j.arr[k], out, indent + 1, pretty);
      }
      nl(indent);
      out += ']';
      break;
    case Json::Object:
      if (j.obj.empty()) { out += "{}"; break; }
      out += '{';
      for (size_t k = 0; k < j.obj.size(); ++k) {
        if (k) out += ',';
        nl(indent + 1);
        json_escape(j.obj[k].first, out);
        out += pretty ? ": " : ":";
        json_write(j.obj[k].second, out, indent + 1, pretty);
      }
      nl(indent);
      out += '}';
      break;
  }
}

}  // namespace host
