#include "json.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace tz {

namespace {
[[noreturn]] void type_error(const char *want) {
  throw std::runtime_error(std::string("json: value is not ") + want);
}
} // namespace

bool Json::as_bool() const {
  if (type_ != Type::Bool) type_error("a bool");
  return b_;
}
int64_t Json::as_int() const {
  if (type_ == Type::Int) return i_;
  if (type_ == Type::Double) return int64_t(d_);
  type_error("a number");
}
double Json::as_double() const {
  if (type_ == Type::Double) return d_;
  if (type_ == Type::Int) return double(i_);
  type_error("a number");
}
const std::string &Json::as_string() const {
  if (type_ != Type::String) type_error("a string");
  return s_;
}
const Json::array_t &Json::as_array() const {
  if (type_ != Type::Array) type_error("an array");
  return *a_;
}
Json::array_t &Json::as_array() {
  if (type_ != Type::Array) type_error("an array");
  detach();
  return *a_;
}
const Json::object_t &Json::as_object() const {
  if (type_ != Type::Object) type_error("an object");
  return *o_;
}
Json::object_t &Json::as_object() {
  if (type_ != Type::Object) type_error("an object");
  detach();
  return *o_;
}

void Json::detach() {
  if (a_ && a_.use_count() > 1) a_ = std::make_shared<array_t>(*a_);
  if (o_ && o_.use_count() > 1) o_ = std::make_shared<object_t>(*o_);
}

bool Json::contains(const std::string &key) const {
  return type_ == Type::Object && o_->count(key);
}
const Json &Json::at(const std::string &key) const {
  const auto &o = as_object();
  auto it = o.find(key);
  if (it == o.end()) throw std::runtime_error("json: missing key '" + key + "'");
  return it->second;
}
Json &Json::operator[](const std::string &key) {
  if (type_ == Type::Null) {
    type_ = Type::Object;
    o_ = std::make_shared<object_t>();
  }
  return as_object()[key];
}
const Json &Json::at(size_t i) const {
  const auto &a = as_array();
  if (i >= a.size()) throw std::runtime_error("json: index out of range");
  return a[i];
}
void Json::push_back(Json v) {
  if (type_ == Type::Null) {
    type_ = Type::Array;
    a_ = std::make_shared<array_t>();
  }
  as_array().push_back(std::move(v));
}
size_t Json::size() const {
  if (type_ == Type::Array) return a_->size();
  if (type_ == Type::Object) return o_->size();
  if (type_ == Type::Null) return 0;
  return 1;
}

bool Json::operator==(const Json &rhs) const {
  if (is_number() && rhs.is_number()) {
    if (type_ == Type::Int && rhs.type_ == Type::Int) return i_ == rhs.i_;
    return as_double() == rhs.as_double();
  }
  if (type_ != rhs.type_) return false;
  switch (type_) {
  case Type::Null: return true;
  case Type::Bool: return b_ == rhs.b_;
  case Type::String: return s_ == rhs.s_;
  case Type::Array: return *a_ == *rhs.a_;
  case Type::Object: return *o_ == *rhs.o_;
  default: return false;
  }
}

static void escape_to(const std::string &s, std::string &out) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
    case '"': out += "\\\""; break;
    case '\\': out += "\\\\"; break;
    case '\n': out += "\\n"; break;
    case '\r': out += "\\r"; break;
    case '\t': out += "\\t"; break;
    case '\b': out += "\\b"; break;
    case '\f': out += "\\f"; break;
    default:
      if (c < 0x20) {
        char buf[8];
        std::snprintf(buf, sizeof(buf), "\\u%04x", c);
        out += buf;
      } else {
        out.push_back(char(c));
      }
    }
  }
  out.push_back('"');
}

void Json::dump_to(std::string &out) const {
  switch (type_) {
  case Type::Null: out += "null"; break;
  case Type::Bool: out += b_ ? "true" : "false"; break;
  case Type::Int: out += std::to_string(i_); break;
  case Type::Double: {
    if (!std::isfinite(d_)) {
      out += "null";
      break;
    }
    char buf[32];
    std::snprintf(buf, sizeof(buf), "%.17g", d_);
    // shortest round-trip representation
    for (int prec = 1; prec <= 17; ++prec) {
      char tmp[32];
      std::snprintf(tmp, sizeof(tmp), "%.*g", prec, d_);
      if (std::strtod(tmp, nullptr) == d_) {
        std::memcpy(buf, tmp, sizeof(tmp));
        break;
      }
    }
    std::string s(buf);
    if (s.find_first_of(".eE") == std::string::npos) s += ".0";
    out += s;
    break;
  }
  case Type::String: escape_to(s_, out); break;
  case Type::Array: {
    out.push_back('[');
    bool first = true;
    for (const auto &v : *a_) {
      if (!first) out.push_back(',');
      first = false;
      v.dump_to(out);
    }
    out.push_back(']');
    break;
  }
  case Type::Object: {
    out.push_back('{');
    bool first = true;
    for (const auto &kv : *o_) {
      if (!first) out.push_back(',');
      first = false;
      escape_to(kv.first, out);
      out.push_back(':');
      kv.second.dump_to(out);
    }
    out.push_back('}');
    break;
  }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out);
  return out;
}

namespace {
struct Parser {
  const std::string &t;
  size_t p = 0;
  explicit Parser(const std::string &text) : t(text) {}

  [[noreturn]] void fail(const char *msg) {
    throw std::runtime_error(std::string("json parse error at ") + std::to_string(p) + ": " + msg);
  }
  void ws() {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\n' || t[p] == '\t' || t[p] == '\r')) ++p;
  }
  bool consume(const char *lit) {
    size_t n = std::strlen(lit);
    if (t.compare(p, n, lit) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  Json value() {
    ws();
    if (p >= t.size()) fail("unexpected end");
    char c = t[p];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return Json(string());
    if (consume("true")) return Json(true);
    if (consume("false")) return Json(false);
    if (consume("null")) return Json();
    return number();
  }
  Json number() {
    size_t start = p;
    bool isDouble = false;
    if (t[p] == '-') ++p;
    while (p < t.size()) {
      char c = t[p];
      if (c >= '0' && c <= '9') {
        ++p;
      } else if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') {
        isDouble = true;
        ++p;
      } else {
        break;
      }
    }
    if (start == p) fail("bad value");
    std::string s = t.substr(start, p - start);
    if (isDouble) return Json(std::strtod(s.c_str(), nullptr));
    return Json((long long)std::strtoll(s.c_str(), nullptr, 10));
  }
  static void put_utf8(std::string &out, unsigned cp) {
    if (cp < 0x80) {
      out.push_back(char(cp));
    } else if (cp < 0x800) {
      out.push_back(char(0xC0 | (cp >> 6)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(char(0xE0 | (cp >> 12)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(char(0xF0 | (cp >> 18)));
      out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    }
  }
  std::string string() {
    ++p; // opening quote
    std::string out;
    while (true) {
      if (p >= t.size()) fail("unterminated string");
      char c = t[p++];
      if (c == '"') break;
      if (c == '\\') {
        if (p >= t.size()) fail("bad escape");
        char e = t[p++];
        switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          if (p + 4 > t.size()) fail("bad unicode escape");
          unsigned cp = std::stoul(t.substr(p, 4), nullptr, 16);
          p += 4;
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
        }
      } else {
        out.push_back(c);
      }
    }
    return out;
  }
  Json array() {
    ++p;
    Json a = Json::array();
    ws();
    if (p < t.size() && t[p] == ']') {
      ++p;
      return a;
    }
    while (true) {
      a.push_back(value());
      ws();
      if (p >= t.size()) fail("unterminated array");
      if (t[p] == ',') {
        ++p;
        continue;
      }
      if (t[p] == ']') {
        ++p;
        break;
      }
      fail("expected , or ]");
    }
    return a;
  }
  Json object() {
    ++p;
    Json o = Json::object();
    ws();
    if (p < t.size() && t[p] == '}') {
      ++p;
      return o;
    }
    while (true) {
      ws();
      if (p >= t.size() || t[p] != '"') fail("expected key");
      std::string k = string();
      ws();
      if (p >= t.size() || t[p] != ':') fail("expected :");
      ++p;
      o[k] = value();
      ws();
      if (p >= t.size()) fail("unterminated object");
      if (t[p] == ',') {
        ++p;
        continue;
      }
      if (t[p] == '}') {
        ++p;
        break;
      }
      fail("expected , or }");
    }
    return o;
  }
};
} // namespace

Json Json::parse(const std::string &text) {
  Parser ps(text);
  Json v = ps.value();
  ps.ws();
  if (ps.p != text.size()) ps.fail("trailing characters");
  return v;
}

} // namespace tz
