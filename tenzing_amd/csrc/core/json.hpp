// Minimal JSON value / parser / serializer for the schedule wire format.
//
// The reference uses nlohmann::json (thirdparty/nlohmann/json.hpp) whose default
// object type is a sorted std::map and whose dump() is compact ("{"a":1,"b":2}").
// Schedules produced here must be byte-compatible with that format
// (reference src/operation_serdes.cpp:14-76), so objects keep
// sorted keys and dump() is compact with integers printed without a fraction.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace tz {

class Json {
public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using array_t = std::vector<Json>;
  using object_t = std::map<std::string, Json>;

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(long v) : type_(Type::Int), i_(v) {}
  Json(long long v) : type_(Type::Int), i_(v) {}
  Json(unsigned v) : type_(Type::Int), i_(v) {}
  Json(unsigned long v) : type_(Type::Int), i_(int64_t(v)) {}
  Json(unsigned long long v) : type_(Type::Int), i_(int64_t(v)) {}
  Json(double v) : type_(Type::Double), d_(v) {}
  Json(const char *s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Json(array_t a) : type_(Type::Array), a_(std::make_shared<array_t>(std::move(a))) {}
  Json(object_t o) : type_(Type::Object), o_(std::make_shared<object_t>(std::move(o))) {}

  static Json array() { return Json(array_t{}); }
  static Json object() { return Json(object_t{}); }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Double; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_int() const;
  double as_double() const;
  const std::string &as_string() const;
  const array_t &as_array() const;
  array_t &as_array();
  const object_t &as_object() const;
  object_t &as_object();

  // object access
  bool contains(const std::string &key) const;
  const Json &at(const std::string &key) const;
  Json &operator[](const std::string &key); // converts null to object
  // array access
  const Json &at(size_t i) const;
  void push_back(Json v); // converts null to array
  size_t size() const;

  std::string dump() const;
  static Json parse(const std::string &text);

  bool operator==(const Json &rhs) const;
  bool operator!=(const Json &rhs) const { return !(*this == rhs); }

private:
  void dump_to(std::string &out) const;
  void detach(); // copy-on-write for shared containers

  Type type_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::shared_ptr<array_t> a_;
  std::shared_ptr<object_t> o_;
};

} // namespace tz
