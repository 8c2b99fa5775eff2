// A small YAML (block + flow) / JSON reader and a JSON writer.
//
// The reference parses its config with sigs.k8s.io/yaml (vendored
// config/v1/config.go:75-99), which converts YAML 1.1 to JSON and then
// json.Unmarshals into typed structs.  The daemon must read the same files
// without a Go runtime, so this implements the subset of YAML that config
// files actually use:
//   * block mappings and sequences (including the compact "key:\n- item"
//     form and "- key: v" mappings inside sequences),
//   * flow collections ([a, b], {k: v}) spanning any number of lines, which
//     also makes every JSON document parseable,
//   * plain, 'single' and "double" quoted scalars, literal (|) and folded (>)
//     block scalars, comments, and a leading "---".
// Anchors, aliases, tags and multi-document streams are rejected with an
// error instead of being misread.
//
// Scalars keep their source text so typed accessors can mirror the
// YAML->JSON conversion rules (e.g. a plain `1` is accepted for a string
// field, but a quoted "1" is rejected for an int field).
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace gfd::yaml {

class Node {
 public:
  enum class Kind { Null, Bool, Int, Float, String, Seq, Map };

  Node() = default;
  static Node null() { return Node(); }
  static Node boolean(bool v);
  static Node integer(int64_t v);
  static Node floating(double v, std::string text = {});
  static Node string(std::string v);
  static Node seq() {
    Node n;
    n.kind_ = Kind::Seq;
    return n;
  }
  static Node map() {
    Node n;
    n.kind_ = Kind::Map;
    return n;
  }

  Kind kind() const { return kind_; }
  bool is_null() const { return kind_ == Kind::Null; }
  bool is_scalar() const { return kind_ != Kind::Seq && kind_ != Kind::Map; }
  bool is_map() const { return kind_ == Kind::Map; }
  bool is_seq() const { return kind_ == Kind::Seq; }

  bool as_bool() const { return b_; }
  int64_t as_int() const { return i_; }
  double as_float() const { return f_; }
  // For String: the value.  For other scalars: canonical source text.
  const std::string& text() const { return s_; }

  const std::vector<Node>& items() const { return seq_; }
  std::vector<Node>& items() { return seq_; }
  const std::vector<std::pair<std::string, Node>>& entries() const { return map_; }

  // Map lookup (last duplicate wins, like encoding/json). nullptr if absent.
  const Node* get(const std::string& key) const;
  // Insert or replace, preserving first-insertion order.
  void set(const std::string& key, Node value);
  void push(Node value) { seq_.push_back(std::move(value)); }

  std::string kind_name() const;

 private:
  Kind kind_ = Kind::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double f_ = 0;
  std::string s_;
  std::vector<Node> seq_;
  std::vector<std::pair<std::string, Node>> map_;
};

// Parse a YAML or JSON document.  Throws gfd::Error with a line number.
Node parse(const std::string& text);

// Serialize as JSON.  indent < 0 → compact; otherwise pretty-printed with
// `indent` spaces per level (Go's json.MarshalIndent(v, "", "  ") shape).
std::string to_json(const Node& n, int indent = -1);
std::string json_quote(const std::string& s);

}  // namespace gfd::yaml
