#include "config/yaml.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <optional>

#include "util/error.h"
#include "util/strings.h"

namespace gfd::yaml {

// ---------------------------------------------------------------------------
// Node

Node Node::boolean(bool v) {
  Node n;
  n.kind_ = Kind::Bool;
  n.b_ = v;
  n.s_ = v ? "true" : "false";
  return n;
}

Node Node::integer(int64_t v) {
  Node n;
  n.kind_ = Kind::Int;
  n.i_ = v;
  n.s_ = std::to_string(v);
  return n;
}

Node Node::floating(double v, std::string text) {
  Node n;
  n.kind_ = Kind::Float;
  n.f_ = v;
  if (text.empty()) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.17g", v);
    text = buf;
  }
  n.s_ = std::move(text);
  return n;
}

Node Node::string(std::string v) {
  Node n;
  n.kind_ = Kind::String;
  n.s_ = std::move(v);
  return n;
}

const Node* Node::get(const std::string& key) const {
  const Node* found = nullptr;
  for (const auto& kv : map_)
    if (kv.first == key) found = &kv.second;
  return found;
}

void Node::set(const std::string& key, Node value) {
  for (auto& kv : map_) {
    if (kv.first == key) {
      kv.second = std::move(value);
      return;
    }
  }
  map_.emplace_back(key, std::move(value));
}

std::string Node::kind_name() const {
  switch (kind_) {
    case Kind::Null: return "null";
    case Kind::Bool: return "bool";
    case Kind::Int: return "number";
    case Kind::Float: return "number";
    case Kind::String: return "string";
    case Kind::Seq: return "array";
    case Kind::Map: return "object";
  }
  return "unknown";
}

// ---------------------------------------------------------------------------
// Scalar resolution (YAML 1.1 rules as used by go-yaml v2 / sigs.k8s.io/yaml)

namespace {

Node resolve_plain(const std::string& s) {
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Node::null();
  static const char* kTrue[] = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"};
  static const char* kFalse[] = {"n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"};
  for (const char* t : kTrue)
    if (s == t) return Node::boolean(true);
  for (const char* f : kFalse)
    if (s == f) return Node::boolean(false);

  // Integers: [-+]?(0x..|0o..|0b..|0..|digits), underscores allowed.
  std::string t;
  for (char c : s)
    if (c != '_') t.push_back(c);
  {
    size_t i = 0;
    bool neg = false;
    if (i < t.size() && (t[i] == '-' || t[i] == '+')) neg = t[i++] == '-';
    std::string body = t.substr(i);
    std::optional<uint64_t> v;
    if (str::starts_with(body, "0x") || str::starts_with(body, "0X")) {
      if (body.size() > 2) v = str::parse_uint(body.substr(2), 16);
    } else if (str::starts_with(body, "0o")) {
      if (body.size() > 2) v = str::parse_uint(body.substr(2), 8);
    } else if (str::starts_with(body, "0b")) {
      if (body.size() > 2) v = str::parse_uint(body.substr(2), 2);
    } else if (!body.empty() && body.find_first_not_of("0123456789") == std::string::npos) {
      v = (body.size() > 1 && body[0] == '0') ? str::parse_uint(body, 8) : str::parse_uint(body, 10);
    }
    if (v && *v <= static_cast<uint64_t>(INT64_MAX)) return Node::integer(neg ? -static_cast<int64_t>(*v) : static_cast<int64_t>(*v));
  }

  // Floats.
  {
    static const char* kInf[] = {".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF"};
    static const char* kNegInf[] = {"-.inf", "-.Inf", "-.INF"};
    static const char* kNan[] = {".nan", ".NaN", ".NAN"};
    for (const char* x : kInf)
      if (s == x) return Node::floating(INFINITY, s);
    for (const char* x : kNegInf)
      if (s == x) return Node::floating(-INFINITY, s);
    for (const char* x : kNan)
      if (s == x) return Node::floating(NAN, s);
    // ^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$
    size_t i = 0;
    if (i < t.size() && (t[i] == '-' || t[i] == '+')) i++;
    auto digit_run = [&] {  // digits at i, skipped; how many
      size_t n = 0;
      for (; i < t.size() && isdigit(static_cast<unsigned char>(t[i])); ++i) ++n;
      return n;
    };
    size_t digits = digit_run(), frac = 0;
    bool dot = false;
    if (i < t.size() && t[i] == '.') {
      dot = true;
      i++;
      frac = digit_run();
    }
    bool ok = digits > 0 || (dot && frac > 0);
    if (ok && i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
      i++;
      if (i < t.size() && (t[i] == '-' || t[i] == '+')) i++;
      ok = digit_run() > 0;
    }
    if (ok && i == t.size()) {
      auto f = str::parse_float(t);
      if (f) return Node::floating(*f, s);
    }
  }
  return Node::string(s);
}

// JSON-number resolution (inside flow collections a JSON number is also a
// valid plain YAML scalar, and resolve_plain handles it identically).

void append_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// ---------------------------------------------------------------------------
// Parser

struct Line {
  int no = 0;           // 1-based source line
  int indent = 0;       // leading spaces
  std::string raw;      // full raw line (no newline)
  std::string content;  // after indent, comment stripped, right-trimmed
  bool comment = false; // the line ends in a comment
};

class Parser {
 public:
  explicit Parser(const std::string& text) { split_lines(text); }

  Node parse_document() {
    size_t idx = next_content(0);
    if (idx >= lines_.size()) return Node::null();
    Node root;
    const Line& l = lines_[idx];
    if (is_flow_start(l.content) || (is_quote_start(l.content) && !split_key(l.content, l.no))) {
      root = parse_inline_value(l.content, idx, -1, false);
    } else {
      root = parse_block(idx, l.indent);
    }
    idx = next_content(idx);
    if (idx < lines_.size()) {
      if (lines_[idx].content == "---" || lines_[idx].content == "...")
        fail(lines_[idx], "multiple YAML documents are not supported");
      fail(lines_[idx], "unexpected content (check indentation)");
    }
    return root;
  }

 private:
  std::vector<Line> lines_;
  // Anchored nodes by name (&name), for aliases (*name) later in the document.
  std::map<std::string, Node> anchors_;

  [[noreturn]] static void fail(const Line& l, const std::string& msg) {
    throw Error("yaml: line " + std::to_string(l.no) + ": " + msg);
  }
  [[noreturn]] static void fail_no(int no, const std::string& msg) {
    throw Error("yaml: line " + std::to_string(no) + ": " + msg);
  }

  // Remove comments outside quoted scalars.  `s` may span lines (flow
  // collections gathered over several lines): quote state carries across
  // line breaks and a comment ends at the next one.
  static std::string strip_comment(const std::string& in) {
    std::string s = in;
    bool sq = false, dq = false;
    size_t closed = std::string::npos;  // just past the last closing quote
    for (size_t i = 0; i < s.size(); ++i) {
      char c = s[i];
      if (dq) {
        if (c == '\\') {
          ++i;
        } else if (c == '"') {
          dq = false;
          closed = i + 1;
        }
      } else if (sq) {
        if (c == '\'') {
          if (i + 1 < s.size() && s[i + 1] == '\'') {
            ++i;
          } else {
            sq = false;
            closed = i + 1;
          }
        }
      } else if (c == '"' && (i == 0 || strchr(" \t\n[{,:", s[i - 1]))) {
        dq = true;
      } else if (c == '\'' && (i == 0 || strchr(" \t\n[{,:", s[i - 1]))) {
        sq = true;
      } else if (c == '#' && (i == 0 || i == closed || s[i - 1] == ' ' || s[i - 1] == '\t' || s[i - 1] == '\n')) {
        // (Right after a closing quote too: the scalar has ended, libyaml and
        // PyYAML read the rest of the line as a comment.)
        size_t nl = s.find('\n', i);
        if (nl == std::string::npos) return s.substr(0, i);
        s.erase(i, nl - i);
        --i;  // the loop's ++i lands on the line break
      }
    }
    return s;
  }

  void split_lines(const std::string& text) {
    std::string t = text;
    // Strip UTF-8 BOM.
    if (t.size() >= 3 && static_cast<unsigned char>(t[0]) == 0xEF && static_cast<unsigned char>(t[1]) == 0xBB &&
        static_cast<unsigned char>(t[2]) == 0xBF)
      t = t.substr(3);
    int no = 0;
    size_t start = 0;
    bool seen_content = false, ended = false;  // ended: a "..." closed the document
    while (start <= t.size()) {
      size_t end = t.find('\n', start);
      if (end == std::string::npos) end = t.size();
      std::string raw = t.substr(start, end - start);
      if (!raw.empty() && raw.back() == '\r') raw.pop_back();
      ++no;
      Line l;
      l.no = no;
      l.raw = raw;
      size_t ind = 0;
      while (ind < raw.size() && raw[ind] == ' ') ++ind;
      if (ind < raw.size() && raw[ind] == '\t' && str::trim(raw).size() > 0 && str::trim(raw)[0] != '#')
        fail_no(no, "found character that cannot start any token (tab indentation)");
      l.indent = static_cast<int>(ind);
      std::string uncommented = strip_comment(raw.substr(ind));
      l.comment = uncommented.size() < raw.size() - ind;
      std::string body = str::trim(uncommented);
      // Directives / document markers before the first content.
      // Markers and directives count only at the start of a line; indented,
      // "---" and "..." are plain text.
      bool col0 = ind == 0;
      if (ended && !body.empty()) fail_no(no, "multiple YAML documents are not supported");
      if (col0 && !seen_content && (body == "---" || str::starts_with(body, "%"))) body.clear();
      if (col0 && !seen_content && str::starts_with(body, "--- ")) {
        body = str::trim(body.substr(4));
        l.indent = static_cast<int>(ind + 4);
      }
      if (col0 && body == "...") {
        body.clear();
        ended = seen_content;
      }
      if (col0 && seen_content && (body == "---" || str::starts_with(body, "--- ")))
        fail_no(no, "multiple YAML documents are not supported");
      l.content = body;
      if (!body.empty()) seen_content = true;
      lines_.push_back(std::move(l));
      if (end == t.size()) break;
      start = end + 1;
    }
  }

  size_t next_content(size_t idx) const {
    while (idx < lines_.size() && lines_[idx].content.empty()) ++idx;
    return idx;
  }

  static bool is_flow_start(const std::string& s) { return !s.empty() && (s[0] == '[' || s[0] == '{'); }
  static bool is_quote_start(const std::string& s) { return !s.empty() && (s[0] == '"' || s[0] == '\''); }
  static bool is_seq_entry(const std::string& s) { return s == "-" || str::starts_with(s, "- ") || str::starts_with(s, "-\t"); }

  // Split "key: rest" outside quotes/brackets.  Returns nullopt if the line is
  // not a mapping entry.
  static std::optional<std::pair<std::string, std::string>> split_key(const std::string& s, int lineno) {
    if (s.empty() || is_flow_start(s)) return std::nullopt;
    size_t i = 0;
    std::string key;
    if (s[0] == '"' || s[0] == '\'') {
      // An implicit key is on one line: a quote still open at the end of the
      // line starts a (multi-line) quoted value instead.
      size_t end;
      try {
        key = parse_quoted(s, 0, &end, lineno);
      } catch (const Error&) {
        return std::nullopt;
      }
      i = end;
      while (i < s.size() && s[i] == ' ') ++i;
      if (i >= s.size() || s[i] != ':') return std::nullopt;
      if (i + 1 < s.size() && s[i + 1] != ' ' && s[i + 1] != '\t') return std::nullopt;
      return std::make_pair(key, str::trim(s.substr(i + 1)));
    }
    if (s[0] == '?' && (s.size() == 1 || s[1] == ' ')) fail_no(lineno, "complex mapping keys are not supported");
    for (i = 0; i < s.size(); ++i) {
      if (s[i] == ':' && (i + 1 == s.size() || s[i + 1] == ' ' || s[i + 1] == '\t')) {
        key = str::trim(s.substr(0, i));
        if (key.empty()) return std::nullopt;
        // A plain key cannot start with these either (see parse_inline_value).
        if (strchr(",]}%@`|>", key[0])) fail_no(lineno, "found character that cannot start a mapping key");
        return std::make_pair(key, str::trim(s.substr(i + 1)));
      }
    }
    return std::nullopt;
  }

  // Line folding inside a quoted scalar, at the line break s[i]: trailing
  // blanks before it and leading blanks after each break are dropped; one
  // break becomes a space, n+1 breaks (n empty lines) become n newlines.
  // Returns the index of the first character of the continuation.
  static size_t fold_line_break(const std::string& s, size_t i, std::string& out) {
    while (!out.empty() && (out.back() == ' ' || out.back() == '\t')) out.pop_back();
    size_t empties = 0;
    size_t j = i + 1;
    for (;;) {
      while (j < s.size() && (s[j] == ' ' || s[j] == '\t')) ++j;
      if (j < s.size() && s[j] == '\n') {
        ++empties;
        ++j;
        continue;
      }
      break;
    }
    if (empties == 0) out.push_back(' ');
    else out.append(empties, '\n');
    return j;
  }

  // Parse a quoted scalar starting at s[pos]; *end is set past the closing quote.
  static std::string parse_quoted(const std::string& s, size_t pos, size_t* end, int lineno) {
    char q = s[pos];
    std::string out;
    size_t i = pos + 1;
    while (i < s.size()) {
      char c = s[i];
      if (q == '\'') {
        if (c == '\'') {
          if (i + 1 < s.size() && s[i + 1] == '\'') {
            out.push_back('\'');
            i += 2;
            continue;
          }
          *end = i + 1;
          return out;
        }
        if (c == '\n') {
          i = fold_line_break(s, i, out);
          continue;
        }
        out.push_back(c);
        ++i;
        continue;
      }
      // Double quoted.
      if (c == '"') {
        *end = i + 1;
        return out;
      }
      if (c == '\n') {
        i = fold_line_break(s, i, out);
        continue;
      }
      if (c == '\\') {
        if (i + 1 >= s.size()) break;
        char e = s[i + 1];
        i += 2;
        switch (e) {
          case '0': out.push_back('\0'); break;
          case 'a': out.push_back('\a'); break;
          case 'b': out.push_back('\b'); break;
          case 't': case '\t': out.push_back('\t'); break;
          case 'n': out.push_back('\n'); break;
          case 'v': out.push_back('\v'); break;
          case 'f': out.push_back('\f'); break;
          case 'r': out.push_back('\r'); break;
          case 'e': out.push_back('\x1b'); break;
          case ' ': out.push_back(' '); break;
          case '"': out.push_back('"'); break;
          case '/': out.push_back('/'); break;
          case '\\': out.push_back('\\'); break;
          case 'N': append_utf8(out, 0x85); break;
          case '_': append_utf8(out, 0xA0); break;
          case 'x':
          case 'u':
          case 'U': {
            size_t n = e == 'x' ? 2 : e == 'u' ? 4 : 8;
            if (i + n > s.size()) fail_no(lineno, "invalid escape in double-quoted scalar");
            auto v = str::parse_uint(s.substr(i, n), 16);
            if (!v) fail_no(lineno, "invalid escape in double-quoted scalar");
            uint32_t cp = static_cast<uint32_t>(*v);
            i += n;
            // JSON surrogate pairs.
            if (e == 'u' && cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              auto lo = str::parse_uint(s.substr(i + 2, 4), 16);
              if (lo && *lo >= 0xDC00 && *lo < 0xE000) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (static_cast<uint32_t>(*lo) - 0xDC00);
                i += 6;
              }
            }
            append_utf8(out, cp);
            break;
          }
          case '\n': {
            // Escaped line break: join without space.
            while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
            break;
          }
          default: fail_no(lineno, std::string("found unknown escape character '") + e + "'");
        }
        continue;
      }
      out.push_back(c);
      ++i;
    }
    fail_no(lineno, "found unexpected end of stream while scanning a quoted scalar");
  }

  // ---- Anchors, aliases and tags (go-yaml v2 resolves the same set).

  static const Node& alias(const std::map<std::string, Node>& anchors, const std::string& name, int lineno) {
    auto it = anchors.find(name);
    if (it == anchors.end()) fail_no(lineno, "unknown anchor '" + name + "' referenced");
    return it->second;
  }

  static void check_anchor_name(const std::string& name, int lineno) {
    if (name.empty()) fail_no(lineno, "did not find expected alphabetic or numeric character");
  }

  // Apply a tag to a parsed value.  `plain` is the untouched text of a plain
  // scalar (has_plain false for quoted/flow/block values).  !!str and the
  // non-specific "!" turn a plain scalar into a string as written.
  static Node apply_tag(const std::string& tag, Node v, bool has_plain, const std::string& plain, int lineno) {
    auto bad = [&](const char* what) -> Node {
      fail_no(lineno, std::string("cannot decode ") + what + " as " + tag);
    };
    if (tag == "!" || tag == "!!str") {
      if (has_plain) return Node::string(plain);
      if (v.kind() == Node::Kind::String) return v;
      if (v.is_null()) return Node::string("");
      if (v.kind() == Node::Kind::Bool) return Node::string(v.as_bool() ? "true" : "false");
      if (v.kind() == Node::Kind::Int) return Node::string(std::to_string(v.as_int()));
      if (v.kind() == Node::Kind::Float) return Node::string(v.text());
      return bad(v.kind_name().c_str());
    }
    // A quoted scalar under a scalar tag is resolved from its content.
    if (v.kind() == Node::Kind::String && !has_plain &&
        (tag == "!!int" || tag == "!!float" || tag == "!!bool" || tag == "!!null"))
      v = resolve_plain(v.text());
    if (tag == "!!int") return v.kind() == Node::Kind::Int ? v : bad(v.kind_name().c_str());
    if (tag == "!!float") {
      if (v.kind() == Node::Kind::Int) return Node::floating(static_cast<double>(v.as_int()));
      return v.kind() == Node::Kind::Float ? v : bad(v.kind_name().c_str());
    }
    if (tag == "!!bool") return v.kind() == Node::Kind::Bool ? v : bad(v.kind_name().c_str());
    if (tag == "!!null") return v.is_null() ? v : bad(v.kind_name().c_str());
    if (tag == "!!map") return v.is_map() ? v : bad(v.kind_name().c_str());
    if (tag == "!!seq") return v.is_seq() ? v : bad(v.kind_name().c_str());
    fail_no(lineno, "unsupported tag " + tag);
  }

  // "<<" entries: keys of the merged mapping(s) that the mapping does not
  // set itself; with a sequence of mappings the earlier one wins.
  static void apply_merges(Node& m, const std::vector<Node>& merges, int lineno) {
    for (const Node& src : merges) {
      std::vector<const Node*> maps;
      if (src.is_map()) {
        maps.push_back(&src);
      } else if (src.is_seq()) {
        for (const Node& item : src.items()) {
          if (!item.is_map()) fail_no(lineno, "map merge requires map or sequence of maps as the value");
          maps.push_back(&item);
        }
      } else {
        fail_no(lineno, "map merge requires map or sequence of maps as the value");
      }
      for (const Node* mp : maps)
        for (const auto& kv : mp->entries())
          if (!m.get(kv.first)) m.set(kv.first, kv.second);
    }
  }

  // ---- Flow parsing over a joined text buffer.
  struct Flow {
    const std::string& s;
    size_t i;
    int lineno;
    std::map<std::string, Node>* anchors;

    // Anchor or tag name: up to a blank or a flow indicator.
    std::string token() {
      size_t start = i;
      while (i < s.size() && !strchr(" \t\n\r,[]{}", s[i])) ++i;
      return s.substr(start, i - start);
    }

    [[noreturn]] void err(const std::string& m) const { fail_no(lineno, m); }
    void ws() {
      while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    Node value() {
      ws();
      if (i >= s.size()) err("unexpected end of flow collection");
      char c = s[i];
      if (c == '{') return mapping();
      if (c == '[') return sequence();
      if (c == '"' || c == '\'') {
        size_t end;
        std::string v = parse_quoted(s, i, &end, lineno);
        i = end;
        return Node::string(v);
      }
      if (c == '&') {
        ++i;
        std::string name = token();
        check_anchor_name(name, lineno);
        Node v = value_or_null();
        (*anchors)[name] = v;
        return v;
      }
      if (c == '*') {
        ++i;
        std::string name = token();
        check_anchor_name(name, lineno);
        return alias(*anchors, name, lineno);
      }
      if (c == '!') {
        std::string tag = token();
        ws();
        bool plain_next = i < s.size() && !strchr("[{\"'&*!,]}", s[i]);
        if (plain_next) {
          std::string text = plain_text(false);
          return apply_tag(tag, resolve_plain(text), true, text, lineno);
        }
        return apply_tag(tag, value_or_null(), false, "", lineno);
      }
      return Node(plain(false));
    }
    // A value that may be empty (before ',', ']' or '}').
    Node value_or_null() {
      ws();
      if (i >= s.size() || s[i] == ',' || s[i] == ']' || s[i] == '}') return Node::null();
      return value();
    }
    std::string plain_text(bool is_key) {
      size_t start = i;
      while (i < s.size()) {
        char c = s[i];
        if (c == ',' || c == ']' || c == '}') break;
        if (c == ':' && (i + 1 >= s.size() || strchr(" \t\n,]}", s[i + 1]))) break;
        if (is_key && c == ':') break;
        ++i;
      }
      // Line breaks fold (one space, or a newline per empty line); blanks
      // inside a line are content.
      std::string t = str::trim(s.substr(start, i - start));
      std::string out;
      for (size_t k = 0; k < t.size();) {
        if (t[k] == '\n') {
          k = fold_line_break(t, k, out);
          continue;
        }
        if (t[k] != '\r') out.push_back(t[k]);
        ++k;
      }
      return out;
    }
    Node plain(bool is_key) { return resolve_plain(plain_text(is_key)); }
    Node sequence() {
      Node n = Node::seq();
      ++i;  // [
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
        return n;
      }
      for (;;) {
        ws();
        if (i < s.size() && s[i] == ']') {  // trailing comma
          ++i;
          return n;
        }
        // "[a: b]" single-pair mappings inside sequences.
        size_t save = i;
        Node item = value();
        ws();
        if (i < s.size() && s[i] == ':' && item.is_scalar()) {
          i = save;
          n.push(single_pair());
        } else {
          n.push(std::move(item));
        }
        ws();
        if (i >= s.size()) err("did not find expected ',' or ']'");
        if (s[i] == ',') {
          ++i;
          continue;
        }
        if (s[i] == ']') {
          ++i;
          return n;
        }
        err("did not find expected ',' or ']'");
      }
    }
    std::string key() {
      ws();
      if (i >= s.size()) err("unexpected end of flow mapping");
      if (s[i] == '"' || s[i] == '\'') {
        size_t end;
        std::string k = parse_quoted(s, i, &end, lineno);
        i = end;
        return k;
      }
      if (s[i] == '{' || s[i] == '[') err("complex mapping keys are not supported");
      return plain_text(true);
    }
    Node single_pair() {
      Node m = Node::map();
      std::string k = key();
      ws();
      ++i;  // ':'
      m.set(k, value());
      return m;
    }
    Node mapping() {
      Node n = Node::map();
      std::vector<Node> merges;
      ++i;  // {
      for (;;) {
        ws();
        if (i >= s.size()) err("did not find expected ',' or '}'");
        if (s[i] == '}') {
          ++i;
          apply_merges(n, merges, lineno);
          return n;
        }
        bool quoted_key = s[i] == '"' || s[i] == '\'';
        std::string k = key();
        ws();
        Node v;
        if (i < s.size() && s[i] == ':') {
          ++i;
          ws();
          if (i < s.size() && (s[i] == ',' || s[i] == '}'))
            v = Node::null();
          else
            v = value();
        }
        if (k == "<<" && !quoted_key)
          merges.push_back(std::move(v));
        else
          n.set(k, std::move(v));
        ws();
        if (i >= s.size()) err("did not find expected ',' or '}'");
        if (s[i] == ',') {
          ++i;
          continue;
        }
        if (s[i] == '}') {
          ++i;
          apply_merges(n, merges, lineno);
          return n;
        }
        err("did not find expected ',' or '}'");
      }
    }
  };

  // Collect flow text starting with `first` (content of line idx-1) plus as
  // many following lines as needed to balance brackets.  Advances idx.
  std::string gather_flow(const std::string& first, size_t& idx, int lineno) {
    std::string raw = first;
    std::string buf = first;
    // A quote opens a quoted scalar only where a flow node starts (after
    // '[', '{', ',' or ": "); inside a plain scalar ("[0']") it is text.
    auto balanced = [](const std::string& t) {
      int depth = 0;
      bool sq = false, dq = false, node_start = true;
      for (size_t i = 0; i < t.size(); ++i) {
        char c = t[i];
        if (dq) {
          if (c == '\\')
            ++i;
          else if (c == '"')
            dq = false;
          continue;
        }
        if (sq) {
          // '' is an escaped quote: the scalar stays open ("'''['" is "'[").
          if (c == '\'') {
            if (i + 1 < t.size() && t[i + 1] == '\'')
              ++i;
            else
              sq = false;
          }
          continue;
        }
        if (c == ' ' || c == '\t' || c == '\n') continue;
        if (node_start && c == '"') dq = true;
        else if (node_start && c == '\'') sq = true;
        else if (c == '[' || c == '{') ++depth;
        else if (c == ']' || c == '}') --depth;
        node_start = c == '[' || c == '{' || c == ',' ||
                     (c == ':' && (i + 1 >= t.size() || t[i + 1] == ' ' || t[i + 1] == '\t' || t[i + 1] == '\n'));
      }
      return depth <= 0 && !sq && !dq;
    };
    while (!balanced(buf)) {
      if (idx >= lines_.size()) fail_no(lineno, "did not find expected end of flow collection");
      raw += "\n" + str::trim(lines_[idx].raw);
      buf = strip_comment(raw);
      ++idx;
    }
    return buf;
  }

  Node parse_flow_text(const std::string& text, int lineno) {
    Flow f{text, 0, lineno, &anchors_};
    Node n = f.value();
    f.ws();
    if (f.i != text.size()) fail_no(lineno, "unexpected trailing content after flow collection");
    return n;
  }

  // Block scalar (| or >) whose header is `header`; content lines follow idx
  // and are indented more than `parent_indent`.
  Node parse_block_scalar(const std::string& header, size_t& idx, int parent_indent, int lineno) {
    bool literal = header[0] == '|';
    char chomp = 'c';  // clip
    int explicit_indent = 0;
    bool chomp_seen = false;
    for (size_t k = 1; k < header.size(); ++k) {
      char c = header[k];
      if ((c == '-' || c == '+') && !chomp_seen) {
        chomp = c == '-' ? 's' : 'k';
        chomp_seen = true;
      } else if (c >= '1' && c <= '9' && !explicit_indent) {
        explicit_indent = c - '0';
      } else if (c == ' ' || c == '\t') {
        if (!str::trim(header.substr(k)).empty()) fail_no(lineno, "did not find expected comment or line break");
        break;
      } else {
        fail_no(lineno, "invalid block scalar header");
      }
    }
    std::vector<std::string> raw;
    int block_indent = explicit_indent ? parent_indent + explicit_indent : -1;
    while (idx < lines_.size()) {
      const Line& l = lines_[idx];
      bool blank = str::trim(l.raw).empty();
      if (!blank) {
        if (block_indent < 0) {
          if (l.indent <= parent_indent) break;
          block_indent = l.indent;
        }
        if (l.indent < block_indent) break;
        raw.push_back(l.raw.substr(static_cast<size_t>(block_indent)));
      } else {
        raw.push_back("");
      }
      ++idx;
    }
    // Trailing blank lines belong to chomping.
    size_t trailing = 0;
    while (!raw.empty() && raw.back().empty()) {
      raw.pop_back();
      ++trailing;
    }
    std::string out;
    if (literal) {
      for (size_t k = 0; k < raw.size(); ++k) {
        if (k > 0) out.push_back('\n');
        out += raw[k];
      }
    } else {
      // Folded: the break between two lines at the block's indentation
      // becomes a space, and when n empty lines separate them the first
      // break is dropped (n newlines).  Around a more-indented line every
      // break is kept.  Leading empty lines are newlines.
      auto more = [](const std::string& l) { return !l.empty() && (l[0] == ' ' || l[0] == '\t'); };
      size_t k = 0;
      while (k < raw.size() && raw[k].empty()) {
        out.push_back('\n');
        ++k;
      }
      while (k < raw.size()) {
        out += raw[k];
        size_t m = k + 1;
        while (m < raw.size() && raw[m].empty()) ++m;
        if (m >= raw.size()) break;  // trailing empties were taken off above
        size_t empties = m - k - 1;
        if (more(raw[k]) || more(raw[m])) out.append(empties + 1, '\n');
        else if (empties == 0) out.push_back(' ');
        else out.append(empties, '\n');
        k = m;
      }
    }
    if (!raw.empty()) {
      if (chomp == 'c') out.push_back('\n');
      else if (chomp == 'k') out.append(trailing + 1, '\n');
    }
    return Node::string(out);
  }

  // Characters that cannot start a block value (go-yaml/libyaml's scanner
  // and parser errors): flow terminators, reserved indicators, and a
  // sequence entry or complex key on the line of a mapping key.
  static void check_value_start(const std::string& rest, bool is_map_value, int lineno) {
    char c = rest[0];
    if (c == ',' || c == ']' || c == '}') fail_no(lineno, "did not find expected node content");
    if (c == '%' || c == '@' || c == '`') fail_no(lineno, "found character that cannot start any token");
    if (is_map_value && (c == '-' || c == '?') && (rest.size() == 1 || rest[1] == ' ' || rest[1] == '\t'))
      fail_no(lineno, c == '-' ? "block sequence entries are not allowed in this context"
                               : "mapping keys are not allowed in this context");
  }

  // Value text appearing inline after "key:" or "- ".  idx points at the line
  // after the one holding `rest`.
  Node parse_inline_value(const std::string& rest, size_t& idx, int parent_indent, bool is_map_value) {
    int lineno = idx > 0 && idx <= lines_.size() ? lines_[idx - 1].no : 0;
    if (idx < lines_.size() && parent_indent < 0) lineno = lines_[idx].no;
    if (rest.empty()) {
      size_t j = next_content(idx);
      if (j < lines_.size()) {
        const Line& l = lines_[j];
        if (l.indent > parent_indent) {
          idx = j;
          return parse_block(idx, l.indent);
        }
        if (is_map_value && l.indent == parent_indent && is_seq_entry(l.content)) {
          idx = j;
          return parse_seq(idx, l.indent);
        }
      }
      return Node::null();
    }
    if (parent_indent < 0) {
      // Document-level flow/quoted value; idx currently points AT the line.
      std::string text = gather_flow(rest, ++idx, lineno);
      if (is_quote_start(text)) {
        size_t end;
        std::string v = parse_quoted(text, 0, &end, lineno);
        if (!str::trim(text.substr(end)).empty()) fail_no(lineno, "unexpected content after quoted scalar");
        return Node::string(v);
      }
      return parse_flow_text(text, lineno);
    }
    char c = rest[0];
    check_value_start(rest, is_map_value, lineno);
    if (c == '[' || c == '{') return parse_flow_text(gather_flow(rest, idx, lineno), lineno);
    if (c == '"' || c == '\'') {
      std::string text = rest;
      size_t end = 0;
      // Multi-line quoted scalars: append following raw lines until it closes.
      for (;;) {
        try {
          std::string v = parse_quoted(text, 0, &end, lineno);
          if (!str::trim(text.substr(end)).empty()) fail_no(lineno, "unexpected content after quoted scalar");
          return Node::string(v);
        } catch (const Error&) {
          if (idx >= lines_.size()) throw;
          text += "\n" + str::trim(lines_[idx].raw);
          ++idx;
        }
      }
    }
    if (c == '|' || c == '>') return parse_block_scalar(rest, idx, parent_indent, lineno);
    if (c == '&' || c == '*' || c == '!') {
      size_t sp = rest.find_first_of(" \t");
      std::string name = rest.substr(c == '!' ? 0 : 1, sp == std::string::npos ? std::string::npos : sp - (c == '!' ? 0 : 1));
      std::string after = sp == std::string::npos ? std::string() : str::trim(rest.substr(sp));
      if (c == '*') {
        check_anchor_name(name, lineno);
        if (!after.empty()) fail_no(lineno, "unexpected content after alias *" + name);
        return alias(anchors_, name, lineno);
      }
      if (c == '&') {
        check_anchor_name(name, lineno);
        Node v = parse_inline_value(after, idx, parent_indent, is_map_value);
        anchors_[name] = v;
        return v;
      }
      if (!after.empty() && !strchr("[{\"'|>&*!", after[0])) {
        check_value_start(after, true, lineno);
        std::string text = gather_plain(after, idx, parent_indent);
        return apply_tag(name, resolve_plain(text), true, text, lineno);
      }
      return apply_tag(name, parse_inline_value(after, idx, parent_indent, is_map_value), false, "", lineno);
    }
    return resolve_plain(gather_plain(rest, idx, parent_indent));
  }

  // Plain scalar text starting with `rest`, continued on more-indented lines.
  // A ':' followed by a blank or the end of the line ends a block plain
  // scalar and would start a mapping value where none may be ("a: b: c",
  // go-yaml/PyYAML: "mapping values are not allowed in this context").
  std::string gather_plain(const std::string& rest, size_t& idx, int parent_indent) {
    auto mapping_indicator = [](const std::string& t) {
      for (size_t k = 0; k < t.size(); ++k)
        if (t[k] == ':' && (k + 1 == t.size() || t[k + 1] == ' ' || t[k + 1] == '\t')) return true;
      return false;
    };
    if (mapping_indicator(rest)) {
      int no = idx > 0 && idx <= lines_.size() ? lines_[idx - 1].no : 0;
      fail_no(no, "mapping values are not allowed in this context");
    }
    std::string text = rest;
    for (;;) {
      // Line folding: one break is a space, a break and n empty lines are n
      // newlines.  A comment line ends the scalar.
      size_t j = idx, empties = 0;
      while (j < lines_.size() && lines_[j].content.empty()) {
        if (str::trim(lines_[j].raw).empty()) {
          ++empties;
        } else {
          return text;  // a comment line
        }
        ++j;
      }
      if (j >= lines_.size() || lines_[j].indent <= parent_indent) break;
      const Line& l = lines_[j];
      // A comment on the previous line ended the scalar.
      if (idx > 0 && lines_[idx - 1].comment) fail(l, "could not find expected ':'");
      // "- x" here is text ("b - x", as libyaml reads it); "x: y" or ": y" is not.
      if (mapping_indicator(l.content)) fail(l, "mapping values are not allowed in this context");
      text += empties ? std::string(empties, '\n') : std::string(" ");
      text += l.content;
      idx = j + 1;
    }
    return text;
  }

  Node parse_block(size_t& idx, int indent) {
    idx = next_content(idx);
    if (idx >= lines_.size()) return Node::null();
    if (is_seq_entry(lines_[idx].content)) return parse_seq(idx, indent);
    const Line& l = lines_[idx];
    if (!split_key(l.content, l.no)) {
      // A bare scalar as a nested block value.
      std::string c = l.content;
      ++idx;
      return parse_inline_value(c, idx, indent - 1, false);
    }
    return parse_map(idx, indent);
  }

  Node parse_map(size_t& idx, int indent) {
    Node m = Node::map();
    std::vector<Node> merges;
    int merge_line = 0;
    for (;;) {
      idx = next_content(idx);
      if (idx >= lines_.size()) break;
      Line& l = lines_[idx];
      if (l.indent < indent) break;
      if (l.indent > indent) fail(l, "bad indentation of a mapping entry");
      if (is_seq_entry(l.content)) break;  // compact sequence owned by caller
      auto kv = split_key(l.content, l.no);
      if (!kv) fail(l, "could not find expected ':'");
      if (kv->first.size() >= 2 && (kv->first[0] == '&' || kv->first[0] == '*' || kv->first[0] == '!'))
        fail(l, "anchors, aliases and tags on mapping keys are not supported");
      int no = l.no;
      bool merge = kv->first == "<<" && l.content[0] == '<';
      ++idx;
      Node v = parse_inline_value(kv->second, idx, indent, true);
      if (merge) {
        merges.emplace_back(std::move(v));
        merge_line = no;
      } else {
        m.set(kv->first, std::move(v));
      }
    }
    apply_merges(m, merges, merge_line);
    return m;
  }

  Node parse_seq(size_t& idx, int indent) {
    Node s = Node::seq();
    for (;;) {
      idx = next_content(idx);
      if (idx >= lines_.size()) break;
      Line& l = lines_[idx];
      if (l.indent < indent) break;
      if (l.indent > indent) fail(l, "bad indentation of a sequence entry");
      if (!is_seq_entry(l.content)) break;
      std::string rest = l.content.size() > 1 ? l.content.substr(1) : std::string();
      size_t pad = 1;
      while (pad < l.content.size() && (l.content[pad] == ' ' || l.content[pad] == '\t')) ++pad;
      rest = str::trim(rest);
      if (rest.empty()) {
        ++idx;
        s.push(parse_inline_value("", idx, indent, false));
        continue;
      }
      if (is_seq_entry(rest) || (!is_flow_start(rest) && split_key(rest, l.no))) {
        // Nested collection starting on the same line: re-anchor the line at
        // the column of `rest` and parse it as a block.
        l.indent = indent + static_cast<int>(pad);
        l.content = rest;
        s.push(parse_block(idx, l.indent));
        continue;
      }
      ++idx;
      s.push(parse_inline_value(rest, idx, indent, false));
    }
    return s;
  }
};

void write_json(std::string& out, const Node& n, int indent, int depth) {
  auto nl = [&](int d) {
    if (indent < 0) return;
    out.push_back('\n');
    out.append(static_cast<size_t>(indent * d), ' ');
  };
  switch (n.kind()) {
    case Node::Kind::Null: out += "null"; break;
    case Node::Kind::Bool: out += n.as_bool() ? "true" : "false"; break;
    case Node::Kind::Int: out += std::to_string(n.as_int()); break;
    case Node::Kind::Float: {
      double f = n.as_float();
      if (std::isnan(f) || std::isinf(f)) {
        out += "null";
      } else {
        char buf[64];
        snprintf(buf, sizeof(buf), "%.17g", f);
        out += buf;
      }
      break;
    }
    case Node::Kind::String: out += json_quote(n.text()); break;
    case Node::Kind::Seq: {
      if (n.items().empty()) {
        out += "[]";
        break;
      }
      out.push_back('[');
      for (size_t k = 0; k < n.items().size(); ++k) {
        if (k) out.push_back(',');
        nl(depth + 1);
        write_json(out, n.items()[k], indent, depth + 1);
      }
      nl(depth);
      out.push_back(']');
      break;
    }
    case Node::Kind::Map: {
      if (n.entries().empty()) {
        out += "{}";
        break;
      }
      out.push_back('{');
      for (size_t k = 0; k < n.entries().size(); ++k) {
        if (k) out.push_back(',');
        nl(depth + 1);
        out += json_quote(n.entries()[k].first);
        out += indent < 0 ? ":" : ": ";
        write_json(out, n.entries()[k].second, indent, depth + 1);
      }
      nl(depth);
      out.push_back('}');
      break;
    }
  }
}

}  // namespace

Node parse(const std::string& text) {
  Parser p(text);
  return p.parse_document();
}

std::string json_quote(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
  return out;
}

std::string to_json(const Node& n, int indent) {
  std::string out;
  write_json(out, n, indent, 0);
  return out;
}

}  // namespace gfd::yaml
