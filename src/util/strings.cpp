#include "util/strings.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

namespace gfd::str {

namespace {
bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
}  // namespace

std::string trim(std::string_view s) {
  size_t b = 0, e = s.size();
  while (b < e && is_space(s[b])) ++b;
  while (e > b && is_space(s[e - 1])) --e;
  return std::string(s.substr(b, e - b));
}

std::vector<std::string> split(std::string_view s, char sep) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == sep) {
      out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return out;
}

std::vector<std::string> split_n(std::string_view s, char sep, size_t n) {
  std::vector<std::string> out;
  if (n == 0) return out;
  size_t start = 0;
  for (size_t i = 0; i < s.size() && out.size() + 1 < n; ++i) {
    if (s[i] == sep) {
      out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  out.emplace_back(s.substr(start));
  return out;
}

std::string join(const std::vector<std::string>& parts, std::string_view sep) {
  std::string out;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) out.append(sep);
    out.append(parts[i]);
  }
  return out;
}

std::string replace_all(std::string s, std::string_view from, std::string_view to) {
  if (from.empty()) return s;
  size_t pos = 0;
  while ((pos = s.find(from, pos)) != std::string::npos) {
    s.replace(pos, from.size(), to);
    pos += to.size();
  }
  return s;
}

std::string to_lower(std::string s) {
  for (auto& c : s)
    if (c >= 'A' && c <= 'Z') c = static_cast<char>(c - 'A' + 'a');
  return s;
}

std::string to_upper(std::string s) {
  for (auto& c : s)
    if (c >= 'a' && c <= 'z') c = static_cast<char>(c - 'a' + 'A');
  return s;
}

bool starts_with(std::string_view s, std::string_view p) { return s.size() >= p.size() && s.compare(0, p.size(), p) == 0; }

std::optional<int64_t> parse_int(std::string_view sv, int base) {
  std::string s = trim(sv);
  if (s.empty()) return std::nullopt;
  errno = 0;
  char* end = nullptr;
  long long v = strtoll(s.c_str(), &end, base);
  if (errno != 0 || end != s.c_str() + s.size()) return std::nullopt;
  return static_cast<int64_t>(v);
}

std::optional<uint64_t> parse_uint(std::string_view sv, int base) {
  std::string s = trim(sv);
  if (s.empty() || s[0] == '-' || s[0] == '+') return std::nullopt;
  errno = 0;
  char* end = nullptr;
  unsigned long long v = strtoull(s.c_str(), &end, base);
  if (errno != 0 || end != s.c_str() + s.size()) return std::nullopt;
  return static_cast<uint64_t>(v);
}

std::optional<uint64_t> parse_uint_auto(std::string_view sv) {
  std::string s = trim(sv);
  if (starts_with(s, "0x") || starts_with(s, "0X")) return parse_uint(std::string_view(s).substr(2), 16);
  return parse_uint(s, 10);
}

std::optional<double> parse_float(std::string_view sv) {
  std::string s = trim(sv);
  if (s.empty()) return std::nullopt;
  errno = 0;
  char* end = nullptr;
  double v = strtod(s.c_str(), &end);
  if (end != s.c_str() + s.size()) return std::nullopt;
  // Like Go's strconv.ParseFloat: overflow is an error, underflow (a
  // subnormal or zero result, also ERANGE for strtod) is not.
  if (errno == ERANGE && std::isinf(v)) return std::nullopt;
  if (errno != 0 && errno != ERANGE) return std::nullopt;
  return v;
}

std::optional<bool> parse_bool(std::string_view s) {
  if (s == "1" || s == "t" || s == "T" || s == "TRUE" || s == "true" || s == "True") return true;
  if (s == "0" || s == "f" || s == "F" || s == "FALSE" || s == "false" || s == "False") return false;
  return std::nullopt;
}

std::string format(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n < 0) return {};
  if (static_cast<size_t>(n) < sizeof(buf)) return std::string(buf, static_cast<size_t>(n));
  std::string out(static_cast<size_t>(n) + 1, '\0');
  va_start(ap, fmt);
  vsnprintf(out.data(), out.size(), fmt, ap);
  va_end(ap);
  out.resize(static_cast<size_t>(n));
  return out;
}

std::string bool_str(bool b) { return b ? "true" : "false"; }

}  // namespace gfd::str
