// Small string helpers used across layers (no locale, no allocation-heavy
// stream machinery on the labeling hot path).
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace gfd::str {

std::string trim(std::string_view s);
std::vector<std::string> split(std::string_view s, char sep);
std::vector<std::string> split_n(std::string_view s, char sep, size_t n);
std::string join(const std::vector<std::string>& parts, std::string_view sep);
std::string replace_all(std::string s, std::string_view from, std::string_view to);
std::string to_lower(std::string s);
std::string to_upper(std::string s);
bool starts_with(std::string_view s, std::string_view prefix);

// Strict parses: the whole (trimmed) string must be consumed.
std::optional<int64_t> parse_int(std::string_view s, int base = 10);
std::optional<uint64_t> parse_uint(std::string_view s, int base = 10);
// Accepts decimal or 0x-prefixed hex.
std::optional<uint64_t> parse_uint_auto(std::string_view s);
std::optional<double> parse_float(std::string_view s);
// Go's strconv.ParseBool: 1,t,T,TRUE,true,True,0,f,F,FALSE,false,False.
std::optional<bool> parse_bool(std::string_view s);

std::string format(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
std::string bool_str(bool b);

}  // namespace gfd::str
