// Command-line flag parsing with urfave/cli v2 + Go `flag` semantics.
//
// Reference: cmd/gpu-feature-discovery/main.go:33-82 (flag table) and the
// vendored urfave/cli v2 behaviour operators rely on:
//   * `-name`, `--name`, `-name=value`, `--name value` (non-bool), aliases
//     (`-o` / `--output` for `--output-file`); parsing stops at the first
//     non-flag argument or `--`;
//   * bool flags take `--flag` or `--flag=false` (never a separate value);
//   * env vars (first one *present* wins, flag.go:400-415): a string env var
//     applies even when empty; bool/duration env vars apply only when
//     non-empty and must parse (flag_bool.go:46-61, flag_duration.go:46-61);
//   * precedence CLI > env > default; IsSet() is true for CLI or env
//     (context.go:53-74) — that is what lets the config file fill in only
//     what neither the CLI nor the environment set;
//   * `--help/-h` and `--version/-v` are built in.
#pragma once

#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "util/duration.h"

namespace gfd::cli {

enum class FlagType { String, Bool, Duration };

struct FlagDef {
  std::string name;
  std::vector<std::string> aliases;
  FlagType type = FlagType::String;
  std::string default_value;  // textual default ("" / "true" / "1m0s")
  std::vector<std::string> env_vars;
  std::string usage;
  bool hidden = false;
};

// Flag parsing failure (urfave prints "Incorrect Usage: <msg>" + help).
class UsageError : public std::runtime_error {
 public:
  explicit UsageError(const std::string& m) : std::runtime_error(m) {}
};

class Context {
 public:
  // Parse argv[1..] against `defs` with `env` lookup (nullptr = getenv).
  static Context parse(const std::vector<FlagDef>& defs, const std::vector<std::string>& args,
                       const std::map<std::string, std::string>* env = nullptr);

  bool help_requested() const { return help_; }
  bool version_requested() const { return version_; }
  const std::vector<std::string>& positional() const { return positional_; }

  bool IsSet(const std::string& name) const;
  std::string String(const std::string& name) const;
  bool Bool(const std::string& name) const;
  Nanos Duration(const std::string& name) const;
  const std::vector<FlagDef>& defs() const { return defs_; }

 private:
  struct Value {
    std::string text;
    bool from_cli = false;
    bool from_env = false;
  };
  const FlagDef* find(const std::string& name) const;

  std::vector<FlagDef> defs_;
  std::map<std::string, Value> values_;  // by canonical name
  std::vector<std::string> positional_;
  bool help_ = false;
  bool version_ = false;
};

// The daemon's flag table (reference flags + AMD extensions).
std::vector<FlagDef> gfd_flags();
// urfave-style help text.
std::string help_text(const std::vector<FlagDef>& defs, const std::string& app_name, const std::string& usage,
                      const std::string& version);

}  // namespace gfd::cli
