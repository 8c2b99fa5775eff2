// libFuzzer target: command-line and environment parsing (urfave/cli
// semantics, src/cli/flags.cpp).  The input is split on NUL bytes into
// arguments; an argument "ENV:NAME=VALUE" becomes an environment variable
// instead.  Parsing must end in a Context or a UsageError / gfd::Error, and
// every flag's typed accessor must then answer or throw gfd::Error.
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "cli/flags.h"
#include "util/error.h"

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  std::string in(reinterpret_cast<const char*>(data), size);
  std::vector<std::string> args;
  std::map<std::string, std::string> env;
  size_t pos = 0;
  while (pos <= in.size()) {
    size_t end = in.find('\0', pos);
    if (end == std::string::npos) end = in.size();
    std::string tok = in.substr(pos, end - pos);
    if (tok.rfind("ENV:", 0) == 0 && tok.find('=') != std::string::npos) {
      env[tok.substr(4, tok.find('=') - 4)] = tok.substr(tok.find('=') + 1);
    } else {
      args.push_back(tok);
    }
    pos = end + 1;
  }
  static const std::vector<gfd::cli::FlagDef> defs = gfd::cli::gfd_flags();
  try {
    auto ctx = gfd::cli::Context::parse(defs, args, &env);
    for (const auto& d : defs) {
      try {
        (void)ctx.IsSet(d.name);
        switch (d.type) {
          case gfd::cli::FlagType::String: (void)ctx.String(d.name); break;
          case gfd::cli::FlagType::Bool: (void)ctx.Bool(d.name); break;
          case gfd::cli::FlagType::Duration: (void)ctx.Duration(d.name); break;
        }
      } catch (const gfd::Error&) {
      }
    }
  } catch (const gfd::cli::UsageError&) {
  } catch (const gfd::Error&) {
  }
  return 0;
}
