// Error type shared by every layer of the daemon.
//
// The reference threads Go `error` values up the stack and wraps them with
// fmt.Errorf("context: %v", err) at each level (e.g. internal/lm/nvml.go:30-32,
// cmd/gpu-feature-discovery/main.go:161-163).  Error paths are cold here (a
// labeling cycle either succeeds or the daemon exits), so we use a single
// exception type and wrap with `wrap()` to keep the same "outer: inner"
// message shape in the logs.
#pragma once

#include <stdexcept>
#include <string>

namespace gfd {

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& msg) : std::runtime_error(msg) {}
};

// Re-throw `e` with `context` prepended, Go-style: "context: inner".
[[noreturn]] inline void rethrow_wrapped(const std::string& context, const std::exception& e) {
  throw Error(context + ": " + e.what());
}

}  // namespace gfd

// Evaluate `expr`; if it throws, re-throw with `ctx` prepended.
#define GFD_WRAP(ctx, expr)                         \
  [&]() -> decltype(auto) {                         \
    try {                                           \
      return (expr);                                \
    } catch (const std::exception& gfd_wrap_e__) {  \
      ::gfd::rethrow_wrapped((ctx), gfd_wrap_e__);  \
    }                                               \
  }()
