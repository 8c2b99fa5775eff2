// Minimal logger with the same line shape as Go's stdlib `log` package
// ("2006/01/02 15:04:05 message"), which the reference uses everywhere
// (e.g. cmd/gpu-feature-discovery/main.go:111-146).  Output goes to stderr so
// that `--output-file=""` (labels on stdout, internal/lm/labels.go:38-41)
// stays machine-readable.
#pragma once

#include <cstdarg>
#include <string>

namespace gfd::log {

// printf-style log line; a trailing newline is added if missing.
void printf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Silence all log output (used by the in-process benchmark binding so that
// timing is not dominated by stderr writes).  Returns the previous setting.
bool set_quiet(bool quiet);
bool quiet();

// While a Hold lives, this thread's log lines (each stamped when logged)
// are collected and written together - in log order, one write(2) - when it
// is flushed or destroyed.  The daemon holds a cycle's lines until the
// feature file is in place: a line to stderr, usually a pipe to the
// container runtime, is a syscall the labels do not wait for.  Warning and
// error lines are written at once (with what was held before them).
class Hold {
 public:
  Hold();
  ~Hold();
  Hold(const Hold&) = delete;
  Hold& operator=(const Hold&) = delete;
  void flush();

 private:
  friend struct HoldChain;
  std::string buf_;
  Hold* prev_;  // the enclosing Hold on this thread, if any
};

}  // namespace gfd::log
