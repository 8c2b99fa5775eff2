#include "util/log.h"

#include <atomic>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <sys/time.h>

namespace gfd::log {

namespace {
std::atomic<bool> g_quiet{false};
thread_local std::string* t_held = nullptr;  // the innermost Hold's buffer

void emit(const char* msg, size_t len) {
  // The stamp only changes once a second: the lines of one cycle share one
  // localtime_r/strftime (per thread).
  thread_local time_t stamp_sec = -1;
  thread_local char stamp[32];
  time_t now = time(nullptr);
  if (now != stamp_sec) {
    struct tm tmv;
    localtime_r(&now, &tmv);
    strftime(stamp, sizeof(stamp), "%Y/%m/%d %H:%M:%S ", &tmv);
    stamp_sec = now;
  }
  // One fwrite per piece; stderr is unbuffered so keep the pieces few.
  std::string out;
  out.reserve(len + 24);
  out.append(stamp);
  out.append(msg, len);
  if (len == 0 || msg[len - 1] != '\n') out.push_back('\n');
  if (t_held) {
    // Warnings and errors are never held: a cycle that then hangs (a wedged
    // library call) or is killed must still have said why.  What is held
    // goes out first, so the order stays.
    bool urgent = len >= 5 && (std::strncmp(msg, "Warning", 7) == 0 || std::strncmp(msg, "WARNING", 7) == 0 ||
                                std::strncmp(msg, "Error", 5) == 0);
    if (!urgent) {
      t_held->append(out);
      return;
    }
    out.insert(0, *t_held);
    t_held->clear();
  }
  fwrite(out.data(), 1, out.size(), stderr);
}
}  // namespace

bool set_quiet(bool q) { return g_quiet.exchange(q); }

Hold::Hold() : prev_(t_held) { t_held = &buf_; }

Hold::~Hold() {
  flush();
  t_held = prev_;
}

void Hold::flush() {
  if (buf_.empty()) return;
  if (prev_) {
    prev_->append(buf_);  // nested: the outer Hold writes it
  } else {
    fwrite(buf_.data(), 1, buf_.size(), stderr);
  }
  buf_.clear();
}
bool quiet() { return g_quiet.load(std::memory_order_relaxed); }

void printf(const char* fmt, ...) {
  if (quiet()) return;
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n < 0) return;
  if (static_cast<size_t>(n) >= sizeof(buf)) {
    std::string big(static_cast<size_t>(n) + 1, '\0');
    va_start(ap, fmt);
    vsnprintf(big.data(), big.size(), fmt, ap);
    va_end(ap);
    emit(big.data(), static_cast<size_t>(n));
    return;
  }
  emit(buf, static_cast<size_t>(n));
}

}  // namespace gfd::log
