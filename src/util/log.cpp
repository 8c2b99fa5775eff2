#include "util/log.h"

#include <atomic>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <sys/time.h>

#include <string>
#include <vector>

namespace gfd::log {

namespace {
std::atomic<bool> g_quiet{false};
thread_local Hold* t_hold = nullptr;  // the innermost Hold of this thread

bool starts_with(const char* msg, size_t len, const char* word) {
  size_t n = std::strlen(word);
  return len >= n && std::memcmp(msg, word, n) == 0;
}
}  // namespace

struct HoldChain {
  // Everything held by the thread's Holds, outermost first (the order the
  // lines were logged in: an inner Hold only holds lines logged after the
  // outer one's), taken out of them.
  static std::string take_all() {
    std::vector<Hold*> chain;
    for (Hold* h = t_hold; h; h = h->prev_) chain.push_back(h);
    std::string out;
    for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
      out.append((*it)->buf_);
      (*it)->buf_.clear();
    }
    return out;
  }
  static void append(const std::string& line) { t_hold->buf_.append(line); }
};

namespace {

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
  if (t_hold) {
    // Warnings and errors are never held: a cycle that then hangs (a wedged
    // library call) or is killed must still have said why.  What every
    // enclosing Hold holds goes out first, so the order stays.
    bool urgent = starts_with(msg, len, "Warning") || starts_with(msg, len, "WARNING") || starts_with(msg, len, "Error");
    if (!urgent) {
      HoldChain::append(out);
      return;
    }
    out.insert(0, HoldChain::take_all());
  }
  fwrite(out.data(), 1, out.size(), stderr);
}
}  // namespace

bool set_quiet(bool q) { return g_quiet.exchange(q); }

Hold::Hold() : prev_(t_hold) { t_hold = this; }

Hold::~Hold() {
  flush();
  t_hold = prev_;
}

void Hold::flush() {
  if (buf_.empty()) return;
  if (prev_) {
    prev_->buf_.append(buf_);  // nested: the outer Hold writes it
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
