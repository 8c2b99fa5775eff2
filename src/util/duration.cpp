#include "util/duration.h"

#include <cstring>
#include <limits>

#include "util/error.h"

namespace gfd {

namespace {

[[noreturn]] void invalid(const std::string& orig) { throw Error("time: invalid duration \"" + orig + "\""); }

struct Unit {
  const char* name;
  uint64_t ns;
};

// Longest names first where one is a prefix of another ("ms" vs "m").
const Unit kUnits[] = {
    {"ns", 1ULL},
    {"us", 1000ULL},
    {"\xC2\xB5s", 1000ULL},  // U+00B5 micro sign
    {"\xCE\xBCs", 1000ULL},  // U+03BC greek mu
    {"ms", 1000000ULL},
    {"s", 1000000000ULL},
    {"m", 60ULL * 1000000000ULL},
    {"h", 3600ULL * 1000000000ULL},
};

// Prints the fraction of v / 10^prec into buf ending at w, omitting trailing
// zeros; returns the new w and stores v / 10^prec in *nv (Go's fmtFrac).
int fmt_frac(char* buf, int w, uint64_t v, int prec, uint64_t* nv) {
  bool print = false;
  for (int i = 0; i < prec; i++) {
    uint64_t digit = v % 10;
    print = print || digit != 0;
    if (print) {
      w--;
      buf[w] = static_cast<char>(digit + '0');
    }
    v /= 10;
  }
  if (print) {
    w--;
    buf[w] = '.';
  }
  *nv = v;
  return w;
}

int fmt_int(char* buf, int w, uint64_t v) {
  if (v == 0) {
    w--;
    buf[w] = '0';
  } else {
    while (v > 0) {
      w--;
      buf[w] = static_cast<char>(v % 10 + '0');
      v /= 10;
    }
  }
  return w;
}

}  // namespace

Nanos parse_duration(const std::string& orig) {
  const std::string& s0 = orig;
  size_t i = 0;
  bool neg = false;
  if (i < s0.size() && (s0[i] == '-' || s0[i] == '+')) {
    neg = s0[i] == '-';
    i++;
  }
  if (s0.substr(i) == "0") return 0;
  if (i == s0.size()) invalid(orig);

  uint64_t total = 0;
  const uint64_t kMax = static_cast<uint64_t>(std::numeric_limits<int64_t>::max());
  while (i < s0.size()) {
    // Integer part.
    if (!(s0[i] == '.' || (s0[i] >= '0' && s0[i] <= '9'))) invalid(orig);
    uint64_t v = 0;
    size_t start = i;
    bool overflow = false;
    while (i < s0.size() && s0[i] >= '0' && s0[i] <= '9') {
      if (v > (kMax - (s0[i] - '0')) / 10) overflow = true;
      v = v * 10 + static_cast<uint64_t>(s0[i] - '0');
      i++;
    }
    if (overflow) invalid(orig);
    bool pre = i != start;
    // Fraction.
    uint64_t f = 0;
    double scale = 1;
    bool post = false;
    if (i < s0.size() && s0[i] == '.') {
      i++;
      size_t fs = i;
      while (i < s0.size() && s0[i] >= '0' && s0[i] <= '9') {
        if (f < (kMax - 9) / 10) {  // drop digits beyond precision, like Go
          f = f * 10 + static_cast<uint64_t>(s0[i] - '0');
          scale *= 10;
        }
        i++;
      }
      post = i != fs;
    }
    if (!pre && !post) invalid(orig);
    // Unit.
    size_t us = i;
    while (i < s0.size() && s0[i] != '.' && !(s0[i] >= '0' && s0[i] <= '9')) i++;
    if (us == i) throw Error("time: missing unit in duration \"" + orig + "\"");
    std::string u = s0.substr(us, i - us);
    uint64_t unit = 0;
    for (const auto& cand : kUnits)
      if (u == cand.name) unit = cand.ns;
    if (unit == 0) throw Error("time: unknown unit \"" + u + "\" in duration \"" + orig + "\"");
    if (v > kMax / unit) invalid(orig);
    v *= unit;
    if (f > 0) {
      v += static_cast<uint64_t>(static_cast<double>(f) * (static_cast<double>(unit) / scale));
      if (v > kMax) invalid(orig);
    }
    total += v;
    if (total > kMax) invalid(orig);
  }
  return neg ? -static_cast<Nanos>(total) : static_cast<Nanos>(total);
}

std::string format_duration(Nanos d) {
  char buf[32];
  int w = sizeof(buf);
  uint64_t u = d < 0 ? static_cast<uint64_t>(-(d + 1)) + 1 : static_cast<uint64_t>(d);
  bool neg = d < 0;
  if (u < static_cast<uint64_t>(kSecond)) {
    int prec = 0;
    w--;
    buf[w] = 's';
    w--;
    if (u == 0) return "0s";
    if (u < 1000ULL) {
      prec = 0;
      buf[w] = 'n';
    } else if (u < 1000000ULL) {
      prec = 3;
      // U+00B5 'µ' as two bytes.
      w--;
      std::memcpy(&buf[w], "\xC2\xB5", 2);
    } else {
      prec = 6;
      buf[w] = 'm';
    }
    w = fmt_frac(buf, w, u, prec, &u);
    w = fmt_int(buf, w, u);
  } else {
    w--;
    buf[w] = 's';
    w = fmt_frac(buf, w, u, 9, &u);
    w = fmt_int(buf, w, u % 60);
    u /= 60;
    if (u > 0) {
      w--;
      buf[w] = 'm';
      w = fmt_int(buf, w, u % 60);
      u /= 60;
      if (u > 0) {
        w--;
        buf[w] = 'h';
        w = fmt_int(buf, w, u);
      }
    }
  }
  if (neg) {
    w--;
    buf[w] = '-';
  }
  return std::string(buf + w, sizeof(buf) - static_cast<size_t>(w));
}

}  // namespace gfd
