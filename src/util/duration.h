// Go-compatible time.Duration parsing and formatting.
//
// The reference's `--sleep-interval` is a urfave DurationFlag
// (cmd/gpu-feature-discovery/main.go:58-63) and the config file's
// `sleepInterval` accepts either a Go duration string or a number of
// nanoseconds (vendored config/v1/duration.go:26-53).  Operators' existing
// manifests use strings like "60s" or "1m30s", so we accept the exact Go
// grammar: [-+]?(<decimal><unit>)+ with units ns, us, µs, μs, ms, s, m, h,
// or the bare string "0".
#pragma once

#include <cstdint>
#include <string>

namespace gfd {

using Nanos = int64_t;

// Throws gfd::Error("time: invalid duration \"x\"") like Go.
Nanos parse_duration(const std::string& s);
// Formats like Go's Duration.String(): "1m0s", "1.5s", "500ms", "0s".
std::string format_duration(Nanos d);

constexpr Nanos kSecond = 1000000000LL;
constexpr Nanos kMillisecond = 1000000LL;

}  // namespace gfd
