// Minimal self-registering unit-test harness (no third-party dependency).
// Each TEST runs in the same process; failures are reported per test and the
// binary exits non-zero if any failed.  `gfd_unit_tests --list` prints the
// test names so pytest can parametrize over them (tests/test_unit_cpp.py).
#pragma once

#include <functional>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace gfdtest {

struct Failure : std::runtime_error {
  explicit Failure(const std::string& m) : std::runtime_error(m) {}
};

struct Registry {
  static std::vector<std::pair<std::string, std::function<void()>>>& tests() {
    static std::vector<std::pair<std::string, std::function<void()>>> t;
    return t;
  }
};

struct Registrar {
  Registrar(const char* name, std::function<void()> fn) { Registry::tests().emplace_back(name, std::move(fn)); }
};

template <typename T>
std::string repr(const T& v) {
  std::ostringstream os;
  os << v;
  return os.str();
}
inline std::string repr(const std::string& v) { return "\"" + v + "\""; }
inline std::string repr(const char* v) { return std::string("\"") + v + "\""; }
inline std::string repr(bool v) { return v ? "true" : "false"; }
inline std::string repr(const std::map<std::string, std::string>& m) {
  std::string s = "{";
  for (const auto& kv : m) s += "\n    " + kv.first + "=" + kv.second;
  return s + "\n  }";
}
inline std::string repr(const std::vector<std::string>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + repr(v[i]);
  return s + "]";
}

}  // namespace gfdtest

#define GFD_CAT2(a, b) a##b
#define GFD_CAT(a, b) GFD_CAT2(a, b)
#define TEST(name)                                                              \
  static void GFD_CAT(test_fn_, name)();                                        \
  static ::gfdtest::Registrar GFD_CAT(test_reg_, name)(#name, GFD_CAT(test_fn_, name)); \
  static void GFD_CAT(test_fn_, name)()

#define GFD_FAIL(msg)                                                                  \
  do {                                                                                 \
    std::ostringstream gfd_os__;                                                       \
    gfd_os__ << __FILE__ << ":" << __LINE__ << ": " << msg;                            \
    throw ::gfdtest::Failure(gfd_os__.str());                                          \
  } while (0)

#define EXPECT_TRUE(c) \
  do {                 \
    if (!(c)) GFD_FAIL("expected true: " #c); \
  } while (0)
#define EXPECT_FALSE(c) \
  do {                  \
    if (c) GFD_FAIL("expected false: " #c); \
  } while (0)
#define EXPECT_EQ(a, b)                                                                                  \
  do {                                                                                                   \
    auto gfd_a__ = (a);                                                                                  \
    auto gfd_b__ = (b);                                                                                  \
    if (!(gfd_a__ == gfd_b__))                                                                           \
      GFD_FAIL(#a " == " #b "\n  left:  " << ::gfdtest::repr(gfd_a__) << "\n  right: " << ::gfdtest::repr(gfd_b__)); \
  } while (0)
#define EXPECT_THROW_MSG(stmt, substr)                                                             \
  do {                                                                                             \
    bool gfd_thrown__ = false;                                                                     \
    try {                                                                                          \
      stmt;                                                                                        \
    } catch (const ::gfdtest::Failure&) {                                                         \
      throw;                                                                                       \
    } catch (const std::exception& gfd_e__) {                                                      \
      gfd_thrown__ = true;                                                                         \
      if (std::string(gfd_e__.what()).find(substr) == std::string::npos)                          \
        GFD_FAIL("exception message '" << gfd_e__.what() << "' does not contain '" << substr << "'"); \
    }                                                                                              \
    if (!gfd_thrown__) GFD_FAIL("expected exception from: " #stmt);                                \
  } while (0)
#define EXPECT_THROW(stmt) EXPECT_THROW_MSG(stmt, "")
#define EXPECT_NO_THROW(stmt)                                           \
  do {                                                                  \
    try {                                                               \
      stmt;                                                             \
    } catch (const ::gfdtest::Failure&) {                              \
      throw;                                                            \
    } catch (const std::exception& gfd_e__) {                           \
      GFD_FAIL("unexpected exception: " << gfd_e__.what() << " from " #stmt); \
    }                                                                   \
  } while (0)
