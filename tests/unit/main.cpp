// Runner for the C++ unit tests.
//   gfd_unit_tests            run everything
//   gfd_unit_tests --list     print test names
//   gfd_unit_tests NAME...    run the named tests (exact match)
#include <cstdio>
#include <cstring>
#include <set>

#include "test.h"
#include "util/log.h"

int main(int argc, char** argv) {
  std::set<std::string> only;
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "--list") == 0) {
      for (const auto& t : gfdtest::Registry::tests()) printf("%s\n", t.first.c_str());
      return 0;
    }
    only.insert(argv[i]);
  }
  gfd::log::set_quiet(getenv("GFD_TEST_VERBOSE") == nullptr);
  int failed = 0, ran = 0;
  for (const auto& [name, fn] : gfdtest::Registry::tests()) {
    if (!only.empty() && !only.count(name)) continue;
    ++ran;
    try {
      fn();
      printf("[ OK ] %s\n", name.c_str());
    } catch (const std::exception& e) {
      ++failed;
      printf("[FAIL] %s\n  %s\n", name.c_str(), e.what());
    }
  }
  if (!only.empty() && ran != static_cast<int>(only.size())) {
    printf("[FAIL] some requested tests were not found\n");
    return 2;
  }
  printf("%d tests, %d failed\n", ran, failed);
  return failed ? 1 : 0;
}
