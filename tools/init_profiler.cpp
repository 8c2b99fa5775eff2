// SIGPROF sampling profiler around amdsmi_init: which library functions
// burn its ~25 ms of user-space CPU (tools/init_sampler.cpp showed it is
// running, not blocked).  Attributes each sample's call stack to symbols
// with dladdr.
//   g++ -O2 -std=c++17 -I/opt/rocm/include tools/init_profiler.cpp -ldl -o build/init_profiler
#include <amd_smi/amdsmi.h>
#include <cxxabi.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

constexpr int kMaxSamples = 20000;
constexpr int kDepth = 24;
static void* g_stacks[kMaxSamples][kDepth];
static int g_depth[kMaxSamples];
static volatile int g_n = 0;

static void on_prof(int, siginfo_t*, void*) {
  int i = g_n;
  if (i >= kMaxSamples) return;
  g_depth[i] = backtrace(g_stacks[i], kDepth);
  g_n = i + 1;
}

static std::string sym(void* ip) {
  Dl_info info;
  if (!dladdr(ip, &info)) return "?";
  std::string lib = info.dli_fname ? info.dli_fname : "?";
  lib = lib.substr(lib.rfind('/') + 1);
  if (!info.dli_sname) {
    char buf[64];
    std::snprintf(buf, sizeof(buf), "+0x%lx", (unsigned long)((char*)ip - (char*)info.dli_fbase));
    return lib + buf;
  }
  int status = 0;
  char* d = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &status);
  std::string name = status == 0 && d ? d : info.dli_sname;
  std::free(d);
  if (name.size() > 110) name = name.substr(0, 110) + "...";
  return lib + ":" + name;
}

int main() {
  void* h = dlopen("libamd_smi.so.26", RTLD_NOW);
  if (!h) h = dlopen("/opt/rocm/lib/libamd_smi.so", RTLD_NOW);
  if (!h) return 1;
  auto init = reinterpret_cast<amdsmi_status_t (*)(uint64_t)>(dlsym(h, "amdsmi_init"));
  auto fini = reinterpret_cast<amdsmi_status_t (*)()>(dlsym(h, "amdsmi_shut_down"));
  void* warm[4];
  backtrace(warm, 4);  // load libgcc's unwinder outside the handler
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  struct itimerval it;
  it.it_interval = {0, 100};
  it.it_value = {0, 100};
  int rounds = 5;
  auto t = std::chrono::steady_clock::now();
  setitimer(ITIMER_PROF, &it, nullptr);
  for (int r = 0; r < rounds; ++r) {
    init(AMDSMI_INIT_AMD_GPUS);
    fini();
  }
  struct itimerval off = {};
  setitimer(ITIMER_PROF, &off, nullptr);
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  int n = g_n;
  std::printf("%d init+shutdown rounds: %.1f ms, %d samples\n", rounds, ms, n);
  // Self (leaf) and inclusive counts per symbol (skip frame 0-1: handler, trampoline).
  std::map<std::string, int> self, incl;
  for (int i = 0; i < n; ++i) {
    std::map<std::string, bool> seen;
    for (int f = 2; f < g_depth[i]; ++f) {
      std::string s = sym(g_stacks[i][f]);
      if (f == 2) self[s]++;
      if (!seen[s]) {
        incl[s]++;
        seen[s] = true;
      }
    }
  }
  auto top = [&](const char* title, std::map<std::string, int>& m, int k) {
    std::vector<std::pair<int, std::string>> v;
    for (auto& [s, c] : m) v.push_back({c, s});
    std::sort(v.rbegin(), v.rend());
    std::printf("\n== %s ==\n", title);
    for (int i = 0; i < k && i < (int)v.size(); ++i) std::printf("%6.1f%%  %s\n", 100.0 * v[i].first / n, v[i].second.c_str());
  };
  top("self (leaf frame)", self, 25);
  top("inclusive", incl, 40);
  return 0;
}
