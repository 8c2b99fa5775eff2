#include "util/affinity.h"

#include <sched.h>

#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "util/fs.h"
#include "util/strings.h"

namespace gfd::affinity {

std::vector<int> parse_cpu_list(const std::string& s) {
  std::vector<int> out;
  for (const auto& part : str::split(str::trim(s), ',')) {
    if (part.empty()) continue;
    auto range = str::split_n(part, '-', 2);
    auto lo = str::parse_uint(range[0]);
    auto hi = range.size() == 2 ? str::parse_uint(range[1]) : lo;
    if (!lo || !hi || *hi < *lo || *hi >= CPU_SETSIZE) return {};
    for (uint64_t c = *lo; c <= *hi; ++c) out.push_back(static_cast<int>(c));
  }
  return out;
}

namespace {
// "0-7,128-135" of the L3 cache of `cpu` (the cache index whose level is 3:
// index3 on x86, but look), or "".
std::string l3_list(int cpu, const std::string& sys_root) {
  std::string base = fs::join(sys_root, "sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache");
  for (const auto& idx : fs::list_dir(base)) {
    if (idx.rfind("index", 0) != 0) continue;
    if (fs::read_trimmed(fs::join(base, idx + "/level")).value_or("") == "3")
      return fs::read_trimmed(fs::join(base, idx + "/shared_cpu_list")).value_or("");
  }
  return "";
}
}  // namespace

std::vector<int> l3_domain(int cpu, const std::string& sys_root) {
  if (cpu < 0) return {};
  std::vector<int> l3;
  {
    static std::mutex mu;
    static std::map<std::pair<std::string, int>, std::vector<int>> known;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair(sys_root, cpu);
    auto it = known.find(key);
    if (it == known.end()) it = known.emplace(key, parse_cpu_list(l3_list(cpu, sys_root))).first;
    l3 = it->second;
  }
  std::vector<int> out;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0)
    for (int c : l3)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
  return out;
}

std::string pin_to_current_l3(const std::string& sys_root) {
  int cpu = sched_getcpu();
  if (cpu < 0) return "";
  std::string list = l3_list(cpu, sys_root);
  std::vector<int> l3 = parse_cpu_list(list);
  if (l3.empty()) return "";
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return "";
  cpu_set_t pin;
  CPU_ZERO(&pin);
  for (int c : l3)
    if (CPU_ISSET(c, &allowed)) CPU_SET(c, &pin);
  int n_pin = CPU_COUNT(&pin), n_allowed = CPU_COUNT(&allowed);
  if (n_pin == 0 || n_pin == n_allowed) return "";
  if (sched_setaffinity(0, sizeof(pin), &pin) != 0) return "";
  return "threads kept on the " + std::to_string(n_pin) + " CPUs sharing cpu" + std::to_string(cpu) +
         "'s L3 cache (" + list + ") of " + std::to_string(n_allowed) + " allowed";
}

}  // namespace gfd::affinity
