#include "util/affinity.h"

#include <sched.h>

#include <map>
#include <mutex>
#include <optional>
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

std::string cache_dir(const std::string& sys_root, int cpu) {
  return fs::join(sys_root, "sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache");
}

// The cache index directory ("index3" on x86) whose level is 3, or "".
std::string l3_index(const std::string& base) {
  for (const auto& idx : fs::list_dir(base)) {
    if (idx.rfind("index", 0) != 0) continue;
    if (fs::read_trimmed(fs::join(base, idx + "/level")).value_or("") == "3") return idx;
  }
  return "";
}

// "0-7,128-135" of the L3 cache of `cpu`, or "".
std::string l3_list(int cpu, const std::string& sys_root) {
  std::string base = cache_dir(sys_root, cpu);
  std::string idx = l3_index(base);
  return idx.empty() ? "" : fs::read_trimmed(fs::join(base, idx + "/shared_cpu_list")).value_or("");
}

}  // namespace

L3Map L3Map::read(const std::string& sys_root) {
  L3Map m;
  std::vector<int> cpus = parse_cpu_list(
      fs::read_trimmed(fs::join(sys_root, "sys/devices/system/cpu/online")).value_or(""));
  std::string idx;  // the L3's index name, found once (the same on every CPU of a host)
  for (int cpu : cpus) {
    if (static_cast<size_t>(cpu) < m.domain_of_.size() && m.domain_of_[cpu] >= 0) continue;
    std::string base = cache_dir(sys_root, cpu);
    std::optional<std::string> list;
    if (!idx.empty()) list = fs::read_trimmed(fs::join(base, idx + "/shared_cpu_list"));
    if (!list) {  // first CPU, or one whose index layout differs
      idx = l3_index(base);
      if (idx.empty()) continue;
      list = fs::read_trimmed(fs::join(base, idx + "/shared_cpu_list"));
    }
    std::vector<int> members = parse_cpu_list(list.value_or(""));
    if (members.empty()) continue;
    int id = static_cast<int>(m.domains_.size());
    for (int c : members) {
      if (static_cast<size_t>(c) >= m.domain_of_.size()) m.domain_of_.resize(static_cast<size_t>(c) + 1, -1);
      m.domain_of_[c] = id;
    }
    m.domains_.push_back(std::move(members));
  }
  return m;
}

int L3Map::id(int cpu) const {
  if (cpu < 0 || static_cast<size_t>(cpu) >= domain_of_.size()) return -1;
  return domain_of_[cpu];
}

const std::vector<int>& L3Map::cpus(int id) const {
  static const std::vector<int> none;
  return id >= 0 && static_cast<size_t>(id) < domains_.size() ? domains_[id] : none;
}

const L3Map& L3Map::host() {
  static const L3Map m = read("/");
  return m;
}

std::vector<int> allowed_subset(const std::vector<int>& cpus) {
  std::vector<int> out;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0)
    for (int c : cpus)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
  return out;
}

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
  return allowed_subset(l3);
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
