// L3 cache domains for the daemon's CPU placement (--cpu-affinity).
//
// A labeling cycle hands work between its thread and a pool worker several
// times (node facts, the SR-IOV scan, per-GPU lanes).  On the MI355X hosts
// (2-socket EPYC 9575F: 16 CCDs of 8 cores, one L3 each) a worker the
// scheduler places on another CCD or socket makes every hand-off and every
// shared cache line cross the fabric (profiles/affinity_ab.txt,
// profiles/affinity_r3.txt).  `follow` keeps only the pool's workers on the
// L3 domain of the CPU each cycle starts on (L3Map, read once at start-up);
// `l3` pins the whole process to the domain it starts on
// (pin_to_current_l3); `none` changes nothing.  CPUs are taken from the
// allowed set only (a pod's cpuset is respected).
#pragma once

#include <string>
#include <vector>

namespace gfd::affinity {

// The host's CPU -> L3 domain map, read from sysfs in one pass: one
// shared_cpu_list per L3 (16 reads on a 256-CPU EPYC host), never per cycle.
class L3Map {
 public:
  static L3Map read(const std::string& sys_root);
  // The map of "/" (read on first use; follow mode reads it at start-up).
  static const L3Map& host();
  // Domain number of `cpu`, -1 if unknown.
  int id(int cpu) const;
  // The CPUs of domain `id` (all of them, allowed or not); empty if unknown.
  const std::vector<int>& cpus(int id) const;
  size_t size() const { return domains_.size(); }

 private:
  std::vector<int> domain_of_;
  std::vector<std::vector<int>> domains_;
};

// The members of `cpus` the calling thread may run on now.
std::vector<int> allowed_subset(const std::vector<int>& cpus);

// Must run before the process starts threads (they inherit the mask).
// Returns what was done, for the log ("" when nothing changed).
std::string pin_to_current_l3(const std::string& sys_root = "/");

// The CPUs sharing the L3 cache of `cpu` that the calling thread may use now
// (the cache topology is read from sysfs once per CPU; the allowed set every
// call, so a cpuset changed under a running pod is followed); empty if
// unknown.
std::vector<int> l3_domain(int cpu, const std::string& sys_root = "/");

// "0-7,128-135" -> CPU numbers; empty on a malformed list.
std::vector<int> parse_cpu_list(const std::string& s);

}  // namespace gfd::affinity
