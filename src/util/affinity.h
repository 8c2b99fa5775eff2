// Keep the daemon's threads on one L3 cache domain.
//
// A labeling cycle hands work between its thread and a pool worker several
// times (node facts, the SR-IOV scan, per-GPU lanes).  On the MI355X hosts
// (2-socket EPYC 9575F: 16 CCDs of 8 cores, one L3 each) a worker the
// scheduler places on another CCD or socket makes every hand-off and every
// shared cache line cross the fabric: pinning the process to the CPUs that
// share the L3 of the CPU it started on took the hot cycle from 0.045-0.047
// to 0.040-0.041 ms with a steadier label phase (profiles/affinity_ab.txt).
// The daemon runs a few threads for a few microseconds a minute, so one CCD
// is plenty; the CPUs are taken from the process's allowed set only (a pod's
// cpuset is respected), and nothing is changed when that set already lies
// within one L3 domain.  GFD_CPU_AFFINITY=none turns it off.
#pragma once

#include <string>
#include <vector>

namespace gfd::affinity {

// Must run before the process starts threads (they inherit the mask).
// Returns what was done, for the log ("" when nothing changed).
std::string pin_to_current_l3(const std::string& sys_root = "/");

// The CPUs sharing the L3 cache of `cpu` that this process may use (read
// from sysfs once per CPU, then cached); empty if unknown.
std::vector<int> l3_domain(int cpu, const std::string& sys_root = "/");

// "0-7,128-135" -> CPU numbers; empty on a malformed list.
std::vector<int> parse_cpu_list(const std::string& s);

}  // namespace gfd::affinity
