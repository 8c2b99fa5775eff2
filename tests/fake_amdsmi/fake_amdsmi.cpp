// A scriptable stand-in for libamd_smi, used to test the amd-smi backend on
// machines without an AMD GPU.  Loaded through GFD_AMDSMI_LIBRARY.
//
// The node is described by fake_amdsmi_configure(spec), one GPU per line:
//   bdf=0000:23:00.0;mode=CPX;parts=8;name=AMD Instinct MI355 OAM;cus=32;xcds=1;vram_mib=36862;links=7;virt=1
// (optional per GPU: serial=<hex asic serial>; visible=3,5 - only those
// partitions are reported, like a pod allocated part of a GPU; kfd_base=N -
// partition p is KFD topology node N+p, else no KFD node is reported)
// plus optional global lines:
//   init_status=34            amdsmi_init returns this status
//   stale_after=N             after N successful queries, queries return NOT_INIT until re-init
//   fail=<function>:<status>  that amd-smi function returns <status> for
//                             every device (repeatable), e.g.
//                             fail=amdsmi_get_gpu_memory_total:2
//   partition_bdf=function    partition p of a GPU at dddd:bb:dd.0 reports
//                             function p (upstream amdgpu on GC 9.4.3-class
//                             parts; the default) - or `shared`: every
//                             partition reports the parent's BDF (older kernels)
//   partition_serials=distinct  each partition reports its own ASIC serial
//                             (the GPU's with the partition index appended),
//                             as a kernel with per-XCP identities would
//   sockets=slot              one socket per PCI slot, i.e. per physical GPU
//                             (what amd-smi does; the default) - or `one`: a
//                             single socket holding every processor
//   lib_major=N               amdsmi_get_lib_version reports major N (26)
//   no_libdrm=1               amd-smi as it behaves when it cannot load
//                             libdrm_amdgpu (measured on MI355X): ASIC info
//                             and virtualization mode NOT_SUPPORTED, the BDF
//                             call succeeds with garbage, the partition
//                             profile table lists SPX only
//   init_latency_us=N         amdsmi_init takes N us (a library that starts
//                             slowly, as the real one does: ~25 ms on MI355X)
//   latency_us=N              every device query except handle-table lookups
//                             (processor type, BDF, ASIC info) busy-waits N us
//                             holding that GPU's lock (amd-smi serialises per
//                             device), to model multi-GPU scaling of the backend
// fake_amdsmi_stage(spec) holds a spec back until the next amdsmi_init, as
// the real library only sees a changed node when it is initialised again.
// Counters are exposed for assertions (fake_amdsmi_init_calls, ...).  The
// spec can also come from the GFD_FAKE_AMDSMI_SPEC environment variable
// ('|' separates lines), read when the library is loaded.
#include <amd_smi/amdsmi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Proc {
  std::string bdf;
  std::string gpu;  // BDF of the physical GPU (its per-device lock)
  uint64_t domain = 0;
  uint32_t bus = 0, dev = 0, fn = 0;
  std::string mode = "SPX";
  std::string nps = "NPS1";
  uint32_t partition_id = 0;
  std::string name = "AMD Instinct MI355 OAM";
  std::string board_name = "AMD Instinct MI355 OAM";
  uint32_t cus = 256;
  uint32_t xcds = 8;
  uint64_t vram = 309220868096ULL;
  int links = 7;
  int virt = AMDSMI_VIRTUALIZATION_MODE_BAREMETAL;
  std::string serial;  // asic_serial ("" = derived from the bus)
  uint32_t kfd_node = 0xFFFFFFFFu;  // KFD topology node (kfd_base + partition)
};

struct State {
  std::mutex mu;
  std::vector<Proc> procs;
  int init_status = 0;
  long stale_after = -1;
  long queries = 0;
  bool initialized = false;
  bool stale = false;
  int init_calls = 0;
  std::atomic<int> virt_calls{0};
  int shutdown_calls = 0;
  long latency_us = 0;
  long init_latency_us = 0;  // amdsmi_init takes this long (a slow library start)
  bool no_libdrm = false;
  uint32_t lib_major = 26;
  std::map<std::string, std::unique_ptr<std::mutex>> device_mu;  // by BDF
  std::map<std::string, int> fail;                               // function -> status
  std::map<std::string, long> calls;                             // function -> device queries made
  bool partition_fn = true;   // partition_bdf=function
  bool socket_per_slot = true;  // sockets=slot
  bool distinct_serials = false;  // partition_serials=distinct
  std::vector<std::vector<uint32_t>> sockets;  // processor indices per socket
  std::unique_ptr<std::string> pending;  // fake_amdsmi_stage: applied by the next amdsmi_init
};

State& S() {
  static State s;
  return s;
}

bool parse_bdf(const std::string& s, Proc& p) {
  unsigned long d = 0;
  unsigned b = 0, dv = 0, f = 0;
  if (sscanf(s.c_str(), "%lx:%x:%x.%x", &d, &b, &dv, &f) != 4) return false;
  p.domain = d;
  p.bus = b;
  p.dev = dv;
  p.fn = f;
  return true;
}

Proc* proc(amdsmi_processor_handle h) {
  auto& s = S();
  uintptr_t i = reinterpret_cast<uintptr_t>(h);
  if (i == 0 || i > s.procs.size()) return nullptr;
  return &s.procs[i - 1];
}

// `cheap`: calls that cost <= 2 us on real hardware (handle table lookups).
amdsmi_status_t check(amdsmi_processor_handle h, Proc** out, bool cheap = false,
                      const char* fn = __builtin_FUNCTION()) {
  auto& s = S();
  std::mutex* dev = nullptr;
  long latency = 0;
  {
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.initialized) return AMDSMI_STATUS_NOT_INIT;
    if (s.stale) return AMDSMI_STATUS_NOT_INIT;
    if (s.stale_after >= 0 && ++s.queries > s.stale_after) {
      s.stale = true;
      return AMDSMI_STATUS_NOT_INIT;
    }
    *out = proc(h);
    if (!*out) return AMDSMI_STATUS_INVAL;
    s.calls[fn]++;
    auto f = s.fail.find(fn);
    if (f != s.fail.end()) return static_cast<amdsmi_status_t>(f->second);
    latency = s.latency_us;
    if (latency > 0 && !cheap) dev = s.device_mu[(*out)->gpu].get();
  }
  if (dev) {
    // Like amd-smi's per-device mutex around its sysfs/ioctl work.
    std::lock_guard<std::mutex> g(*dev);
    auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(latency);
    while (std::chrono::steady_clock::now() < until) {
    }
  }
  return AMDSMI_STATUS_SUCCESS;
}

void copy(char* dst, size_t n, const std::string& src) {
  std::strncpy(dst, src.c_str(), n - 1);
  dst[n - 1] = 0;
}

}  // namespace

extern "C" {

// ---- control API ----
static int configure_locked(State& s, const char* spec);

int fake_amdsmi_configure(const char* spec) {
  auto& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  s.pending.reset();
  return configure_locked(s, spec);
}

// The node as the next amdsmi_init will find it: like the real library,
// which enumerates the GPUs when it is initialised and keeps answering for
// the processors it found until it is shut down and initialised again (a
// partition switch or a driver reload in between leaves its handles stale).
int fake_amdsmi_stage(const char* spec) {
  auto& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  s.pending = std::make_unique<std::string>(spec);
  return 0;
}

static int configure_locked(State& s, const char* spec) {
  s.procs.clear();
  s.init_status = 0;
  s.stale_after = -1;
  s.latency_us = 0;
  s.init_latency_us = 0;
  s.no_libdrm = false;
  s.lib_major = 26;
  s.fail.clear();
  s.calls.clear();
  s.queries = 0;
  s.stale = false;
  s.partition_fn = true;
  s.socket_per_slot = true;
  s.distinct_serials = false;
  s.sockets.clear();
  std::istringstream in(spec);
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    if (line.rfind("init_status=", 0) == 0) {
      s.init_status = std::atoi(line.c_str() + 12);
      continue;
    }
    if (line.rfind("stale_after=", 0) == 0) {
      s.stale_after = std::atol(line.c_str() + 12);
      continue;
    }
    if (line.rfind("fail=", 0) == 0) {
      size_t colon = line.rfind(':');
      if (colon == std::string::npos || colon < 5) return -1;
      s.fail[line.substr(5, colon - 5)] = std::atoi(line.c_str() + colon + 1);
      continue;
    }
    if (line.rfind("partition_bdf=", 0) == 0) {
      s.partition_fn = line.substr(14) == "function";
      continue;
    }
    if (line.rfind("partition_serials=", 0) == 0) {
      s.distinct_serials = line.substr(18) == "distinct";
      continue;
    }
    if (line.rfind("sockets=", 0) == 0) {
      s.socket_per_slot = line.substr(8) == "slot";
      continue;
    }
    if (line.rfind("lib_major=", 0) == 0) {
      s.lib_major = static_cast<uint32_t>(std::atoi(line.c_str() + 10));
      continue;
    }
    if (line.rfind("no_libdrm=", 0) == 0) {
      s.no_libdrm = line.substr(10) == "1";
      if (s.no_libdrm) {
        s.fail["amdsmi_get_gpu_asic_info"] = AMDSMI_STATUS_NOT_SUPPORTED;
        s.fail["amdsmi_get_gpu_virtualization_mode"] = AMDSMI_STATUS_NOT_SUPPORTED;
      }
      continue;
    }
    if (line.rfind("init_latency_us=", 0) == 0) {
      s.init_latency_us = std::atol(line.c_str() + 16);
      continue;
    }
    if (line.rfind("latency_us=", 0) == 0) {
      s.latency_us = std::atol(line.c_str() + 11);
      continue;
    }
    Proc base;
    int parts = 1;
    std::vector<int> visible;  // partitions the process may see (empty: all)
    // key=value pairs separated by ';' (values may contain spaces).
    std::vector<std::pair<std::string, std::string>> kv;
    std::istringstream fields(line);
    std::string field;
    while (std::getline(fields, field, ';')) {
      size_t eq = field.find('=');
      if (eq != std::string::npos) kv.emplace_back(field.substr(0, eq), field.substr(eq + 1));
    }
    for (auto& [k, v] : kv) {
      if (k == "bdf") {
        base.bdf = v;
        if (!parse_bdf(v, base)) return -1;
      } else if (k == "mode") base.mode = v;
      else if (k == "nps") base.nps = v;
      else if (k == "parts") parts = std::atoi(v.c_str());
      else if (k == "name") base.name = v;
      else if (k == "board") base.board_name = v;
      else if (k == "cus") base.cus = static_cast<uint32_t>(std::atoi(v.c_str()));
      else if (k == "xcds") base.xcds = static_cast<uint32_t>(std::atoi(v.c_str()));
      else if (k == "vram_mib") base.vram = std::strtoull(v.c_str(), nullptr, 10) << 20;
      else if (k == "links") base.links = std::atoi(v.c_str());
      else if (k == "virt") base.virt = std::atoi(v.c_str());
      else if (k == "serial") base.serial = v;
      else if (k == "kfd_base") base.kfd_node = static_cast<uint32_t>(std::atoi(v.c_str()));
      else if (k == "visible") {
        std::istringstream ids(v);
        std::string id;
        while (std::getline(ids, id, ',')) visible.push_back(std::atoi(id.c_str()));
      }
    }
    // Enumerate partitions in reverse to prove the backend orders them.
    for (int p = parts - 1; p >= 0; --p) {
      if (!visible.empty() && std::find(visible.begin(), visible.end(), p) == visible.end()) continue;
      Proc q = base;
      q.gpu = base.bdf;
      q.partition_id = static_cast<uint32_t>(p);
      if (base.kfd_node != 0xFFFFFFFFu) q.kfd_node = base.kfd_node + static_cast<uint32_t>(p);
      if (parts > 1 && s.distinct_serials)
        q.serial = (base.serial.empty() ? "3A7C178B7C5E" + base.bdf.substr(5, 2) + "5C" : base.serial) + std::to_string(p);
      if (parts > 1 && s.partition_fn) {
        // kfd_topology.c: location_id = pci_dev_id | xcp node id.
        q.fn = base.fn | static_cast<uint32_t>(p);
        char buf[32];
        snprintf(buf, sizeof(buf), "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(q.domain), q.bus, q.dev, q.fn);
        q.bdf = buf;
      }
      if (!s.device_mu.count(base.bdf)) s.device_mu[base.bdf] = std::make_unique<std::mutex>();
      s.procs.push_back(q);
    }
  }
  // amd-smi's socket id is domain:bus:device (one socket per physical GPU).
  std::map<std::string, size_t> slot_socket;
  for (uint32_t i = 0; i < s.procs.size(); ++i) {
    std::string slot = s.socket_per_slot ? s.procs[i].bdf.substr(0, s.procs[i].bdf.rfind('.')) : "";
    auto it = slot_socket.find(slot);
    if (it == slot_socket.end()) {
      it = slot_socket.emplace(slot, s.sockets.size()).first;
      s.sockets.emplace_back();
    }
    s.sockets[it->second].push_back(i);
  }
  return 0;
}
int fake_amdsmi_init_calls() { return S().init_calls; }
// Device queries made through `fn` (e.g. "amdsmi_get_gpu_memory_total") since
// the last configure.
long fake_amdsmi_calls(const char* fn) {
  auto& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.calls.find(fn);
  return it == s.calls.end() ? 0 : it->second;
}
int fake_amdsmi_virt_calls() { return S().virt_calls.load(); }
int fake_amdsmi_shutdown_calls() { return S().shutdown_calls; }
int fake_amdsmi_initialized() { return S().initialized ? 1 : 0; }

// ---- amd-smi API subset ----
amdsmi_status_t amdsmi_init(uint64_t) {
  auto& s = S();
  std::unique_lock<std::mutex> g(s.mu);
  if (long us = s.init_latency_us; us > 0) {
    g.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    g.lock();
  }
  s.init_calls++;
  if (s.pending) {
    std::string spec = std::move(*s.pending);
    s.pending.reset();
    if (configure_locked(s, spec.c_str()) != 0) return AMDSMI_STATUS_INVAL;
  }
  if (s.init_status) return static_cast<amdsmi_status_t>(s.init_status);
  s.initialized = true;
  if (s.stale) s.stale_after = -1;  // handles go stale once; a re-init fixes them
  s.stale = false;
  s.queries = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  auto& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  s.shutdown_calls++;
  s.initialized = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_status_code_to_string(amdsmi_status_t status, const char** str) {
  switch (status) {
    case AMDSMI_STATUS_NOT_INIT: *str = "AMDSMI_STATUS_NOT_INIT: Processor not initialized"; break;
    case AMDSMI_STATUS_DRIVER_NOT_LOADED: *str = "AMDSMI_STATUS_DRIVER_NOT_LOADED: Processor driver not loaded."; break;
    case AMDSMI_STATUS_NOT_SUPPORTED: *str = "AMDSMI_STATUS_NOT_SUPPORTED: Command not supported."; break;
    default: *str = "AMDSMI_STATUS_FAKE";
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* handles) {
  auto& s = S();
  if (!s.initialized) return AMDSMI_STATUS_NOT_INIT;
  uint32_t n = static_cast<uint32_t>(s.sockets.size());
  if (handles)
    for (uint32_t i = 0; i < n && i < *count; ++i) handles[i] = reinterpret_cast<amdsmi_socket_handle>(uintptr_t(i + 1));
  *count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle sock, uint32_t* count, amdsmi_processor_handle* handles) {
  auto& s = S();
  if (!s.initialized) return AMDSMI_STATUS_NOT_INIT;
  uintptr_t si = reinterpret_cast<uintptr_t>(sock);
  if (si == 0 || si > s.sockets.size()) return AMDSMI_STATUS_INVAL;
  const auto& members = s.sockets[si - 1];
  uint32_t n = static_cast<uint32_t>(members.size());
  if (handles)
    for (uint32_t i = 0; i < n && i < *count; ++i)
      handles[i] = reinterpret_cast<amdsmi_processor_handle>(uintptr_t(members[i] + 1));
  *count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle h, processor_type_t* t) {
  Proc* p;
  if (auto st = check(h, &p, true)) return st;
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* b) {
  Proc* p;
  if (auto st = check(h, &p, true)) return st;
  std::memset(b, 0, sizeof(*b));
  if (S().no_libdrm) {  // uninitialised bytes, as measured: "5ddf28c0:c2:1a.0"
    b->domain_number = 0x5ddf28c0;
    b->bus_number = 0xc2;
    b->device_number = 0x1a;
    return AMDSMI_STATUS_SUCCESS;
  }
  b->domain_number = p->domain;
  b->bus_number = p->bus;
  b->device_number = p->dev;
  b->function_number = p->fn;
  return AMDSMI_STATUS_SUCCESS;
}

// The first processor at that address, in enumeration order - the
// library's lookup (its CLI resolves a partition's primary through it,
// amdsmi_helpers.py get_primary_partition_gpu_id).
amdsmi_status_t amdsmi_get_processor_handle_from_bdf(amdsmi_bdf_t bdf, amdsmi_processor_handle* h) {
  auto& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  if (!s.initialized) return AMDSMI_STATUS_NOT_INIT;
  if (!h) return AMDSMI_STATUS_INVAL;
  for (size_t i = 0; i < s.procs.size(); ++i) {
    const Proc& p = s.procs[i];
    if (p.domain == bdf.domain_number && p.bus == bdf.bus_number && p.dev == bdf.device_number &&
        p.fn == bdf.function_number) {
      *h = reinterpret_cast<amdsmi_processor_handle>(uintptr_t(i + 1));
      return AMDSMI_STATUS_SUCCESS;
    }
  }
  return AMDSMI_STATUS_API_FAILED;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* a) {
  Proc* p;
  if (auto st = check(h, &p, true)) return st;
  std::memset(a, 0, sizeof(*a));
  copy(a->market_name, sizeof(a->market_name), p->name);
  a->vendor_id = 0x1002;
  a->device_id = 0x75a3;
  a->num_of_compute_units = p->cus;
  a->target_graphics_version = 0x950;
  // A 64-bit hex serial, here derived from the bus (the real library's
  // spelling of the prefix varies; both forms are exercised).
  copy(a->asic_serial, sizeof(a->asic_serial),
       !p->serial.empty() ? p->serial
                          : std::string(p->bus & 0x10 ? "0x" : "") + "3A7C178B7C5E" + p->gpu.substr(5, 2) + "5C");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_board_info(amdsmi_processor_handle h, amdsmi_board_info_t* b) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(b, 0, sizeof(*b));
  copy(b->product_name, sizeof(b->product_name), p->board_name);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t, uint64_t* total) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  *total = p->vram;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* k) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(k, 0, sizeof(*k));
  k->kfd_id = 1000;
  k->node_id = p->kfd_node;  // default none: the backend falls back to xcd_counter
  k->current_partition_id = p->partition_id;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xcd_counter(amdsmi_processor_handle h, uint16_t* x) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  *x = static_cast<uint16_t>(p->xcds);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle h, char* buf, uint32_t len) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  copy(buf, len, p->mode);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle h, char* buf, uint32_t len) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  copy(buf, len, p->nps);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition_config(amdsmi_processor_handle h, amdsmi_memory_partition_config_t* c) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(c, 0, sizeof(*c));
  c->partition_caps.nps_cap_mask = 0x3;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_accelerator_partition_profile_config(amdsmi_processor_handle h,
                                                                     amdsmi_accelerator_partition_profile_config_t* c) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(c, 0, sizeof(*c));
  if (S().no_libdrm) {
    c->num_profiles = 1;
    c->profiles[0].profile_type = AMDSMI_ACCELERATOR_PARTITION_SPX;
    return AMDSMI_STATUS_SUCCESS;
  }
  c->num_profiles = 4;
  c->profiles[0].profile_type = AMDSMI_ACCELERATOR_PARTITION_SPX;
  c->profiles[1].profile_type = AMDSMI_ACCELERATOR_PARTITION_DPX;
  c->profiles[2].profile_type = AMDSMI_ACCELERATOR_PARTITION_QPX;
  c->profiles[3].profile_type = AMDSMI_ACCELERATOR_PARTITION_CPX;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_accelerator_partition_profile(amdsmi_processor_handle h,
                                                             amdsmi_accelerator_partition_profile_t* prof,
                                                             uint32_t* ids) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(prof, 0, sizeof(*prof));
  prof->num_partitions = 1;
  prof->num_resources = AMDSMI_ACCELERATOR_MAX;
  prof->resources[0][AMDSMI_ACCELERATOR_XCC] = p->xcds;
  prof->resources[0][AMDSMI_ACCELERATOR_ENCODER] = 0;
  prof->resources[0][AMDSMI_ACCELERATOR_DECODER] = 1;
  prof->resources[0][AMDSMI_ACCELERATOR_DMA] = 2;
  prof->resources[0][AMDSMI_ACCELERATOR_JPEG] = 4;
  ids[0] = p->partition_id;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h, amdsmi_xgmi_link_status_t* ls) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(ls, 0, sizeof(*ls));
  ls->total_links = 8;
  ls->status[0] = AMDSMI_XGMI_LINK_DISABLE;
  for (int i = 1; i < 8; ++i) ls->status[i] = i <= p->links ? AMDSMI_XGMI_LINK_UP : AMDSMI_XGMI_LINK_DOWN;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_virtualization_mode(amdsmi_processor_handle h, amdsmi_virtualization_mode_t* m) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  S().virt_calls++;
  *m = static_cast<amdsmi_virtualization_mode_t>(p->virt);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_driver_info(amdsmi_processor_handle h, amdsmi_driver_info_t* d) {
  Proc* p;
  if (auto st = check(h, &p)) return st;
  std::memset(d, 0, sizeof(*d));
  copy(d->driver_version, sizeof(d->driver_version), "6.12.12");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_lib_version(amdsmi_version_t* v) {
  std::memset(v, 0, sizeof(*v));
  v->major = S().lib_major;
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"

namespace {
// A process that cannot call fake_amdsmi_configure (the daemon binary under a
// Python test) describes the node in GFD_FAKE_AMDSMI_SPEC instead, with '|'
// or newlines between lines.
__attribute__((constructor)) void configure_from_env() {
  const char* spec = std::getenv("GFD_FAKE_AMDSMI_SPEC");
  if (!spec || !*spec) return;
  std::string text(spec);
  for (char& ch : text)
    if (ch == '|') ch = '\n';
  fake_amdsmi_configure(text.c_str());
}
}  // namespace
