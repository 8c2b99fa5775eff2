#include "resource/amdsmi.h"

#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "resource/amdsmi_lib.h"
#include "resource/pci_ids.h"
#include "resource/physical.h"
#include "resource/sysfs.h"
#include "resource/versions.h"
#include "util/error.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/pool.h"
#include "util/strings.h"
#include "util/trace.h"

namespace gfd::resource {

// ---------------------------------------------------------------------------
// Snapshot helpers

namespace {

// A failed amd-smi call.  The status (not the message) decides whether the
// persistent session's handles went stale.
class CallError : public Error {
 public:
  CallError(const std::string& msg, amdsmi_status_t st) : Error(msg), status(st) {}
  amdsmi_status_t status;
};

[[noreturn]] void call_failed(AmdSmiLib& L, const char* fn, amdsmi_status_t st) {
  throw CallError(std::string(fn) + ": " + L.status_str(st), st);
}

// Statuses meaning "the session/handles are stale; re-initialise": a
// processor handle from before a driver reload or partition switch.
bool is_stale(amdsmi_status_t st) { return st == AMDSMI_STATUS_NOT_INIT || st == AMDSMI_STATUS_NOT_FOUND; }

// Raw per-processor facts (one amd-smi processor = a GPU or a partition).
struct ProcInfo {
  amdsmi_processor_handle h = nullptr;
  std::string bdf;      // as amd-smi reports it (a partition's may carry its index)
  std::string gpu_bdf;  // parent PCI function of its physical GPU (GPU-wide attributes)
  bool identified = false;  // query_identity ran this cycle
  std::string market_name;
  uint32_t vendor_id = 0;
  uint32_t device_id = 0;
  uint32_t cus = 0;
  uint64_t gfx = 0;
  uint64_t vram = 0;
  uint32_t partition_id = 0;
  uint32_t xcds = 0;
  int sdma = -1;  // KFD node num_sdma_engines (-1: node unknown)
  std::string compute_partition;
  std::string memory_partition;
  std::string uuid;
};

// Facts queried once per physical GPU.
struct GpuExtras {
  int xgmi_links = -1;
  std::string virtualization;
  std::vector<std::string> available_memory;
  std::vector<std::string> available_compute;
  Attributes engines;  // engines.* of each partition (partition_engine_counts)
};

const char* virt_name(amdsmi_virtualization_mode_t m) {
  switch (m) {
    case AMDSMI_VIRTUALIZATION_MODE_BAREMETAL: return "baremetal";
    case AMDSMI_VIRTUALIZATION_MODE_HOST: return "host";
    case AMDSMI_VIRTUALIZATION_MODE_GUEST: return "guest";
    case AMDSMI_VIRTUALIZATION_MODE_PASSTHROUGH: return "passthrough";
    default: return "";
  }
}

const char* accel_name(amdsmi_accelerator_partition_type_t t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_PARTITION_SPX: return "SPX";
    case AMDSMI_ACCELERATOR_PARTITION_DPX: return "DPX";
    case AMDSMI_ACCELERATOR_PARTITION_TPX: return "TPX";
    case AMDSMI_ACCELERATOR_PARTITION_QPX: return "QPX";
    case AMDSMI_ACCELERATOR_PARTITION_CPX: return "CPX";
    default: return nullptr;
  }
}

std::vector<std::string> nps_list(uint32_t mask) {
  std::vector<std::string> out;
  if (mask & 1u) out.push_back("NPS1");
  if (mask & 2u) out.push_back("NPS2");
  if (mask & 4u) out.push_back("NPS4");
  if (mask & 8u) out.push_back("NPS8");
  return out;
}

// GFD_AMDSMI_CALL_TRACE=1 records every amd-smi call as a trace phase
// ("amdsmi:<call>") - used to build the cost table in docs/BACKENDS.md.
bool call_trace() {
  static const bool on = std::getenv("GFD_AMDSMI_CALL_TRACE") != nullptr;
  return on;
}

template <typename F>
auto timed(const char* name, F&& f) -> decltype(f()) {
  if (!call_trace()) return f();
  int64_t t0 = trace::now_ns();
  auto r = f();
  trace::record(std::string("amdsmi:") + name, trace::now_ns() - t0);
  return r;
}
#define AMDSMI_CALL(name, expr) timed(name, [&] { return (expr); })

// libdrm's marketing-name table is consulted by amd-smi; when the process
// already carries another libdrm (e.g. PyTorch's bundled copy, whose
// amdgpu.ids path does not exist) it degrades to this generic string -
// observed on the MI355X pool.
bool is_generic_name(const std::string& s) { return s.empty() || s == "AMD Radeon Graphics" || s == "N/A"; }

constexpr uint32_t kNoNode = 0xFFFFFFFFu;

// A numeric field of a KFD node's properties text ("key value" lines).
std::optional<uint64_t> kfd_field(const std::string& text, const std::string& key) {
  for (size_t pos = text.find(key); pos != std::string::npos; pos = text.find(key, pos + 1)) {
    size_t end = pos + key.size();
    if ((pos == 0 || text[pos - 1] == '\n') && end < text.size() && text[end] == ' ')
      return std::strtoull(text.c_str() + end + 1, nullptr, 10);
  }
  return std::nullopt;
}

fs::ReadResult kfd_properties(const std::string& root, uint32_t node_id) {
  return fs::attrs().read(fs::join(root, "sys/class/kfd/kfd/topology/nodes/" + std::to_string(node_id) + "/properties"));
}

// XCD and SDMA-engine counts of a KFD node (num_xcc, num_sdma_engines) -
// ~15 us versus ~140 us for amdsmi_get_gpu_xcd_counter, which decodes the
// full gpu_metrics table.  Zero / -1 when the node cannot be read.
struct KfdCounts {
  uint32_t num_xcc = 0;
  int num_sdma = -1;
};
KfdCounts kfd_counts(const std::string& root, uint32_t node_id) {
  KfdCounts c;
  auto r = kfd_properties(root, node_id);
  if (!r.ok()) return c;
  if (auto v = kfd_field(r.data, "num_xcc")) c.num_xcc = static_cast<uint32_t>(*v);
  if (auto v = kfd_field(r.data, "num_sdma_engines")) c.num_sdma = static_cast<int>(*v);
  return c;
}
uint32_t kfd_num_xcc(const std::string& root, uint32_t node_id) { return kfd_counts(root, node_id).num_xcc; }

// KFD node and partition id of a processor (amdsmi_get_gpu_kfd_info).
bool query_kfd(AmdSmiLib& L, ProcInfo& p, uint32_t* node_id) {
  if (!L.get_gpu_kfd_info) return false;
  amdsmi_kfd_info_t kfd;
  std::memset(&kfd, 0, sizeof(kfd));
  if (AMDSMI_CALL("kfd_info", L.get_gpu_kfd_info(p.h, &kfd)) != AMDSMI_STATUS_SUCCESS) return false;
  if (kfd.current_partition_id != 0xFFFFFFFFu) p.partition_id = kfd.current_partition_id;
  *node_id = kfd.node_id;
  return true;
}

// KFD's gfx_target_version (major*10000 + minor*100 + stepping, decimal) in
// amd-smi's spelling (hex digits naming the target: 90500 -> 0x950).
uint64_t amdsmi_gfx_from_kfd(uint64_t v) {
  uint64_t major = v / 10000, minor = (v / 100) % 100, step = v % 100;
  uint64_t maj_hex = 0;
  for (uint64_t shift = 0; major; major /= 10, shift += 4) maj_hex |= (major % 10) << shift;
  return (maj_hex << 8) | ((minor & 0xF) << 4) | (step & 0xF);
}

// The processor's identity from its KFD node - the same facts amd-smi's
// ASIC info reports (vendor/device ID, CUs, ISA target, serial), for when
// that call is refused.  amd-smi answers it through libdrm_amdgpu, which it
// dlopens; without that library (a slim image) asic_info returns
// NOT_SUPPORTED for every processor (measured on the pool,
// tests/test_gpu.py::test_amdsmi_without_libdrm_labels_identically).  The
// name comes from the board's product_name attribute (fix_market_name).
bool identity_from_kfd(AmdSmiLib& L, const std::string& root, ProcInfo& p) {
  uint32_t node = kNoNode;
  if (!query_kfd(L, p, &node) || node == kNoNode) return false;
  auto r = kfd_properties(root, node);
  if (!r.ok()) return false;
  uint64_t gfx = kfd_field(r.data, "gfx_target_version").value_or(0);
  uint64_t device = kfd_field(r.data, "device_id").value_or(0);
  if (gfx == 0 || device == 0) return false;
  uint64_t simds = kfd_field(r.data, "simd_count").value_or(0), per_cu = kfd_field(r.data, "simd_per_cu").value_or(0);
  p.market_name.clear();
  p.vendor_id = static_cast<uint32_t>(kfd_field(r.data, "vendor_id").value_or(0));
  p.device_id = static_cast<uint32_t>(device);
  p.cus = per_cu ? static_cast<uint32_t>(simds / per_cu) : 0;
  p.gfx = amdsmi_gfx_from_kfd(gfx);
  p.uuid = amd_uuid(kfd_field(r.data, "unique_id").value_or(0), p.device_id);
  return true;
}

// Identity of a processor from its ASIC info (the library caches it after
// the first call: ~2 us), or from its KFD node when amd-smi cannot answer.
void query_identity(AmdSmiLib& L, const std::string& root, ProcInfo& p) {
  if (p.identified) return;
  amdsmi_status_t st = AMDSMI_STATUS_NOT_SUPPORTED;
  amdsmi_asic_info_t asic;
  std::memset(&asic, 0, sizeof(asic));
  if (!L.asic_info_unsupported.load(std::memory_order_relaxed))
    st = AMDSMI_CALL("asic_info", L.get_gpu_asic_info(p.h, &asic));
  if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
    if (!identity_from_kfd(L, root, p)) call_failed(L, "amdsmi_get_gpu_asic_info", st);
    L.asic_info_unsupported.store(true, std::memory_order_relaxed);
    p.identified = true;
    return;
  }
  if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_gpu_asic_info", st);
  p.market_name = str::trim(asic.market_name);
  p.vendor_id = asic.vendor_id;
  p.device_id = static_cast<uint32_t>(asic.device_id);
  p.cus = asic.num_of_compute_units == 0xFFFFFFFFu ? 0 : asic.num_of_compute_units;
  p.gfx = asic.target_graphics_version;
  // amd-smi's UUID is a spelling of the ASIC serial: derive it here instead
  // of paying amdsmi_get_gpu_device_uuid per processor.
  // The library spells the serial in hex, with or without "0x".
  std::string serial_hex = str::trim(asic.asic_serial);
  if (serial_hex.size() > 2 && serial_hex[0] == '0' && (serial_hex[1] == 'x' || serial_hex[1] == 'X'))
    serial_hex.erase(0, 2);
  if (auto serial = str::parse_uint(serial_hex, 16)) p.uuid = amd_uuid(*serial, p.device_id);
  p.identified = true;
}

void fix_market_name(AmdSmiLib& L, const std::string& root, ProcInfo& p) {
  if (!is_generic_name(p.market_name)) return;
  // The board FRU product name: amdgpu publishes it in sysfs (~5 us); the
  // amd-smi board-info call returns the same string for ~155 us.
  auto v = fs::attrs().read_trimmed(fs::join(root, "sys/bus/pci/devices/" + p.gpu_bdf + "/product_name"));
  if (v && !is_generic_name(*v)) {
    p.market_name = *v;
  } else if (L.get_gpu_board_info) {
    amdsmi_board_info_t b;
    std::memset(&b, 0, sizeof(b));
    if (AMDSMI_CALL("board_info", L.get_gpu_board_info(p.h, &b)) == AMDSMI_STATUS_SUCCESS &&
        !is_generic_name(str::trim(b.product_name)))
      p.market_name = str::trim(b.product_name);
  }
  // Nothing better known (no libdrm, no FRU): the model of the device ID,
  // the KFD backend's fallback too.
  if (p.market_name.empty() && p.device_id) p.market_name = device_name(p.device_id);
}

// The GPU's compute partition mode for the session: `mode` (the session
// cache entry) when known, else read from the parent function's
// current_compute_partition - once per session, not per cycle.  amdgpu
// answers that attribute by reading the XCP control register, which "may
// momentarily wake the GPU up" (AMD's own CLI stopped reading it by
// default: /opt/rocm/libexec/amdsmi_cli/amdsmi_commands.py:463-466).  The
// mode only changes with a partition switch, which rebuilds the KFD
// topology and bumps its generation, and a new generation re-initialises the
// session, which clears the cache (AmdSmiManager::compute_mode_).  False
// when the attribute is missing or unknown.  `read_ns`: the read's time, if
// it happened (reported by the cycle thread as "compute_partition(read)").
bool session_compute_mode(const std::string& pci, std::string* mode, int64_t* read_ns) {
  if (!mode->empty()) return true;
  int64_t t0 = trace::now_ns();
  auto cp = fs::attrs().read_trimmed(pci + "/current_compute_partition");
  *read_ns += trace::now_ns() - t0;
  if (!cp) return false;
  *mode = partition_mode(*cp);
  return !mode->empty();
}

// The only processor at its PCI address and in SPX mode: its values are
// the amdgpu attributes amd-smi reads for the same calls
// (mem_info_vram_total for memory_total(VRAM), current_compute_partition /
// current_memory_partition for the partition getters), read directly -
// once per session (`kept`, AmdSmiManager::session_values_), like the
// compute mode: none of them changes while a driver instance lives but with
// a partition or NPS switch, which rebuilds the KFD topology, and a new
// generation re-initialises the session.  Measured on the pool: 2.0 + 1.0
// us per GPU per cycle for the two reads, and 1.7 us for xgmi_num_links
// (query_gpu_caps); the 8-GPU snapshot 0.0378 -> 0.0328 ms back to back
// (profiles/hybrid_amdsmi_scaling_r6.txt).  `node_id` is the
// session-cached KFD node (kNoNode = not yet known: queried and returned
// through it).  Returns false when the GPU is partitioned or an attribute
// is missing; the caller then queries amd-smi.
bool query_unpartitioned(AmdSmiLib& L, const std::string& root, ProcInfo& p, AmdSmiManager::KfdNodeFacts* kfd,
                         std::string* mode, int64_t* read_ns, AmdSmiManager::SessionValues* kept) {
  uint32_t* node_id = &kfd->node_id;
  std::string pci;  // built only for a read (a steady cycle makes none)
  auto pci_dir = [&]() -> const std::string& {
    if (pci.empty()) pci = fs::join(root, "sys/bus/pci/devices/" + p.gpu_bdf);
    return pci;
  };
  if (mode->empty() && !session_compute_mode(pci_dir(), mode, read_ns)) return false;
  if (*mode != "SPX") return false;
  std::string mp_mode;
  std::optional<uint64_t> vram;
  if (kept && !kept->memory_partition.empty() && kept->vram) {
    mp_mode = kept->memory_partition;
    vram = kept->vram;
  } else {
    pci_dir();
    auto mp = AMDSMI_CALL("memory_partition(sysfs)", fs::attrs().read_trimmed(pci + "/current_memory_partition"));
    mp_mode = mp ? partition_mode(*mp) : "";
    if (mp_mode.empty()) return false;
    auto vram_s = AMDSMI_CALL("memory_total(sysfs)", fs::attrs().read_trimmed(pci + "/mem_info_vram_total"));
    vram = vram_s ? str::parse_uint(*vram_s) : std::nullopt;
    if (!vram || *vram == 0) return false;
    if (kept) {
      kept->memory_partition = mp_mode;
      kept->vram = *vram;
    }
  }
  if (!kfd->known && *node_id == kNoNode && !query_kfd(L, p, node_id)) return false;
  query_identity(L, root, p);
  p.compute_partition = "SPX";
  p.memory_partition = mp_mode;
  p.vram = *vram;
  if (!kfd->known) {
    // The XCD count from the KFD node, else (no node: amd-smi reports none
    // for a GPU whose node this container cannot read) the library's
    // counter - once per session; a failed count is tried again next cycle.
    uint32_t x = *node_id != kNoNode ? AMDSMI_CALL("kfd_num_xcc(sysfs)", kfd_num_xcc(root, *node_id)) : 0;
    uint16_t c = 0;
    if (x == 0 && L.get_gpu_xcd_counter && L.get_gpu_xcd_counter(p.h, &c) == AMDSMI_STATUS_SUCCESS) x = c;
    kfd->num_xcc = x;
    kfd->known = x != 0;
  }
  p.xcds = kfd->num_xcc;
  fix_market_name(L, root, p);
  return true;
}

// The processors of one partitioned GPU (DPX/QPX/CPX, or the partitions of
// it this container may see): per cycle, the compute and memory partition
// modes from the parent function's amdgpu attributes (shared by every
// partition) and each processor's ASIC info; per session (`facts`, aligned
// with `procs`; node_id kNoNode = not known yet) each partition's KFD node
// (amdsmi_get_gpu_kfd_info) and from it the partition id, XCD/SDMA counts
// and memory.  Returns false when the parent reports SPX or an attribute or
// node is missing; the caller then queries every value through amd-smi.
bool query_partitioned(AmdSmiLib& L, const std::string& root, std::vector<ProcInfo>& procs,
                       std::vector<AmdSmiManager::PartitionFacts>& facts, std::string* mode, int64_t* read_ns) {
  std::string pci = fs::join(root, "sys/bus/pci/devices/" + procs.front().gpu_bdf);
  if (!session_compute_mode(pci, mode, read_ns) || *mode == "SPX") return false;
  const std::string cp = *mode;
  auto mp_raw = AMDSMI_CALL("memory_partition(sysfs)", fs::attrs().read_trimmed(pci + "/current_memory_partition"));
  std::string mp = mp_raw ? partition_mode(*mp_raw) : "";
  if (mp.empty()) return false;
  for (size_t i = 0; i < procs.size(); ++i) {
    ProcInfo& p = procs[i];
    AmdSmiManager::PartitionFacts& f = facts[i];
    if (f.node_id == kNoNode) {
      uint32_t node = kNoNode;
      if (!query_kfd(L, p, &node) || node == kNoNode) return false;
      KfdCounts c = AMDSMI_CALL("kfd_counts(sysfs)", kfd_counts(root, node));
      uint64_t mem = kfd_node_memory_bytes(fs::join(root, "sys/class/kfd/kfd/topology/nodes/" + std::to_string(node)));
      if (c.num_xcc == 0 || mem == 0) return false;
      f.handle = p.h;
      f.node_id = node;
      f.partition_id = p.partition_id;
      f.num_xcc = c.num_xcc;
      f.sdma = c.num_sdma;
      f.mem_bytes = mem;
    }
    query_identity(L, root, p);
    p.partition_id = f.partition_id;
    p.xcds = f.num_xcc;
    p.sdma = f.sdma;
    p.vram = f.mem_bytes;
    p.compute_partition = cp;
    p.memory_partition = mp;
  }
  fix_market_name(L, root, procs.front());
  for (auto& p : procs) p.market_name = procs.front().market_name;
  return true;
}

// Every value through amd-smi (partitioned GPUs, or sysfs values disabled).
void query_proc(AmdSmiLib& L, const std::string& root, ProcInfo& p) {
  query_identity(L, root, p);

  uint64_t total = 0;
  if (AMDSMI_CALL("memory_total", L.get_gpu_memory_total(p.h, AMDSMI_MEM_TYPE_VRAM, &total)) == AMDSMI_STATUS_SUCCESS)
    p.vram = total;

  uint32_t node_id = kNoNode;
  query_kfd(L, p, &node_id);
  if (node_id != kNoNode) {
    KfdCounts c = AMDSMI_CALL("kfd_counts(sysfs)", kfd_counts(root, node_id));
    p.xcds = c.num_xcc;
    p.sdma = c.num_sdma;
  }
  char buf[64];
  if (L.get_gpu_compute_partition) {
    std::memset(buf, 0, sizeof(buf));
    if (AMDSMI_CALL("compute_partition", L.get_gpu_compute_partition(p.h, buf, sizeof(buf))) == AMDSMI_STATUS_SUCCESS)
      p.compute_partition = partition_mode(buf);
  }
  if (L.get_gpu_memory_partition) {
    std::memset(buf, 0, sizeof(buf));
    if (AMDSMI_CALL("memory_partition", L.get_gpu_memory_partition(p.h, buf, sizeof(buf))) == AMDSMI_STATUS_SUCCESS)
      p.memory_partition = partition_mode(buf);
  }
  if (p.xcds == 0 && L.get_gpu_xcd_counter) {
    uint16_t x = 0;
    if (L.get_gpu_xcd_counter(p.h, &x) == AMDSMI_STATUS_SUCCESS) p.xcds = x;
  }
  fix_market_name(L, root, p);
}

// xGMI links to hive peers from amdgpu's per-peer table ("01 01 ... 00 01",
// measured on the pool: 7 links).  The same count amd-smi's link-status call
// derives, but that call decodes the gpu_metrics table through the SMU and
// costs ~280 us per GPU per cycle (GFD_AMDSMI_CALL_TRACE on MI355X) versus
// ~5 us here.
int sysfs_xgmi_links(const std::string& root, const std::string& bdf) {
  auto v = fs::attrs().read_trimmed(fs::join(root, "sys/bus/pci/devices/" + bdf + "/xgmi_num_links"));
  if (!v) return -1;
  int total = 0;
  bool any = false;
  for (const auto& tok : str::split(*v, ' ')) {
    if (tok.empty()) continue;
    auto n = str::parse_uint(tok, 16);
    if (!n) return -1;
    total += static_cast<int>(*n);
    any = true;
  }
  return any ? total : -1;
}

// GPU-level capabilities: xGMI links, virtualization mode, supported
// partition modes.  Any processor handle of the GPU will do.
void query_gpu_caps(AmdSmiLib& L, const ProcInfo& p, const std::string& root, GpuExtras& x,
                    const AmdSmiManager::AvailableModes* kept_avail, AmdSmiManager::AvailableModes& avail) {
  // Pre-filled from the session (AmdSmiManager::session_values_) when kept.
  if (x.xgmi_links < 0) x.xgmi_links = AMDSMI_CALL("xgmi_num_links(sysfs)", sysfs_xgmi_links(root, p.gpu_bdf));
  if (x.xgmi_links < 0 && L.get_gpu_xgmi_link_status) {
    amdsmi_xgmi_link_status_t ls;
    std::memset(&ls, 0, sizeof(ls));
    if (AMDSMI_CALL("xgmi_link_status", L.get_gpu_xgmi_link_status(p.h, &ls)) == AMDSMI_STATUS_SUCCESS) {
      int up = 0;
      for (uint32_t i = 0; i < ls.total_links && i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i)
        if (ls.status[i] == AMDSMI_XGMI_LINK_UP) ++up;
      x.xgmi_links = up;
    }
  }
  // Pre-filled from the session cache when already known (see snapshot()).
  // Without an answer from amd-smi (it refuses the query when it could not
  // load libdrm_amdgpu) the driver's classification from sysfs, as the KFD
  // backend labels it.
  if (x.virtualization.empty() && L.get_gpu_virtualization_mode) {
    amdsmi_virtualization_mode_t vm = AMDSMI_VIRTUALIZATION_MODE_UNKNOWN;
    if (AMDSMI_CALL("virtualization_mode", L.get_gpu_virtualization_mode(p.h, &vm)) == AMDSMI_STATUS_SUCCESS)
      x.virtualization = virt_name(vm);
  }
  if (x.virtualization.empty()) {
    std::string pci = fs::join(root, "sys/bus/pci/devices/" + p.gpu_bdf);
    if (fs::exists(pci))
      x.virtualization = classify_virtualization(pci, p.device_id, running_in_vm(root), fs::exists(pci + "/physfn"));
  }
  // Kept from an earlier cycle of the session (AmdSmiManager::available_).
  if (kept_avail && kept_avail->known) {
    x.available_memory = kept_avail->memory;
    x.available_compute = kept_avail->compute;
    return;
  }
  // Supported memory partition modes: world-readable in sysfs (~5 us);
  // the amd-smi partition-config call (~25 us) only as a fallback.
  if (auto v = AMDSMI_CALL("available_memory_partition(sysfs)",
                           fs::attrs().read_trimmed(fs::join(root, "sys/bus/pci/devices/" + p.gpu_bdf + "/available_memory_partition")))) {
    x.available_memory = partition_mode_list(*v);
  } else if (L.get_gpu_memory_partition_config) {
    amdsmi_memory_partition_config_t cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    if (AMDSMI_CALL("memory_partition_config", L.get_gpu_memory_partition_config(p.h, &cfg)) == AMDSMI_STATUS_SUCCESS)
      x.available_memory = nps_list(cfg.partition_caps.nps_cap_mask);
  }
  // Supported compute partition modes: world-readable in sysfs, the source
  // amd-smi reads too; the library's profile table (root only: NO_PERM for
  // a pod, and a partial table when amd-smi runs without libdrm_amdgpu)
  // only as a fallback.
  if (auto v = AMDSMI_CALL("available_compute_partition(sysfs)",
                           fs::attrs().read_trimmed(fs::join(root, "sys/bus/pci/devices/" + p.gpu_bdf + "/available_compute_partition")))) {
    x.available_compute = partition_mode_list(*v);
  }
  if (x.available_compute.empty() && L.get_gpu_accelerator_partition_profile_config) {
    amdsmi_accelerator_partition_profile_config_t cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    if (AMDSMI_CALL("partition_profile_config", L.get_gpu_accelerator_partition_profile_config(p.h, &cfg)) ==
        AMDSMI_STATUS_SUCCESS) {
      for (uint32_t i = 0; i < cfg.num_profiles && i < AMDSMI_MAX_ACCELERATOR_PROFILE; ++i)
        if (const char* n = accel_name(cfg.profiles[i].profile_type)) x.available_compute.push_back(n);
    }
  }
  // Kept only when both lists were found.
  if (!x.available_memory.empty() && !x.available_compute.empty())
    avail = {true, x.available_memory, x.available_compute};
  else
    avail = {};
}

std::string format_bdf(const amdsmi_bdf_t& b) {
  return str::format("%04llx:%02x:%02x.%x", static_cast<unsigned long long>(b.domain_number),
                     static_cast<unsigned>(b.bus_number), static_cast<unsigned>(b.device_number),
                     static_cast<unsigned>(b.function_number));
}


// The PCI address of a processor, decided once per session.  amd-smi's
// answer stands when it is a PCI function under <root>/sys, or when nothing
// better is known; otherwise (amd-smi without libdrm_amdgpu reports garbage
// such as "5ddf28c0:c2:1a.0" with success) the address KFD reports for the
// processor's node (domain, location_id) - what amd-smi reports when libdrm
// works, including a partition's index in the function bits.
std::string checked_bdf(AmdSmiLib& L, const std::string& root, amdsmi_processor_handle h, const amdsmi_bdf_t& b) {
  std::string bdf = format_bdf(b);
  if (fs::exists(fs::join(root, "sys/bus/pci/devices/" + bdf))) return bdf;
  ProcInfo p;
  p.h = h;
  uint32_t node = kNoNode;
  if (!query_kfd(L, p, &node) || node == kNoNode) return bdf;
  auto r = kfd_properties(root, node);
  if (!r.ok()) return bdf;
  uint64_t location = kfd_field(r.data, "location_id").value_or(0);
  if (location == 0) return bdf;
  uint64_t domain = kfd_field(r.data, "domain").value_or(0);
  return str::format("%04llx:%02x:%02x.%x", static_cast<unsigned long long>(domain),
                     static_cast<unsigned>((location >> 8) & 0xff), static_cast<unsigned>((location >> 3) & 0x1f),
                     static_cast<unsigned>(location & 0x7));
}

}  // namespace

// The node's GPU processors grouped into physical GPUs (each group ordered
// as amd-smi listed it), ordered by parent PCI function; every processor's
// gpu_bdf set.  `parents` caches the parent function per group for the
// session (resolve_parent_bdf reads sysfs).
using IdentityCache = std::map<void*, AmdSmiManager::Identity>;

// Fills p's identity from the session cache; true if it was there.
static bool identity_from_cache(const IdentityCache& cache, ProcInfo& p) {
  auto it = cache.find(p.h);
  if (it == cache.end()) return false;
  const auto& id = it->second;
  p.market_name = id.market_name;
  p.vendor_id = id.vendor_id;
  p.device_id = id.device_id;
  p.cus = id.cus;
  p.gfx = id.gfx;
  p.uuid = id.uuid;
  p.identified = true;
  return true;
}

static std::vector<std::vector<ProcInfo>> collect_physical_gpus(AmdSmiLib& L, const std::string& root,
                                                                std::map<std::string, std::string>& parents,
                                                                std::map<void*, std::string>& proc_bdfs,
                                                                const IdentityCache& identities) {
  uint32_t ns = 0;
  amdsmi_status_t st = L.get_socket_handles(&ns, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_socket_handles", st);
  std::vector<amdsmi_socket_handle> sockets(ns);
  if (ns) {
    st = L.get_socket_handles(&ns, sockets.data());
    if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_socket_handles", st);
    sockets.resize(ns);
  }

  // Collect GPU processors by PCI slot (domain:bus:device - amd-smi's own
  // socket id, the same for every partition of a GPU under both KFD
  // location layouts; resource/physical.h).
  std::map<std::string, std::vector<ProcInfo>> slots;
  for (auto s : sockets) {
    uint32_t np = 0;
    st = L.get_processor_handles(s, &np, nullptr);
    if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_processor_handles", st);
    std::vector<amdsmi_processor_handle> procs(np);
    if (np) {
      st = L.get_processor_handles(s, &np, procs.data());
      if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_processor_handles", st);
      procs.resize(np);
    }
    for (auto h : procs) {
      processor_type_t t;
      if (L.get_processor_type(h, &t) != AMDSMI_STATUS_SUCCESS || t != AMDSMI_PROCESSOR_TYPE_AMD_GPU) continue;
      auto known = proc_bdfs.find(h);
      if (known == proc_bdfs.end()) {
        amdsmi_bdf_t b;
        std::memset(&b, 0, sizeof(b));
        st = L.get_gpu_device_bdf(h, &b);
        if (st != AMDSMI_STATUS_SUCCESS) call_failed(L, "amdsmi_get_gpu_device_bdf", st);
        known = proc_bdfs.emplace(h, checked_bdf(L, root, h, b)).first;
      }
      ProcInfo p;
      p.h = h;
      p.bdf = known->second;
      identity_from_cache(identities, p);
      slots[bdf_slot(p.bdf)].push_back(std::move(p));
    }
  }

  // Split slots into physical GPUs.  One processor: a GPU (the hot path, no
  // further calls).  Several: the partitions of one GPU when the family puts
  // partitions on one slot and they share the device ID - not the ASIC
  // serial, which a kernel reporting one per partition would split a CPX GPU
  // by (split_by_identity); otherwise distinct GPUs that happen to share a
  // slot.
  std::vector<std::vector<ProcInfo>> physical;
  for (auto& [slot, procs] : slots) {
    if (procs.size() == 1) {
      physical.push_back(std::move(procs));
      continue;
    }
    std::map<std::string, std::vector<ProcInfo>> by_gpu;
    for (auto& p : procs) {
      query_identity(L, root, p);
      bool partitions = partition_index_in_function_bits(gfx_target_from_amdsmi(p.gfx));
      by_gpu[partitions ? "device:" + std::to_string(p.device_id) : "bdf:" + p.bdf].push_back(std::move(p));
    }
    for (auto& [key, members] : by_gpu)
      for (auto& g : split_by_identity(
               root, std::move(members), [](const ProcInfo& p) { return p.uuid; },
               [](const ProcInfo& p) { return p.bdf; }))
        physical.push_back(std::move(g));
  }
  // Parent PCI function of each GPU, resolved once per session.
  for (auto& procs : physical) {
    std::vector<std::string> bdfs;
    for (const auto& p : procs) bdfs.push_back(p.bdf);
    std::string key = procs.size() == 1 ? procs[0].bdf : str::join(bdfs, ",");
    auto it = parents.find(key);
    if (it == parents.end()) {
      uint32_t device_id = 0;
      if (procs.size() > 1) device_id = procs.front().device_id;  // identified above
      it = parents.emplace(key, resolve_parent_bdf(root, bdfs, device_id)).first;
    }
    for (auto& p : procs) p.gpu_bdf = it->second;
  }
  std::sort(physical.begin(), physical.end(),
            [](const std::vector<ProcInfo>& a, const std::vector<ProcInfo>& b) { return a[0].gpu_bdf < b[0].gpu_bdf; });

  return physical;
}

// ---------------------------------------------------------------------------
// AmdSmiManager



AmdSmiManager::AmdSmiManager(AmdSmiOptions opts)
    : opts_(std::move(opts)), generation_attr_(fs::join(opts_.root, "sys/class/kfd/kfd/topology/generation_id")) {
  opts_.versions.root = opts_.root;
}

AmdSmiManager::~AmdSmiManager() {
  if (lib_initialized_) library_shutdown();
}

void AmdSmiManager::library_init() {
  trace::Span span("amdsmi_init");
  std::lock_guard<std::mutex> g(lib_->mu);
  amdsmi_status_t st = lib_->init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) throw Error("amdsmi_init failed: " + lib_->status_str(st));
  lib_->users++;
  lib_->asic_info_unsupported = false;
  lib_initialized_ = true;
  virt_mode_.clear();
  kfd_node_.clear();
  partition_facts_.clear();
  parent_bdf_.clear();
  proc_bdf_.clear();
  identity_.clear();
  available_.clear();
  compute_mode_.clear();
  session_values_.clear();
  ++init_count_;
}

void AmdSmiManager::library_shutdown() {
  std::lock_guard<std::mutex> g(lib_->mu);
  lib_initialized_ = false;
  if (--lib_->users == 0) lib_->shut_down();
}

std::string AmdSmiManager::read_generation() const {
  std::string gen;
  if (!generation_attr_.read(&gen)) gen.clear();
  return gen;
}

void AmdSmiManager::Init() {
  if (!lib_) {
    std::string err;
    lib_ = AmdSmiLib::get(&err);
    if (!lib_) throw Error("failed to load amd-smi: " + err);
  }
  if (opts_.persistent && lib_initialized_) {
    // A partition-mode change or driver reload bumps the KFD generation and
    // invalidates every processor handle.
    std::string gen = read_generation();
    if (gen != generation_) {
      fs::attrs().clear();  // KFD node paths of the old topology are gone
      library_shutdown();
      library_init();
      generation_ = gen;
    }
  } else if (!lib_initialized_) {
    library_init();
    if (opts_.persistent) generation_ = read_generation();
  }
  in_window_ = true;
  have_snapshot_ = false;
}

void AmdSmiManager::Shutdown() {
  in_window_ = false;
  have_snapshot_ = false;
  snapshot_.clear();
  if (!opts_.persistent && lib_initialized_) library_shutdown();
}

std::vector<DevicePtr> AmdSmiManager::GetDevices() {
  if (!in_window_) throw Error("amd-smi manager not initialized");
  if (have_snapshot_) return snapshot_;
  try {
    snapshot_ = snapshot();
  } catch (const CallError& e) {
    if (!opts_.persistent || !is_stale(e.status)) throw;
    log::printf("amd-smi handles are stale (%s); re-initializing", e.what());
    library_shutdown();
    library_init();
    generation_ = read_generation();
    snapshot_ = snapshot();
  }
  have_snapshot_ = true;
  return snapshot_;
}

std::vector<DevicePtr> AmdSmiManager::snapshot() {
  AmdSmiLib& L = *lib_;
  trace::Span span("amdsmi.snapshot");
  int64_t handles_t0 = trace::stamp();
  std::vector<std::vector<ProcInfo>> physical = collect_physical_gpus(L, opts_.root, parent_bdf_, proc_bdf_, identity_);
  trace::record_since("amdsmi.handles", handles_t0);

  // Apply the visible-device filter on physical GPUs (index = parent BDF order).
  struct Gpu {
    int index = 0;
    std::string bdf;
    std::vector<ProcInfo>* procs = nullptr;
    GpuExtras extras;
    std::exception_ptr error;
    int64_t proc_ns = 0, caps_ns = 0;
    KfdNodeFacts kfd;  // session cache entry (unpartitioned GPUs)
    std::string mode;  // session cache entry: compute partition mode
    SessionValues values;  // session cache entry: memory partition, VRAM, xGMI links
    int64_t mode_read_ns = -1;  // >= 0: read this cycle (not from the cache)
    AvailableModes avail;  // read this cycle (kept_avail: null)
    std::vector<PartitionFacts> parts;  // session cache entries (partitioned GPUs), aligned with procs
    // Which values came from the session's entries (then nothing is written
    // back: work() changes no value it was given).
    bool kept_virt = false, kept_kfd = false, kept_mode = false, kept_values = false;
    const AvailableModes* kept_avail = nullptr;
  };
  std::vector<Gpu> gpus;
  gpus.reserve(physical.size());
  for (size_t i = 0; i < physical.size(); ++i) {
    const std::string& bdf = physical[i][0].gpu_bdf;
    if (opts_.filter.matches(static_cast<int>(i), bdf)) {
      Gpu g;
      g.index = static_cast<int>(i);
      g.bdf = bdf;
      g.procs = &physical[i];
      gpus.push_back(std::move(g));
      Gpu& e = gpus.back();
      auto v = virt_mode_.find(bdf);
      if (v != virt_mode_.end()) {
        e.extras.virtualization = v->second;
        e.kept_virt = true;
      }
      auto k = kfd_node_.find(bdf);
      if (k != kfd_node_.end()) {
        e.kfd = k->second;
        e.kept_kfd = e.kfd.known;
      }
      auto a = available_.find(bdf);
      if (a != available_.end() && a->second.known) e.kept_avail = &a->second;
      auto sv = session_values_.find(bdf);
      if (sv != session_values_.end()) {
        e.values = sv->second;
        e.extras.xgmi_links = sv->second.xgmi_links;
        e.kept_values = true;
      }
      auto m = compute_mode_.find(bdf);
      if (m != compute_mode_.end()) {
        e.mode = m->second;
        e.kept_mode = !e.mode.empty();
      } else {
        e.mode_read_ns = 0;
      }
      e.parts.reserve(physical[i].size());
      for (const auto& p : physical[i]) {
        auto f = partition_facts_.find(p.h);
        e.parts.push_back(f != partition_facts_.end() ? f->second : PartitionFacts{});
      }
    }
  }
  if (!opts_.filter.all()) {  // checked when the set of GPUs changes, not every cycle
    bool same = selected_from_.size() == physical.size();
    for (size_t i = 0; same && i < physical.size(); ++i) same = selected_from_[i] == physical[i][0].gpu_bdf;
    if (!same) {
      selected_from_.clear();
      for (const auto& procs : physical) selected_from_.push_back(procs[0].gpu_bdf);
      opts_.filter.check_selection(selected_from_);
    }
  }
  const bool sysfs_values = opts_.sysfs_values;

  // One GPU's values and capabilities, always on one thread: amdgpu
  // serialises a device's queries on its own locks (amd-smi adds a
  // per-device mutex), so splitting one GPU's reads over threads makes each
  // of them slower - measured 273 us sequential vs 472 us split with amd-smi
  // calls, and 2-3x slower sysfs reads (profiles/README.md).  fast: only
  // through the unpartitioned (attribute) path - returns false if that path
  // does not apply; otherwise every processor through the library.
  // Lanes run on pool threads, which record nothing: this cycle's tracing
  // decides whether a GPU's work is timed.
  const bool traced = trace::active();
  auto work = [&](Gpu& g, bool fast) -> bool {
    try {
      int64_t t0 = trace::stamp(traced);
      auto& procs = *g.procs;
      if (fast) {
        int64_t* rd = &g.mode_read_ns;
        bool done = procs.size() == 1 && query_unpartitioned(L, opts_.root, procs[0], &g.kfd, &g.mode, rd, &g.values);
        if (!done && !query_partitioned(L, opts_.root, procs, g.parts, &g.mode, rd)) return false;
        std::sort(procs.begin(), procs.end(),
                  [](const ProcInfo& a, const ProcInfo& b) { return a.partition_id < b.partition_id; });
      } else {
        for (auto& p : procs) query_proc(L, opts_.root, p);
        std::sort(procs.begin(), procs.end(),
                  [](const ProcInfo& a, const ProcInfo& b) { return a.partition_id < b.partition_id; });
      }
      int64_t t1 = trace::stamp(traced);
      const ProcInfo& first = procs.front();
      query_gpu_caps(L, first, opts_.root, g.extras, g.kept_avail, g.avail);
      if (procs.size() > 1 || (!first.compute_partition.empty() && first.compute_partition != "SPX"))
        g.extras.engines = AMDSMI_CALL("partition_engines(sysfs)", partition_engine_counts(opts_.root, first.gpu_bdf));
      g.proc_ns = t1 - t0;
      g.caps_ns = trace::stamp(traced) - t1;
    } catch (...) {
      g.error = std::current_exception();
    }
    return true;
  };
  // One pass over the GPUs; each tries the attribute path first (SPX: ~7 us
  // of preads and cached library lookups; partitioned: two preads plus the
  // session-cached partition facts) and falls back to library calls in the
  // same lane.  (Two passes - all attribute attempts, then the library
  // fallbacks - left the second pass's helper lanes queued behind the first
  // pass's, so its items ran mostly serially on the caller: 8 GPUs 0.94 ms
  // instead of 0.22 ms over the latency-modelled fake.)  Lanes: one GPU per
  // lane (gpu_lanes: a cycle after the daemon's sleep runs on cold,
  // down-clocked cores - 8 GPUs' reads 170 us on one thread vs 36 us on four
  // lanes, profiles/multi_gpu_read_probe.txt - and with the pinned pool one
  // GPU per lane is also fastest back to back).
  int64_t t_gpus = trace::stamp();
  size_t lanes = opts_.threads > 0 ? static_cast<size_t>(opts_.threads) : gpu_lanes(gpus.size());
  // Nothing to read: every GPU is an unpartitioned one whose values the
  // session already holds (the steady state).  Its work is then a few
  // lookups, ~0.2 us warm, and waking helper lanes costs more than it: on
  // this thread.  8 GPUs over the host's real attributes (fake library):
  // back to back 0.0207 vs 0.0262 ms with one lane per GPU, the GPUs'
  // part 1.6 vs 5.0 us; 1 s apart 4-6 vs 15-20 us
  // (profiles/hybrid_amdsmi_scaling_r6.txt).
  if (sysfs_values && lanes > 1) {
    bool all_cached = true;
    for (const auto& g : gpus) {
      all_cached = all_cached && g.procs->size() == 1 && g.mode == "SPX" && g.values.vram != 0 &&
                   g.kfd.known && g.kept_avail &&
                   !g.extras.virtualization.empty() && g.extras.xgmi_links >= 0 && (*g.procs)[0].identified &&
                   !is_generic_name((*g.procs)[0].market_name);
      if (!all_cached) break;
    }
    if (all_cached) lanes = 1;
  }
  WorkerPool::ParallelStats lane_stats;
  WorkerPool::instance().parallel_for(
      gpus.size(),
      [&](size_t i) {
        if (sysfs_values && work(gpus[i], true)) return;
        work(gpus[i], false);
      },
      lanes, gpus.size() > 1 && traced ? &lane_stats : nullptr);
  trace::record_since("amdsmi.gpus", t_gpus);
  if (gpus.size() > 1 && traced) {
    // Where a multi-GPU snapshot's lanes spend it: the hand-off (enqueue
    // and wake the helpers, on this thread), how late the last GPU started
    // (a helper's wake-up), the slowest GPU's own work, and how many GPUs
    // this thread ran itself (a count, recorded as that many milliseconds).
    trace::record("amdsmi.lanes.handoff", lane_stats.handoff_ns);
    trace::record("amdsmi.lanes.last_start", lane_stats.last_start_ns);
    trace::record("amdsmi.lanes.max_gpu", lane_stats.max_item_ns);
    trace::record("amdsmi.lanes.caller_gpus(count_as_ms)", static_cast<int64_t>(lane_stats.caller_items) * 1000000);
  }
  // Per-GPU phase times: the slowest GPU (items may have run on pool
  // threads, whose trace records are their own).
  int64_t proc_ns = 0, caps_ns = 0;
  for (const auto& g : gpus) {
    proc_ns = std::max(proc_ns, g.proc_ns);
    caps_ns = std::max(caps_ns, g.caps_ns);
  }
  for (const auto& g : gpus)
    if (g.error) std::rethrow_exception(g.error);
  trace::record("amdsmi.proc", proc_ns);
  // The compute-mode reads of GPUs new to the session (none on a steady cycle).
  for (const auto& g : gpus)
    if (g.mode_read_ns > 0) trace::record("compute_partition(read)", g.mode_read_ns);
  trace::record("amdsmi.extras", caps_ns);
  for (const auto& g : gpus) {
    for (const auto& p : *g.procs)
      if (p.identified && !identity_.count(p.h))
        identity_[p.h] = Identity{p.market_name, p.vendor_id, p.device_id, p.cus, p.gfx, p.uuid};
    if (!g.kept_virt && !g.extras.virtualization.empty()) virt_mode_[g.bdf] = g.extras.virtualization;
    if (!g.kept_kfd && g.kfd.known) kfd_node_[g.bdf] = g.kfd;
    if (!g.kept_mode && !g.mode.empty()) compute_mode_[g.bdf] = g.mode;
    if (!g.kept_values && g.values.vram && g.extras.xgmi_links >= 0) {
      SessionValues v = g.values;
      v.xgmi_links = g.extras.xgmi_links;
      session_values_[g.bdf] = v;
    }
    if (!g.kept_avail) {
      if (!g.avail.known)
        available_.erase(g.bdf);
      else
        available_[g.bdf] = g.avail;
    }
    for (const auto& f : g.parts)
      if (f.node_id != kNoNode) partition_facts_[f.handle] = f;
  }

  std::vector<DevicePtr> out;
  for (auto& g : gpus) {
    const ProcInfo& first = g.procs->front();
    DeviceInfo info;
    info.index = g.index;
    info.bdf = g.bdf;
    info.name = first.market_name;
    info.uuid = first.uuid;
    info.vendor_id = first.vendor_id;
    info.device_id = first.device_id;
    info.gfx = gfx_target_from_amdsmi(first.gfx);
    info.compute_partition = first.compute_partition;
    info.memory_partition = first.memory_partition;
    info.available_compute_partitions = std::move(g.extras.available_compute);
    info.available_memory_partitions = std::move(g.extras.available_memory);
    info.xgmi_links = g.extras.xgmi_links;
    info.virtualization = g.extras.virtualization;
    bool partitioned = g.procs->size() > 1 || (!first.compute_partition.empty() && first.compute_partition != "SPX");

    std::vector<std::shared_ptr<SnapshotDevice>> parts;
    uint64_t mem = 0;
    uint32_t cus = 0, xcds = 0;
    for (const auto& p : *g.procs) {
      mem += p.vram;
      cus += p.cus;
      xcds += p.xcds;
      if (!partitioned) continue;
      DeviceInfo pi;
      pi.partition_id = static_cast<int>(p.partition_id);
      pi.bdf = p.bdf;
      pi.uuid = p.uuid;
      pi.vendor_id = p.vendor_id;
      pi.device_id = p.device_id;
      pi.compute_units = p.cus;
      pi.xcds = p.xcds;
      pi.memory_mib = p.vram >> 20;
      pi.compute_partition = p.compute_partition;
      pi.memory_partition = p.memory_partition;
      pi.name = partition_profile_name(pi.compute_partition, pi.xcds, pi.memory_mib);
      pi.attributes = partition_attributes(pi.memory_mib, pi.compute_units, pi.xcds, p.sdma, g.extras.engines,
                                           pi.compute_partition, pi.memory_partition);
      parts.push_back(SnapshotDevice::partition(std::move(pi)));
    }
    info.memory_mib = mem >> 20;
    info.compute_units = cus;
    info.xcds = xcds;
    bool capable = info.available_compute_partitions.size() > 1;
    auto dev = SnapshotDevice::gpu(std::move(info), partitioned, capable);
    dev->set_partitions(std::move(parts));
    out.push_back(dev);
  }
  return out;
}

std::string AmdSmiManager::GetDriverVersion() {
  // amdsmi_get_gpu_driver_info reports /sys/module/amdgpu/version for a DKMS
  // driver and the kernel banner for an in-tree one (measured on the pool:
  // "Linuxversion6.18.54-ant.1(...)").  Reading those sources directly gives
  // the same answer without the ~130 us library round trip per cycle.
  return driver_version(opts_.root);
}

std::optional<RuntimeVersion> AmdSmiManager::GetRuntimeVersion() { return rocm_version(opts_.versions); }

}  // namespace gfd::resource
