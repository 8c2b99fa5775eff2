#include "resource/sysfs.h"

#if defined(__x86_64__)
#include <cpuid.h>
#endif

#include <algorithm>
#include <cerrno>
#include <map>
#include <tuple>

#include "resource/pci_ids.h"
#include "resource/physical.h"
#include "resource/versions.h"
#include "util/error.h"
#include "util/fs.h"
#include "util/pool.h"
#include "util/strings.h"
#include "util/trace.h"

namespace gfd::resource {

namespace {

constexpr const char* kTopology = "sys/class/kfd/kfd/topology/nodes";

// The subset of KFD node properties the labels need.
struct KfdNode {
  int id = -1;
  uint64_t gfx_target_version = 0;
  uint64_t simd_count = 0;
  uint64_t simd_per_cu = 0;
  uint64_t num_xcc = 0;
  uint64_t location_id = 0;
  uint64_t domain = 0;
  uint64_t vendor_id = 0;
  uint64_t device_id = 0;
  uint64_t unique_id = 0;
  uint64_t drm_render_minor = 0;
  uint64_t num_sdma_engines = 0;
  uint64_t local_mem_size = 0;
  uint64_t mem_bytes = 0;  // device-local memory of the node (mem_banks), read with the properties
  std::string dir;
};

// Parse "key value\n" lines, picking only known keys (one pass, no maps).
void parse_properties(const std::string& text, KfdNode& n) {
  struct Key {
    const char* name;
    size_t len;
    uint64_t KfdNode::*field;
  };
#define K(f) \
  { #f, sizeof(#f) - 1, &KfdNode::f }
  static const Key keys[] = {K(gfx_target_version), K(simd_count), K(simd_per_cu),      K(num_xcc),
                             K(location_id),        K(domain),     K(vendor_id),        K(device_id),
                             K(unique_id),          K(drm_render_minor), K(num_sdma_engines), K(local_mem_size)};
#undef K
  size_t pos = 0;
  while (pos < text.size()) {
    size_t eol = text.find('\n', pos);
    if (eol == std::string::npos) eol = text.size();
    size_t sp = text.find(' ', pos);
    if (sp != std::string::npos && sp < eol) {
      size_t klen = sp - pos;
      for (const auto& k : keys) {
        if (k.len == klen && text.compare(pos, klen, k.name) == 0) {
          uint64_t v = 0;
          for (size_t i = sp + 1; i < eol && text[i] >= '0' && text[i] <= '9'; ++i)
            v = v * 10 + static_cast<uint64_t>(text[i] - '0');
          n.*(k.field) = v;
          break;
        }
      }
    }
    pos = eol + 1;
  }
}

// "01 01 01 01 01 01 00 01" -> 7 (links to each hive peer; self is 00).
int sum_links(const std::string& s) {
  int total = 0;
  bool any = false;
  for (auto& tok : str::split(str::replace_all(s, "\n", " "), ' ')) {
    std::string t = str::trim(tok);
    if (t.empty()) continue;
    auto v = str::parse_uint(t, 16);
    if (!v) return -1;
    total += static_cast<int>(*v);
    any = true;
  }
  return any ? total : -1;
}

std::string bdf_of(const KfdNode& n) {
  unsigned bus = static_cast<unsigned>((n.location_id >> 8) & 0xff);
  unsigned dev = static_cast<unsigned>((n.location_id >> 3) & 0x1f);
  unsigned fn = static_cast<unsigned>(n.location_id & 0x7);
  return str::format("%04x:%02x:%02x.%x", static_cast<unsigned>(n.domain), bus, dev, fn);
}
}  // namespace

bool running_in_vm(const std::string& root) {
#if defined(__x86_64__)
  // The kernel's "hypervisor" flag is CPUID leaf 1, ECX bit 31: asking the
  // CPU costs 0.08 us on the pool versus 15-90 us for the kernel to format
  // the start of /proc/cpuinfo (profiles/cpuinfo_probe.txt).
  if (root.empty() || root == "/") {
    unsigned a = 0, b = 0, c = 0, d = 0;
    if (__get_cpuid(1, &a, &b, &c, &d)) return (c >> 31) & 1u;
  }
#endif
  // The first processor's "flags" line (synthetic trees, other
  // architectures): read the start of the file, more only if that line is
  // not complete yet (all of /proc/cpuinfo on a 256-thread host is ~400 KB).
  for (size_t max : {size_t{4096}, size_t{16384}}) {
    auto r = fs::read_file(fs::join(root, "proc/cpuinfo"), max);
    if (!r.ok()) return false;
    auto flags = r.data.find("\nflags");
    if (flags == std::string::npos) {
      if (r.data.size() < max) return false;
      continue;
    }
    auto eol = r.data.find('\n', flags + 1);
    if (eol == std::string::npos && r.data.size() >= max) continue;
    std::string line = r.data.substr(flags, eol == std::string::npos ? std::string::npos : eol - flags);
    return (line + " ").find(" hypervisor ") != std::string::npos;
  }
  return false;
}

bool has_kfd_topology(const std::string& root, std::string* reason) {
  std::string dir = fs::join(root, kTopology);
  int err = 0;
  auto nodes = fs::list_dir(dir, &err);
  if (err != 0) {
    if (reason) *reason = "could not read " + dir + ": " + fs::errno_str(err);
    return false;
  }
  if (reason) *reason = "found KFD topology at " + dir + " (" + std::to_string(nodes.size()) + " nodes)";
  return true;
}

SysfsManager::SysfsManager(SysfsOptions opts)
    : opts_(std::move(opts)), generation_attr_(fs::join(opts_.root, "sys/class/kfd/kfd/topology/generation_id")) {
  opts_.versions.root = opts_.root;
  topology_ = fs::join(opts_.root, kTopology);
  in_vm_ = running_in_vm(opts_.root);
}

void SysfsManager::Init() {
  // generation_id lives next to nodes/; when it is readable the topology is
  // there.  Otherwise list nodes/ (kernels without generation_id, or to get
  // the error to report).
  if (!generation_attr_.read(&generation_)) generation_.clear();
  if (generation_.empty()) {
    int err = 0;
    fs::list_dir(topology_, &err);
    if (err != 0) throw Error("KFD topology not available at " + topology_ + ": " + fs::errno_str(err));
  }
  initialized_ = true;
  have_snapshot_ = false;
}

void SysfsManager::Shutdown() {
  initialized_ = false;
  have_snapshot_ = false;
  snapshot_.clear();
}

std::vector<DevicePtr> SysfsManager::GetDevices() {
  if (!initialized_) throw Error("sysfs manager not initialized");
  if (!have_snapshot_) {
    snapshot_ = enumerate();
    have_snapshot_ = true;
  }
  return snapshot_;
}

// One physical GPU (and its partitions) from its KFD nodes and PCI attributes.
// `bdf` is the parent PCI function (see resource/physical.h): every GPU-wide
// attribute is read there, whichever addresses the partitions report.
static DevicePtr describe_gpu(const std::string& root, bool in_vm, int index, const std::string& bdf,
                              const std::vector<const KfdNode*>& members, bool has_physfn,
                              const std::string& compute_partition) {
  const KfdNode& first = *members.front();
  std::string pci = fs::join(root, "sys/bus/pci/devices/" + bdf);

  DeviceInfo info;
  info.index = index;
  info.bdf = bdf;
  info.vendor_id = static_cast<uint32_t>(first.vendor_id);
  info.device_id = static_cast<uint32_t>(first.device_id);
  info.uuid = amd_uuid(first.unique_id, static_cast<uint32_t>(first.device_id));
  info.gfx = gfx_target_from_kfd(first.gfx_target_version);
  auto product = fs::attrs().read_trimmed(fs::join(pci, "product_name"));
  info.name = product && !product->empty() ? *product : device_name(static_cast<uint32_t>(first.device_id));
  info.compute_partition = compute_partition;
  info.memory_partition = partition_mode(fs::attrs().read_trimmed(fs::join(pci, "current_memory_partition")).value_or(""));
  info.available_compute_partitions =
      partition_mode_list(fs::attrs().read_trimmed(fs::join(pci, "available_compute_partition")).value_or(""));
  info.available_memory_partitions =
      partition_mode_list(fs::attrs().read_trimmed(fs::join(pci, "available_memory_partition")).value_or(""));
  if (auto x = fs::attrs().read_trimmed(fs::join(pci, "xgmi_num_links"))) info.xgmi_links = sum_links(*x);
  info.virtualization = classify_virtualization(pci, info.device_id, in_vm, has_physfn);

  bool partitioned = members.size() > 1 || (!info.compute_partition.empty() && info.compute_partition != "SPX");
  uint64_t vram = 0;
  if (auto v = fs::attrs().read_trimmed(fs::join(pci, "mem_info_vram_total"))) vram = str::parse_uint(*v).value_or(0);

  // Per-partition HBM: each partition node's memory banks, read with the
  // node properties (a partition's share of HBM only changes with a
  // partition or NPS switch, which rebuilds the KFD topology).

  Attributes engines;
  if (partitioned) engines = partition_engine_counts(root, bdf);
  // Partition ids: where the partitions' KFD locations carry their index in
  // the function bits (upstream amdgpu on GC 9.4.3-class parts,
  // resource/physical.h), that index - the current_partition_id amd-smi
  // reports and AMD's CLI keys primary partitions on
  // (amdsmi_cli/amdsmi_helpers.py:1691-1725), also when the container sees
  // only some partitions.  Otherwise (every partition at the parent's
  // location) the position among the GPU's nodes.
  bool index_in_function = false;
  if (partition_index_in_function_bits(info.gfx))
    for (const KfdNode* n : members) index_in_function = index_in_function || (n->location_id & 7) != 0;
  std::vector<std::shared_ptr<SnapshotDevice>> parts;
  uint32_t cus = 0, xcds = 0;
  uint64_t part_mem_sum = 0;
  for (size_t p = 0; p < members.size(); ++p) {
    const KfdNode& n = *members[p];
    uint32_t pcus = n.simd_per_cu ? static_cast<uint32_t>(n.simd_count / n.simd_per_cu) : 0;
    cus += pcus;
    xcds += static_cast<uint32_t>(n.num_xcc);
    if (!partitioned) continue;
    DeviceInfo pi;
    pi.partition_id = index_in_function ? static_cast<int>(n.location_id & 7) : static_cast<int>(p);
    pi.bdf = bdf_of(n);
    pi.vendor_id = info.vendor_id;
    pi.device_id = info.device_id;
    pi.compute_units = pcus;
    pi.xcds = static_cast<uint32_t>(n.num_xcc);
    uint64_t mem = n.mem_bytes;
    pi.memory_mib = mem >> 20;
    part_mem_sum += mem;
    pi.compute_partition = info.compute_partition;
    pi.memory_partition = info.memory_partition;
    pi.name = partition_profile_name(pi.compute_partition, pi.xcds, pi.memory_mib);
    pi.attributes = partition_attributes(pi.memory_mib, pcus, pi.xcds, static_cast<int>(n.num_sdma_engines), engines,
                                         pi.compute_partition, pi.memory_partition);
    parts.push_back(SnapshotDevice::partition(std::move(pi)));
  }
  info.compute_units = cus;
  info.xcds = xcds;
  if (vram == 0) vram = partitioned ? part_mem_sum : first.mem_bytes;
  info.memory_mib = vram >> 20;

  bool capable = info.available_compute_partitions.size() > 1;
  auto dev = SnapshotDevice::gpu(std::move(info), partitioned, capable);
  dev->set_partitions(std::move(parts));
  return dev;
}

struct SysfsManager::Topology {
  std::vector<KfdNode> nodes;  // accessible GPU nodes, by node id
  struct Gpu {
    std::string bdf;                       // parent PCI function
    std::vector<const KfdNode*> members;   // its partitions' nodes, by node id
    // A `physfn` link (the function is an SR-IOV VF), fixed when the PCI
    // function is created - looked up here, not with a path walk per cycle.
    bool has_physfn = false;
    // Its compute partition mode (current_compute_partition), read once per
    // topology generation: amdgpu answers that attribute by reading the XCP
    // control register, which "may momentarily wake the GPU up" - AMD's own
    // CLI stopped reading it by default for that reason
    // (/opt/rocm/libexec/amdsmi_cli/amdsmi_commands.py:463-466).  A
    // partition switch rebuilds the GPU's KFD nodes and bumps the
    // generation, which re-reads the topology and this with it.
    std::string compute_partition;
  };
  std::vector<Gpu> gpus;  // ordered by parent BDF (the enumeration index)
};

std::shared_ptr<const SysfsManager::Topology> SysfsManager::read_topology() const {
  // 1. Read every accessible GPU node.  A CPX node has 64 of them, so the
  //    reads are spread over the worker pool in chunks.
  std::vector<KfdNode> nodes;
  for (const auto& name : fs::list_dir(topology_)) {
    auto id = str::parse_uint(name);
    if (!id) continue;
    KfdNode n;
    n.id = static_cast<int>(*id);
    n.dir = fs::join(topology_, name);
    nodes.push_back(std::move(n));
  }
  std::vector<char> usable(nodes.size(), 0);
  constexpr size_t kChunk = 8;
  fs::Dir top(topology_);  // "<id>/properties" relative to it: no path walk per node
  auto read_chunk = [&](size_t c) {
    for (size_t i = c * kChunk; i < std::min(nodes.size(), (c + 1) * kChunk); ++i) {
      auto r = top.read_attr((std::to_string(nodes[i].id) + "/properties").c_str());
      if (!r.ok()) continue;  // EPERM: GPU not allocated to this container
      parse_properties(r.data, nodes[i]);
      usable[i] = nodes[i].gfx_target_version != 0 && nodes[i].simd_count != 0;  // else a CPU node
      if (usable[i])
        nodes[i].mem_bytes = nodes[i].local_mem_size ? nodes[i].local_mem_size : kfd_node_memory_bytes(nodes[i].dir);
    }
  };
  size_t chunks = (nodes.size() + kChunk - 1) / kChunk;
  int64_t t0 = trace::stamp();
  // Lanes on parked workers only: a oneshot Job's 10-node host topology is
  // read faster by this thread than by a worker created for it.
  WorkerPool::instance().parallel_for(chunks, read_chunk, 1 + WorkerPool::instance().idle_workers());
  trace::record_since("sysfs.nodes", t0);
  auto topo = std::make_shared<Topology>();
  for (size_t i = 0; i < nodes.size(); ++i)
    if (usable[i]) topo->nodes.push_back(std::move(nodes[i]));
  std::sort(topo->nodes.begin(), topo->nodes.end(), [](const KfdNode& a, const KfdNode& b) { return a.id < b.id; });

  // 2. Group partitions by physical GPU: (domain, location, device ID), with
  //    the PCI function bits - where partition-capable parts put the
  //    partition index - masked (resource/physical.h).  Not the ASIC serial
  //    (unique_id): every partition of a GPU reports the GPU's on current
  //    kernels, but a kernel reporting one per partition must not turn a CPX
  //    GPU into 8 GPUs (split_by_identity).
  struct Key {
    uint64_t domain, location, device_id;
    bool operator<(const Key& o) const {
      return std::tie(domain, location, device_id) < std::tie(o.domain, o.location, o.device_id);
    }
  };
  std::map<Key, std::vector<const KfdNode*>> groups;
  for (const auto& n : topo->nodes) {
    bool masked = partition_index_in_function_bits(gfx_target_from_kfd(n.gfx_target_version));
    groups[Key{n.domain, masked ? (n.location_id & ~uint64_t{7}) : n.location_id, n.device_id}].push_back(&n);
  }
  std::vector<std::vector<const KfdNode*>> physical;
  for (auto& [key, members] : groups)
    for (auto& g : split_by_identity(
             opts_.root, std::move(members), [](const KfdNode* n) { return n->unique_id; },
             [](const KfdNode* n) { return bdf_of(*n); }))
      physical.push_back(std::move(g));
  for (auto& members : physical) {
    std::vector<std::string> bdfs;
    for (const auto* n : members) bdfs.push_back(bdf_of(*n));
    Topology::Gpu g;
    g.bdf = resolve_parent_bdf(opts_.root, bdfs, static_cast<uint32_t>(members.front()->device_id));
    g.members = std::move(members);
    g.has_physfn = fs::exists(fs::join(opts_.root, "sys/bus/pci/devices/" + g.bdf + "/physfn"));
    int64_t r0 = trace::stamp();
    g.compute_partition = partition_mode(
        fs::attrs().read_trimmed(fs::join(opts_.root, "sys/bus/pci/devices/" + g.bdf + "/current_compute_partition"))
            .value_or(""));
    trace::record_since("compute_partition(read)", r0);
    topo->gpus.push_back(std::move(g));
  }
  std::sort(topo->gpus.begin(), topo->gpus.end(),
            [](const Topology::Gpu& a, const Topology::Gpu& b) { return a.bdf < b.bdf; });
  return topo;
}

std::vector<DevicePtr> SysfsManager::enumerate() {
  std::shared_ptr<const Topology> topo;
  bool fresh = false;
  if (!generation_.empty() && generation_ == cached_generation_ && cached_) {
    topo = cached_;
  } else {
    if (!cached_generation_.empty()) fs::attrs().clear();  // paths of the old topology
    topo = read_topology();
    fresh = true;
    cached_ = generation_.empty() ? nullptr : topo;
    cached_generation_ = generation_;
  }

  // 3. Describe each visible physical GPU (~10 sysfs reads each), in
  //    parallel across GPUs.
  std::vector<std::pair<int, const Topology::Gpu*>> visible;
  for (size_t i = 0; i < topo->gpus.size(); ++i)
    if (opts_.filter.matches(static_cast<int>(i), topo->gpus[i].bdf))
      visible.emplace_back(static_cast<int>(i), &topo->gpus[i]);
  if (fresh && !opts_.filter.all()) {  // the GPUs can only change with the topology
    std::vector<std::string> bdfs;
    for (const auto& g : topo->gpus) bdfs.push_back(g.bdf);
    opts_.filter.check_selection(bdfs);
  }
  std::vector<DevicePtr> out(visible.size());
  trace::Span span("sysfs.gpus");
  // ~10 attribute preads per GPU (a partitioned one also its partitions'
  // engine counts), one GPU per lane (gpu_lanes, see AmdSmiManager::snapshot).
  size_t lanes = gpu_lanes(visible.size());
  WorkerPool::instance().parallel_for(
      visible.size(),
      [&](size_t i) {
        const Topology::Gpu& g = *visible[i].second;
        out[i] = describe_gpu(opts_.root, in_vm_, visible[i].first, g.bdf, g.members, g.has_physfn, g.compute_partition);
      },
      lanes);
  return out;
}

std::string SysfsManager::GetDriverVersion() { return driver_version(opts_.root); }

std::optional<RuntimeVersion> SysfsManager::GetRuntimeVersion() { return rocm_version(opts_.versions); }

}  // namespace gfd::resource
