// Python bindings for the native core (module gpu_feature_discovery_amd._gfd).
//
// The daemon itself is the C++ binary; this module exposes the same code
// paths in-process so the test-suite can drive labelers directly (like the
// reference's in-package Go tests calling run()) and bench.py can time
// labeling cycles without process-spawn noise.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "cli/daemon.h"
#include "cli/flags.h"
#include "config/config.h"
#include "config/yaml.h"
#include "info/version.h"
#include "lm/labels.h"
#include "lm/node.h"
#include "resource/amdsmi.h"
#include "resource/factory.h"
#include "resource/managers.h"
#include "resource/sysfs.h"
#include "sriov/bound.h"
#include "sriov/sriov.h"
#include "util/duration.h"
#include "util/error.h"
#include "util/log.h"
#include "util/pool.h"

namespace py = pybind11;
using namespace gfd;

namespace {

py::dict cycle_to_dict(const cli::CycleResult& r) {
  py::dict d;
  d["labels"] = r.labels;
  d["total_ns"] = r.total_ns;
  py::list phases;
  for (const auto& p : r.phases) phases.append(py::make_tuple(p.first, p.second));
  d["phases"] = phases;
  d["rendered"] = lm::render(r.labels);
  return d;
}

py::object node_to_py(const yaml::Node& n) {
  using K = yaml::Node::Kind;
  switch (n.kind()) {
    case K::Null: return py::none();
    case K::Bool: return py::bool_(n.as_bool());
    case K::Int: return py::int_(n.as_int());
    case K::Float: return py::float_(n.as_float());
    case K::String: return py::str(n.text());
    case K::Seq: {
      py::list l;
      for (const auto& i : n.items()) l.append(node_to_py(i));
      return l;
    }
    case K::Map: {
      py::dict d;
      for (const auto& kv : n.entries()) d[py::str(kv.first)] = node_to_py(kv.second);
      return d;
    }
  }
  return py::none();
}

py::dict device_to_dict(const resource::Device& d) {
  const auto& i = d.Info();
  py::dict o;
  o["name"] = i.name;
  o["bdf"] = i.bdf;
  o["uuid"] = i.uuid;
  o["index"] = i.index;
  o["vendor_id"] = i.vendor_id;
  o["device_id"] = i.device_id;
  o["gfx"] = i.gfx.name();
  o["compute_units"] = i.compute_units;
  o["xcds"] = i.xcds;
  o["memory_mib"] = i.memory_mib;
  o["compute_partition"] = i.compute_partition;
  o["memory_partition"] = i.memory_partition;
  o["available_compute_partitions"] = i.available_compute_partitions;
  o["available_memory_partitions"] = i.available_memory_partitions;
  o["xgmi_links"] = i.xgmi_links;
  o["virtualization"] = i.virtualization;
  o["partition_id"] = i.partition_id;
  o["attributes"] = i.attributes;
  o["is_partition"] = d.IsPartition();
  if (!d.IsPartition()) {
    o["partitioned"] = d.IsPartitioned();
    o["partition_capable"] = d.IsPartitionCapable();
    py::list parts;
    for (const auto& p : d.GetPartitions()) parts.append(device_to_dict(*p));
    o["partitions"] = parts;
  }
  return o;
}

// A configured daemon instance: config + manager + SR-IOV lib built once,
// exactly as `start` does, then any number of labeling cycles.
class Session {
 public:
  // A library leaves the host process's CPU placement alone: --cpu-affinity=l3
  // is applied by gfd_main only, never here.  The default, follow, moves
  // only the pool's own worker threads (to the L3 domain of the thread that
  // runs a cycle), as in the daemon.
  Session(const std::vector<std::string>& args, const std::map<std::string, std::string>& env, bool use_env,
          bool amdsmi_library_only) {
    auto ctx = cli::Context::parse(cli::gfd_flags(), args, use_env ? &env : nullptr);
    config_ = cli::load_config(ctx);
    config::disable_resource_renaming(config_);
    config_.amdsmi_library_only = amdsmi_library_only;
    WorkerPool::instance().set_follow(ctx.String("cpu-affinity") == "follow");
    if (!config_.oneshot()) WorkerPool::instance().load_topology();
    // As cli::start does: the first SR-IOV scan runs on a worker while the
    // backend is selected (and, here, while the caller does whatever it does
    // before the first cycle).
    sriov_ = sriov::new_sriov_lib(config_.sysfs_root());
    auto lib = sriov_;
    if (!config_.oneshot())
      prefetch_ = WorkerPool::instance().submit([lib] {
        try {
          lib->Devices();
        } catch (...) {
        }
      });
    manager_ = resource::new_manager(config_);
    timestamp_ = lm::NewTimestampLabeler(config_);
  }
  // A loop-mode session's writes keep the swapped-out feature file for the
  // next write (lm::write_to_file): do not leave it behind.
  ~Session() {
    prefetch_.cancel_or_wait();
    // This session's output only: another live session's kept files stay.
    if (!config_.oneshot()) lm::release_kept_files(config_.output_file());
  }
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;

  py::dict cycle(bool write) {
    cli::CycleResult r;
    {
      py::gil_scoped_release nogil;
      r = cli::label_cycle(*manager_, sriov_, config_, timestamp_, write && true);
    }
    return cycle_to_dict(r);
  }

  // Tight loop in native code: `warmup` untimed cycles, then `steps` timed
  // cycles; returns per-cycle wall time in ns.  With `traced` the timed
  // cycles' phase times are kept for bench_phases(); without, the cycles
  // record no phase (as the daemon's without --trace-timing).
  std::vector<int64_t> bench(int steps, int warmup, bool write, bool traced) {
    std::vector<int64_t> out;
    out.reserve(static_cast<size_t>(steps));
    py::gil_scoped_release nogil;
    bool was_quiet = log::set_quiet(true);
    phases_.clear();
    try {
      for (int i = 0; i < warmup; ++i) cli::label_cycle(*manager_, sriov_, config_, timestamp_, write, traced);
      for (int i = 0; i < steps; ++i) {
        int64_t t0 = trace::now_ns();
        cli::CycleResult r = cli::label_cycle(*manager_, sriov_, config_, timestamp_, write, traced);
        out.push_back(trace::now_ns() - t0);
        for (const auto& [name, ns] : r.phases) phases_[name].push_back(ns);
      }
    } catch (...) {
      log::set_quiet(was_quiet);
      throw;
    }
    log::set_quiet(was_quiet);
    return out;
  }

  // Enumerate through the configured backend (Init/GetDevices/Shutdown).
  py::list devices() {
    py::list l;
    manager_->Init();
    try {
      for (const auto& d : manager_->GetDevices()) l.append(device_to_dict(*d));
    } catch (...) {
      manager_->Shutdown();
      throw;
    }
    manager_->Shutdown();
    return l;
  }

  // Per-phase times (ns) of the last bench()'s timed cycles.
  std::map<std::string, std::vector<int64_t>> bench_phases() const { return phases_; }

  std::string backend() const { return manager_->Name(); }
  std::string config_json() const { return config::to_json(config_); }

  // Run the full daemon loop (run()) in-process: used by loop tests.
  bool run_loop() {
    py::gil_scoped_release nogil;
    return cli::run(*manager_, sriov_, config_, nullptr);
  }

 private:
  config::Config config_;
  WorkerPool::Task prefetch_;
  resource::ManagerPtr manager_;
  std::shared_ptr<sriov::Interface> sriov_;
  lm::LabelerPtr timestamp_;
  std::map<std::string, std::vector<int64_t>> phases_;
};

}  // namespace

PYBIND11_MODULE(_gfd, m) {
  m.doc() = "MI355X GPU feature discovery native core";
  py::register_exception<Error>(m, "GfdError");
  py::register_exception<cli::UsageError>(m, "UsageError");

  m.def("version", [] { return info::version_string(); });
  m.def("set_quiet", &log::set_quiet, py::arg("quiet"));
  // dlopen libamd_smi now (no amdsmi_init).  A host process that will also
  // import PyTorch should call this first: PyTorch bundles its own libdrm,
  // and whichever copy is loaded first is the one amd-smi binds to.
  m.def("load_amdsmi", [] {
    std::string reason;
    bool ok = resource::has_amdsmi(&reason);
    return py::make_tuple(ok, reason);
  });
  // The SR-IOV function sources side by side: "bound" (the functions the
  // listed drivers bind and their VFs, nothing else), "daemon" (the daemon's
  // and a Job's source: those, plus - inside a VM - the bus's AMD functions
  // no listed driver binds) or "bus" (every function on the PCI bus, the
  // reference's approach).
  auto pci_source = [](const std::string& root, const std::string& source) -> std::shared_ptr<sriov::AmdPCI> {
    if (source == "bound") return std::make_shared<sriov::BoundAmdPCI>(root);
    if (source == "daemon")
      return std::make_shared<sriov::BoundAmdPCI>(root, std::make_shared<sriov::SysfsAmdPCI>(root),
                                                  resource::running_in_vm(root));
    if (source == "bus") return std::make_shared<sriov::SysfsAmdPCI>(root);
    throw Error("unknown PCI function source '" + source + "' (expected bound, daemon or bus)");
  };
  m.def(
      "pci_functions",
      [pci_source](const std::string& root, const std::string& source) {
        std::vector<sriov::PCIDevice> devs;
        {
          auto src = pci_source(root, source);
          py::gil_scoped_release nogil;
          devs = src->Devices();
        }
        py::list out;
        for (const auto& d : devs) {
          py::dict o;
          o["address"] = d.address;
          o["device"] = d.device;
          o["class"] = d.class_code;
          o["sriov_totalvfs"] = d.sriov_totalvfs;
          o["sriov_numvfs"] = d.sriov_numvfs;
          o["sriov_vf_device"] = d.sriov_vf_device;
          o["physfn"] = d.physfn;
          o["config_bytes"] = d.config.size();
          out.append(o);
        }
        return out;
      },
      py::arg("root") = "/", py::arg("source") = "bound");
  // The SR-IOV labels (lm::NewSriovLabeler) over one of those sources.
  m.def(
      "sriov_labels",
      [pci_source](const std::string& root, const std::string& source) {
        auto lib = std::make_shared<sriov::Lib>(pci_source(root, source), root);
        py::gil_scoped_release nogil;
        return lm::NewSriovLabeler(lib)->GetLabels();
      },
      py::arg("root") = "/", py::arg("source") = "bound");
  m.def("parse_duration", &parse_duration);
  m.def("format_duration", &format_duration);
  m.def("parse_yaml", [](const std::string& text) { return node_to_py(yaml::parse(text)); });
  m.def("yaml_to_json", [](const std::string& text, int indent) { return yaml::to_json(yaml::parse(text), indent); },
        py::arg("text"), py::arg("indent") = -1);
  m.def("parse_config", [](const std::string& text) { return config::to_json(config::parse_config_text(text)); });
  m.def("new_resource_name", &config::new_resource_name);
  m.def("sanitize_label_value", &lm::sanitize_label_value);

  py::class_<Session>(m, "Session")
      .def(py::init([](const std::vector<std::string>& args, py::object env, bool amdsmi_library_only) {
             if (env.is_none())
               return std::make_unique<Session>(args, std::map<std::string, std::string>{}, false, amdsmi_library_only);
             return std::make_unique<Session>(args, env.cast<std::map<std::string, std::string>>(), true,
                                              amdsmi_library_only);
           }),
           py::arg("args") = std::vector<std::string>{}, py::arg("env") = py::none(),
           py::arg("amdsmi_library_only") = false)
      .def("cycle", &Session::cycle, py::arg("write") = true)
      .def("bench", &Session::bench, py::arg("steps"), py::arg("warmup") = 0, py::arg("write") = true,
           py::arg("traced") = true)
      .def("bench_phases", &Session::bench_phases)
      .def("devices", &Session::devices)
      .def("run_loop", &Session::run_loop)
      .def_property_readonly("backend", &Session::backend)
      .def_property_readonly("config_json", &Session::config_json);

  // Run the CLI entry point in-process (argv[0] is supplied).
  m.def("main", [](const std::vector<std::string>& args) {
    std::vector<std::string> argv{"gpu-feature-discovery"};
    argv.insert(argv.end(), args.begin(), args.end());
    std::vector<char*> cargv;
    for (auto& a : argv) cargv.push_back(a.data());
    cargv.push_back(nullptr);
    py::gil_scoped_release nogil;
    return cli::gfd_main(static_cast<int>(argv.size()), cargv.data());
  });
}
