#include "resource/amdsmi_lib.h"

#include <cstdlib>
#include <vector>

#include "resource/amdsmi.h"
#include "util/fs.h"
#include "util/log.h"

namespace gfd::resource {

namespace {
// amdsmi_get_lib_version's struct, with room to spare: the library being
// probed may be of another major version, whose struct is laid out
// differently (older ones started with a `year` field).
union VersionBuf {
  amdsmi_version_t v;
  unsigned char slack[128];
  VersionBuf() : slack{} {}
};
}  // namespace

bool AmdSmiLib::load(std::string* err) {
  const std::string versioned = "libamd_smi.so." + std::to_string(AMDSMI_LIB_VERSION_MAJOR);
  std::vector<std::string> candidates;
  if (const char* p = std::getenv("GFD_AMDSMI_LIBRARY"); p && *p) candidates.push_back(p);
  if (const char* rp = std::getenv("ROCM_PATH"); rp && *rp) {
    candidates.push_back(fs::join(rp, "lib/" + versioned));
    candidates.push_back(fs::join(rp, "lib/libamd_smi.so"));
  }
  candidates.push_back("/opt/rocm/lib/" + versioned);
  candidates.push_back("/opt/rocm/lib/libamd_smi.so");
  candidates.push_back(versioned);
  candidates.push_back("libamd_smi.so");
  // The structs the backend passes to the library are laid out by the
  // amdsmi.h it was compiled against; a library of another major version
  // (an unversioned libamd_smi.so from a different ROCm) may lay them out
  // differently, so it is skipped in favour of the next candidate.
  std::string mismatch;
  bool opened = false;
  for (const auto& c : candidates) {
    if (!lib_.open({c})) continue;
    amdsmi_status_t (*lib_version)(amdsmi_version_t*) = nullptr;
    VersionBuf buf;
    const amdsmi_version_t& v = buf.v;
    if (lib_.bind("amdsmi_get_lib_version", lib_version) && lib_version(&buf.v) == AMDSMI_STATUS_SUCCESS &&
        v.major != AMDSMI_LIB_VERSION_MAJOR) {
      mismatch = c + " is amd-smi " + std::to_string(v.major) + "." + std::to_string(v.minor) +
                 ", this build needs major version " + std::to_string(AMDSMI_LIB_VERSION_MAJOR);
      log::printf("Skipping %s", mismatch.c_str());
      lib_.close();
      continue;
    }
    opened = true;
    break;
  }
  if (!opened) {
    *err = mismatch.empty() ? lib_.last_error() : mismatch;
    return false;
  }
  bool ok = true;
  auto need = [&](const char* sym, auto& fn) {
    if (!lib_.bind(sym, fn)) {
      ok = false;
      *err = std::string("symbol ") + sym + " not found in " + lib_.path();
    }
  };
  need("amdsmi_init", init);
  need("amdsmi_shut_down", shut_down);
  need("amdsmi_get_socket_handles", get_socket_handles);
  need("amdsmi_get_processor_handles", get_processor_handles);
  need("amdsmi_get_processor_type", get_processor_type);
  need("amdsmi_get_gpu_asic_info", get_gpu_asic_info);
  need("amdsmi_get_gpu_device_bdf", get_gpu_device_bdf);
  need("amdsmi_get_gpu_memory_total", get_gpu_memory_total);
  need("amdsmi_get_gpu_driver_info", get_gpu_driver_info);
  // Optional: newer partition / topology queries degrade gracefully.
  lib_.bind("amdsmi_get_gpu_device_uuid", get_gpu_device_uuid);
  lib_.bind("amdsmi_get_gpu_kfd_info", get_gpu_kfd_info);
  lib_.bind("amdsmi_get_gpu_compute_partition", get_gpu_compute_partition);
  lib_.bind("amdsmi_get_gpu_memory_partition", get_gpu_memory_partition);
  lib_.bind("amdsmi_get_gpu_memory_partition_config", get_gpu_memory_partition_config);
  lib_.bind("amdsmi_get_gpu_accelerator_partition_profile_config", get_gpu_accelerator_partition_profile_config);
  lib_.bind("amdsmi_get_gpu_xgmi_link_status", get_gpu_xgmi_link_status);
  lib_.bind("amdsmi_get_gpu_virtualization_mode", get_gpu_virtualization_mode);
  lib_.bind("amdsmi_get_gpu_xcd_counter", get_gpu_xcd_counter);
  lib_.bind("amdsmi_get_gpu_board_info", get_gpu_board_info);
  lib_.bind("amdsmi_get_lib_version", get_lib_version);
  lib_.bind("amdsmi_status_code_to_string", status_code_to_string);
  return ok;
}

bool has_amdsmi(std::string* reason) {
  std::string err;
  AmdSmiLib* l = AmdSmiLib::get(&err);
  if (!l) {
    if (reason) *reason = "could not load libamd_smi: " + err;
    return false;
  }
  if (reason) {
    *reason = "found " + l->path();
    VersionBuf buf;
    const amdsmi_version_t& v = buf.v;
    if (l->get_lib_version && l->get_lib_version(&buf.v) == AMDSMI_STATUS_SUCCESS)
      *reason += " (amd-smi library " + std::to_string(v.major) + "." + std::to_string(v.minor) + "." +
                 std::to_string(v.release) + ")";
  }
  return true;
}

}  // namespace gfd::resource
