// The process-wide binding to libamd_smi: dlopen'ed once - the first
// candidate whose major version matches the amdsmi.h this build was
// compiled against - with every entry point bound once; optional entry
// points stay null and the backend degrades without them.  Reference
// analogue: go-nvml's Init + updateVersionedSymbols
// (vendor/github.com/NVIDIA/go-nvml/pkg/nvml/init.go:25-218), which the
// reference pays on every labeling cycle.
#pragma once

#include <amd_smi/amdsmi.h>

#include <atomic>
#include <mutex>
#include <string>

#include "util/dynlib.h"

namespace gfd::resource {

class AmdSmiLib {
 public:
  static AmdSmiLib* get(std::string* err) {
    static std::once_flag once;
    static AmdSmiLib* inst = nullptr;
    static std::string load_error;
    std::call_once(once, [] {
      auto* l = new AmdSmiLib();
      if (l->load(&load_error)) {
        inst = l;
      } else {
        delete l;
      }
    });
    if (!inst && err) *err = load_error;
    return inst;
  }

  std::string status_str(amdsmi_status_t st) const {
    const char* s = nullptr;
    if (status_code_to_string && status_code_to_string(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
    return "amdsmi status " + std::to_string(static_cast<int>(st));
  }

  const std::string& path() const { return lib_.path(); }

  // Process-wide init state (amdsmi_init is global).
  std::mutex mu;
  int users = 0;
  // Set once amd-smi has refused asic_info with NOT_SUPPORTED (see
  // identity_from_kfd); reset by every amdsmi_init, so a session asks once.
  std::atomic<bool> asic_info_unsupported{false};

#define GFD_AMDSMI_FN(name, ...) amdsmi_status_t (*name)(__VA_ARGS__) = nullptr
  GFD_AMDSMI_FN(init, uint64_t);
  GFD_AMDSMI_FN(shut_down, void);
  GFD_AMDSMI_FN(get_socket_handles, uint32_t*, amdsmi_socket_handle*);
  GFD_AMDSMI_FN(get_processor_handles, amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
  GFD_AMDSMI_FN(get_processor_type, amdsmi_processor_handle, processor_type_t*);
  GFD_AMDSMI_FN(get_gpu_asic_info, amdsmi_processor_handle, amdsmi_asic_info_t*);
  GFD_AMDSMI_FN(get_gpu_device_bdf, amdsmi_processor_handle, amdsmi_bdf_t*);
  GFD_AMDSMI_FN(get_gpu_device_uuid, amdsmi_processor_handle, unsigned int*, char*);
  GFD_AMDSMI_FN(get_gpu_kfd_info, amdsmi_processor_handle, amdsmi_kfd_info_t*);
  GFD_AMDSMI_FN(get_gpu_memory_total, amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*);
  GFD_AMDSMI_FN(get_gpu_compute_partition, amdsmi_processor_handle, char*, uint32_t);
  GFD_AMDSMI_FN(get_gpu_memory_partition, amdsmi_processor_handle, char*, uint32_t);
  GFD_AMDSMI_FN(get_gpu_memory_partition_config, amdsmi_processor_handle, amdsmi_memory_partition_config_t*);
  GFD_AMDSMI_FN(get_gpu_accelerator_partition_profile_config, amdsmi_processor_handle,
                amdsmi_accelerator_partition_profile_config_t*);
  GFD_AMDSMI_FN(get_gpu_xgmi_link_status, amdsmi_processor_handle, amdsmi_xgmi_link_status_t*);
  GFD_AMDSMI_FN(get_gpu_virtualization_mode, amdsmi_processor_handle, amdsmi_virtualization_mode_t*);
  GFD_AMDSMI_FN(get_gpu_xcd_counter, amdsmi_processor_handle, uint16_t*);
  GFD_AMDSMI_FN(get_gpu_driver_info, amdsmi_processor_handle, amdsmi_driver_info_t*);
  GFD_AMDSMI_FN(get_gpu_board_info, amdsmi_processor_handle, amdsmi_board_info_t*);
  GFD_AMDSMI_FN(get_lib_version, amdsmi_version_t*);
#undef GFD_AMDSMI_FN
  amdsmi_status_t (*status_code_to_string)(amdsmi_status_t, const char**) = nullptr;

 private:
  bool load(std::string* err);

  DynLib lib_;
};

}  // namespace gfd::resource
