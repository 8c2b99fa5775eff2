// RAII wrapper around dlopen/dlsym/dlclose.
//
// Reference analogue: vendored go-nvml `pkg/dl` (dl.go:22-82), which the
// reference drives far too often — go-nvlib re-dlopens libnvidia-ml on every
// IsMigCapable/IsMigEnabled call (nvlib/device/device.go:55-88, :327-338).
// Here a library is opened once per process and its symbols are resolved
// once into a function table (AmdSmiLib in resource/amdsmi.cpp).
#pragma once

#include <string>
#include <vector>

namespace gfd {

class DynLib {
 public:
  DynLib() = default;
  ~DynLib();
  DynLib(const DynLib&) = delete;
  DynLib& operator=(const DynLib&) = delete;

  // Try each candidate path in order (RTLD_LAZY | RTLD_LOCAL).  Returns false
  // and records the last dlerror() if none loads.
  bool open(const std::vector<std::string>& candidates);
  void close();

  void* symbol(const char* name) const;
  template <typename Fn>
  bool bind(const char* name, Fn*& out) const {
    out = reinterpret_cast<Fn*>(symbol(name));
    return out != nullptr;
  }

  const std::string& path() const { return path_; }
  const std::string& last_error() const { return error_; }

 private:
  void* handle_ = nullptr;
  std::string path_;
  std::string error_;
};

}  // namespace gfd
