#include "util/dynlib.h"

#include <dlfcn.h>

namespace gfd {

DynLib::~DynLib() { close(); }

bool DynLib::open(const std::vector<std::string>& candidates) {
  close();
  for (const auto& c : candidates) {
    void* h = ::dlopen(c.c_str(), RTLD_LAZY | RTLD_LOCAL);
    if (h) {
      handle_ = h;
      path_ = c;
      error_.clear();
      return true;
    }
    const char* e = ::dlerror();
    error_ = e ? e : ("unable to load " + c);
  }
  return false;
}

void DynLib::close() {
  if (handle_) {
    ::dlclose(handle_);
    handle_ = nullptr;
  }
}

void* DynLib::symbol(const char* name) const {
  if (!handle_) return nullptr;
  ::dlerror();
  return ::dlsym(handle_, name);
}

}  // namespace gfd
