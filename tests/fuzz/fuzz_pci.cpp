// libFuzzer target: PCI configuration-space walkers (SR-IOV discovery).
//
// The config space is read from sysfs (`config`, 64 bytes unprivileged, up
// to 4 KiB privileged) and is device-controlled data: the capability and
// extended-capability walks must stop on loops, broken chains and pointers
// past the end, whatever the bytes - or throw gfd::Error for a truncated
// space (the reference's "entire PCI configuration is not read" case).
#include <cstdint>
#include <string>

#include "sriov/pci.h"
#include "util/error.h"

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  const int caps[] = {0x01, 0x05, 0x09, 0x10, 0x11, 0xff};
  const int ext_caps[] = {0x0001, 0x000B, 0x000E, 0x0010};
  gfd::sriov::PCIDevice d;
  d.address = "0000:00:00.0";
  d.config.assign(reinterpret_cast<const char*>(data), size > 4096 ? 4096 : size);
  for (int id : caps) {
    try {
      auto cap = d.GetCapability(id);
      if (cap && cap->size() > d.config.size()) __builtin_trap();
    } catch (const gfd::Error&) {
    }
  }
  for (int id : ext_caps) {
    try {
      auto cap = d.GetExtendedCapability(id, 64);
      if (cap && cap->size() > 64) __builtin_trap();
    } catch (const gfd::Error&) {
    }
  }
  return 0;
}
