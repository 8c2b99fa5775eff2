// libFuzzer target: the config-file reader (YAML/JSON -> v1 Config).
//
// A config file comes from a ConfigMap or a host path; whatever its bytes,
// the reader must either accept it or throw gfd::Error - never crash, hang,
// read out of bounds or leak another exception type.  Accepted documents
// must also survive the JSON round trip the daemon logs at start-up
// (config::to_json): its output must parse again, and one more round trip
// must not change it (the first may normalise: a YAML float -0.0 is written
// "-0" like Go's encoder, which then reads back as the integer 0).
//
//   make fuzz   (builds build-fuzz/, runs every target over tests/fuzz/corpus)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "config/config.h"
#include "config/yaml.h"
#include "util/error.h"

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  std::string text(reinterpret_cast<const char*>(data), size);
  try {
    gfd::yaml::Node n = gfd::yaml::parse(text);
    std::string json = gfd::yaml::to_json(n);
    std::string again = gfd::yaml::to_json(gfd::yaml::parse(json));
    std::string third = gfd::yaml::to_json(gfd::yaml::parse(again));
    if (third != again) {
      std::fprintf(stderr, "JSON round trip does not settle:\n%s\n%s\n%s\n", json.c_str(), again.c_str(),
                   third.c_str());
      std::abort();
    }
  } catch (const gfd::Error&) {
  }
  try {
    gfd::config::Config c = gfd::config::parse_config_text(text);
    std::string json = gfd::config::to_json(c);
    (void)gfd::config::parse_config_text(json);
  } catch (const gfd::Error&) {
  }
  return 0;
}
