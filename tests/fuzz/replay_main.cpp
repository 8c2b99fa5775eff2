// Replays fuzz inputs without libFuzzer (any compiler): every file named on
// the command line, or inside a directory named there, is passed once to
// the target's LLVMFuzzerTestOneInput.  The default build links each target
// with this driver so the CPU test-suite re-runs tests/fuzz/corpus (seeds and
// past crashers) on every change; `make fuzz` does the actual fuzzing.
#include <dirent.h>
#include <sys/stat.h>

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size);
extern "C" __attribute__((weak)) int LLVMFuzzerInitialize(int* argc, char*** argv);

namespace {
void collect(const std::string& path, std::vector<std::string>& out) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return;
  if (!S_ISDIR(st.st_mode)) {
    out.push_back(path);
    return;
  }
  DIR* d = opendir(path.c_str());
  if (!d) return;
  while (dirent* e = readdir(d))
    if (e->d_name[0] != '.') collect(path + "/" + e->d_name, out);
  closedir(d);
}
}  // namespace

int main(int argc, char** argv) {
  if (LLVMFuzzerInitialize) LLVMFuzzerInitialize(&argc, &argv);
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i) collect(argv[i], files);
  for (const auto& f : files) {
    std::ifstream in(f, std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    std::string data = ss.str();
    LLVMFuzzerTestOneInput(reinterpret_cast<const uint8_t*>(data.data()), data.size());
  }
  std::printf("replayed %zu inputs\n", files.size());
  return files.empty() ? 1 : 0;
}
