// gpu-feature-discovery: MI355X-native node labeler for Kubernetes/NFD.
// Reference entry point: cmd/gpu-feature-discovery/main.go:22-90.
#include <unistd.h>

#include <cstdio>

#include "cli/daemon.h"
#include "resource/managers.h"

int main(int argc, char** argv) {
  int rc = gfd::cli::gfd_main(argc, argv);
  if (gfd::resource::warmer_left_running()) {
    // A background amd-smi initialisation is still running (its manager
    // gave up waiting for it at teardown): running static destructors -
    // libamd_smi's among them - under it could crash the exit.  Everything
    // of ours is already flushed or removed; leave without them.
    std::fflush(nullptr);
    _exit(rc);
  }
  return rc;
}
