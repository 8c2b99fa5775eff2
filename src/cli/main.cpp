// gpu-feature-discovery: MI355X-native node labeler for Kubernetes/NFD.
// Reference entry point: cmd/gpu-feature-discovery/main.go:22-90.
#include "cli/daemon.h"

int main(int argc, char** argv) { return gfd::cli::gfd_main(argc, argv); }
