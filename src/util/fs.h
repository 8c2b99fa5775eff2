// Filesystem helpers built directly on POSIX calls.  The sysfs backend and
// the PCI walker read hundreds of tiny files per cycle, so these avoid
// iostreams and do a single open/read/close per file.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

namespace gfd::fs {

// Result of reading a small file.  `err` is the errno on failure (0 on success).
struct ReadResult {
  std::string data;
  int err = 0;
  bool ok() const { return err == 0; }
};

ReadResult read_file(const std::string& path, size_t max_bytes = 1 << 20);
// read_file + trim; nullopt on any error.
std::optional<std::string> read_trimmed(const std::string& path);
// Throws gfd::Error("<what> '<path>': <strerror>") on failure.
std::string read_file_or_throw(const std::string& path);

bool exists(const std::string& path);
bool is_dir(const std::string& path);
// Directory entries (excluding . and ..), sorted by name.  Empty on error;
// `err` (optional) receives errno.
std::vector<std::string> list_dir(const std::string& path, int* err = nullptr);
// Like list_dir but also returns each entry's inode number (d_ino), which
// changes when a sysfs object is removed and re-created (hot-plug).
std::vector<std::pair<std::string, uint64_t>> list_dir_ino(const std::string& path, int* err = nullptr);
// A directory listing re-read every call through a descriptor kept open
// across calls: one lseek + getdents64 pass, no path walk, no per-entry
// work when nothing changed.  Whether anything changed is decided on the raw
// getdents64 records (name, inode, position cookie), which sysfs (kernfs)
// produces identically for an unchanged directory.  The descriptor is
// reopened when the directory was removed (st_nlink 0) or `path` differs.
class DirListing {
 public:
  DirListing() = default;
  ~DirListing();
  DirListing(const DirListing&) = delete;
  DirListing& operator=(const DirListing&) = delete;
  // Re-reads `path`.  Returns 0 or errno; `changed` is true when the listing
  // differs from the previous successful read (always on the first).
  int read(const std::string& path, bool* changed);
  // Entries of the last read, without . and .., sorted by name.
  std::vector<std::pair<std::string, uint64_t>> entries() const;

 private:
  int read_raw();
  std::string path_;
  int fd_ = -1;
  std::string raw_, prev_;
};

// readlink(2); empty on failure.
std::string read_link(const std::string& path);
// Final path component of realpath(path), or empty.
std::string real_basename(const std::string& path);

std::string join(const std::string& a, const std::string& b);
std::string dirname(const std::string& path);
std::string basename(const std::string& path);
// Make `path` absolute against the current working directory (no symlink
// resolution, like Go's filepath.Abs).
std::string absolute(const std::string& path);

// mkdir -p; throws on failure.
void mkdir_all(const std::string& path, unsigned mode = 0777);
// rm -rf; returns 0 or errno.  Missing paths are not an error.
int remove_all(const std::string& path);

std::string errno_str(int err);

}  // namespace gfd::fs
