// Filesystem helpers built directly on POSIX calls.  The sysfs backend and
// the PCI walker read hundreds of tiny files per cycle, so these avoid
// iostreams and do a single open/read/close per file.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <optional>
#include <string>
#include <unordered_map>
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

bool exists(const std::string& path);
bool is_dir(const std::string& path);
// Directory entries (excluding . and ..), sorted by name.  Empty on error;
// `err` (optional) receives errno.
std::vector<std::string> list_dir(const std::string& path, int* err = nullptr);
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
  // Forget the last listing: the next read reports a change.
  void reset() {
    raw_.clear();
    prev_.clear();
  }

 private:
  int read_raw();
  std::string path_;
  int fd_ = -1;
  std::string raw_, prev_;
};

// sysfs attribute reads through descriptors kept open across calls.
//
// Every read is `pread(fd, ..., 0)`: kernfs regenerates an attribute's text
// (calls the driver's show()) for each read at offset 0, so the value is as
// live as with open/read/close - but the path walk, open and close, which
// are ~85% of a small attribute read and contend across cores, are paid
// once.  Measured on an 8xMI355X host: six amdgpu attributes of one GPU in
// 2.9 us instead of 20.7 us (profiles/multi_gpu_read_probe.txt).
//
// Only files on sysfs are kept open (checked with fstatfs): a kernfs file
// that is removed makes reads on old descriptors fail with ENODEV, which
// drops the descriptor and opens the path again.  Files elsewhere (regular
// files, synthetic test trees) could be replaced under an open descriptor,
// so they are opened for every read.  Thread-safe.
class AttrReader {
 public:
  AttrReader() = default;
  ~AttrReader();
  AttrReader(const AttrReader&) = delete;
  AttrReader& operator=(const AttrReader&) = delete;
  ReadResult read(const std::string& path, size_t max_bytes = 64 * 1024);
  std::optional<std::string> read_trimmed(const std::string& path);
  // A regular file that may be replaced (e.g. a package's version file):
  // kept open too, but a stat() of the path confirms it is still the same
  // file (device + inode) before every pread - cheaper than open/read/close,
  // and a replaced or removed file is seen at once.
  ReadResult read_checked(const std::string& path, size_t max_bytes = 64 * 1024);
  std::optional<std::string> read_checked_trimmed(const std::string& path);
  // Close every kept descriptor (e.g. when the topology generation changed
  // and some paths will never be read again).
  void clear();
  size_t open_count() const;
  // Keep descriptors of files on any filesystem (tests only).
  void keep_all_for_testing(bool on) { keep_all_ = on; }

 private:
  // Shared so that a descriptor dropped by one thread stays open (and its
  // number unused) until every thread still reading it is done.
  struct Fd {
    explicit Fd(int f) : fd(f) {}
    Fd(const Fd&) = delete;
    Fd& operator=(const Fd&) = delete;
    ~Fd();
    int fd;
  };
  // Lookups (every read) share the lock; only opening and dropping a
  // descriptor take it exclusively, so per-GPU lanes do not queue on it.
  mutable std::shared_mutex mu_;
  std::unordered_map<std::string, std::shared_ptr<const Fd>> fds_;
  struct Checked {
    std::shared_ptr<const Fd> fd;
    uint64_t dev = 0, ino = 0;
  };
  std::unordered_map<std::string, Checked> checked_;
  bool keep_all_ = false;
};

// The process-wide reader used for per-cycle attribute reads.
AttrReader& attrs();

// A DMI identification attribute (e.g. the machine type's product_name).
// The kernel copies these strings from the firmware's SMBIOS tables once at
// boot (dmi_scan) and every read of sysfs devices/virtual/dmi/id/<attr>
// returns them unchanged until the next boot, so the first successful read
// of such a file is kept for the life of the process.  Any other file - a
// synthetic tree, a regular file mounted over the default path - is read
// through attrs() every time.
ReadResult read_dmi(const std::string& path);

// readlink(2); empty on failure.
std::string read_link(const std::string& path);

// A directory opened once (O_PATH) whose entries are then read relative to
// it: no path walk per attribute - a PCI function's sysfs path goes through
// a symlink and a dozen components, which is most of a cold attribute read.
class Dir {
 public:
  explicit Dir(const std::string& path);
  ~Dir();
  Dir(const Dir&) = delete;
  Dir& operator=(const Dir&) = delete;
  int err() const { return err_; }  // 0 if the directory was opened
  // A sysfs attribute in one read(2): kernfs hands over the whole value (at
  // most a page; a binary attribute up to `max_bytes`) in the first read,
  // so no second read for end-of-file.
  ReadResult read_attr(const char* name, size_t max_bytes = 4096) const;
  std::optional<std::string> read_trimmed(const char* name) const;
  std::string read_link(const char* name) const;
  // Whether `name` exists in the directory (not following a final symlink):
  // 0 if it does, else the errno (ENOENT: it does not).
  int lookup(const char* name) const;

 private:
  int fd_ = -1;
  int err_ = 0;
};
// Resolve `rel` under `root` the way a process chrooted at `root` would:
// component by component, following symlinks, with absolute link targets
// re-rooted under `root` (a host's /opt/rocm -> /opt/rocm-7.2.0 seen through
// a mount of the host's /opt at /host/opt).  ".." never leaves `root`.
// Returns the resolved path under `root`, or "" if a component does not
// exist or links nest deeper than 40.  `dirs` (optional) receives every
// directory a component was looked up in, symlink targets' included: the
// directories whose entries decide the answer.
std::string resolve_in_root(const std::string& root, const std::string& rel, std::vector<std::string>* dirs = nullptr);

// One small attribute read every cycle (the KFD topology generation, the
// kernel's uevent counter): on sysfs through a descriptor kept open, read
// with one pread into a stack buffer - no path lookup, no allocation; off
// sysfs (synthetic trees, whose files tests replace) opened for each read,
// as AttrReader does.  Not thread-safe: one per reader.
class KeptAttr {
 public:
  explicit KeptAttr(std::string path) : path_(std::move(path)) {}
  ~KeptAttr();
  KeptAttr(const KeptAttr&) = delete;
  KeptAttr& operator=(const KeptAttr&) = delete;
  // The trimmed contents (up to 255 bytes) into *out; false if unreadable.
  bool read(std::string* out);
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  int fd_ = -1;  // kept: a sysfs attribute
};

// Whether the file system of `fd` is local, so that this kernel sees every
// change to it (ext4, xfs, btrfs, tmpfs, overlayfs): a lease or an inotify
// watch there misses nothing another node did.
bool is_local_fs(int fd);

// Whether the entries of a set of directories changed: an inotify watch on
// each (an entry created, removed or renamed; the directory itself removed
// or moved).  A lookup's answer - a symlink chain resolved to a file, or the
// file not found - stands while its directories are unchanged.
//
// All DirWatches share one inotify instance, created on the first arm() and
// kept for the process: closing an instance waits for an SRCU grace period
// in the kernel (40-70 ms measured on the MI355X pool, at exit of a process
// that had one), so none is closed while the process runs; a watch no set
// needs any more is removed (inotify_rm_watch does not wait).  A oneshot
// Job never arms one (resource::VersionSources::keep).
class DirWatch {
 public:
  DirWatch() = default;
  ~DirWatch();
  DirWatch(const DirWatch&) = delete;
  DirWatch& operator=(const DirWatch&) = delete;
  // Watch `dirs` from now on (the previous set is dropped).  False, and
  // nothing watched, when one of them cannot be watched or is not on a
  // local file system (is_local_fs): then unchanged() stays false.
  bool arm(const std::vector<std::string>& dirs);
  // True while nothing changed in the armed directories since arm(): one
  // non-blocking read of the shared inotify queue.  The first change
  // disarms.
  bool unchanged();

 private:
  std::vector<int> wds_;
  bool armed_ = false;
  bool dirty_ = false;
  friend struct DirWatchRegistry;
};

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

// The whole of an open file, from offset 0, up to `max_bytes` (pread: no
// file position involved).  0 or an errno.
// `short_read_is_all`: the file is a sysfs attribute or a regular file, so a
// first read shorter than a page is the whole of it (no second read).
int pread_all(int fd, size_t max_bytes, std::string* out, bool short_read_is_all = false);

std::string errno_str(int err);

}  // namespace gfd::fs
