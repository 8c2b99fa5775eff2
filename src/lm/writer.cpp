// The feature-file writer (lm/labels.h: write_to_file and friends): atomic
// replacement through gfd-tmp/; in loop mode the swapped-out feature file is
// kept and rewritten by the next write.  The labelers are in labels.cpp.
#include "lm/labels.h"

#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <string>
#include <utility>

#include <cerrno>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "util/error.h"
#include "util/fs.h"
#include "util/trace.h"

namespace gfd::lm {

namespace {

bool write_all(int fd, const std::string& data) {
  size_t off = 0;
  while (off < data.size()) {
    ssize_t n = ::write(fd, data.data() + off, data.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += static_cast<size_t>(n);
  }
  return true;
}

// The process umask, from /proc/self/status (reading it with umask(2) would
// briefly change it for every thread); 022 if unavailable.
mode_t process_umask() {
  static const mode_t mask = [] {
    auto r = fs::read_file("/proc/self/status", 8192);
    auto pos = r.ok() ? r.data.find("\nUmask:") : std::string::npos;
    if (pos == std::string::npos) return static_cast<mode_t>(022);
    return static_cast<mode_t>(std::strtoul(r.data.c_str() + pos + 7, nullptr, 8));
  }();
  return mask;
}

// Prefix of this daemon's temporary files in gfd-tmp/.  NVIDIA's GFD, which
// may run on the same node (GPUs of both vendors), keeps its own files there
// as gfd-XXXXXX (labels.go:90): everything here that removes temporary files
// removes only names with this prefix, never the other daemon's in-flight
// file.
constexpr const char kTempPrefix[] = "gfd-amd-";

// mkstemp with the final permission bits: "<dir>/gfd-amd-XXXXXX" with a
// random suffix, O_EXCL.  Returns the fd (name in *name) or -1 with errno set.
int create_temp(const std::string& dir, unsigned perm, std::string* name) {
  static const char kChars[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
  static thread_local uint64_t state = static_cast<uint64_t>(::getpid()) * 0x9E3779B97F4A7C15ULL ^
                                       static_cast<uint64_t>(reinterpret_cast<uintptr_t>(&state));
  for (int attempt = 0; attempt < 100; ++attempt) {
    *name = dir + "/" + kTempPrefix;
    for (int i = 0; i < 6; ++i) {
      state ^= state << 13;
      state ^= state >> 7;
      state ^= state << 17;
      name->push_back(kChars[state % (sizeof(kChars) - 1)]);
    }
    int fd = ::open(name->c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, perm);
    if (fd >= 0 || errno != EEXIST) return fd;
  }
  errno = EEXIST;
  return -1;
}

// Whether to fallocate the temporary file before writing it.
//
// ext4 (default `auto_da_alloc`) treats a rename that replaces an existing
// file as "replace-via-rename" and, if the new file still has delayed-
// allocation blocks, flushes it inside rename(2): measured 52-62 ms per
// rename on an ext4 root (profiles/write_ext4_ab.txt) - 1000x the rest of a
// cycle, and the NFD features.d hostPath is usually on the node's root fs.
// A file whose blocks were allocated up front has nothing delayed, so the
// rename is a plain directory update (0.03 ms).  Overlayfs is included
// because its upper layer is commonly ext4 (the call passes through).
// Elsewhere (tmpfs, xfs, ...) the extra allocation would be pure cost.
bool wants_prealloc(int fd) {
  struct statfs sf;
  if (::fstatfs(fd, &sf) != 0) return false;
  constexpr unsigned long kExt4 = 0xEF53, kOverlay = 0x794c7630;
  return static_cast<unsigned long>(sf.f_type) == kExt4 || static_cast<unsigned long>(sf.f_type) == kOverlay;
}

}  // namespace

bool reuse_is_safe(int fd) { return fs::is_local_fs(fd); }

namespace {

// Removes this daemon's files from gfd-tmp/ (kTempPrefix) and any
// subdirectory (only this daemon's round-2 layout made them; NVIDIA's GFD
// keeps plain files there), then the directory if nothing else is left in
// it.  Something that is not a directory where gfd-tmp/ belongs blocks
// every write, and is removed.  Returns 0 or an errno.
int remove_own_temps(const std::string& tmp_dir) {
  int err = 0;
  auto names = fs::list_dir(tmp_dir, &err);
  if (err == ENOENT) return 0;
  if (err == ENOTDIR) return ::unlink(tmp_dir.c_str()) == 0 || errno == ENOENT ? 0 : errno;
  if (err != 0) return err;
  int first = 0;
  for (const auto& n : names) {
    std::string p = tmp_dir + "/" + n;
    int e = 0;
    if (n.rfind(kTempPrefix, 0) == 0) {
      e = ::unlink(p.c_str()) == 0 || errno == ENOENT ? 0 : errno;
      if (e == EISDIR || e == EPERM) e = fs::remove_all(p);
    } else if (fs::is_dir(p)) {
      e = fs::remove_all(p);
    }
    if (e && !first) first = e;
  }
  if (::rmdir(tmp_dir.c_str()) != 0 && errno != ENOTEMPTY && errno != EEXIST && errno != ENOENT && !first) first = errno;
  return first;
}

}  // namespace

namespace {

// The reference's temporary file (labels.go:68-114): a new file in tmp_dir
// (its name in *tmpl) holding `contents`; the rename is the caller's.  With
// `kept` the descriptor is left open and returned there, else closed.
void create_and_write(const std::string& tmp_dir, const std::string& contents, unsigned perm, std::string* tmpl,
                      int* kept) {
  int64_t t0 = trace::stamp();
  // The temporary directory normally exists from the previous cycle: try the
  // create first and make the directory only when it is missing.
  int fd = create_temp(tmp_dir, perm, tmpl);
  if (fd < 0 && errno == ENOENT) {
    try {
      fs::mkdir_all(tmp_dir);
    } catch (const std::exception& e) {
      throw Error(std::string("failed to create temporary directory: ") + e.what());
    }
    fd = create_temp(tmp_dir, perm, tmpl);
  }
  // Failures remove gfd-tmp/ like the reference (labels.go:81-85).
  if (fd < 0) {
    int e = errno;
    remove_own_temps(tmp_dir);
    throw Error("fail to create temporary output file: " + fs::errno_str(e));
  }
  auto fail = [&](const std::string& msg) {
    ::close(fd);
    ::unlink(tmpl->c_str());
    remove_own_temps(tmp_dir);
    throw Error(msg);
  };
  int64_t t1 = trace::stamp();
  trace::record("write.create", t1 - t0);
  // Best effort: a file system without fallocate(2) just takes the write.
  if (wants_prealloc(fd)) (void)::fallocate(fd, 0, 0, static_cast<off_t>(contents.size()));
  if (!write_all(fd, contents)) fail("error writing temporary file '" + *tmpl + "': " + fs::errno_str(errno));
  // Created with `perm` already; chmod only what the umask took away.
  if ((perm & process_umask()) != 0 && ::fchmod(fd, perm) != 0)
    fail("error setting permissions on '" + *tmpl + "': " + fs::errno_str(errno));
  if (kept) {
    *kept = fd;
  } else if (::close(fd) != 0) {
    int e = errno;
    ::unlink(tmpl->c_str());
    remove_own_temps(tmp_dir);
    throw Error("error writing temporary file '" + *tmpl + "': " + fs::errno_str(e));
  }
  trace::record_since("write.data", t1);
}

std::string temp_dir_of(const std::string& path) { return fs::join(fs::dirname(fs::absolute(path)), "gfd-tmp"); }

// Loop mode: the two files of one feature file.  `live` is the file now at
// the output path (written by the last write); `spare` the one before it,
// which that write swapped out to a name in gfd-tmp/ - the file the next
// write rewrites.  Both stay open (writable).
//
// Why, measured on the pool's overlayfs: creating a file took 17-64 us on a
// fresh box (2 us on tmpfs) and, done ahead on a worker as round 4 did,
// held gfd-tmp/'s directory lock against the cycle's own rename, which then
// waited for it (rename 0.049 ms against 0.004 ms alone,
// profiles/fs_probe_r5.txt); on ext4 (the usual file system of NFD's
// features.d hostPath) a rename over the old file frees its inode inside
// rename(2), 0.34-0.58 ms cold vs 0.03 ms for an exchange
// (profiles/rename_exchange_ab.txt), and unlinking it later costs the same
// eviction.  Rewriting the swapped-out file needs none of these: a lease
// check, a write into its existing blocks, the exchange.
struct File {
  std::string name;  // spare only: its name in gfd-tmp/
  int fd = -1;
  dev_t dev = 0;
  ino_t ino = 0;
  bool local = false;  // on a file system where a lease sees every reader (reuse_is_safe)
};
struct Slot {
  File live, spare;
};

std::mutex g_mu;
std::map<std::string, Slot>& slots() {
  static auto* m = new std::map<std::string, Slot>();  // never destroyed: read at exit
  return *m;
}

void close_file(File& f, bool unlink_name) {
  if (f.fd >= 0) ::close(f.fd);
  if (unlink_name && !f.name.empty()) {
    // Only if the name is still this file's.
    struct stat st;
    if (::lstat(f.name.c_str(), &st) == 0 && st.st_dev == f.dev && st.st_ino == f.ino) ::unlink(f.name.c_str());
  }
  f = File{};
}

// Rewrites the spare with `contents` if nobody else has it open; false (the
// spare dropped) if it cannot be used.
bool rewrite_spare(File& spare, const std::string& contents) {
  if (spare.fd < 0) return false;
  int64_t t0 = trace::stamp();
  struct stat st;
  // On a local file system (a network one's readers elsewhere hold no lease
  // this kernel could see), still ours under its name (gfd-tmp/ was not
  // emptied behind our back)...
  bool usable = spare.local && ::lstat(spare.name.c_str(), &st) == 0 && st.st_dev == spare.dev &&
                st.st_ino == spare.ino;
  int64_t t1 = trace::stamp();
  // ...and no reader that opened it while it was the feature file still has
  // it open: a write lease is granted only to the sole opener.  EAGAIN: a
  // reader; EINVAL/EACCES: no leases here (a file system without them,
  // leases disabled).  Then the spare is left to its reader (unlinked) and
  // this write creates a new file.
  if (usable && ::fcntl(spare.fd, F_SETLEASE, F_WRLCK) != 0) usable = false;
  int64_t t2 = trace::stamp();
  if (!usable) {
    close_file(spare, true);
    return false;
  }
  bool ok = ::pwrite(spare.fd, contents.data(), contents.size(), 0) == static_cast<ssize_t>(contents.size());
  // Shorter than before: cut the rest (same length, the steady case: no
  // size change at all).
  if (ok && static_cast<size_t>(st.st_size) > contents.size())
    ok = ::ftruncate(spare.fd, static_cast<off_t>(contents.size())) == 0;
  int64_t t3 = trace::stamp();
  // Released before the exchange: an open of the feature file must not wait
  // for a lease break.
  (void)::fcntl(spare.fd, F_SETLEASE, F_UNLCK);
  if (!ok) {
    close_file(spare, true);
    return false;
  }
  int64_t t4 = trace::stamp();
  // The rewrite's parts (a cycle after an idle second spends most of its
  // write here and in the exchange, write.rename).
  trace::record("write.check", t1 - t0);
  trace::record("write.lease", t2 - t1);
  trace::record("write.pwrite", t3 - t2);
  trace::record("write.unlease", t4 - t3);
  trace::record("write.reuse", t4 - t0);
  return true;
}

void write_kept(const std::string& path, const std::string& tmp_dir, const std::string& contents, unsigned perm) {
  std::lock_guard<std::mutex> lk(g_mu);
  Slot& s = slots()[path];
  File next;
  if (rewrite_spare(s.spare, contents)) {
    next = std::move(s.spare);
    s.spare = File{};
  } else {
    create_and_write(tmp_dir, contents, perm, &next.name, &next.fd);
    struct stat st;
    if (::fstat(next.fd, &st) == 0) {
      next.dev = st.st_dev;
      next.ino = st.st_ino;
    }
    next.local = reuse_is_safe(next.fd);
    // A lease break (an open that raced with the exchange and reached the
    // file while this process held its lease) signals the holder: SIGIO by
    // default, which would terminate the daemon.  SIGURG is ignored unless
    // handled, and the breaker only waits for the lease's release anyway.
    (void)::fcntl(next.fd, F_SETSIG, SIGURG);
  }
  // Swap it with the feature file when that is a regular file; anything else
  // at `path` (nothing yet, a directory that must fail like rename(2)
  // would, a file system without the exchange) takes a plain rename.
  int64_t t0 = trace::stamp();
  struct stat old;
  bool swapped = false;
  if (::lstat(path.c_str(), &old) == 0 && S_ISREG(old.st_mode)) {
    swapped = ::renameat2(AT_FDCWD, next.name.c_str(), AT_FDCWD, path.c_str(), RENAME_EXCHANGE) == 0;
  }
  if (!swapped && ::rename(next.name.c_str(), path.c_str()) != 0) {
    int e = errno;
    close_file(next, true);
    remove_own_temps(tmp_dir);
    throw Error("error moving temporary file to '" + path + "': " + fs::errno_str(e));
  }
  trace::record_since("write.rename", t0);
  if (swapped && s.live.fd >= 0 && old.st_dev == s.live.dev && old.st_ino == s.live.ino) {
    // The old feature file, ours, is now under the temporary name.
    s.spare = std::move(s.live);
    s.spare.name = next.name;
  } else {
    // Someone else's file was at `path` (now under the temporary name, to be
    // removed as a rename would have), or nothing was.
    if (swapped) ::unlink(next.name.c_str());
    close_file(s.live, false);
  }
  next.name.clear();
  s.live = std::move(next);
}

}  // namespace

void write_file_atomically(const std::string& path, const std::string& contents, unsigned perm) {
  std::string tmp_dir = temp_dir_of(path);
  std::string tmpl;
  create_and_write(tmp_dir, contents, perm, &tmpl, nullptr);
  int64_t t0 = trace::stamp();
  if (::rename(tmpl.c_str(), path.c_str()) != 0) {
    int e = errno;
    ::unlink(tmpl.c_str());
    remove_own_temps(tmp_dir);
    throw Error("error moving temporary file to '" + path + "': " + fs::errno_str(e));
  }
  trace::record_since("write.rename", t0);
}

void release_kept_files() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& [path, s] : slots()) {
    close_file(s.spare, true);
    close_file(s.live, false);
  }
  slots().clear();
}

void release_kept_files(const std::string& path) {
  if (path.empty()) return;
  std::string abs = fs::absolute(path);
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = slots().find(abs);
  if (it == slots().end()) return;
  close_file(it->second.spare, true);
  close_file(it->second.live, false);
  slots().erase(it);
}

void sweep_temp_dir(const std::string& path) {
  if (path.empty()) return;
  std::string tmp_dir = temp_dir_of(path);
  if (int e = remove_own_temps(tmp_dir))
    throw Error("failed to remove stale temporary files in '" + tmp_dir + "': " + fs::errno_str(e));
}

void write_to_file(const Labels& labels, const std::string& path, bool reuse) {
  std::string out = render(labels);
  if (path.empty()) {
    if (fwrite(out.data(), 1, out.size(), stdout) != out.size() || fflush(stdout) != 0)
      throw Error("error writing labels to stdout");
    return;
  }
  try {
    if (reuse) {
      std::string abs = fs::absolute(path);
      write_kept(abs, temp_dir_of(abs), out, 0644);
    } else {
      write_file_atomically(path, out, 0644);
    }
  } catch (const std::exception& e) {
    throw Error("error atomically writing file '" + path + "': " + e.what());
  }
}

void remove_output_file(const std::string& path) {
  std::string abs = fs::absolute(path);
  release_kept_files(abs);
  std::string tmp_dir = temp_dir_of(abs);
  if (int e = remove_own_temps(tmp_dir)) throw Error("failed to remove temporary output directory: " + fs::errno_str(e));
  if (::unlink(abs.c_str()) != 0) throw Error("failed to remove output file: " + fs::errno_str(errno));
}

}  // namespace gfd::lm
