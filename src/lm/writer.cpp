// The feature-file writer (lm/labels.h: write_to_file and friends): atomic
// replacement through gfd-tmp/, with temporary files prepared by a worker
// between cycles in loop mode.  The labelers are in labels.cpp.
#include "lm/labels.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

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

// Loop-mode state of the writer, kept between cycles: up to two temporary
// files made ahead of the writes that will use them, and the old feature
// files writes swapped out, until the next preparer job unlinks them (one
// between cycles; two if a write came before the job that was to unlink its
// predecessor had started).  All live in <dir>/gfd-tmp/, which the daemon
// empties at start-up (sweep_temp_dir) and removes at exit, so a crash leaves
// at most these files behind until the next start.
//
// Why each exists, measured with the daemon's cycles 1 s apart (the deployed
// cadence is 60 s, so every cycle starts cold):
//   * The prepared file: a cold create on the box's overlayfs costs 0.1-0.2
//     ms, more than the rest of the write.  The cycle's worker makes the next
//     file after its node-facts and SR-IOV tasks, off the critical path:
//     write p50 0.055-0.090 ms vs 0.147-0.282 ms creating in the write
//     (profiles/writer_ab_r3.txt).  Two, not one: the job runs while its own
//     cycle writes, so the file a write uses must come from an earlier
//     cycle's job - with one, every other write made its own file.  Each
//     job tops the queue up to two (and makes gfd-tmp/ if the first cycle's
//     write has not yet), so every write after the first takes one
//     (tests/test_daemon.py::test_loop_writes_take_prepared_files).
//   * The exchange: a rename over the old feature file frees its inode
//     inside rename(2); on ext4 (the usual file system of NFD's features.d
//     hostPath) that is most of a cold replace, 0.34-0.58 ms vs 0.03 ms for
//     renameat2(RENAME_EXCHANGE), which leaves the old file under the
//     temporary name for the next cycle's preparer job to unlink
//     (profiles/rename_exchange_ab.txt).  Readers see the old file or the
//     new one under `path`, never neither, exactly as with a rename.  A
//     write exchanges even when an earlier old file still waits (its job
//     had not started yet): waiting for it made 3 of 14 cold ext4 writes
//     rename over the old file and pay the eviction, 0.35-0.39 ms; waking a
//     worker for the unlink right after the write cost 0.1 ms every cycle.
constexpr size_t kMaxPrepared = 2;
constexpr size_t kMinPrealloc = 4096;

struct Prepared {
  std::string name;
  int fd = -1;
  size_t allocated = 0;  // bytes preallocated beyond EOF
};

struct WriterState {
  std::mutex mu;
  std::condition_variable cv;   // job finished
  std::string dir;              // gfd-tmp/ of the prepared files
  std::vector<Prepared> ready;  // oldest first
  std::vector<std::string> retired;  // swapped-out feature files to unlink
  std::string no_exchange_dir;  // whose file system refused RENAME_EXCHANGE
  bool job = false;             // a preparer job is handed out, not yet finished or dropped
  size_t last_size = 0;         // of the last write: the next file's preallocation
};

WriterState& writer() {
  static auto* w = new WriterState;  // never destroyed: a worker may still use it at exit
  return *w;
}

void drop_ready(WriterState& w) {  // caller holds mu
  for (auto& f : w.ready) {
    ::close(f.fd);
    ::unlink(f.name.c_str());
  }
  w.ready.clear();
}

// Takes the oldest prepared file if it is in `tmp_dir` (fd, name,
// preallocation), else -1; prepared files elsewhere are removed.
int take_prepared(const std::string& tmp_dir, std::string* name, size_t* allocated) {
  WriterState& w = writer();
  std::lock_guard<std::mutex> lk(w.mu);
  if (w.dir != tmp_dir) drop_ready(w);
  if (w.ready.empty()) return -1;
  Prepared f = std::move(w.ready.front());
  w.ready.erase(w.ready.begin());
  *name = std::move(f.name);
  *allocated = f.allocated;
  return f.fd;
}

// Replaces `path` by the finished temporary file `tmpl`.  `exchange` (loop
// mode): swap the two names when `path` is a regular file; the old file,
// now under `tmpl`, waits for the next preparer job.  Anything else - no
// feature file yet, a directory or other non-file at `path` (which must fail
// like rename(2) would), a file system without the exchange - is a plain
// rename.  Returns 0 or an errno.
int replace_file(const std::string& tmpl, const std::string& path, const std::string& tmp_dir, bool exchange) {
  WriterState& w = writer();
  if (exchange) {
    std::lock_guard<std::mutex> lk(w.mu);
    exchange = w.no_exchange_dir != tmp_dir;
  }
  struct stat st;
  if (exchange && ::lstat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) {
    if (::renameat2(AT_FDCWD, tmpl.c_str(), AT_FDCWD, path.c_str(), RENAME_EXCHANGE) == 0) {
      std::lock_guard<std::mutex> lk(w.mu);
      w.retired.push_back(tmpl);
      return 0;
    }
    if (errno == EINVAL || errno == ENOSYS || errno == EOPNOTSUPP) {
      std::lock_guard<std::mutex> lk(w.mu);
      w.no_exchange_dir = tmp_dir;
    }
  }
  return ::rename(tmpl.c_str(), path.c_str()) == 0 ? 0 : errno;
}

// One attempt: false (nothing thrown, nothing left behind) when a prepared
// file vanished before its rename - the caller retries with a fresh one.
bool write_atomically_once(const std::string& path, const std::string& tmp_dir, const std::string& contents,
                           unsigned perm, bool use_prepared) {
  std::string tmpl;
  size_t allocated = 0;
  int64_t t0 = trace::now_ns();
  int fd = use_prepared ? take_prepared(tmp_dir, &tmpl, &allocated) : -1;
  bool prepared_fd = fd >= 0;
  // The temporary directory normally exists from the previous cycle: try the
  // create first and make the directory only when it is missing.
  if (fd < 0) fd = create_temp(tmp_dir, perm, &tmpl);
  if (fd < 0 && errno == ENOENT) {
    try {
      fs::mkdir_all(tmp_dir);
    } catch (const std::exception& e) {
      throw Error(std::string("failed to create temporary directory: ") + e.what());
    }
    fd = create_temp(tmp_dir, perm, &tmpl);
  }
  // Failures remove gfd-tmp/ like the reference (labels.go:81-85): a
  // prepared file lost with it is a vanished prepared file (retried).
  if (fd < 0) {
    int e = errno;
    remove_own_temps(tmp_dir);
    throw Error("fail to create temporary output file: " + fs::errno_str(e));
  }
  auto fail = [&](const std::string& msg) {
    ::close(fd);
    ::unlink(tmpl.c_str());
    remove_own_temps(tmp_dir);
    throw Error(msg);
  };
  int64_t t1 = trace::now_ns();
  trace::record(prepared_fd ? "write.take" : "write.create", t1 - t0);
  // Best effort: a file system without fallocate(2) just takes the write.
  if (contents.size() > allocated && wants_prealloc(fd))
    (void)::fallocate(fd, 0, 0, static_cast<off_t>(contents.size()));
  if (!write_all(fd, contents)) fail("error writing temporary file '" + tmpl + "': " + fs::errno_str(errno));
  // Created with `perm` already; chmod only what the umask took away.
  if ((perm & process_umask()) != 0 && ::fchmod(fd, perm) != 0)
    fail("error setting permissions on '" + tmpl + "': " + fs::errno_str(errno));
  if (::close(fd) != 0) {
    int e = errno;
    ::unlink(tmpl.c_str());
    remove_own_temps(tmp_dir);
    throw Error("error writing temporary file '" + tmpl + "': " + fs::errno_str(e));
  }
  int64_t t2 = trace::now_ns();
  trace::record("write.data", t2 - t1);
  if (int e = replace_file(tmpl, path, tmp_dir, prepared_fd)) {
    ::unlink(tmpl.c_str());
    // A prepared file removed behind our back (gfd-tmp/ deleted between
    // cycles): not an error of this cycle.
    if (prepared_fd && e == ENOENT) return false;
    remove_own_temps(tmp_dir);
    throw Error("error moving temporary file to '" + path + "': " + fs::errno_str(e));
  }
  trace::record("write.rename", trace::now_ns() - t2);
  return true;
}

std::string temp_dir_of(const std::string& path) { return fs::join(fs::dirname(fs::absolute(path)), "gfd-tmp"); }

}  // namespace

void write_file_atomically(const std::string& path, const std::string& contents, unsigned perm) {
  std::string tmp_dir = temp_dir_of(path);
  // Prepared files are created 0644 - the feature file's mode.
  WriterState& w = writer();
  if (!write_atomically_once(path, tmp_dir, contents, perm, perm == 0644)) {
    {
      // gfd-tmp/ was removed under us: the other prepared files went with it.
      std::lock_guard<std::mutex> lk(w.mu);
      drop_ready(w);
    }
    write_atomically_once(path, tmp_dir, contents, perm, false);
  }
  std::lock_guard<std::mutex> lk(w.mu);
  w.last_size = contents.size();
}

std::function<void()> temp_preparer(const std::string& path) {
  if (path.empty()) return {};
  std::string tmp_dir = temp_dir_of(path);
  WriterState& w = writer();
  size_t hint;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    size_t have = w.dir == tmp_dir ? w.ready.size() : 0;
    if (w.job || (have >= kMaxPrepared && w.retired.empty())) return {};
    w.job = true;
    // Before the first write no size is known: a block, which holds the
    // label file of a node of 8 GPUs.  Without it the first two loop writes
    // allocated inside the write (write.data 0.066-0.089 ms vs 0.022-0.043,
    // profiles/cold_rows_r4.txt).
    hint = std::max<size_t>(w.last_size, kMinPrealloc);
  }
  // Clears `job` when the job has run or was dropped unrun.
  std::shared_ptr<void> ticket(nullptr, [](void*) {
    WriterState& q = writer();
    std::lock_guard<std::mutex> lk(q.mu);
    q.job = false;
    q.cv.notify_all();
  });
  return [tmp_dir, hint, ticket] {
    WriterState& q = writer();
    std::vector<std::string> old;
    size_t want;
    {
      std::lock_guard<std::mutex> lk(q.mu);
      old.swap(q.retired);
      size_t have = q.dir == tmp_dir ? q.ready.size() : 0;
      want = have < kMaxPrepared ? kMaxPrepared - have : 0;
    }
    for (const auto& name : old) ::unlink(name.c_str());
    // Top the queue up to kMaxPrepared, not one file per job: a job that
    // runs after its own cycle's write (the worker is free only after the
    // node facts and the SR-IOV scan) must still leave the next write one.
    // Back to back too: the driver's 20-step headline 0.063-0.068 ms vs
    // 0.073-0.076 with one file per job (profiles/headline_ab_r4.txt).
    for (size_t i = 0; i < want; ++i) {
      // The first cycle's job usually runs before gfd-tmp/ exists: make it
      // (and the output directory), as that cycle's write is about to.
      Prepared f;
      f.fd = create_temp(tmp_dir, 0644, &f.name);
      if (f.fd < 0 && errno == ENOENT) {
        try {
          fs::mkdir_all(tmp_dir);
        } catch (const std::exception&) {
          return;  // the write reports it
        }
        f.fd = create_temp(tmp_dir, 0644, &f.name);
      }
      if (f.fd < 0) return;
      if (wants_prealloc(f.fd) && ::fallocate(f.fd, FALLOC_FL_KEEP_SIZE, 0, static_cast<off_t>(hint)) == 0)
        f.allocated = hint;
      std::lock_guard<std::mutex> lk(q.mu);
      if (q.dir != tmp_dir) drop_ready(q);
      q.dir = tmp_dir;
      q.ready.push_back(std::move(f));
    }
  };
}

void discard_prepared_temps() {
  WriterState& w = writer();
  std::unique_lock<std::mutex> lk(w.mu);
  // A job handed out runs soon (or is dropped): its file must not outlive
  // this call.  Bounded all the same - exit must not hang on a worker stuck
  // in the file system; a file it makes later stays in gfd-tmp/ until the
  // next start's sweep.  system_clock: a steady_clock wait is
  // pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not intercept.
  w.cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::seconds(1), [&] { return !w.job; });
  drop_ready(w);
  for (const auto& name : w.retired) ::unlink(name.c_str());
  w.retired.clear();
}

void sweep_temp_dir(const std::string& path) {
  if (path.empty()) return;
  std::string tmp_dir = temp_dir_of(path);
  if (int e = remove_own_temps(tmp_dir))
    throw Error("failed to remove stale temporary files in '" + tmp_dir + "': " + fs::errno_str(e));
}

void write_to_file(const Labels& labels, const std::string& path) {
  std::string out = render(labels);
  if (path.empty()) {
    if (fwrite(out.data(), 1, out.size(), stdout) != out.size() || fflush(stdout) != 0)
      throw Error("error writing labels to stdout");
    return;
  }
  try {
    write_file_atomically(path, out, 0644);
  } catch (const std::exception& e) {
    throw Error("error atomically writing file '" + path + "': " + e.what());
  }
}

void remove_output_file(const std::string& path) {
  discard_prepared_temps();
  std::string abs = fs::absolute(path);
  std::string tmp_dir = temp_dir_of(abs);
  if (int e = remove_own_temps(tmp_dir)) throw Error("failed to remove temporary output directory: " + fs::errno_str(e));
  if (::unlink(abs.c_str()) != 0) throw Error("failed to remove output file: " + fs::errno_str(errno));
}


}  // namespace gfd::lm
