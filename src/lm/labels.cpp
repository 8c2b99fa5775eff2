#include "lm/labels.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include <cerrno>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "util/error.h"
#include "util/fs.h"
#include "util/pool.h"
#include "util/trace.h"

namespace gfd::lm {

namespace {

class FixedLabeler : public Labeler {
 public:
  explicit FixedLabeler(Labels l) : labels_(std::move(l)) {}
  Labels GetLabels() override { return labels_; }
  void AppendTo(Labels& out) override {
    if (out.empty()) {
      out = labels_;
      return;
    }
    for (const auto& kv : labels_) out[kv.first] = kv.second;
  }

 private:
  Labels labels_;
};

class ListLabeler : public Labeler {
 public:
  explicit ListLabeler(std::vector<LabelerPtr> l) : labelers_(std::move(l)) {}
  Labels GetLabels() override {
    Labels all;
    AppendTo(all);
    return all;
  }
  void AppendTo(Labels& out) override {
    for (const auto& l : labelers_) {
      if (!l) continue;
      try {
        l->AppendTo(out);
      } catch (const std::exception& e) {
        throw Error(std::string("error generating labels: ") + e.what());
      }
    }
  }

 private:
  std::vector<LabelerPtr> labelers_;
};

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

// mkstemp with the final permission bits: "<dir>/gfd-XXXXXX" with a random
// suffix, O_EXCL.  Returns the fd (name in *name) or -1 with errno set.
int create_temp(const std::string& dir, unsigned perm, std::string* name) {
  static const char kChars[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
  static thread_local uint64_t state = static_cast<uint64_t>(::getpid()) * 0x9E3779B97F4A7C15ULL ^
                                       static_cast<uint64_t>(reinterpret_cast<uintptr_t>(&state));
  for (int attempt = 0; attempt < 100; ++attempt) {
    *name = dir + "/gfd-";
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
// GFD_WRITE_PREALLOC=always|never overrides the file-system check (A/B).
bool wants_prealloc(int fd) {
  static const int forced = [] {
    const char* v = std::getenv("GFD_WRITE_PREALLOC");
    if (!v) return -1;
    std::string s(v);
    return s == "always" ? 1 : s == "never" ? 0 : -1;
  }();
  if (forced >= 0) return forced == 1;
  struct statfs sf;
  if (::fstatfs(fd, &sf) != 0) return false;
  constexpr unsigned long kExt4 = 0xEF53, kOverlay = 0x794c7630;
  return static_cast<unsigned long>(sf.f_type) == kExt4 || static_cast<unsigned long>(sf.f_type) == kOverlay;
}

}  // namespace

LabelerPtr from_labels(Labels l) { return std::make_shared<FixedLabeler>(std::move(l)); }
LabelerPtr empty() { return std::make_shared<FixedLabeler>(Labels{}); }
LabelerPtr merge(std::vector<LabelerPtr> labelers) { return std::make_shared<ListLabeler>(std::move(labelers)); }

std::string render(const Labels& labels) {
  size_t n = 0;
  for (const auto& kv : labels) n += kv.first.size() + kv.second.size() + 2;
  std::string out;
  out.reserve(n);
  for (const auto& kv : labels) {
    out.append(kv.first);
    out.push_back('=');
    out.append(kv.second);
    out.push_back('\n');
  }
  return out;
}

namespace {

// Temporary files created ahead of the writes that use them (loop mode):
// the daemon's cycle hands temp_preparer()'s job to the worker that already
// runs its node facts and SR-IOV scan, after those, so the next cycle's file
// is created - and, where the write preallocates (wants_prealloc), its blocks
// allocated beyond EOF for the last size (FALLOC_FL_KEEP_SIZE) - while this
// cycle enumerates and writes.  A write then is write + close + rename; the
// ~7 us create plus allocation (more on some hosts' overlayfs) are off its
// critical path (profiles/write_prepare_ab.txt).  At most kMaxPrepared files
// are ready or being made; a write takes the oldest in its directory and
// creates its own when none is ready, never waiting for a worker.
//
// Four, not two: back to back, a worker's create (and the unlink of the file
// the last exchange swapped out) can take longer than a whole cycle, and
// with two ready some writes still made their own file - bench p90
// 0.024-0.036 -> 0.021-0.024 ms with four, p50 and cold cycles unchanged
// (profiles/write_prepare_ab.txt, last section).  An empty file and a
// descriptor each.
constexpr size_t kMaxPrepared = 4;

// GFD_WRITE_PREPARE_MAX=N (1-8): another bound (A/B measurements).
size_t max_prepared() {
  static const size_t n = [] {
    const char* v = std::getenv("GFD_WRITE_PREPARE_MAX");
    long x = v ? std::strtol(v, nullptr, 10) : 0;
    return x >= 1 && x <= 8 ? static_cast<size_t>(x) : kMaxPrepared;
  }();
  return n;
}

struct Prepared {
  std::string dir, name;
  int fd = -1;
  size_t allocated = 0;  // bytes of blocks preallocated
};

// Old feature files swapped out of place by a write's RENAME_EXCHANGE, now
// under a temporary name in gfd-tmp/<x>/, waiting for a worker to unlink them.
struct Retired {
  std::string dir, name;
};

struct PreparedTemps {
  std::mutex mu;
  std::condition_variable cv;  // in_flight or jobs dropped
  std::deque<Prepared> ready;
  std::vector<Retired> retired;
  std::string no_exchange_dir;  // temporary directory whose file system refused RENAME_EXCHANGE
  size_t in_flight = 0;  // files being made by preparer jobs handed out and not yet finished or dropped
  size_t jobs = 0;       // preparer jobs handed out and not yet finished or dropped
  size_t last_size = 0;  // of the last write: the next file's preallocation
  size_t serial = 0;     // files handed out to be made so far (picks the subdirectory)
};

PreparedTemps& prepared() {
  static auto* p = new PreparedTemps;  // never destroyed: a worker may still use it at exit
  return *p;
}

void drop(Prepared& f) {
  ::close(f.fd);
  ::unlink(f.name.c_str());
}

// The oldest prepared file in `tmp_dir` (fd, name and preallocation), or -1;
// prepared files of other directories are removed.
int take_prepared(const std::string& tmp_dir, std::string* name, size_t* allocated) {
  PreparedTemps& p = prepared();
  std::lock_guard<std::mutex> lk(p.mu);
  while (!p.ready.empty()) {
    Prepared f = std::move(p.ready.front());
    p.ready.pop_front();
    if (f.dir != tmp_dir) {
      drop(f);
      continue;
    }
    *name = std::move(f.name);
    *allocated = f.allocated;
    return f.fd;
  }
  return -1;
}

// Counts a handed-out preparer job (and the file it makes, if it makes one)
// until it has run (finish) or was dropped unrun (the job, and with it this
// ticket, destroyed).
struct InFlight {
  bool creates = false;
  bool finished = false;
  void finish() {
    PreparedTemps& p = prepared();
    std::lock_guard<std::mutex> lk(p.mu);
    if (finished) return;
    finished = true;
    p.in_flight -= creates;
    --p.jobs;
    p.cv.notify_all();
  }
  ~InFlight() { finish(); }
};

// Replace `path` with the finished temporary file `tmpl`.
//
// In loop mode (a prepared file, so a preparer job comes every cycle) the two
// names are swapped with renameat2(RENAME_EXCHANGE) and the old feature file,
// now under the temporary name, is left for the next preparer job to unlink.
// A rename over the old file drops its inode inside the call - on ext4 (the
// usual file system of NFD's features.d hostPath) that eviction is most of a
// cold replace: 0.46 ms vs 0.05 ms for the exchange, cycles 1 s apart
// (profiles/rename_exchange_ab.txt).  Readers see the same thing either way:
// the old file or the new one under `path`, never neither.  No feature file
// yet (first write), a file system without the exchange, or something other
// than a file at `path` (a directory must fail like rename(2) would, not be
// swapped into gfd-tmp/): a plain rename.  GFD_WRITE_EXCHANGE=never: always a
// plain rename (A/B).  Returns 0 or an errno.
int replace_file(const std::string& tmpl, const std::string& path, const std::string& tmp_dir, bool exchange) {
  static const bool never = [] {
    const char* v = std::getenv("GFD_WRITE_EXCHANGE");
    return v && std::string(v) == "never";
  }();
  PreparedTemps& p = prepared();
  if (exchange && !never) {
    {
      std::lock_guard<std::mutex> lk(p.mu);
      exchange = p.no_exchange_dir != tmp_dir;
    }
    if (exchange && ::renameat2(AT_FDCWD, tmpl.c_str(), AT_FDCWD, path.c_str(), RENAME_EXCHANGE) == 0) {
      struct stat st;
      if (::lstat(tmpl.c_str(), &st) == 0 && !S_ISDIR(st.st_mode)) {
        std::lock_guard<std::mutex> lk(p.mu);
        p.retired.push_back({tmp_dir, tmpl});
        return 0;
      }
      // Swapped a directory out of `path`: put it back, rename decides.
      if (::renameat2(AT_FDCWD, tmpl.c_str(), AT_FDCWD, path.c_str(), RENAME_EXCHANGE) != 0) return errno;
    } else if (exchange && (errno == EINVAL || errno == ENOSYS || errno == EOPNOTSUPP)) {
      std::lock_guard<std::mutex> lk(p.mu);
      p.no_exchange_dir = tmp_dir;
    }
  }
  return ::rename(tmpl.c_str(), path.c_str()) == 0 ? 0 : errno;
}

void unlink_retired(std::vector<Retired>& files) {
  for (const auto& f : files) ::unlink(f.name.c_str());
  files.clear();
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
  if (fd < 0) {
    int e = errno;
    fs::remove_all(tmp_dir);
    throw Error("fail to create temporary output file: " + fs::errno_str(e));
  }
  auto fail = [&](const std::string& msg) {
    ::close(fd);
    ::unlink(tmpl.c_str());
    fs::remove_all(tmp_dir);
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
    fs::remove_all(tmp_dir);
    throw Error("error writing temporary file '" + tmpl + "': " + fs::errno_str(e));
  }
  int64_t t2 = trace::now_ns();
  trace::record("write.data", t2 - t1);
  if (int e = replace_file(tmpl, path, tmp_dir, prepared_fd)) {
    ::unlink(tmpl.c_str());
    // A prepared file removed behind our back (gfd-tmp/ deleted between
    // cycles): not an error of this cycle.
    if (prepared_fd && e == ENOENT) return false;
    fs::remove_all(tmp_dir);
    throw Error("error moving temporary file to '" + path + "': " + fs::errno_str(e));
  }
  trace::record("write.rename", trace::now_ns() - t2);
  return true;
}

}  // namespace

void write_file_atomically(const std::string& path, const std::string& contents, unsigned perm) {
  std::string abs = fs::absolute(path);
  std::string tmp_dir = fs::join(fs::dirname(abs), "gfd-tmp");
  // Prepared files are created 0644 - the feature file's mode.
  if (!write_atomically_once(path, tmp_dir, contents, perm, perm == 0644))
    write_atomically_once(path, tmp_dir, contents, perm, false);
  PreparedTemps& p = prepared();
  std::lock_guard<std::mutex> lk(p.mu);
  p.last_size = contents.size();
}

std::function<void()> temp_preparer(const std::string& path) {
  // GFD_WRITE_PREPARE=never: every write creates its own file (A/B).
  static const bool never = [] {
    const char* v = std::getenv("GFD_WRITE_PREPARE");
    return v && std::string(v) == "never";
  }();
  if (never || path.empty()) return {};
  std::string tmp_dir = fs::join(fs::dirname(fs::absolute(path)), "gfd-tmp");
  PreparedTemps& p = prepared();
  size_t hint, serial;
  auto ticket = std::make_shared<InFlight>();
  {
    std::lock_guard<std::mutex> lk(p.mu);
    size_t have = p.in_flight;
    for (const auto& f : p.ready) have += f.dir == tmp_dir;
    ticket->creates = have < max_prepared();
    if (!ticket->creates && p.retired.empty()) {
      ticket->finished = true;  // never handed out
      return {};
    }
    p.in_flight += ticket->creates;
    ++p.jobs;
    hint = p.last_size;
    serial = ticket->creates ? p.serial++ : 0;
  }
  return [tmp_dir, hint, serial, ticket] {
    // Old feature files the last writes swapped out (replace_file): unlinked
    // here, off the write's path.  After this job's create, which the next
    // write may need sooner.
    std::vector<Retired> old;
    auto take_retired = [&] {
      PreparedTemps& q = prepared();
      std::lock_guard<std::mutex> lk(q.mu);
      old.swap(q.retired);
    };
    if (!ticket->creates) {
      take_retired();
      unlink_retired(old);
      ticket->finish();
      return;
    }
    Prepared f;
    f.dir = tmp_dir;
    // Round-robin over one subdirectory more than files can be ready or
    // being made (gfd-tmp/a, b, ...): writes take files in the order they
    // were made, so the file a write swaps out of gfd-tmp/<x>/ - and the old
    // feature file left there, which a later job unlinks - never shares <x>
    // with a create or unlink in flight, and those (tens of us on some
    // overlayfs hosts) never hold the directory lock the exchange needs.
    // With two subdirectories and four files they did: exchange 4 -> 54 us
    // on a slow-create box (profiles/write_prepare_ab.txt).  gfd-tmp/ itself
    // is not re-created: a missing one is the next write's business.
    std::string sub = tmp_dir + "/" + static_cast<char>('a' + serial % (max_prepared() + 1));
    f.fd = create_temp(sub, 0644, &f.name);
    if (f.fd < 0 && errno == ENOENT && ::mkdir(sub.c_str(), 0755) == 0) f.fd = create_temp(sub, 0644, &f.name);
    if (f.fd >= 0) {
      if (hint > 0 && wants_prealloc(f.fd) &&
          ::fallocate(f.fd, FALLOC_FL_KEEP_SIZE, 0, static_cast<off_t>(hint)) == 0)
        f.allocated = hint;
      PreparedTemps& q = prepared();
      std::lock_guard<std::mutex> lk(q.mu);
      q.ready.push_back(std::move(f));
    }
    take_retired();
    unlink_retired(old);
    ticket->finish();
  };
}

void discard_prepared_temps() {
  PreparedTemps& p = prepared();
  std::unique_lock<std::mutex> lk(p.mu);
  // A job handed out runs soon (or is dropped): its file must not outlive
  // this call.  Bounded all the same - exit must not hang on a worker stuck
  // in the file system; its file would then stay behind in gfd-tmp/.
  // system_clock: a steady_clock wait is pthread_cond_clockwait, which GCC
  // 11's ThreadSanitizer does not intercept (it then reports the job's lock
  // of `mu` as a double lock); a clock step only moves this safety bound.
  p.cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::seconds(5), [&] { return p.jobs == 0; });
  for (auto& f : p.ready) drop(f);
  p.ready.clear();
  unlink_retired(p.retired);
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
  std::string tmp_dir = fs::join(fs::dirname(abs), "gfd-tmp");
  if (int e = fs::remove_all(tmp_dir)) throw Error("failed to remove temporary output directory: " + fs::errno_str(e));
  if (::unlink(abs.c_str()) != 0) throw Error("failed to remove output file: " + fs::errno_str(errno));
}

std::string sanitize_label_value(const std::string& v) {
  auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); };
  // Fast path (every label of a healthy node): already a valid value.
  if (v.empty()) return v;
  if (v.size() <= 63 && alnum(v.front()) && alnum(v.back())) {
    bool ok = true;
    for (char c : v) ok &= alnum(c) || c == '.' || c == '_' || c == '-';
    if (ok) return v;
  }
  std::string out;
  out.reserve(v.size());
  for (char c : v) {
    out.push_back((alnum(c) || c == '.' || c == '_' || c == '-') ? c : '-');
  }
  if (out.size() > 63) out.resize(63);
  size_t b = 0, e = out.size();
  while (b < e && !alnum(out[b])) ++b;
  while (e > b && !alnum(out[e - 1])) --e;
  return out.substr(b, e - b);
}

}  // namespace gfd::lm
