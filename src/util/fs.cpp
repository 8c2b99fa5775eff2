#include "util/fs.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "util/error.h"
#include "util/strings.h"

namespace gfd::fs {

ReadResult read_file(const std::string& path, size_t max_bytes) {
  ReadResult r;
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    r.err = errno;
    return r;
  }
  // sysfs attributes are at most a page; PCI config space is 4 KiB.
  char buf[4096];
  for (;;) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0) {
      if (errno == EINTR) continue;
      r.err = errno;
      break;
    }
    if (n == 0) break;
    r.data.append(buf, static_cast<size_t>(n));
    if (r.data.size() >= max_bytes) {
      r.data.resize(max_bytes);
      break;
    }
  }
  ::close(fd);
  return r;
}

std::optional<std::string> read_trimmed(const std::string& path) {
  auto r = read_file(path, 64 * 1024);
  if (!r.ok()) return std::nullopt;
  return str::trim(r.data);
}

bool exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

bool is_dir(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<std::string> list_dir(const std::string& path, int* err) {
  std::vector<std::string> out;
  DIR* d = ::opendir(path.c_str());
  if (!d) {
    if (err) *err = errno;
    return out;
  }
  if (err) *err = 0;
  while (struct dirent* e = ::readdir(d)) {
    if (e->d_name[0] == '.' && (e->d_name[1] == 0 || (e->d_name[1] == '.' && e->d_name[2] == 0))) continue;
    out.emplace_back(e->d_name);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

DirListing::~DirListing() {
  if (fd_ >= 0) ::close(fd_);
}

int DirListing::read_raw() {
  raw_.clear();
  if (::lseek(fd_, 0, SEEK_SET) < 0) return errno;
  char buf[32768];
  for (;;) {
    long n = ::syscall(SYS_getdents64, fd_, buf, sizeof(buf));
    if (n < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (n == 0) return 0;
    raw_.append(buf, static_cast<size_t>(n));
  }
}

int DirListing::read(const std::string& path, bool* changed) {
  if (fd_ >= 0 && path != path_) {
    ::close(fd_);
    fd_ = -1;
  }
  prev_.swap(raw_);
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (fd_ < 0) {
      fd_ = ::open(path.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
      if (fd_ < 0) {
        int e = errno;
        raw_.clear();
        prev_.clear();
        return e;
      }
      path_ = path;
    }
    int e = read_raw();
    struct stat st;
    if (e == 0 && ::fstat(fd_, &st) == 0 && st.st_nlink > 0) break;
    // Removed (or unreadable) since it was opened: look the path up again.
    ::close(fd_);
    fd_ = -1;
    if (attempt == 1) {
      raw_.clear();
      prev_.clear();
      return e ? e : ENOENT;
    }
  }
  *changed = raw_ != prev_;
  return 0;
}

std::vector<std::pair<std::string, uint64_t>> DirListing::entries() const {
  // struct linux_dirent64: u64 d_ino, s64 d_off, u16 d_reclen, u8 d_type,
  // NUL-terminated d_name.
  constexpr size_t kReclen = 16, kName = 19;
  std::vector<std::pair<std::string, uint64_t>> out;
  for (size_t pos = 0; pos + kName < raw_.size();) {
    uint64_t ino = 0;
    uint16_t reclen = 0;
    std::memcpy(&ino, raw_.data() + pos, sizeof(ino));
    std::memcpy(&reclen, raw_.data() + pos + kReclen, sizeof(reclen));
    if (reclen == 0 || pos + reclen > raw_.size()) break;
    const char* name = raw_.data() + pos + kName;
    if (!(name[0] == '.' && (name[1] == 0 || (name[1] == '.' && name[2] == 0)))) out.emplace_back(name, ino);
    pos += reclen;
  }
  std::sort(out.begin(), out.end());
  return out;
}

int pread_all(int fd, size_t max_bytes, std::string* out, bool short_read_is_all) {
  out->clear();
  char buf[8192];
  off_t off = 0;
  for (;;) {
    ssize_t n = ::pread(fd, buf, sizeof(buf), off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (n == 0) return 0;
    out->append(buf, static_cast<size_t>(n));
    off += n;
    // A sysfs attribute's show() fills at most a page, returned by one read;
    // a regular file reads short only at its end.  Then the read that would
    // return 0 is a syscall for nothing (one per attribute read per cycle).
    if (short_read_is_all && off == n && n < 4096) {
      if (out->size() > max_bytes) out->resize(max_bytes);
      return 0;
    }
    if (out->size() >= max_bytes) {
      out->resize(max_bytes);
      return 0;
    }
  }
}

namespace {

constexpr long kSysfsMagic = 0x62656572;  // SYSFS_MAGIC
constexpr size_t kMaxKeptOpen = 1024;


}  // namespace

AttrReader::Fd::~Fd() { ::close(fd); }

AttrReader::~AttrReader() { clear(); }

void AttrReader::clear() {
  std::unique_lock<std::shared_mutex> g(mu_);
  fds_.clear();
  checked_.clear();
}

size_t AttrReader::open_count() const {
  std::shared_lock<std::shared_mutex> g(mu_);
  return fds_.size() + checked_.size();
}

ReadResult AttrReader::read(const std::string& path, size_t max_bytes) {
  ReadResult r;
  std::shared_ptr<const Fd> kept;
  {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto it = fds_.find(path);
    if (it != fds_.end()) kept = it->second;
  }
  if (kept) {
    // Kept descriptors are sysfs attributes (or, in tests, regular files).
    if (pread_all(kept->fd, max_bytes, &r.data, true) == 0) return r;
    // Removed since it was opened (ENODEV) or otherwise unusable: forget it
    // and look the path up again.
    std::unique_lock<std::shared_mutex> g(mu_);
    auto it = fds_.find(path);
    if (it != fds_.end() && it->second == kept) fds_.erase(it);
  }
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    r.err = errno;
    return r;
  }
  if (int e = pread_all(fd, max_bytes, &r.data)) {
    ::close(fd);
    r.err = e;
    r.data.clear();
    return r;
  }
  struct statfs sfs;
  bool keep = keep_all_ || (::fstatfs(fd, &sfs) == 0 && static_cast<long>(sfs.f_type) == kSysfsMagic);
  if (keep) {
    auto holder = std::make_shared<const Fd>(fd);
    std::unique_lock<std::shared_mutex> g(mu_);
    if (fds_.size() >= kMaxKeptOpen) fds_.clear();
    fds_.emplace(path, std::move(holder));  // if another thread kept one first, ours closes here
    return r;
  }
  ::close(fd);
  return r;
}

ReadResult AttrReader::read_checked(const std::string& path, size_t max_bytes) {
  ReadResult r;
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) {
    r.err = errno;
    std::unique_lock<std::shared_mutex> g(mu_);
    checked_.erase(path);
    return r;
  }
  std::shared_ptr<const Fd> kept;
  {
    std::shared_lock<std::shared_mutex> g(mu_);
    auto it = checked_.find(path);
    if (it != checked_.end() && it->second.dev == static_cast<uint64_t>(st.st_dev) &&
        it->second.ino == static_cast<uint64_t>(st.st_ino))
      kept = it->second.fd;
  }
  if (kept && pread_all(kept->fd, max_bytes, &r.data) == 0) return r;
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    r.err = errno;
    return r;
  }
  auto holder = std::make_shared<const Fd>(fd);
  struct stat fst;
  if (int e = pread_all(fd, max_bytes, &r.data); e != 0 || ::fstat(fd, &fst) != 0) {
    r.err = e ? e : errno;
    r.data.clear();
    return r;
  }
  std::unique_lock<std::shared_mutex> g(mu_);
  if (checked_.size() >= kMaxKeptOpen) checked_.clear();
  checked_[path] = Checked{std::move(holder), static_cast<uint64_t>(fst.st_dev), static_cast<uint64_t>(fst.st_ino)};
  return r;
}

std::optional<std::string> AttrReader::read_checked_trimmed(const std::string& path) {
  auto r = read_checked(path);
  if (!r.ok()) return std::nullopt;
  return str::trim(r.data);
}

std::optional<std::string> AttrReader::read_trimmed(const std::string& path) {
  auto r = read(path);
  if (!r.ok()) return std::nullopt;
  return str::trim(r.data);
}

AttrReader& attrs() {
  // Leaked on purpose: pool threads may read attributes during exit.
  static AttrReader* reader = new AttrReader();
  return *reader;
}

ReadResult read_dmi(const std::string& path) {
  static std::mutex mu;
  // path -> the kept value, or nullopt for a file found not to be DMI's.
  // Leaked: workers may read at exit.
  static auto* kept = new std::unordered_map<std::string, std::optional<std::string>>();
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = kept->find(path);
    if (it != kept->end()) {
      if (it->second) return ReadResult{*it->second, 0};
    }
    if (it != kept->end() || kept->size() >= 64) return attrs().read(path, 4096);
  }
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return ReadResult{{}, errno};
  ReadResult r;
  r.err = pread_all(fd, 4096, &r.data);
  bool constant = false;
  struct statfs sfs;
  if (r.err == 0 && ::fstatfs(fd, &sfs) == 0 && static_cast<long>(sfs.f_type) == kSysfsMagic) {
    // Where the descriptor really points (any sysfs mount shows the one tree).
    char link[64], real[PATH_MAX];
    std::snprintf(link, sizeof(link), "/proc/self/fd/%d", fd);
    ssize_t n = ::readlink(link, real, sizeof(real) - 1);
    constant = n > 0 && std::string(real, static_cast<size_t>(n)).find("/devices/virtual/dmi/id/") != std::string::npos;
  }
  ::close(fd);
  if (r.err) {
    r.data.clear();
    return r;  // asked again next time
  }
  std::lock_guard<std::mutex> g(mu);
  kept->emplace(path, constant ? std::optional<std::string>(r.data) : std::nullopt);
  return r;
}

Dir::Dir(const std::string& path) {
  fd_ = ::open(path.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
  if (fd_ < 0) err_ = errno;
}

Dir::~Dir() {
  if (fd_ >= 0) ::close(fd_);
}

ReadResult Dir::read_attr(const char* name, size_t max_bytes) const {
  ReadResult r;
  if (fd_ < 0) {
    r.err = err_;
    return r;
  }
  int fd = ::openat(fd_, name, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    r.err = errno;
    return r;
  }
  r.data.resize(max_bytes);
  ssize_t n;
  do {
    n = ::read(fd, r.data.data(), max_bytes);
  } while (n < 0 && errno == EINTR);
  if (n < 0) {
    r.err = errno;
    r.data.clear();
  } else {
    r.data.resize(static_cast<size_t>(n));
  }
  ::close(fd);
  return r;
}

std::optional<std::string> Dir::read_trimmed(const char* name) const {
  auto r = read_attr(name);
  if (!r.ok()) return std::nullopt;
  return str::trim(r.data);
}

std::string Dir::read_link(const char* name) const {
  if (fd_ < 0) return {};
  char buf[PATH_MAX];
  ssize_t n = ::readlinkat(fd_, name, buf, sizeof(buf) - 1);
  if (n < 0) return {};
  return std::string(buf, static_cast<size_t>(n));
}

int Dir::lookup(const char* name) const {
  if (fd_ < 0) return err_;
  struct stat st;
  return ::fstatat(fd_, name, &st, AT_SYMLINK_NOFOLLOW) == 0 ? 0 : errno;
}

std::string read_link(const std::string& path) {
  char buf[PATH_MAX];
  ssize_t n = ::readlink(path.c_str(), buf, sizeof(buf) - 1);
  if (n < 0) return {};
  return std::string(buf, static_cast<size_t>(n));
}

std::string resolve_in_root(const std::string& root, const std::string& rel, std::vector<std::string>* dirs) {
  std::vector<std::string> todo;  // components still to walk, in reverse order
  auto push_path = [&](const std::string& p) {
    auto parts = str::split(p, '/');
    for (auto it = parts.rbegin(); it != parts.rend(); ++it)
      if (!it->empty() && *it != ".") todo.push_back(*it);
  };
  push_path(rel);
  std::vector<std::string> cur;
  int links = 0;
  auto path_of = [&](const std::vector<std::string>& comps) {
    std::string p = root.empty() ? "/" : root;
    for (const auto& c : comps) p = join(p, c);
    return p;
  };
  while (!todo.empty()) {
    std::string c = std::move(todo.back());
    todo.pop_back();
    if (c == "..") {
      if (!cur.empty()) cur.pop_back();
      continue;
    }
    if (dirs) {
      std::string parent = path_of(cur);
      if (std::find(dirs->begin(), dirs->end(), parent) == dirs->end()) dirs->push_back(parent);
    }
    cur.push_back(c);
    std::string p = path_of(cur);
    struct stat st;
    if (::lstat(p.c_str(), &st) != 0) return {};
    if (!S_ISLNK(st.st_mode)) continue;
    if (++links > 40) return {};
    std::string target = read_link(p);
    if (target.empty()) return {};
    cur.pop_back();
    if (target.front() == '/') cur.clear();
    push_path(target);
  }
  return path_of(cur);
}

KeptAttr::~KeptAttr() {
  if (fd_ >= 0) ::close(fd_);
}

bool KeptAttr::read(std::string* out) {
  char buf[256];
  ssize_t n = -1;
  if (fd_ >= 0) {
    n = ::pread(fd_, buf, sizeof(buf), 0);
    if (n < 0) {  // removed since it was opened (ENODEV): look the path up again
      ::close(fd_);
      fd_ = -1;
    }
  }
  if (fd_ < 0) {
    int fd = ::open(path_.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    n = ::pread(fd, buf, sizeof(buf), 0);
    struct statfs sfs;
    if (n >= 0 && ::fstatfs(fd, &sfs) == 0 && static_cast<long>(sfs.f_type) == kSysfsMagic)
      fd_ = fd;
    else
      ::close(fd);
  }
  if (n < 0) return false;
  size_t b = 0, e = static_cast<size_t>(n);
  auto space = [](char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; };
  while (b < e && space(buf[b])) ++b;
  while (e > b && space(buf[e - 1])) --e;
  out->assign(buf + b, e - b);
  return true;
}

bool is_local_fs(int fd) {
  struct statfs sf;
  if (::fstatfs(fd, &sf) != 0) return false;
  switch (static_cast<unsigned long>(sf.f_type)) {
    case 0xEF53:      // ext2/3/4
    case 0x58465342:  // xfs
    case 0x9123683E:  // btrfs
    case 0x01021994:  // tmpfs
    case 0x794c7630:  // overlayfs (a container's root; its upper layer is local)
      return true;
    default:
      return false;
  }
}

// The shared inotify instance and, per watch descriptor, the DirWatches
// that need it (one descriptor per directory and instance).
struct DirWatchRegistry {
  std::mutex mu;
  int fd = -1;
  std::map<int, std::vector<DirWatch*>> owners;

  static DirWatchRegistry& get() {
    static auto* r = new DirWatchRegistry();  // leaked: pool threads may read at exit
    return *r;
  }
  // Reads every queued event and marks the sets whose directories changed.
  void poll() {
    alignas(struct inotify_event) char buf[4096];
    for (;;) {
      ssize_t n = ::read(fd, buf, sizeof(buf));
      if (n <= 0) return;  // EAGAIN: nothing (more) queued
      for (ssize_t off = 0; off < n;) {
        const auto* e = reinterpret_cast<const struct inotify_event*>(buf + off);
        off += static_cast<ssize_t>(sizeof(struct inotify_event) + e->len);
        if (e->mask & IN_Q_OVERFLOW) {
          for (auto& [wd, ws] : owners)
            for (auto* w : ws) w->dirty_ = true;
          continue;
        }
        auto it = owners.find(e->wd);
        if (it != owners.end())
          for (auto* w : it->second) w->dirty_ = true;
      }
    }
  }
  void release(DirWatch* w) {
    for (int wd : w->wds_) {
      auto it = owners.find(wd);
      if (it == owners.end()) continue;
      auto& ws = it->second;
      ws.erase(std::remove(ws.begin(), ws.end(), w), ws.end());
      if (ws.empty()) {
        (void)::inotify_rm_watch(fd, wd);
        owners.erase(it);
      }
    }
    w->wds_.clear();
    w->armed_ = false;
  }
};

DirWatch::~DirWatch() {
  auto& r = DirWatchRegistry::get();
  std::lock_guard<std::mutex> g(r.mu);
  r.release(this);
}

bool DirWatch::arm(const std::vector<std::string>& dirs) {
  auto& r = DirWatchRegistry::get();
  std::lock_guard<std::mutex> g(r.mu);
  if (r.fd >= 0) r.poll();  // events so far belong to the sets armed so far
  r.release(this);
  dirty_ = false;
  if (dirs.empty()) return false;
  if (r.fd < 0) r.fd = ::inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (r.fd < 0) return false;  // e.g. the user's inotify instances used up
  constexpr uint32_t kMask =
      IN_CREATE | IN_DELETE | IN_MOVED_FROM | IN_MOVED_TO | IN_DELETE_SELF | IN_MOVE_SELF | IN_ONLYDIR;
  for (const auto& d : dirs) {
    int dfd = ::open(d.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    bool local = dfd >= 0 && is_local_fs(dfd);
    if (dfd >= 0) ::close(dfd);
    int wd = local ? ::inotify_add_watch(r.fd, d.c_str(), kMask) : -1;
    if (wd < 0) {
      r.release(this);
      return false;
    }
    auto& ws = r.owners[wd];
    if (std::find(ws.begin(), ws.end(), this) == ws.end()) ws.push_back(this);
    if (std::find(wds_.begin(), wds_.end(), wd) == wds_.end()) wds_.push_back(wd);
  }
  armed_ = true;
  return true;
}

bool DirWatch::unchanged() {
  auto& r = DirWatchRegistry::get();
  std::lock_guard<std::mutex> g(r.mu);
  if (!armed_) return false;
  r.poll();
  if (!dirty_) return true;
  r.release(this);  // a change: look again
  return false;
}

std::string join(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  if (b.empty()) return a;
  if (a.back() == '/') return b.front() == '/' ? a + b.substr(1) : a + b;
  return b.front() == '/' ? a + b : a + "/" + b;
}

std::string dirname(const std::string& path) {
  auto pos = path.find_last_of('/');
  if (pos == std::string::npos) return ".";
  if (pos == 0) return "/";
  return path.substr(0, pos);
}

std::string basename(const std::string& path) {
  std::string p = path;
  while (p.size() > 1 && p.back() == '/') p.pop_back();
  auto pos = p.find_last_of('/');
  return pos == std::string::npos ? p : p.substr(pos + 1);
}

std::string absolute(const std::string& path) {
  std::string p = path;
  if (p.empty() || p[0] != '/') {
    char cwd[PATH_MAX];
    if (!::getcwd(cwd, sizeof(cwd))) throw Error("getwd: " + errno_str(errno));
    p = join(cwd, p);
  }
  // Lexical clean (like Go's filepath.Clean): collapse //, ., ..
  std::vector<std::string> parts;
  for (auto& seg : str::split(p, '/')) {
    if (seg.empty() || seg == ".") continue;
    if (seg == "..") {
      if (!parts.empty()) parts.pop_back();
      continue;
    }
    parts.push_back(seg);
  }
  return "/" + str::join(parts, "/");
}

void mkdir_all(const std::string& path, unsigned mode) {
  if (path.empty() || is_dir(path)) return;
  mkdir_all(dirname(path), mode);
  if (::mkdir(path.c_str(), mode) != 0 && errno != EEXIST)
    throw Error("mkdir " + path + ": " + errno_str(errno));
}

int remove_all(const std::string& path) {
  struct stat st;
  if (::lstat(path.c_str(), &st) != 0) return errno == ENOENT ? 0 : errno;
  if (S_ISDIR(st.st_mode)) {
    for (const auto& name : list_dir(path)) {
      int e = remove_all(join(path, name));
      if (e) return e;
    }
    if (::rmdir(path.c_str()) != 0 && errno != ENOENT) return errno;
    return 0;
  }
  if (::unlink(path.c_str()) != 0 && errno != ENOENT) return errno;
  return 0;
}

std::string errno_str(int err) {
  char buf[256];
  // GNU strerror_r returns a char* that may not be `buf`.
  const char* s = strerror_r(err, buf, sizeof(buf));
  return s ? std::string(s) : std::string("errno ") + std::to_string(err);
}

}  // namespace gfd::fs
