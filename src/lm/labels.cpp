#include "lm/labels.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>

#include "util/error.h"
#include "util/fs.h"

namespace gfd::lm {

namespace {

class FixedLabeler : public Labeler {
 public:
  explicit FixedLabeler(Labels l) : labels_(std::move(l)) {}
  Labels GetLabels() override { return labels_; }

 private:
  Labels labels_;
};

class ListLabeler : public Labeler {
 public:
  explicit ListLabeler(std::vector<LabelerPtr> l) : labelers_(std::move(l)) {}
  Labels GetLabels() override {
    Labels all;
    for (const auto& l : labelers_) {
      if (!l) continue;
      Labels part;
      try {
        part = l->GetLabels();
      } catch (const std::exception& e) {
        throw Error(std::string("error generating labels: ") + e.what());
      }
      for (auto& kv : part) all[kv.first] = std::move(kv.second);
    }
    return all;
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

void write_file_atomically(const std::string& path, const std::string& contents, unsigned perm) {
  std::string abs = fs::absolute(path);
  std::string tmp_dir = fs::join(fs::dirname(abs), "gfd-tmp");
  try {
    fs::mkdir_all(tmp_dir);
  } catch (const std::exception& e) {
    throw Error(std::string("failed to create temporary directory: ") + e.what());
  }
  std::string tmpl = fs::join(tmp_dir, "gfd-XXXXXX");
  int fd = ::mkstemp(tmpl.data());
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
  if (!write_all(fd, contents)) fail("error writing temporary file '" + tmpl + "': " + fs::errno_str(errno));
  if (::fchmod(fd, perm) != 0) fail("error setting permissions on '" + tmpl + "': " + fs::errno_str(errno));
  if (::close(fd) != 0) {
    int e = errno;
    ::unlink(tmpl.c_str());
    fs::remove_all(tmp_dir);
    throw Error("error writing temporary file '" + tmpl + "': " + fs::errno_str(e));
  }
  if (::rename(tmpl.c_str(), path.c_str()) != 0) {
    int e = errno;
    ::unlink(tmpl.c_str());
    fs::remove_all(tmp_dir);
    throw Error("error moving temporary file to '" + path + "': " + fs::errno_str(e));
  }
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
  std::string abs = fs::absolute(path);
  std::string tmp_dir = fs::join(fs::dirname(abs), "gfd-tmp");
  if (int e = fs::remove_all(tmp_dir)) throw Error("failed to remove temporary output directory: " + fs::errno_str(e));
  if (::unlink(abs.c_str()) != 0) throw Error("failed to remove output file: " + fs::errno_str(errno));
}

std::string sanitize_label_value(const std::string& v) {
  auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); };
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
