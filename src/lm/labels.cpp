#include "lm/labels.h"

#include <string>
#include <utility>
#include <vector>

#include "util/error.h"

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
  void MoveTo(Labels& out) override { move_labels(out, std::move(labels_)); }

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
  void AppendTo(Labels& out) override { append(out, false); }
  void MoveTo(Labels& out) override { append(out, true); }

 private:
  void append(Labels& out, bool move) {
    for (const auto& l : labelers_) {
      if (!l) continue;
      try {
        if (move)
          l->MoveTo(out);
        else
          l->AppendTo(out);
      } catch (const std::exception& e) {
        throw Error(std::string("error generating labels: ") + e.what());
      }
    }
  }
  std::vector<LabelerPtr> labelers_;
};

}  // namespace

void move_labels(Labels& out, Labels&& from) {
  if (out.empty()) {
    out.swap(from);
    from.clear();
    return;
  }
  while (!from.empty()) {
    auto r = out.insert(from.extract(from.begin()));
    if (!r.inserted) r.position->second = std::move(r.node.mapped());  // later labels win
  }
}

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
