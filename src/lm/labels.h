// Label model, labeler composition and the NFD feature-file writer.
//
// Reference: internal/lm/labels.go:29-114 (Labels, WriteToFile, WriteTo,
// writeFileAtomically), labeler.go:28-30 (Labeler), list.go:22-46 (Merge:
// later labelers override earlier ones), empty.go:20-24.
//
// Differences by design:
//   * Labels is an ordered map, so the feature file is written sorted by key
//     and is byte-for-byte reproducible (the reference writes in Go's random
//     map order, labels.go:57), which is what makes golden files possible.
//   * Values are sanitised to valid Kubernetes label values (<=63 chars of
//     [A-Za-z0-9._-], alphanumeric at both ends); the reference only replaces
//     spaces, so a DMI string like "Server (X)" would be rejected by NFD.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace gfd::lm {

using Labels = std::map<std::string, std::string>;

class Labeler {
 public:
  virtual ~Labeler() = default;
  virtual Labels GetLabels() = 0;
  // Adds this labeler's labels to `out` (overriding same keys) - what a
  // merge does with each of its labelers, without an intermediate map.
  virtual void AppendTo(Labels& out) {
    for (auto& kv : GetLabels()) out[kv.first] = std::move(kv.second);
  }
  // AppendTo for a labeler used once (a cycle's own): fixed labels are moved
  // into `out` - map nodes and all - instead of copied; the labeler is left
  // empty.  Other labelers append as usual.
  virtual void MoveTo(Labels& out) { AppendTo(out); }
};
using LabelerPtr = std::shared_ptr<Labeler>;

// Moves every label of `from` into `out`, overriding same keys (map nodes
// are moved, not copied); `from` is left empty.
void move_labels(Labels& out, Labels&& from);

// A fixed set of labels (Labels implements Labeler in the reference).
LabelerPtr from_labels(Labels l);
// The null labeler.
LabelerPtr empty();
// Composite: evaluates in order, later keys win; errors are wrapped as
// "error generating labels: <inner>".
LabelerPtr merge(std::vector<LabelerPtr> labelers);

// "key=value\n" per label, sorted by key.
std::string render(const Labels& labels);

// Write labels to `path` atomically (temp file in <dir>/gfd-tmp, rename,
// 0644).  An empty path writes to stdout.  Throws gfd::Error.
//
// `reuse` (loop mode): the write swaps the new file with the old feature file
// (renameat2 RENAME_EXCHANGE) and keeps the old one, under its temporary
// name, to be rewritten by the next write to `path` - once a write lease
// (F_SETLEASE) shows that no reader still has it open; otherwise, or where
// leases are not available, the next write creates a new file as a oneshot
// write does.  So a daemon's steady cycles create, unlink and evict no file.
// Only on local file systems (reuse_is_safe): the lease check sees only this
// kernel's openers, so on a shared or network file system a reader on
// another machine could read a half-rewritten file; there every write
// creates a new file, as the reference always does.
void write_to_file(const Labels& labels, const std::string& path, bool reuse = false);
// Whether the file system of `fd` is one where a write lease sees every
// reader: a local one (ext4, xfs, btrfs, tmpfs, overlayfs).
bool reuse_is_safe(int fd);
// Atomic write of arbitrary contents (labels.go:68-114).
void write_file_atomically(const std::string& path, const std::string& contents, unsigned perm);
// Closes and removes every file kept for reuse (a session that ends).
void release_kept_files();
// The same for the files kept for one output path only (one of several
// sessions in a process ends); the feature file itself stays.
void release_kept_files(const std::string& path);
// Start-up: removes <dir>/gfd-tmp left by a process that did not exit
// cleanly (one GFD per node writes there, as the reference assumes).
void sweep_temp_dir(const std::string& path);
// Removes <dir>/gfd-tmp and the output file (main.go:212-232).
void remove_output_file(const std::string& path);

// Kubernetes label-value sanitiser: spaces and invalid characters become
// '-' (so "AMD Instinct MI355X" -> "AMD-Instinct-MI355X" exactly like the
// reference's space replacement), the result is truncated to 63 characters
// and trimmed to alphanumeric ends.
std::string sanitize_label_value(const std::string& v);

}  // namespace gfd::lm
