#!/usr/bin/env python3
"""Mutation check of tests/test_differential.py: in a copy of the tree
(built in place there), remove one kept fact's invalidation at a time,
rebuild and run the differential test; it must fail for each.

    python tools/differential_mutations.py COPY_DIR [M1 M2 ...]

COPY_DIR: a scratch copy of the repository (e.g. `git worktree add`), built
once with `make build`.  Results: profiles/differential_mutations_r6.txt.
(Round 6: M5 was the supported-mode lists keyed by the current modes -
unobservable, deleted; it is now the session's compute mode.  M11 and M12
are new; M11 applies to VMs, the only nodes whose bus the SR-IOV source
reads.  M10 and M13 guard the ROCm version kept under a directory watch, M14 the kept
SR-IOV classification.)
"""
import os
import subprocess
import sys

os.chdir(sys.argv[1])
M = [
 ("M1 SR-IOV result kept across uevents", "src/sriov/bound.cpp", "if (have_ && seqnum && *seqnum == seqnum_) {", "if (have_) {"),
 ("M2 SR-IOV check ignores the driver listing", "src/sriov/bound.cpp", "if (!have_ || fell_back_ || bound != bound_ || unbound != unbound_) return false;", "if (!have_ || fell_back_ || unbound != unbound_) return false;"),
 ("M3 SR-IOV check ignores VF links", "src/sriov/bound.cpp", "    if (d.sriov_totalvfs <= 0) continue;\n    // The kernel links", "    continue;\n    // The kernel links"),
 ("M4 amd-smi identity kept across re-init", "src/resource/amdsmi.cpp", "  identity_.clear();\n", ""),
 ("M5 amd-smi compute partition mode kept across re-init", "src/resource/amdsmi.cpp", "  compute_mode_.clear();\n", ""),
 ("M6 amdgpu module directory never reopened", "src/resource/versions.cpp", 'if (!d || d->lookup("initstate") != 0) d =', 'if (!d) d ='),
 ("M7 sysfs topology kept across generations", "src/resource/sysfs.cpp", "if (!generation_.empty() && generation_ == cached_generation_ && cached_) {", "if (cached_) {"),
 ("M8 amd-smi session kept across generations", "src/resource/amdsmi.cpp", "    if (gen != generation_) {", "    if (false) {"),
 ("M9 DMI kept for any file", "src/util/fs.cpp", "  kept->emplace(path, constant ? std::optional<std::string>(r.data) : std::nullopt);", "  kept->emplace(path, std::optional<std::string>(r.data));"),
 ("M11 SR-IOV check ignores the bus's unbound functions (VMs)", "src/sriov/bound.cpp", "bound != bound_ || unbound != unbound_) return false;", "bound != bound_) return false;"),
 ("M12 amd-smi session values kept across re-init", "src/resource/amdsmi.cpp", "  session_values_.clear();\n", ""),
 ("M10 ROCm version kept without its directory watch", "src/resource/versions.cpp", "if (k->valid && k->watch.unchanged()) {", "if (k->valid) {"),
 ("M14 SR-IOV classification kept after the source re-read", "src/sriov/sriov.cpp", "    if (!pci_->DevicesIfChanged(&devices)) {", "    if (!pci_->DevicesIfChanged(&devices) || have_) {"),
 ("M13 ROCm version lookup watches no directory behind a symlink", "src/util/fs.cpp", "    if (dirs) {\n      std::string parent", "    if (dirs && links == 0) {\n      std::string parent"),
]
sel = sys.argv[2:] or [m[0].split()[0] for m in M]
for name, f, a, b in M:
    if name.split()[0] not in sel: continue
    src = open(f).read()
    assert a in src, (name, a)
    open(f, 'w').write(src.replace(a, b, 1))
    try:
        r = subprocess.run("cmake --build build -j8 > /tmp/mut_b.log 2>&1 && GFD_DIFF_SEQUENCES=200 timeout 600 python -m pytest tests/test_differential.py -x -q 2>&1 | tail -30",
                           shell=True, capture_output=True, text=True)
        out = r.stdout
        verdict = "CAUGHT" if "1 failed" in out else ("MISSED" if "1 passed" in out else "BUILD/OTHER")
        hint = ""
        for line in out.splitlines():
            if "AssertionError: sequence" in line:
                hint = line.strip()[:200]
        print(f"{name}: {verdict} {hint}", flush=True)
    finally:
        open(f, 'w').write(src)
subprocess.run("cmake --build build -j8 > /tmp/mut_b.log 2>&1", shell=True)
