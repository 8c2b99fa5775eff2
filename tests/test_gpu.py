"""Real-hardware tests (MI355X).  Run with ``pytest -m gpu`` on the GPU box.

BASELINE.json configs 2-3: the amd-smi backend on real MI355X GPUs, full-GPU
amd.com/* labels, per-GPU count/memory/xGMI labels.  Every test drives the
native core (the _gfd extension or the daemon binary) - there is no Python
fallback.  The amd-smi and KFD-sysfs backends are cross-checked against
each other on the same node.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, TESTS, has_amd_gpu, run_daemon
from test_deployments import MANIFEST_PODS, check_manifest_run, manifest_pod
from gpu_feature_discovery_amd.utils import golden

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_amd_gpu(), reason="no /dev/kfd")]


@pytest.fixture(scope="module")
def amdsmi_devices(native):
    return native.Session(["--backend=amdsmi"]).devices()


@pytest.fixture(scope="module")
def sysfs_devices(native):
    return native.Session(["--backend=sysfs"]).devices()


def test_amdsmi_enumerates_mi355x(amdsmi_devices):
    assert amdsmi_devices, "amd-smi reported no GPU"
    for d in amdsmi_devices:
        assert d["gfx"] == "gfx950", d
        assert "MI355" in d["name"], d
        assert d["compute_units"] == 256, d
        assert d["xcds"] == 8, d
        assert 280 * 1024 <= d["memory_mib"] <= 300 * 1024, d  # 288 GB HBM3E
        assert d["compute_partition"] in ("SPX", "DPX", "QPX", "CPX"), d
        assert d["memory_partition"] in ("NPS1", "NPS2", "NPS4", "NPS8"), d
        assert 0 <= d["xgmi_links"] <= 7, d
        assert d["virtualization"] in ("baremetal", "host", "guest", "passthrough"), d
        assert d["vendor_id"] == 0x1002
        # Against the driver's own attributes, whatever mode the box is in
        # (the pool runs SPX/NPS1 and cannot switch; profiles/hw_probe.md).
        pci = f"/sys/bus/pci/devices/{d['bdf']}"
        mode = open(pci + "/current_compute_partition").read().strip().upper()
        assert d["compute_partition"] == mode, (d, mode)
        assert d["memory_partition"] == open(pci + "/current_memory_partition").read().strip().upper()
        assert d["partitioned"] == (mode != "SPX")
        assert len(d["partitions"]) == {"SPX": 0, "DPX": 2, "QPX": 4, "CPX": 8}[mode] or d["partitions"], d


def test_sysfs_backend_agrees_with_amdsmi(amdsmi_devices, sysfs_devices):
    assert len(sysfs_devices) == len(amdsmi_devices)
    keys = ("name", "bdf", "gfx", "compute_units", "xcds", "memory_mib", "compute_partition", "memory_partition",
            "partitioned", "partition_capable")
    for a, s in zip(amdsmi_devices, sysfs_devices):
        assert {k: a[k] for k in keys} == {k: s[k] for k in keys}


def test_amdsmi_sysfs_values_match_library_calls(native, amdsmi_devices):
    """An unpartitioned GPU's per-cycle values are read from the amdgpu
    attributes amd-smi itself reads; with that turned off (the bindings'
    test hook, amdsmi_library_only) every value comes from the library calls,
    and the devices and the label files must be identical."""
    lib = native.Session(["--backend=amdsmi"], amdsmi_library_only=True)
    assert lib.devices() == amdsmi_devices
    common = ["--backend=amdsmi", "--no-timestamp", "--output-file="]
    assert (native.Session(common, amdsmi_library_only=True).cycle(False)["labels"]
            == native.Session(common).cycle(False)["labels"])


def test_label_sets_identical_across_backends(native, tmp_path):
    common = ["--oneshot", "--no-timestamp", "--output-file="]
    a = native.Session(["--backend=amdsmi", *common]).cycle(False)["labels"]
    s = native.Session(["--backend=sysfs", *common]).cycle(False)["labels"]
    assert a == s


def test_daemon_amdsmi_oneshot_matches_regex_golden(binary, tmp_path):
    out = tmp_path / "gfd"
    cp = run_daemon(binary, "--oneshot", "--backend=amdsmi", f"--output-file={out}", "--trace-timing", check=True,
                    timeout=120)
    assert "Using amd-smi manager" in cp.stderr and "failed to initialize" not in cp.stderr
    text = out.read_text()
    golden.check_regex_golden(text, TESTS / "expected-output.txt", select=lambda ln: "sriov" not in ln)
    labels = golden.parse_labels(text)
    assert golden.k8s_label_problems(labels) == []
    assert labels["amd.com/gpu.arch"] == "gfx950"
    assert labels["amd.com/gpu.family"] == "cdna4"
    assert labels["amd.com/gpu.compute-units"] == "256"


def test_oneshot_auto_skips_amdsmi_with_identical_labels(binary, tmp_path):
    """Job mode (--oneshot, --backend=auto) reads the KFD topology and never
    loads amd-smi; its feature file is byte-identical to the amd-smi
    backend's, and the whole process stays under 4 ms (p50 of 15)."""
    import statistics

    files = {}
    for backend in ("auto", "amdsmi"):
        out = tmp_path / f"gfd-{backend}"
        cp = run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--output-file={out}",
                        check=True, timeout=120)
        files[backend] = out.read_text()
        if backend == "auto":
            assert "oneshot: amd-smi not loaded" in cp.stderr
            assert "amd-smi platform" not in cp.stderr
    assert files["auto"] == files["amdsmi"]
    from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms

    walls = [spawn_wait_ms([binary, "--oneshot", f"--output-file={tmp_path / 'gfd'}"]) for _ in range(15)]
    assert statistics.median(walls) < 4.0, walls  # measured 1.05-1.43 ms


def _daemon_files(binary, tmp_path, env_extra=None, until="", timeout=60):
    """Run the daemon loop (20 ms sleeps; the timestamp is fixed per run) and collect the
    feature file after every cycle until a log line containing `until` has
    been seen and one more cycle completed; returns (files, stderr)."""
    import signal
    import time

    out = tmp_path / "gfd"
    env = {k: v for k, v in os.environ.items() if not k.startswith("GFD_")}
    env.update(env_extra or {})
    p = subprocess.Popen([binary, "--sleep-interval=20ms", f"--output-file={out}"], env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    files, err, seen = [], [], False
    try:
        deadline = time.monotonic() + timeout
        for line in p.stderr:
            err.append(line)
            if "Sleeping for" in line:
                files.append(out.read_text())
                if seen:
                    break
            seen = seen or (until in line)
            if time.monotonic() > deadline:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        _, rest = p.communicate(timeout=30)
        err.append(rest or "")
    return files, "".join(err)


def test_auto_backend_falls_back_to_sysfs_on_hardware(binary, tmp_path):
    """An amd-smi library that loads but cannot initialise (the scriptable
    fake, told to fail amdsmi_init) on a real node: the auto backend of the
    daemon loop labels the GPU from the KFD topology instead, with the same
    label set."""
    fake = REPO / "build" / "libfake_amdsmi.so"
    files, err = _daemon_files(binary, tmp_path, {"GFD_AMDSMI_LIBRARY": str(fake),
                                                  "GFD_FAKE_AMDSMI_SPEC": "init_status=34"},
                               until="Using the sysfs manager")
    assert "Using the sysfs manager" in err, err[-3000:]
    golden.check_regex_golden(files[-1], TESTS / "expected-output.txt", select=lambda ln: "sriov" not in ln)
    assert golden.parse_labels(files[-1])["amd.com/gpu.arch"] == "gfx950"


def test_daemon_first_cycle_from_kfd_then_amdsmi_with_identical_labels(binary, tmp_path):
    """Daemon mode, --backend=auto on a real MI355X: the first cycle is
    labelled from the KFD topology while amd-smi initialises in the
    background (~25 ms); then amd-smi takes over.  Every feature file of the
    run - before and after the switch - is the same."""
    files, err = _daemon_files(binary, tmp_path, until="Using the amdsmi(persistent) manager")
    assert "labeling from the sysfs manager meanwhile" in err, err[-3000:]
    assert "Using the amdsmi(persistent) manager (initialized in the background" in err, err[-3000:]
    assert "failed to initialize" not in err
    assert "describes the GPUs differently" not in err, err[-3000:]  # the switch-over comparison
    assert len(files) >= 2
    assert all(f == files[0] for f in files), files
    golden.check_regex_golden(files[0], TESTS / "expected-output.txt", select=lambda ln: "sriov" not in ln)


@pytest.mark.parametrize("backend,ready", [("auto", "Using the amdsmi(persistent) manager"),
                                           ("amdsmi", "Start running"),
                                           ("amdsmi-per-cycle", "Start running"),
                                           ("sysfs", "Start running")])
def test_sleeping_daemon_holds_nothing_on_the_gpu(binary, tmp_path, backend, ready):
    """Between cycles the daemon is no GPU client.  The reference initialises
    NVML and shuts it down every cycle (internal/lm/nvml.go:30-33), so it
    holds nothing while it sleeps; here the amd-smi session stays
    initialised across cycles (persistent, the default).  While the loop
    sleeps (--sleep-interval=5s) - after the warm start switched to amd-smi
    for auto - the daemon holds no /dev/kfd or /dev/dri descriptor, maps
    neither, and KFD does not list it as a process: amd-smi's session keeps
    no device open between calls (measured r6, profiles/gpu_holds_r6.txt).
    A render node held would make it a DRM client with its own GPU VM, a KFD
    process one that amdgpu counts when it refuses a partition switch."""
    import signal

    from gpu_feature_discovery_amd.utils.proc import gpu_holds

    args = [binary, "--sleep-interval=5s", f"--output-file={tmp_path / 'gfd'}"]
    if backend == "amdsmi-per-cycle":
        args += ["--backend=amdsmi", "--amdsmi-session=per-cycle"]
    else:
        args.append(f"--backend={backend}")
    env = {k: v for k, v in os.environ.items() if not k.startswith("GFD_")}
    p = subprocess.Popen(args, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    seen, holds, err = False, None, []
    try:
        for line in p.stderr:
            err.append(line)
            seen = seen or ready in line
            if seen and "Sleeping for" in line:
                import time

                time.sleep(0.5)  # well inside the sleep
                holds = gpu_holds(p.pid)
                break
    finally:
        p.send_signal(signal.SIGTERM)
        _, rest = p.communicate(timeout=30)
        err.append(rest or "")
    assert holds is not None, "".join(err)[-3000:]
    assert p.returncode == 0, "".join(err)[-3000:]
    assert holds["device_fds"] == {}, holds
    assert holds["device_maps"] == [], holds
    assert not holds["kfd_process"], holds


def test_daemon_sysfs_backend_oneshot(binary, tmp_path):
    out = tmp_path / "gfd"
    run_daemon(binary, "--oneshot", "--backend=sysfs", f"--output-file={out}", check=True, timeout=60)
    golden.check_regex_golden(out.read_text(), TESTS / "expected-output.txt", select=lambda ln: "sriov" not in ln)


def test_persistent_session_initialises_once(native):
    s = native.Session(["--backend=amdsmi", "--output-file="])
    phases = [dict(s.cycle(False)["phases"]) for _ in range(5)]
    assert "amdsmi_init" in phases[0]
    assert all("amdsmi_init" not in p for p in phases[1:])


def test_per_cycle_session_reinitialises(native):
    s = native.Session(["--backend=amdsmi", "--amdsmi-session=per-cycle", "--output-file="])
    phases = [dict(s.cycle(False)["phases"]) for _ in range(3)]
    assert all("amdsmi_init" in p for p in phases)
    labels = [s.cycle(False)["labels"] for _ in range(2)]
    labels[0].pop("amd.com/gfd.timestamp"), labels[1].pop("amd.com/gfd.timestamp")
    assert labels[0] == labels[1]


def test_visible_devices_filter(native, amdsmi_devices):
    bdf = amdsmi_devices[0]["bdf"]
    only = native.Session(["--backend=amdsmi", f"--visible-devices={bdf}"]).devices()
    assert [d["bdf"] for d in only] == [bdf]
    none = native.Session(["--backend=amdsmi", "--visible-devices=63"]).devices()
    assert none == []


def test_real_pci_scan_succeeds(native, amdsmi_devices):
    """The SR-IOV scan on the box: it must find the allocated GPU's physical
    function (an SR-IOV capable PF on the pool) and, as its VFs are not
    enabled (sriov_numvfs 0, bare metal), emit no amd.com/sriov.* label -
    the reference's vGPU labeler is silent on a passthrough GPU the same way
    (internal/vgpu/vgpu_test.go:36-74).  On an SR-IOV node the labels must
    match the SR-IOV golden instead."""
    r = native.Session(["--backend=sysfs", "--output-file="]).cycle(False)
    assert "sriov(overlapped)" in dict(r["phases"])
    sriov = {k: v for k, v in r["labels"].items() if "sriov" in k}
    for d in amdsmi_devices:
        pf = f"/sys/bus/pci/devices/{d['bdf']}"
        assert os.path.exists(pf + "/vendor"), pf
        assert open(pf + "/vendor").read().strip() == "0x1002"
        numvfs = open(pf + "/sriov_numvfs").read().strip() if os.path.exists(pf + "/sriov_numvfs") else "0"
        if d["virtualization"] == "baremetal" and numvfs == "0":
            assert sriov == {}, sriov
    if sriov:
        golden.check_regex_golden("".join(f"{k}={v}\n" for k, v in sorted(sriov.items())),
                                  TESTS / "expected-output-sriov.txt")
    assert r["labels"]["amd.com/gpu.virtualization-mode"] == amdsmi_devices[0]["virtualization"]


def test_bound_sriov_source_matches_the_whole_bus_on_the_box(native, amdsmi_devices):
    """Round 4 reads SR-IOV state only from the functions amdgpu / gim bind
    (plus their VFs) instead of every function on the bus.  On the real
    host - 8 MI355X bound to amdgpu, ~370 PCI functions, the allocated GPU
    among them - both sources must hand the labeler the same functions,
    field for field, and the bound one must be much cheaper."""
    import time

    def timed(source):
        t0 = time.perf_counter()
        r = native.pci_functions("/", source)
        return r, (time.perf_counter() - t0) * 1e3

    bus, bus_ms = timed("bus")
    bound, bound_ms = timed("bound")
    assert bound == bus, (bound, bus)
    addrs = {f["address"] for f in bound}
    for d in amdsmi_devices:
        assert d["bdf"] in addrs, (d["bdf"], addrs)
    print(f"bound {len(bound)} functions in {bound_ms:.3f} ms, whole bus {bus_ms:.3f} ms")


def test_vf_links_are_the_pfs_numvfs_on_the_box():
    """The SR-IOV check after an unrelated uevent counts a PF's VFs by its
    virtfn* links instead of reading sriov_numvfs (src/sriov/bound.cpp).
    On the real host every amdgpu/gim-bound PF with an SR-IOV capability
    must have exactly sriov_numvfs links."""
    checked = 0
    for drv in ("amdgpu", "gim"):
        d = f"/sys/bus/pci/drivers/{drv}"
        if not os.path.isdir(d):
            continue
        for name in os.listdir(d):
            pf = os.path.join(d, name)
            if ":" not in name or not os.path.exists(os.path.join(pf, "sriov_totalvfs")):
                continue
            with open(os.path.join(pf, "sriov_numvfs")) as f:
                numvfs = int(f.read())
            links = [e for e in os.listdir(pf) if e.startswith("virtfn")]
            assert len(links) == numvfs, (pf, numvfs, links)
            checked += 1
    print(f"{checked} SR-IOV PFs checked")


def test_kept_partition_mode_lists_match_the_driver_every_cycle(native):
    """The supported compute / memory partition modes are read once per
    amd-smi session (AmdSmiManager::available_): cycle after cycle they must
    still be what amdgpu reports."""
    s = native.Session(["--backend=amdsmi", "--no-timestamp", "--output-file="])
    for _ in range(4):
        s.cycle(False)
        for d in s.devices():
            pci = f"/sys/bus/pci/devices/{d['bdf']}"
            for attr, key in (("available_compute_partition", "available_compute_partitions"),
                              ("available_memory_partition", "available_memory_partitions")):
                path = os.path.join(pci, attr)
                if not os.path.exists(path):
                    continue
                with open(path) as f:
                    want = [m.strip() for m in f.read().split(",") if m.strip()]
                assert d[key] == want, (d["bdf"], attr, d[key], want)


def _kfd_gpu_nodes():
    """(properties text) of every readable GPU node of the KFD topology."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    out = []
    for n in sorted(os.listdir(base), key=lambda x: int(x) if x.isdigit() else -1):
        try:
            with open(f"{base}/{n}/properties") as f:
                text = f.read()
        except OSError:
            continue
        props = dict(ln.split(" ", 1) for ln in text.splitlines() if " " in ln)
        if int(props.get("simd_count", "0")) > 0:
            out.append(props)
    return out


@pytest.mark.parametrize("backend", ["amdsmi", "sysfs"])
def test_compute_partition_read_once_and_agrees_with_the_driver(native, backend):
    """current_compute_partition makes amdgpu read an XCP register, which can
    wake the GPU (AMD's CLI stopped reading it by default,
    /opt/rocm/libexec/amdsmi_cli/amdsmi_commands.py:463-466): the daemon
    reads it when the session starts or the KFD generation changes, not on
    steady cycles (no "compute_partition(read)" record after the first).
    The kept mode agrees with the attribute read now, with the library's own
    getter, and with the KFD topology: in SPX one node holds all of the GPU's
    XCDs."""
    s = native.Session([f"--backend={backend}", "--no-timestamp", "--output-file="])
    reads = []
    for _ in range(5):
        r = s.cycle(False)
        reads.append(sum(1 for name, _ in r["phases"] if name == "compute_partition(read)"))
    assert reads[0] >= 1 and reads[1:] == [0, 0, 0, 0], reads
    nodes = _kfd_gpu_nodes()
    for d in s.devices():
        with open(f"/sys/bus/pci/devices/{d['bdf']}/current_compute_partition") as f:
            live = f.read().strip()
        assert d["compute_partition"] == live, (d["bdf"], d["compute_partition"], live)
        if live == "SPX":
            loc = int(d["bdf"][5:7], 16) << 8 | int(d["bdf"][8:10], 16) << 3 | int(d["bdf"][11], 16)
            node = [n for n in nodes if int(n["location_id"]) == loc]
            assert len(node) == 1 and int(node[0]["num_xcc"]) == d["xcds"], (d["bdf"], node, d["xcds"])
    if backend == "amdsmi":
        lib = native.Session(["--backend=amdsmi", "--no-timestamp", "--output-file="], amdsmi_library_only=True)
        assert [d["compute_partition"] for d in lib.devices()] == [d["compute_partition"] for d in s.devices()]


def test_idle_cycles_on_hardware_are_attributed_and_create_no_file(binary, tmp_path):
    """The deployed daemon (auto backend) with idle time between cycles, on
    the real node: every cycle's named phases account for all but a few
    microseconds of it (round-3 verdict: 0.369 ms of a 0.683 ms cycle were
    unnamed), and every write after the second rewrites the old feature
    file instead of creating one."""
    import signal
    import statistics

    from test_daemon import TOP_LEVEL, _timing_fields

    out = tmp_path / "features.d" / "gfd"
    p = subprocess.Popen([binary, "--sleep-interval=300ms", "--trace-timing", f"--output-file={out}"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                         env={k: v for k, v in os.environ.items() if not k.startswith("GFD_")})
    rows = []
    try:
        for line in p.stderr:
            if "Timing:" in line:
                rows.append(_timing_fields(line))
                if len(rows) >= 8:
                    break
    finally:
        p.send_signal(signal.SIGTERM)
        p.communicate(timeout=30)
    assert len(rows) == 8
    for r in rows:
        assert abs(sum(v for k, v in r.items() if k in TOP_LEVEL) + r["other"] - r["total"]) <= 0.013, r
    assert statistics.median(r["other"] for r in rows[1:]) <= 0.02, rows
    assert all("write.reuse" in r and "write.create" not in r for r in rows[2:]), rows


def test_auto_backend_switch_with_library_values_keeps_the_labels(native):
    """The daemon's default backend (auto) labels its first cycles from the
    KFD topology and then from amd-smi; with the amd-smi backend's own sysfs
    shortcuts off (amdsmi_library_only: every value through the library
    calls), the label file must not change across the switch."""
    import time

    s = native.Session(["--backend=auto", "--no-timestamp", "--output-file="], amdsmi_library_only=True)
    first = s.cycle(False)
    assert s.backend == "sysfs", s.backend
    for _ in range(500):
        if s.backend.startswith("amdsmi"):
            break
        time.sleep(0.01)
        s.cycle(False)
    assert s.backend.startswith("amdsmi"), s.backend
    after = s.cycle(False)
    assert after["rendered"] == first["rendered"]


def test_product_name_survives_torch_libdrm(tmp_path):
    """PyTorch ships a libdrm whose amdgpu.ids path does not exist; with it
    loaded first, amd-smi's market name degrades to "AMD Radeon Graphics".
    The backend must still report the board's product name."""
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import torch\n"
        "torch.cuda.is_available()\n"
        "import gpu_feature_discovery_amd as g\n"
        "print(g.native().Session(['--backend=amdsmi']).devices()[0]['name'])\n" % str(REPO)
    )
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert cp.returncode == 0, cp.stderr[-2000:]
    assert "MI355" in cp.stdout.strip().splitlines()[-1]


def test_amdsmi_without_libdrm_labels_identically(binary, tmp_path):
    """amd-smi dlopens libdrm_amdgpu for the marketing-name table.  A slim
    runtime image may lack it: emulated here with a copy of libamd_smi whose
    libdrm_amdgpu soname is altered (same length) so the dlopen fails.  The
    library must still initialise and the feature file must not change."""
    import glob

    libs = sorted(glob.glob("/opt/rocm/lib/libamd_smi.so.*.*"))
    if not libs:
        pytest.skip("no versioned libamd_smi under /opt/rocm/lib")
    blob = open(libs[-1], "rb").read()
    name = b"libdrm_amdgpu.so.1\x00"
    assert name in blob
    patched = tmp_path / "libamd_smi.so"
    patched.write_bytes(blob.replace(name, b"libdrm_amdgpX.so.1\x00"))
    files = {}
    for lib in (libs[-1], str(patched)):
        out = tmp_path / "gfd"
        cp = run_daemon(binary, "--oneshot", "--no-timestamp", "--backend=amdsmi", f"--output-file={out}",
                        env={"GFD_AMDSMI_LIBRARY": lib}, check=True, timeout=120)
        assert "Using amd-smi manager" in cp.stderr, cp.stderr[-2000:]
        files[lib] = out.read_text()
    with_drm, without = golden.parse_labels(files[libs[-1]]), golden.parse_labels(files[str(patched)])
    assert without == with_drm, {k: (with_drm.get(k), without.get(k)) for k in set(with_drm) | set(without)
                                 if with_drm.get(k) != without.get(k)}
    assert "MI355" in without["amd.com/gpu.product"]


def test_bench_contract_on_gpu(tmp_path):
    cp = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "20", "--warmup", "2", "--no-extras"],
                        capture_output=True, text=True, timeout=600, cwd=str(REPO))
    assert cp.returncode == 0, cp.stderr[-2000:]
    line = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["labels_ok"] is True, r
    assert r["config"]["backend"].startswith("amdsmi")
    assert r["higher_is_better"] is False and r["unit"] == "ms"
    assert r["value"] > 0 and r["n_gpus"] == 1


def _bench_json(args: list[str], env: dict | None = None, timeout: float = 600) -> dict:
    cp = subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                        timeout=timeout, cwd=str(REPO), env=env)
    assert cp.returncode == 0, cp.stderr[-2000:]
    return json.loads([ln for ln in cp.stdout.splitlines() if ln.startswith("{")][-1])


def _within_bounds(measure, bounds) -> None:
    """Run `measure`, check every (name, value_of, limit) bound; if any is
    exceeded, measure once more and require the second run to meet all of
    them - a real drift fails both runs, one noisy run of a shared box does
    not fail the suite (round-5 advice)."""
    first = measure()
    over = [(name, f(first), lim) for name, f, lim in bounds if f(first) > lim]
    if not over:
        return
    print("over its bounds on the first run, measuring again:", over)
    second = measure()
    over2 = [(name, f(second), lim) for name, f, lim in bounds if f(second) > lim]
    assert not over2, (over, over2)


def test_driver_bench_command_stays_within_its_bounds(tmp_path):
    """The driver's own command (bench.py --gpus 1 --steps 20 --warmup 5):
    a drift of the headline or of the deployed cadence's cycle fails here,
    not three rounds later in the driver's records (round-4 verdict: 0.021 ->
    0.0251 -> 0.0288 ms went unnoticed).  Bounds (round-5 verdict, Next #5:
    a +25% drift must fail): headline 0.016 ms (round 6's final code
    0.0116-0.0125 on its boxes, profiles/bench_fresh_r6.txt; a 20-step p50
    on a shared box strays up to 0.015 now and then, hence the margin),
    cycles 1 s apart 0.28 ms (0.17-0.22), their unattributed time 0.02 ms; the Job
    process: its fastest of 15 spawns 1.15 ms (0.778-0.928 on the round-6
    boxes, +24 % over the slowest) - the p50 of 15 spawns right after the idle second cycles is
    bimodal on some boxes (spawns of 0.8 or 1.5-1.9 ms, the slow ones on
    idle cores: p50 0.799-1.538, profiles/bench_fresh_r6.txt), so it is
    bounded only against gross drift, 2.0 ms; and no write after the second
    creates a file.  A run over a bound is repeated once (_within_bounds)."""

    def measure():
        r = _bench_json(["--gpus", "1", "--steps", "20", "--warmup", "5"])
        print(json.dumps({k: r[k] for k in ("value", "p90_ms", "first_cycle_ms", "oneshot_process_p50_ms")}),
              json.dumps({"job_runs_ms": r["extras"]["oneshot_process"]["runs_ms"]}),
              json.dumps({"cold": r["cold_cycle"]["p50_ms"], "cold_other": r["cold_cycle"]["other_p50_ms"]}))
        assert r["labels_ok"] is True and r["config"]["backend"].startswith("amdsmi"), r
        assert "write.create" not in r["phases_p50_ms"], r["phases_n"]
        return r

    _within_bounds(measure, [("headline_ms", lambda r: r["value"], 0.016),
                             ("cold_p50_ms", lambda r: r["cold_cycle"]["p50_ms"], 0.28),
                             ("cold_other_ms", lambda r: r["cold_cycle"]["other_p50_ms"], 0.02),
                             ("job_fastest_ms", lambda r: min(r["extras"]["oneshot_process"]["runs_ms"]), 1.15),
                             ("job_p50_ms", lambda r: r["oneshot_process_p50_ms"], 2.0)])


def test_amdsmi_backend_over_all_the_hosts_gpus(tmp_path):
    """The 8-GPU node the daemon is built for, as close as a one-GPU box gets:
    the fake libamd_smi reports every MI355X of the host at its real PCI
    address (tools/hybrid_amdsmi_spec.py), so the amd-smi backend's per-GPU
    lanes read each GPU's live amdgpu attributes.  The label set must be
    right for all of them and a back-to-back cycle stay within 0.022 ms."""
    fake = REPO / "build" / "libfake_amdsmi.so"
    spec = subprocess.run([sys.executable, str(REPO / "tools" / "hybrid_amdsmi_spec.py")], capture_output=True, text=True)
    if spec.returncode != 0 or not fake.exists():
        pytest.skip("no MI355X in sysfs or fake library not built")
    n = min(8, spec.stdout.count("bdf="))
    if n < 2:
        pytest.skip("one GPU on this host")
    env = {**os.environ, "GFD_AMDSMI_LIBRARY": str(fake), "GFD_FAKE_AMDSMI_SPEC": spec.stdout.strip()}

    def measure():
        r = _bench_json(["--gpus", str(n), "--backend", "amdsmi", "--steps", "2000", "--warmup", "200", "--no-extras"],
                        env=env, timeout=300)
        print(json.dumps({k: r[k] for k in ("n_gpus", "value", "p90_ms", "p99_ms", "labels_ok")}))
        assert r["labels_ok"] is True and r["n_gpus"] == n, r.get("label_problems")
        return r

    # Round-5 verdict, Next #5: a +25% drift fails - 0.022 ms at 8 GPUs
    # against round 6's final 0.0164-0.0166 (2000-step p50s, stable;
    # profiles/hybrid_amdsmi_scaling_r6.txt).
    _within_bounds(measure, [("hybrid_%d_gpu_ms" % n, lambda r: r["value"], 0.022)])


def test_smoke_entry_point():
    cp = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], capture_output=True, text=True,
                        timeout=300, cwd=str(REPO), env={**os.environ})
    assert cp.returncode == 0, cp.stderr[-2000:]
    assert "smoke:" in cp.stdout


AMD_SMI_CLI = "/opt/rocm/bin/amd-smi"


def _amd_smi_json(*args: str):
    cp = subprocess.run([AMD_SMI_CLI, *args, "--json"], capture_output=True, text=True, timeout=180)
    assert cp.returncode == 0, cp.stderr[-2000:]
    return json.loads(cp.stdout)


@pytest.mark.skipif(not os.path.exists(AMD_SMI_CLI), reason="amd-smi CLI not installed")
def test_devices_match_amd_smi_cli(amdsmi_devices, sysfs_devices):
    """Independent oracle: AMD's own `amd-smi` tool (a separate Python
    program over the same library) must report the same facts the labels
    are built from, for both backends."""
    static = {g["bus"]["bdf"]: g for g in _amd_smi_json("static")["gpu_data"]}
    listed = {g["bdf"]: g for g in _amd_smi_json("list")}
    part = _amd_smi_json("partition")
    current = {p["gpu_id"]: p for p in part["current_partition"]}
    memcaps = {p["gpu_id"]: p for p in part["memory_partition"]}
    ports = {p["bdf"]: p["link_status"] for p in _amd_smi_json("xgmi")["link_port_status"]}
    assert set(static) == {d["bdf"] for d in amdsmi_devices}
    for backend in (amdsmi_devices, sysfs_devices):
        for d in backend:
            s = static[d["bdf"]]
            gpu = s["gpu"]
            assert d["name"] in (s["asic"]["market_name"], s["board"]["product_name"]), (d["name"], s["asic"])
            assert d["device_id"] == int(s["asic"]["device_id"], 16)
            assert d["vendor_id"] == int(s["asic"]["vendor_id"], 16)
            assert d["gfx"] == s["asic"]["target_graphics_version"]
            assert d["memory_mib"] == s["vram"]["size"]["value"] and s["vram"]["size"]["unit"] == "MB"
            assert d["uuid"] == listed[d["bdf"]]["uuid"]
            assert d["compute_partition"] == current[gpu]["accelerator_type"]
            assert d["memory_partition"] == current[gpu]["memory"] == memcaps[gpu]["current_memory_partition"]
            assert d["available_memory_partitions"] == [m.strip() for m in
                                                        memcaps[gpu]["memory_partition_caps"].split(",")]
            assert d["xgmi_links"] == sum(1 for x in ports[d["bdf"]] if x == "U")
            if d["compute_partition"] == "SPX":
                assert d["compute_units"] == s["asic"]["num_compute_units"]


@pytest.mark.skipif(not os.path.exists(AMD_SMI_CLI), reason="amd-smi CLI not installed")
def test_version_labels_match_amd_smi_cli(binary, tmp_path):
    """The version labels against AMD's tool: amd.com/driver.* is the amdgpu
    version `amd-smi static --driver` reports and amd.com/rocm.runtime.* the
    ROCm version `amd-smi version` reports, for both backends."""
    import re

    data = _amd_smi_json("static", "--driver")
    gpus = data["gpu_data"] if isinstance(data, dict) else data
    drivers = {str(g["driver"]["version"]) for g in gpus if isinstance(g.get("driver"), dict)}
    ver = _amd_smi_json("version")
    ver = ver[0] if isinstance(ver, list) else ver
    rocm = str(ver.get("rocm_version", ""))
    print("amd-smi: driver", drivers, "rocm", rocm)
    assert len(drivers) == 1, drivers
    want_driver = [int(x) for x in re.findall(r"\d+", drivers.pop())[:3]]
    want_rocm = [int(x) for x in re.findall(r"\d+", rocm)[:2]]
    for backend in ("amdsmi", "sysfs"):
        out = tmp_path / f"gfd-{backend}"
        run_daemon(binary, "--oneshot", f"--backend={backend}", f"--output-file={out}", check=True, timeout=120)
        labels = golden.parse_labels(out.read_text())
        got = [int(labels[f"amd.com/driver.{k}"]) for k in ("major", "minor", "rev") if f"amd.com/driver.{k}" in labels]
        assert len(got) >= 2 and got == want_driver[:len(got)], (backend, got, want_driver)
        if len(want_rocm) == 2:  # this amd-smi reports the ROCm release
            assert [int(labels["amd.com/rocm.runtime.major"]), int(labels["amd.com/rocm.runtime.minor"])] == want_rocm


def test_devices_match_the_hip_runtime(amdsmi_devices, sysfs_devices):
    """A third oracle, independent of amd-smi: the HIP runtime, as PyTorch-ROCm
    reports each visible GPU (its own path through the KFD thunk), in a
    separate process - loading it changes what amd-smi reads in this one
    (test_product_name_survives_torch_libdrm).  Architecture, compute units
    and device memory must be the ones the labels are built from."""
    code = (
        "import json, torch\n"
        "out = []\n"
        "for i in range(torch.cuda.device_count()):\n"
        "    p = torch.cuda.get_device_properties(i)\n"
        "    out.append({'bdf': '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id),\n"
        "                'arch': p.gcnArchName, 'cus': p.multi_processor_count, 'mem': p.total_memory,\n"
        "                'warp': p.warp_size})\n"
        "print(json.dumps(out))\n"
    )
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert cp.returncode == 0, cp.stderr[-2000:]
    hip = {g["bdf"]: g for g in json.loads(cp.stdout.strip().splitlines()[-1])}
    print("hip runtime:", hip)
    assert set(hip) == {d["bdf"] for d in amdsmi_devices}
    for backend in (amdsmi_devices, sysfs_devices):
        for d in backend:
            h = hip[d["bdf"]]
            assert h["arch"].split(":")[0] == d["gfx"], (h, d["gfx"])
            assert h["warp"] == 64
            if d["compute_partition"] == "SPX":
                assert h["cus"] == d["compute_units"], (h, d["compute_units"])
                assert h["mem"] // (1 << 20) == d["memory_mib"], (h, d["memory_mib"])


def test_attribute_descriptors_kept_open_and_stable(native):
    """Per-cycle sysfs attributes are read through descriptors kept open
    across cycles (pread at offset 0 re-runs the driver's show()): after a
    few cycles the process holds descriptors on the GPU's amdgpu attributes,
    their number does not grow, and the labels do not change."""
    s = native.Session(["--backend=amdsmi", "--no-timestamp", "--output-file="])
    first = s.cycle(False)["labels"]

    def sysfs_fds():
        out = []
        for fd in os.listdir("/proc/self/fd"):
            try:
                target = os.readlink(f"/proc/self/fd/{fd}")
            except OSError:
                continue
            if target.startswith("/sys/"):
                out.append(target)
        return sorted(out)

    before = sysfs_fds()
    for _ in range(50):
        assert s.cycle(False)["labels"] == first
    after = sysfs_fds()
    assert any(t.endswith("/current_compute_partition") for t in after), after
    assert any(t.endswith("/mem_info_vram_total") for t in after), after
    assert len(after) == len(before), (before, after)


def test_eight_gpu_node_from_live_attributes(binary, tmp_path):
    """BASELINE config 3 (8xMI355X SPX/NPS1) from a one-GPU box: the host's
    other seven GPUs' KFD nodes are not readable here, but every GPU's
    amdgpu PCI attributes are (sysfs is not namespaced).  tools/hybrid_root.py
    builds a root whose PCI tree is the live one and whose KFD topology
    repeats the allocated GPU's node at each GPU's address; the labels must
    describe all of the host's MI355X from their live attributes."""
    root = tmp_path / "hybrid"
    cp = subprocess.run([sys.executable, str(REPO / "tools" / "hybrid_root.py"), str(root)], capture_output=True,
                        text=True, timeout=60)
    assert cp.returncode == 0, cp.stderr
    n = int(cp.stdout.strip())
    assert n >= 1
    for visible, want in (("", n), (f"0-{min(n, 4) - 1}", min(n, 4))):
        out = tmp_path / f"gfd-{want}"
        run_daemon(binary, "--oneshot", "--no-timestamp", "--backend=sysfs", f"--sysfs-root={root}",
                   f"--machine-type-file={root}/sys/class/dmi/id/product_name", f"--visible-devices={visible}",
                   f"--output-file={out}", check=True, timeout=60)
        labels = golden.parse_labels(out.read_text())
        assert labels["amd.com/gpu.count"] == str(want), labels
        assert "MI355" in labels["amd.com/gpu.product"]
        assert labels["amd.com/gpu.memory"] == "294896"
        assert labels["amd.com/gpu.compute-partition"] == "SPX"
        assert labels["amd.com/gpu.memory-partition"] == "NPS1"
        assert labels["amd.com/gpu.xgmi.links"] == "7"  # minimum over the GPUs: every one has its 7 hive links


@pytest.mark.parametrize("var", ["ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                 "GPU_DEVICE_ORDINAL"])
def test_runtime_visibility_masks_do_not_hide_gpus(binary, tmp_path, var):
    """A node labeler describes the node, not the GPUs a runtime mask leaves
    to one process: a pod that inherits a device plugin's or user's
    visibility variable (pointing at a GPU that does not exist) still labels
    every GPU, through amd-smi and KFD alike (profiles/env_probe.txt)."""
    files = {}
    for backend in ("amdsmi", "sysfs"):
        out = tmp_path / f"gfd-{backend}"
        run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--output-file={out}",
                   env={var: "63"}, check=True, timeout=120)
        files[backend] = out.read_text()
    assert files["amdsmi"] == files["sysfs"]
    assert int(golden.parse_labels(files["amdsmi"])["amd.com/gpu.count"]) >= 1


def test_daemon_pins_itself_to_one_l3_domain_only_when_asked(binary, tmp_path):
    """CPU placement: by default (follow) the process is not pinned - only
    the pool's workers are kept on the labeling thread's L3 domain; with
    --cpu-affinity=l3 (GFD_CPU_AFFINITY=l3) every thread stays on the CPUs
    sharing one L3 cache (util/affinity.h), within the allowed set.
    (Started with every CPU of the box allowed.)"""
    def run(env):
        def widen():
            os.sched_setaffinity(0, range(os.cpu_count()))  # the kernel keeps the cgroup's share

        e = {k: v for k, v in os.environ.items() if not k.startswith("GFD_")}
        e.update(env)
        return subprocess.run([binary, "--oneshot", "--backend=null", "--output-file="], capture_output=True,
                              text=True, timeout=60, env=e, preexec_fn=widen, check=True)

    default = run({}).stderr
    assert "sharing cpu" not in default and "workers follow" in default
    assert "CPU affinity:" not in run({"GFD_CPU_AFFINITY": "none"}).stderr
    on = run({"GFD_CPU_AFFINITY": "l3"})
    lines = [ln for ln in on.stderr.splitlines() if "CPU affinity:" in ln]
    assert len(lines) == 1, on.stderr[-2000:]
    assert "sharing cpu" in lines[0] and "L3 cache" in lines[0], lines[0]


# ---- The deployment manifests' own argv / env / mounts on the MI355X -------

def _box_rocm() -> str:
    text = open(os.path.realpath("/opt/rocm/.info/version")).read().strip()
    return ".".join(text.split("-")[0].split(".")[:2])


@pytest.mark.parametrize("name,source,strategy", MANIFEST_PODS, ids=[m[0] for m in MANIFEST_PODS])
def test_manifest_pod_labels_the_real_node(native, image, tmp_path, name, source, strategy):
    """The stand-in for the reference's container integration test
    (tests/integration-tests.py:36-78): each manifest's labeler container -
    static DaemonSets, the Job template, the Helm chart's defaults - run with
    exactly its argv and environment, its hostPath mounts reproduced (the
    box's real /sys at /sys; a copy of the box's /opt/rocm/.info/version
    under the --host-root mount).  The labels must match the regex golden in
    both directions and carry the box's ROCm release; the DaemonSet must
    remove its file on SIGTERM."""
    import manifest_pods

    pod = manifest_pod(native, source)
    croot = tmp_path / "container"
    manifest_pods.materialise(pod, croot)
    r = manifest_pods.run(pod, image, croot, timeout=120)
    check_manifest_run(r, pod, strategy, _box_rocm())
    if pod.env.get("GFD_BACKEND", "auto") == "auto" and pod.kind == "DaemonSet":
        assert "failed to initialize" not in r["stderr"], r["stderr"][-3000:]


def test_image_labels_the_real_node_with_its_own_libraries(binary, image, tmp_path):
    """The image (the Dockerfile's runtime stage, tests/e2e/fakes/_image.py)
    on the MI355X with the amd-smi backend: amd-smi and the libdrm_amdgpu it
    loads for the marketing names come from the image (its COPY --from=build
    and apt-get lines), nothing from the host's library directories, and the
    labels equal the in-tree build's."""
    sys.path.insert(0, str(TESTS / "e2e" / "fakes"))
    import _image

    args = ["--oneshot", "--backend=amdsmi", "--no-timestamp", "--host-root=/"]
    trace = tmp_path / "ld"
    argv, env = _image.command(image, [*args, f"--output-file={tmp_path / 'image'}"], {}, base=dict(os.environ),
                               trace=trace)
    cp = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=60)
    assert cp.returncode == 0, cp.stderr[-3000:]
    run_daemon(binary, *args, f"--output-file={tmp_path / 'host'}", check=True)
    assert (tmp_path / "image").read_text() == (tmp_path / "host").read_text()
    loaded = _image.loaded_objects(trace)
    for lib in ("libamd_smi.so*", "libdrm_amdgpu.so*"):
        assert [o for o in _image.matches(loaded, lib) if o.startswith(str(image))], (lib, loaded)
    assert not _image.foreign_libraries(image, trace)


# ---- tests/e2e scripts (the reference's integration / e2e tests) on the node -

def test_integration_script_on_the_real_node(tmp_path):
    """tests/e2e/integration_docker.py as it is, its `docker run` served by
    the fake runtime (tests/e2e/fakes): the labeler with the host's real
    /sys and /opt, labels checked against the regex golden."""
    from test_e2e_scripts import assert_ran_from_the_image, e2e_env, run_integration, stop_all

    env = e2e_env(tmp_path)
    try:
        cp = run_integration(env, "none", timeout=120)
    finally:
        stop_all(env)
    assert cp.returncode == 0, cp.stdout + cp.stderr
    assert "integration test passed" in cp.stdout and "amd.com/gpu.arch=gfx950" in cp.stdout
    assert_ran_from_the_image(env)


def test_e2e_script_on_the_real_node(tmp_path):
    """tests/e2e/e2e_kubectl.py as it is, against the fake one-node cluster
    on the real MI355X: NFD's PCI source must match the node (class 0x12
    whitelisted) for the DaemonSet to schedule, and its local source must
    publish the amd.com labels."""
    from test_e2e_scripts import assert_ran_from_the_image, e2e_env, run_e2e, stop_all

    env = e2e_env(tmp_path)
    try:
        cp = run_e2e(env, timeout=150)
    finally:
        stop_all(env)
    assert cp.returncode == 0, cp.stdout + cp.stderr
    assert "e2e test passed" in cp.stdout and '"amd.com/gpu.family": "cdna4"' in cp.stdout
    assert_ran_from_the_image(env)


def test_helm_chart_installs_on_the_real_node(tmp_path):
    """The Helm chart's defaults rendered (tests/helm_lite.py) and applied to
    the fake one-node cluster backed by the real MI355X: NFD's PCI source
    must see the GPU for the DaemonSet to schedule, and the published
    amd.com labels must describe it."""
    from test_e2e_scripts import e2e_env, helm_install, stop_all, wait_for_node_labels

    env = e2e_env(tmp_path)
    try:
        cp = helm_install(env, tmp_path)
        assert cp.returncode == 0, cp.stderr
        labels = wait_for_node_labels(env, timeout=90)
    finally:
        stop_all(env)
    assert labels.get("feature.node.kubernetes.io/pci-1002.present") == "true", labels
    assert labels.get("amd.com/gpu.arch") == "gfx950" and labels.get("amd.com/gpu.family") == "cdna4", labels
