"""The labeler image's runtime stage, assembled offline from
deployments/container/Dockerfile - the stand-in for `docker build` that the
fake `docker` and `kubectl` (this directory) and tests/manifest_pods.py run.

There is no image builder or registry here or on the GPU box, and no
ubuntu:22.04 base to pull.  What the runtime stage's instructions say is
interpreted instead, into a directory tree (the image's root file system):

* FROM ubuntu:<ver>: the base image's shared libraries - every shared object
  of the packages an Ubuntu base image is made of (Priority required or
  Essential, plus apt), with their dependencies, taken from this machine's
  dpkg database (the same Ubuntu release: the build stage's FROM image is
  this one);
* RUN apt-get install PKG...: the packages' files and their dependencies'
  (only the apt-get line is interpreted; the rest of that RUN is cleanup);
* COPY --from=build SRC DST: SRC from the build stage - this machine, with
  the stage's WORKDIR (/src, filled by `COPY . .`) being the repository and
  its build/ the in-tree build of the same CMake project;
* COPY SRC DST: from the build context (the repository);
* ENV / ENTRYPOINT: what `command()` runs.

`command()` starts the ENTRYPOINT through the image's own dynamic loader
with the image's library directories as the search path and the loader
cache off.  Without a mount namespace the loader's last resort is still the
host's system directories, so a library the image lacks would be found
there: `foreign_libraries()` reads the loader's trace of a run and names
every object that came from the host's library directories, and the tests
require that list to be empty.  Likewise an absolute path the daemon opens
(/sys, /opt/rocm/...) is the host's: the manifests' hostPath mounts are
reproduced by the callers, who re-root the path settings.
"""

from __future__ import annotations

import fcntl
import fnmatch
import glob
import hashlib
import json
import os
import re
import shlex
import shutil
import subprocess
from pathlib import Path

REPO = Path(__file__).resolve().parents[3]
DOCKERFILE = REPO / "deployments" / "container" / "Dockerfile"
HOST_LIB_DIRS = ("/lib/", "/lib64/", "/usr/lib/", "/usr/lib64/", "/opt/")
DEFAULT_DEST = Path(os.environ.get("TMPDIR", "/tmp")) / "gfd-image"
LIB_DIRS = ("lib/x86_64-linux-gnu", "usr/lib/x86_64-linux-gnu", "lib", "usr/lib", "lib64")


def _stages(text: str, build_args: dict[str, str] | None = None) -> list[dict]:
    """The Dockerfile's stages: name, base and (instruction, argument) list,
    ARGs substituted (`build_args` over the declared defaults)."""
    text = re.sub(r"\\\n", " ", text)
    args: dict[str, str] = dict(build_args or {})
    stages: list[dict] = []

    def subst(s: str) -> str:
        return re.sub(r"\$\{(\w+)\}|\$(\w+)", lambda m: args.get(m.group(1) or m.group(2), m.group(0)), s)

    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        ins, _, rest = line.partition(" ")
        ins = ins.upper()
        if ins == "ARG":
            k, _, v = rest.strip().partition("=")
            args.setdefault(k, v)
            continue
        if ins == "FROM":
            parts = subst(rest).split()
            stages.append({"base": parts[0], "name": parts[2] if len(parts) > 2 else None, "steps": []})
            continue
        stages[-1]["steps"].append((ins, subst(rest.strip())))
    return stages


def _packages() -> dict[str, list[str]]:
    """Installed packages and their (first-alternative) dependencies."""
    out = subprocess.run(["dpkg-query", "-W", "-f=${Package}\t${Priority}\t${Essential}\t${Depends}, ${Pre-Depends}\n"],
                         capture_output=True, text=True, check=True).stdout
    deps: dict[str, list[str]] = {}
    base: list[str] = []
    for line in out.splitlines():
        name, prio, ess, dep = line.split("\t")
        deps[name] = [re.split(r"[\s(:]", alt.split("|")[0].strip())[0] for alt in dep.split(",") if alt.strip()]
        if prio == "required" or ess == "yes" or name == "apt":
            base.append(name)
    deps["__base__"] = base
    return deps


def _closure(roots: list[str], deps: dict[str, list[str]]) -> list[str]:
    seen: list[str] = []
    todo = list(roots)
    while todo:
        p = todo.pop()
        if p in seen or p not in deps:
            continue
        seen.append(p)
        todo.extend(deps[p])
    return seen


def _files_of(pkg: str) -> list[str]:
    cp = subprocess.run(["dpkg-query", "-L", pkg], capture_output=True, text=True)
    return [f for f in cp.stdout.splitlines() if f.startswith("/")]


def _is_shared_object(path: str) -> bool:
    base = os.path.basename(path)
    return base.startswith("ld-linux") or ".so" in base and any(path.startswith("/" + d + "/") for d in LIB_DIRS)


def _place(src: str, root: Path, dst: str) -> None:
    """Copy `src` to root/dst; a symbolic link stays one, its absolute target
    made relative so that it resolves inside the image."""
    target = root / dst.lstrip("/")
    if target.exists() or target.is_symlink():
        return
    if os.path.isdir(src) and not os.path.islink(src):
        return
    target.parent.mkdir(parents=True, exist_ok=True)
    if os.path.islink(src):
        link = os.readlink(src)
        if os.path.isabs(link):
            link = os.path.relpath(root / link.lstrip("/"), target.parent)
        target.symlink_to(link)
        real = os.path.join(os.path.dirname(src), os.readlink(src))
        _place(os.path.normpath(real), root, os.path.normpath(os.path.join(os.path.dirname(dst), os.readlink(src))))
    elif os.path.isfile(src):
        shutil.copy2(src, target)


def _usr_merge(root: Path) -> None:
    """ubuntu:22.04 is usr-merged: /lib, /lib64, /bin and /sbin are links into /usr."""
    for d in ("lib", "lib64", "bin", "sbin"):
        (root / "usr" / d).mkdir(parents=True, exist_ok=True)
        link = root / d
        if not link.exists() and not link.is_symlink():
            link.symlink_to("usr/" + d)


def _install(pkgs: list[str], root: Path, deps: dict[str, list[str]], libs_only: bool) -> None:
    for p in _closure(pkgs, deps):
        for f in _files_of(p):
            if libs_only and not _is_shared_object(f):
                continue
            _place(f, root, f)


def _copy(src_pattern: str, dst: str, src_root: Path, root: Path) -> None:
    srcs = sorted(glob.glob(str(src_root / src_pattern.lstrip("/")))) if any(c in src_pattern for c in "*?[") \
        else [str(src_root / src_pattern.lstrip("/"))]
    if not srcs or not all(os.path.lexists(s) for s in srcs):
        # docker build fails the same way: a COPY source must exist, and a
        # wildcard must match something.
        raise FileNotFoundError(f"COPY {src_pattern}: nothing at {src_root}")
    for s in srcs:
        d = os.path.join(dst, os.path.basename(s)) if dst.endswith("/") else dst
        _place(s, root, d)


def _map_build_path(path: str, workdir: str | None, src: Path) -> tuple[str, Path]:
    """Where a build-stage path is: under its WORKDIR, `src` (the stage's
    `COPY . .` and what its RUN built there); anywhere else, this machine."""
    if workdir and (path == workdir or path.startswith(workdir.rstrip("/") + "/")):
        return path[len(workdir.rstrip("/")):], src
    return path, Path("/")


def _ignore_patterns(context: Path) -> list[re.Pattern]:
    """.dockerignore's patterns (no `!` exceptions: this one has none)."""
    f = context / ".dockerignore"
    out = []
    for line in (f.read_text().splitlines() if f.exists() else []):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("!"):
            raise ValueError(".dockerignore exceptions are not emulated")
        rx = re.escape(line.strip("/")).replace(r"\*\*/", "(.*/)?").replace(r"\*", "[^/]*").replace(r"\?", "[^/]")
        out.append(re.compile(rx + "$"))
    return out


def context_files(context: Path = REPO) -> list[str]:
    """The build context `docker build` would send: every file under
    `context` (relative paths) that .dockerignore does not exclude; an
    excluded directory excludes everything under it."""
    pats = _ignore_patterns(context)
    out = []
    for d, dirs, files in os.walk(context):
        rel = os.path.relpath(d, context)
        rel = "" if rel == "." else rel + "/"
        dirs[:] = [x for x in dirs if not any(p.match(rel + x) for p in pats)]
        out += [rel + f for f in files if not any(p.match(rel + f) for p in pats)]
    return sorted(out)


def run_build_stage(work: Path, log=print, build_args: dict[str, str] | None = None) -> Path:
    """Run the Dockerfile's build stage: the build context copied to
    work/<WORKDIR> (`COPY . .`), then each RUN there, package installs
    skipped (no network; this machine is the stage's base image).  Raises
    on the first failing step; returns the WORKDIR."""
    stages = _stages(DOCKERFILE.read_text(), build_args)
    stage = next(s for s in stages if s["name"] == "build")
    src = work
    for ins, arg in stage["steps"]:
        if ins == "WORKDIR":
            src = work / arg.lstrip("/")
            src.mkdir(parents=True, exist_ok=True)
        elif ins == "COPY":
            if arg.split() != [".", "."]:
                raise ValueError(f"COPY {arg} in the build stage is not emulated")
            for rel in context_files():
                (src / rel).parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(REPO / rel, src / rel, follow_symlinks=False)
        elif ins == "RUN":
            steps = [c.strip() for c in arg.split("&&")]
            steps = [c for c in steps if not c.startswith(("apt-get", "rm -rf /var/lib/apt"))]
            if not steps:
                continue
            cmd = " && ".join(steps)
            log(f"RUN {cmd}")
            subprocess.run(["bash", "-e", "-c", cmd], cwd=src, check=True)
        elif ins in ("ARG", "ENV", "LABEL"):
            pass
        else:
            raise ValueError(f"{ins} in the build stage is not emulated")
    return src


def _key(src: Path) -> str:
    h = hashlib.sha256(DOCKERFILE.read_bytes())
    for f in (src / "build" / "gpu-feature-discovery", Path("/opt/rocm/lib")):
        st = f.stat()
        h.update(f"{f}:{st.st_mtime_ns}:{st.st_size}".encode())
    return h.hexdigest()[:16]


def build(dest: Path = DEFAULT_DEST, build_src: Path = REPO) -> Path:
    """Assemble the runtime stage under `dest` (reused while the Dockerfile,
    the daemon binary and the ROCm libraries are unchanged; concurrent
    builders wait for each other); returns the image's root.  The build
    stage's WORKDIR is `build_src`: by default the repository with its
    in-tree build, or what `run_build_stage` produced."""
    dest.mkdir(parents=True, exist_ok=True)
    root = dest / f"rootfs-{_key(build_src)}"
    with open(dest / ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not (root / ".complete").exists():
            for old in dest.glob("rootfs-*"):
                shutil.rmtree(old, ignore_errors=True)
            _assemble(root, build_src)
    return root


def _assemble(root: Path, build_src: Path) -> None:
    stages = _stages(DOCKERFILE.read_text())
    build_stage = next(s for s in stages if s["name"] == "build")
    workdir = next((a for i, a in build_stage["steps"] if i == "WORKDIR"), None)
    stage = stages[-1]
    root.mkdir(parents=True)
    _usr_merge(root)
    deps = _packages()
    if not stage["base"].startswith("ubuntu:"):
        raise ValueError(f"runtime stage FROM {stage['base']}: only ubuntu bases are emulated")
    _install(deps["__base__"], root, deps, libs_only=True)
    env: dict[str, str] = {}
    entry: list[str] = []
    for ins, arg in stage["steps"]:
        if ins == "RUN":
            m = re.search(r"apt-get install ([^&;]+)", arg)
            if not m:
                raise ValueError(f"RUN {arg!r}: only apt-get install is emulated")
            pkgs = [w for w in shlex.split(m.group(1)) if not w.startswith("-")]
            missing = [p for p in pkgs if p not in deps]
            if missing:
                raise ValueError(f"RUN apt-get install: {missing} not installed on this machine")
            _install(pkgs, root, deps, libs_only=False)
        elif ins == "COPY":
            words = shlex.split(arg)
            frm = next((w.split("=", 1)[1] for w in words if w.startswith("--from=")), None)
            words = [w for w in words if not w.startswith("--")]
            *srcs, dst = words
            for s in srcs:
                if frm == "build":
                    path, src_root = _map_build_path(s, workdir, build_src)
                    _copy(path, dst, src_root, root)
                elif frm is None:
                    _copy(s, dst, REPO, root)
                else:
                    raise ValueError(f"COPY --from={frm}: unknown stage")
        elif ins == "ENV":
            for w in shlex.split(arg):
                k, _, v = w.partition("=")
                env[k] = v
        elif ins == "ENTRYPOINT":
            entry = json.loads(arg)
        elif ins in ("LABEL", "WORKDIR", "USER", "EXPOSE"):
            pass
        else:
            raise ValueError(f"{ins} in the runtime stage is not emulated")
    (root / ".image.env").write_text("\n".join(f"{k}={v}" for k, v in env.items()))
    (root / ".image.entrypoint").write_text("\n".join(entry))
    (root / ".complete").write_text("")


def command(root: Path, args: list[str], env: dict[str, str], base: dict[str, str],
            trace: Path | None = None) -> tuple[list[str], dict]:
    """argv and environment that start the image's ENTRYPOINT with `args`:
    the image's loader, the image's library directories only.  The
    environment is `base` (the calling process's), then the image's ENV,
    then `env` (the container's own); the image's path settings are
    re-rooted into the image.  With `trace`, the loader writes its library
    trace to trace.<pid>."""
    ienv = dict(base)
    ienv.update(line.split("=", 1) for line in (root / ".image.env").read_text().splitlines() if line)
    entry = (root / ".image.entrypoint").read_text().splitlines()
    ienv.update(env)
    lib_path = [str(root) + p for p in ienv.get("LD_LIBRARY_PATH", "").split(":") if p]
    lib_path += [str(root / d) for d in LIB_DIRS]
    if "ROCM_PATH" in ienv:
        ienv["ROCM_PATH"] = str(root) + ienv["ROCM_PATH"]
    ienv["LD_LIBRARY_PATH"] = ":".join(lib_path)
    if trace is not None:
        ienv["LD_DEBUG"] = "libs"
        ienv["LD_DEBUG_OUTPUT"] = str(trace)
    loader = root / "lib64" / "ld-linux-x86-64.so.2"
    argv = [str(loader), "--inhibit-cache", "--library-path", ":".join(lib_path), str(root) + entry[0], *entry[1:],
            *args]
    return argv, ienv


def loaded_objects(trace_prefix: Path) -> list[str]:
    """Every object the loader initialised, from the trace files of a run."""
    objs: list[str] = []
    for f in sorted(glob.glob(str(trace_prefix) + ".*")):
        for line in Path(f).read_text(errors="replace").splitlines():
            m = re.search(r"calling init: (\S+)", line)
            if m and m.group(1) not in objs:
                objs.append(m.group(1))
    return objs


def foreign_libraries(root: Path, trace_prefix: Path) -> list[str]:
    """Objects of a run that came from the host's library directories rather
    than the image (objects the environment preloads live elsewhere)."""
    r = str(root) + "/"
    return [o for o in loaded_objects(trace_prefix) if not o.startswith(r) and o.startswith(HOST_LIB_DIRS)]


def matches(objs: list[str], pattern: str) -> list[str]:
    return [o for o in objs if fnmatch.fnmatch(os.path.basename(o), pattern)]
