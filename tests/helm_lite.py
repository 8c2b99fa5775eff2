"""A small renderer for the Go-template subset the in-repo NFD subchart uses
(deployments/helm/gpu-feature-discovery-amd/charts/nfd-minimal), so the
chart's default install can be rendered and checked without helm (not in
this image, and no network to fetch it):

* ``{{ .Values.a.b }}``, ``{{ .Release.Name }}``, ``{{ .Release.Namespace }}``
* ``{{ toYaml <path> | nindent N }}``
* ``{{- range <path> }} ... {{ . }} ... {{- end }}``
* ``{{-`` / ``-}}`` whitespace trimming

Anything else raises, so a template that grows past this subset fails the
test instead of rendering wrongly.
"""

from __future__ import annotations

import re

import yaml

_ACTION = re.compile(r"{{(-?)\s*(.*?)\s*(-?)}}", re.S)


def _lookup(path: str, ctx: dict, dot):
    if path == ".":
        return dot
    if not path.startswith("."):
        raise ValueError(f"unsupported expression {path!r}")
    node = ctx
    for part in path[1:].split("."):
        if not isinstance(node, dict) or part not in node:
            raise KeyError(f"{path}: no {part!r}")
        node = node[part]
    return node


def _scalar(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _tokens(text: str):
    pos = 0
    for m in _ACTION.finditer(text):
        lit = text[pos:m.start()]
        if m.group(1):
            lit = lit.rstrip()
        yield "text", lit
        yield "action", m.group(2)
        pos = m.end()
        if m.group(3):
            while pos < len(text) and text[pos] in " \t\r\n":
                pos += 1
    yield "text", text[pos:]


def _render(toks: list, i: int, ctx: dict, dot, out: list[str], stop_at_end: bool) -> int:
    while i < len(toks):
        kind, val = toks[i]
        i += 1
        if kind == "text":
            out.append(val)
            continue
        if val == "end":
            if not stop_at_end:
                raise ValueError("unexpected {{ end }}")
            return i
        if val.startswith("range "):
            items = _lookup(val[6:].strip(), ctx, dot)
            start = i
            if not items:  # skip the body
                i = _render(toks, start, ctx, dot, [], True)
            for item in items or []:
                i = _render(toks, start, ctx, item, out, True)
            continue
        m = re.fullmatch(r"toYaml\s+(\S+)\s*\|\s*nindent\s+(\d+)", val)
        if m:
            data = _lookup(m.group(1), ctx, dot)
            pad = " " * int(m.group(2))
            dumped = yaml.safe_dump(data, default_flow_style=False, sort_keys=False).rstrip("\n")
            out.append("\n" + "\n".join(pad + ln for ln in dumped.splitlines()))
            continue
        out.append(_scalar(_lookup(val, ctx, dot)))
    if stop_at_end:
        raise ValueError("missing {{ end }}")
    return i


def render(text: str, values: dict, release_name: str = "gfd", namespace: str = "gpu-feature-discovery") -> str:
    ctx = {"Values": values, "Release": {"Name": release_name, "Namespace": namespace}}
    out: list[str] = []
    _render(list(_tokens(text)), 0, ctx, None, out, False)
    return "".join(out)


def merge(base: dict, override: dict) -> dict:
    """Helm's value coalescing: maps merge key by key, anything else replaces."""
    out = dict(base)
    for k, v in override.items():
        out[k] = merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out
