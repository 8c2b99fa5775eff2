"""A small Go-template interpreter for rendering this repository's Helm chart
(deployments/helm/gpu-feature-discovery-amd, with its in-repo NFD subchart)
without helm, which is not in this image (and there is no network to fetch
it).  It implements what the chart's templates use, and raises on anything
else, so a template that grows past it fails the tests instead of rendering
wrongly:

* actions with ``{{-`` / ``-}}`` trimming, comments, ``if/else if/else``,
  ``with/else``, ``range`` (with ``$v :=`` / ``$k, $v :=``), ``define`` /
  ``include``, variables (``$x := ...``, ``$x = ...``), pipelines, parenthesised
  sub-pipelines, field chains on ``.``, ``$`` and variables;
* the sprig/Helm functions the chart calls: ``default``, ``trunc``,
  ``trimSuffix``, ``ternary``, ``printf``, ``contains``, ``dict``, ``list``,
  ``keys``, ``sortAlpha``, ``get``, ``has``, ``kindIs``, ``toString``,
  ``quote``, ``merge``, ``sha256sum``, ``replace``, ``toYaml``, ``indent``,
  ``nindent``, ``fail``, ``and``, ``or``, ``not``, ``eq``, ``ne``.

``render_chart`` renders every manifest template of a chart (and of its
enabled file:// dependencies) the way ``helm template`` does for one release.
"""

from __future__ import annotations

import hashlib
import json
import re
from pathlib import Path

import yaml


class HelmFail(Exception):
    """The template called ``fail`` (or an unsupported construct was met)."""


# ---------------------------------------------------------------------------
# Lexing and parsing

_ACTION = re.compile(r"{{(-?)(\s*)(.*?)(\s*)(-?)}}", re.S)


def _lex(text: str):
    out, pos = [], 0
    for m in _ACTION.finditer(text):
        lit = text[pos:m.start()]
        if m.group(1) == "-":
            lit = lit.rstrip(" \t\r\n")
        out.append(("text", lit))
        body = m.group(3)
        if not (body.startswith("/*") and body.endswith("*/")):
            out.append(("action", body))
        pos = m.end()
        if m.group(5) == "-":
            while pos < len(text) and text[pos] in " \t\r\n":
                pos += 1
    out.append(("text", text[pos:]))
    return out


_TOKEN = re.compile(r"""\s*(?:
    (?P<str>"(?:[^"\\]|\\.)*") |
    (?P<raw>`[^`]*`) |
    (?P<num>-?\d+(?:\.\d+)?) |
    (?P<assign>:=|=) |
    (?P<pipe>\|) |
    (?P<lp>\() | (?P<rp>\)) |
    (?P<comma>,) |
    (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*) |
    (?P<field>(?:\.[A-Za-z0-9_]+)+|\.) |
    (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
    )""", re.X)


def _tokens(expr: str) -> list[tuple[str, str]]:
    out, pos = [], 0
    expr = expr.strip()
    while pos < len(expr):
        m = _TOKEN.match(expr, pos)
        if not m or m.end() == pos:
            raise HelmFail(f"cannot parse {expr[pos:]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


def _parse(toks: list, i: int, stop: tuple) -> tuple[list, int, str | None]:
    """Nodes until an action in `stop` (its keyword returned) or the end."""
    nodes = []
    while i < len(toks):
        kind, val = toks[i]
        i += 1
        if kind == "text":
            if val:
                nodes.append(("text", val))
            continue
        word = val.split(None, 1)[0] if val else ""
        if word in stop or (word == "else" and "else" in stop):
            return nodes, i, val
        if word in ("if", "with", "range"):
            body, i, end = _parse(toks, i, ("end", "else"))
            node = [word, val[len(word):].strip(), body, []]
            if end and end.startswith("else"):
                rest = end[4:].strip()
                if rest.startswith("if ") or rest.startswith("with "):
                    # `else if` / `else with`: a nested block sharing our {{ end }}
                    kw = rest.split(None, 1)[0]
                    sub, i, end2 = _parse(toks, i, ("end", "else"))
                    inner = [kw, rest[len(kw):].strip(), sub, []]
                    if end2 and end2.startswith("else"):
                        inner[3], i, _ = _parse(toks, i, ("end",))
                    node[3] = [tuple(inner)]
                else:
                    node[3], i, _ = _parse(toks, i, ("end",))
            nodes.append(tuple(node))
            continue
        if word == "define":
            name = json.loads(val[len("define"):].strip())
            body, i, _ = _parse(toks, i, ("end",))
            nodes.append(("define", name, body))
            continue
        if word in ("end", "else"):
            raise HelmFail(f"unexpected {{{{ {val} }}}}")
        nodes.append(("action", val))
    if stop:
        raise HelmFail(f"missing {{{{ end }}}} (want {stop})")
    return nodes, i, None


# ---------------------------------------------------------------------------
# Values and functions


def _truthy(v) -> bool:
    return not (v is None or v is False or v == 0 and not isinstance(v, bool) or v == "" or v == [] or v == {})


def _to_string(v) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return json.dumps(v, separators=(",", ":"))
    return str(v)


def _quote(s: str) -> str:
    return json.dumps(s)  # Go %q for the strings the chart quotes


def _printf(fmt: str, *args) -> str:
    out, ai = [], 0

    def sub(m):
        nonlocal ai
        verb = m.group(1)
        if verb == "%":
            return "%"
        a = args[ai]
        ai += 1
        return _quote(_to_string(a)) if verb == "q" else _to_string(a)

    out = re.sub(r"%([sdvq%])", sub, fmt)
    return out


def _kind(v) -> str:
    if v is None:
        return "invalid"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, dict):
        return "map"
    if isinstance(v, list):
        return "slice"
    return type(v).__name__


def _merge(dst: dict, *srcs: dict) -> dict:
    """sprig merge: keys already in dst win (deeply)."""
    for src in srcs:
        for k, v in (src or {}).items():
            if k not in dst:
                dst[k] = v
            elif isinstance(dst[k], dict) and isinstance(v, dict):
                _merge(dst[k], v)
    return dst


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _fail(msg):
    raise HelmFail(msg)


FUNCS = {
    "default": lambda d, v=None: v if _truthy(v) else d,
    "trunc": lambda n, s: s[:n],
    "trimSuffix": lambda suf, s: s[: -len(suf)] if suf and s.endswith(suf) else s,
    "ternary": lambda a, b, c: a if _truthy(c) else b,
    "printf": _printf,
    "contains": lambda sub, s: sub in s,
    "dict": lambda *kv: {kv[i]: kv[i + 1] for i in range(0, len(kv), 2)},
    "list": lambda *xs: list(xs),
    "keys": lambda d: list(d.keys()),
    "sortAlpha": lambda xs: sorted(_to_string(x) for x in xs),
    "get": lambda d, k: d.get(k, ""),
    "has": lambda item, xs: item in (xs or []),
    "kindIs": lambda kind, v: _kind(v) == kind,
    "toString": _to_string,
    "quote": lambda *xs: " ".join(_quote(_to_string(x)) for x in xs),
    "merge": _merge,
    "sha256sum": lambda s: hashlib.sha256(s.encode()).hexdigest(),
    "replace": lambda old, new, s: s.replace(old, new),
    "toYaml": _to_yaml,
    "indent": lambda n, s: "\n".join(" " * n + ln for ln in s.split("\n")),
    "nindent": lambda n, s: "\n" + "\n".join(" " * n + ln for ln in s.split("\n")),
    "fail": _fail,
    "not": lambda v: not _truthy(v),
    "and": lambda *xs: next((x for x in xs if not _truthy(x)), xs[-1]),
    "or": lambda *xs: next((x for x in xs if _truthy(x)), xs[-1]),
    "eq": lambda a, *bs: any(a == b for b in bs),
    "ne": lambda a, b: a != b,
}


class _Env:
    def __init__(self, root, defines: dict):
        self.root = root
        self.defines = defines

    # -- expressions --
    def _field(self, base, chain: str):
        v = base
        for part in [p for p in chain.split(".") if p]:
            if isinstance(v, dict):
                v = v.get(part)
            else:
                return None
        return v

    def _operand(self, toks, i, dot, vars_):
        kind, val = toks[i]
        if kind == "lp":
            depth, j = 1, i + 1
            while depth:
                if toks[j][0] == "lp":
                    depth += 1
                elif toks[j][0] == "rp":
                    depth -= 1
                j += 1
            return self.pipeline(toks[i + 1:j - 1], dot, vars_), j
        if kind == "str":
            return json.loads(val), i + 1
        if kind == "raw":
            return val[1:-1], i + 1
        if kind == "num":
            return (float(val) if "." in val else int(val)), i + 1
        if kind == "field":
            return (dot if val == "." else self._field(dot, val)), i + 1
        if kind == "var":
            name, _, chain = val.partition(".")
            if name == "$":
                base = self.root
            elif name in vars_:
                base = vars_[name]
            else:
                raise HelmFail(f"undefined variable {name}")
            return self._field(base, chain) if chain else base, i + 1
        if kind == "ident" and val in ("true", "false"):
            return val == "true", i + 1
        if kind == "ident" and val == "nil":
            return None, i + 1
        if kind == "ident" and val in FUNCS:  # a function as an argument: called with no arguments
            return FUNCS[val](), i + 1
        raise HelmFail(f"unexpected {val!r}")

    def _command(self, toks, dot, vars_, piped, has_piped):
        kind, val = toks[0]
        if kind == "ident" and val not in ("true", "false", "nil"):
            args, i = [], 1
            while i < len(toks):
                a, i = self._operand(toks, i, dot, vars_)
                args.append(a)
            if has_piped:
                args.append(piped)
            if val == "include":
                return self.include(args[0], args[1])
            if val not in FUNCS:
                raise HelmFail(f"unsupported function {val}")
            return FUNCS[val](*args)
        v, i = self._operand(toks, 0, dot, vars_)
        if i != len(toks) or has_piped:
            raise HelmFail(f"cannot apply {toks}")
        return v

    def pipeline(self, toks, dot, vars_):
        cmds, cur, depth = [], [], 0
        for t in toks:
            if t[0] == "lp":
                depth += 1
            elif t[0] == "rp":
                depth -= 1
            if t[0] == "pipe" and depth == 0:
                cmds.append(cur)
                cur = []
            else:
                cur.append(t)
        cmds.append(cur)
        v, has = None, False
        for c in cmds:
            v = self._command(c, dot, vars_, v, has)
            has = True
        return v

    def expr(self, text, dot, vars_):
        toks = _tokens(text)
        if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] == "assign":
            v = self.pipeline(toks[2:], dot, vars_)
            vars_[toks[0][1]] = v
            return None
        return self.pipeline(toks, dot, vars_)

    # -- execution --
    def include(self, name, data):
        if name not in self.defines:
            raise HelmFail(f"no template {name!r}")
        out: list[str] = []
        self.run(self.defines[name], data, {}, out)
        return "".join(out)

    def run(self, nodes, dot, vars_, out):
        for n in nodes:
            kind = n[0]
            if kind == "text":
                out.append(n[1])
            elif kind == "action":
                v = self.expr(n[1], dot, vars_)
                if v is not None or not re.match(r"\s*\$\w+\s*:?=", n[1]):
                    out.append(_to_string(v))
            elif kind == "define":
                continue
            elif kind == "if":
                branch = n[2] if _truthy(self.expr(n[1], dot, vars_)) else n[3]
                self.run(branch, dot, vars_, out)
            elif kind == "with":
                v = self.expr(n[1], dot, vars_)
                if _truthy(v):
                    self.run(n[2], v, vars_, out)
                else:
                    self.run(n[3], dot, vars_, out)
            elif kind == "range":
                head = n[1]
                names = []
                m = re.match(r"(\$\w+)(?:\s*,\s*(\$\w+))?\s*:=\s*(.*)", head, re.S)
                if m:
                    names = [x for x in (m.group(1), m.group(2)) if x]
                    head = m.group(3)
                items = self.expr(head, dot, vars_)
                seq = list(items.items()) if isinstance(items, dict) else list(enumerate(items or []))
                if not seq:
                    self.run(n[3], dot, vars_, out)
                for k, v in seq:
                    inner = dict(vars_)
                    if len(names) == 1:
                        inner[names[0]] = v
                    elif len(names) == 2:
                        inner[names[0]], inner[names[1]] = k, v
                    self.run(n[2], v, inner, out)
            else:
                raise HelmFail(f"unknown node {kind}")


def _collect_defines(nodes, into: dict):
    for n in nodes:
        if n[0] == "define":
            into[n[1]] = n[2]


def render(text: str, values: dict, release_name: str = "gfd", namespace: str = "gpu-feature-discovery",
           chart: dict | None = None, defines: dict | None = None) -> str:
    """Render one template (the subchart tests use this directly)."""
    nodes, _, _ = _parse(_lex(text), 0, ())
    defs = dict(defines or {})
    _collect_defines(nodes, defs)
    root = {"Values": values, "Release": {"Name": release_name, "Namespace": namespace, "Service": "Helm"},
            "Chart": chart or {}}
    env = _Env(root, defs)
    out: list[str] = []
    env.run(nodes, root, {}, out)
    return "".join(out)


def merge(base: dict, override: dict) -> dict:
    """Helm's value coalescing: maps merge key by key (so an empty map
    changes nothing), null deletes the key, anything else replaces."""
    out = dict(base)
    for k, v in override.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def _chart_meta(path: Path) -> dict:
    meta = yaml.safe_load((path / "Chart.yaml").read_text())
    return {"Name": meta["name"], "Version": str(meta["version"]), "AppVersion": str(meta.get("appVersion", "")),
            "_deps": meta.get("dependencies", [])}


def render_chart(chart_dir: str | Path, values: dict | None = None, release_name: str = "gfd",
                 namespace: str = "gpu-feature-discovery") -> dict[str, str]:
    """``helm template`` for one release: {template path: rendered text} for
    the chart and its enabled file:// dependencies (alias-scoped values)."""
    chart_dir = Path(chart_dir)
    meta = _chart_meta(chart_dir)
    vals = merge(yaml.safe_load((chart_dir / "values.yaml").read_text()) or {}, values or {})
    tdir = chart_dir / "templates"
    defines: dict = {}
    for t in sorted(tdir.glob("*.tpl")):
        _collect_defines(_parse(_lex(t.read_text()), 0, ())[0], defines)
    chart = {k: v for k, v in meta.items() if not k.startswith("_")}
    out = {}
    for t in sorted(tdir.iterdir()):
        if t.suffix not in (".yaml", ".yml"):
            continue  # helpers, NOTES.txt
        out[str(t.relative_to(chart_dir))] = render(t.read_text(), vals, release_name, namespace, chart, defines)
    for dep in meta["_deps"]:
        key = dep.get("alias", dep["name"])
        cond = dep.get("condition")
        if cond and not any(_truthy(_Env({}, {})._field(vals, c)) for c in cond.split(",")):
            continue
        repo = dep["repository"]
        if not repo.startswith("file://"):
            raise HelmFail(f"dependency {dep['name']} is not in the repository ({repo})")
        sub = render_chart(chart_dir / repo[len("file://"):], vals.get(key, {}), release_name, namespace)
        out.update({f"charts/{key}/{k}": v for k, v in sub.items()})
    return out


def documents(rendered: dict[str, str]) -> list[dict]:
    """Every non-empty YAML document of a render_chart result."""
    docs = []
    for text in rendered.values():
        for d in yaml.safe_load_all(text):
            if d:
                docs.append(d)
    return docs
