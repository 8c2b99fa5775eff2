#!/usr/bin/env python3
"""Differential run of the daemon's YAML reader against PyYAML on random
token soups rooted in a mapping (the shape of a config file): counts the
documents one reader rejects and the other accepts, and those both accept
with different values, and prints the shortest examples of each.  PyYAML is
YAML 1.1 like go-yaml v2 (the reference's reader) but not identical to it:
tab handling (documents with tabs are skipped), sexagesimal ints, non-string keys and a few indentation
leniencies differ, and those remain in the output by design.

    python tools/yaml_diff.py [SEED] [N]
"""
import math
import os
import random
import sys

import yaml

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_feature_discovery_amd as gfd  # noqa: E402

n = gfd.native()
toks = ["a", "b", "c", "x y", "1", "-1", "1.5", "true", "null", "~", "'q'", '"d"', "'a: b'", "http://h:8/p",
        ": ", ":", " ", "  ", "- ", "-", "#c", " #c", "[", "]", "{", "}", ",", ", ", "&a ", "*a", "!!str ", "|", ">",
        "\n", "\n  ", "\n    ", "\n- ", "\n  - ", "<<: ", "'", '"', "\t", "%", "@", "`", "...", "---"]
def gen(rng):
    return rng.choice(["k: ", "k:\n  ", "k:\n- ", "- k: "]) + "".join(rng.choice(toks) for _ in range(rng.randint(1, 10))) + "\n"
def same(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return a == b or (math.isnan(a) and math.isnan(b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    return type(a) is type(b) and a == b
rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
cats = {}
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 20000):
    t = gen(rng)
    if "\t" in t:
        continue  # PyYAML rejects tabs where libyaml (go-yaml) takes them as blanks
    try:
        py = yaml.safe_load(t); pe = None
    except Exception as e:
        pe = type(e).__name__
    try:
        ours = n.parse_yaml(t); oe = None
    except Exception as e:
        oe = str(e)
    if pe and not oe:
        k = "py rejects, ours accepts"
    elif oe and not pe:
        k = "ours rejects, py accepts"
    elif not pe and not oe and not same(ours, py):
        k = "values differ"
    else:
        continue
    cats.setdefault(k, []).append((t, py if not pe else pe, ours if not oe else oe))
for k, v in cats.items():
    print(f"== {k}: {len(v)}")
    for t, p, o in sorted({x[0]: x for x in v}.values(), key=lambda x: len(x[0]))[:12]:
        print(f"   {t!r}\n      py={p!r}\n      ours={o!r}")
