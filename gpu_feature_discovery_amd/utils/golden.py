"""Golden-file helpers.

Two kinds of goldens live in ``tests/``:

* byte goldens (``tests/golden/*.txt``): the exact feature file for a
  deterministic input (mock or synthetic backend, ``--no-timestamp``); the
  daemon writes labels sorted by key so these compare byte-for-byte.
* regex goldens (``tests/expected-output*.txt``): one full-match regex per
  line, in the style of the reference's tests/expected-output*.txt, checked
  *bidirectionally* (every label matches exactly one regex and every regex
  is used) - the reference's check (main_test.go:403-435) is one-directional,
  unanchored and uses ``[true|false]`` character classes; those gaps are fixed
  here.
"""

from __future__ import annotations

import re
from pathlib import Path


def parse_labels(text: str) -> dict[str, str]:
    """Parse ``key=value`` lines; duplicate keys are an error
    (buildLabelMapFromOutput, main_test.go:382-401)."""
    labels: dict[str, str] = {}
    for line in text.rstrip("\n").split("\n"):
        if not line:
            continue
        if line.count("=") != 1:
            raise ValueError(f"unexpected format in line: {line!r}")
        k, v = line.split("=", 1)
        if k in labels:
            raise ValueError(f"duplicate label {k!r}")
        labels[k] = v
    return labels


def load_regexes(path: str | Path) -> list[re.Pattern]:
    return [re.compile(line) for line in Path(path).read_text().splitlines() if line and not line.startswith("#")]


def check_regex_golden(output: str, golden: str | Path, select=None) -> None:
    """Every selected output line must fully match exactly one regex and every
    regex must be matched exactly once."""
    regexes = load_regexes(golden)
    used = [0] * len(regexes)
    lines = [ln for ln in output.rstrip("\n").split("\n") if ln and (select is None or select(ln))]
    for line in lines:
        hits = [i for i, r in enumerate(regexes) if r.fullmatch(line)]
        if not hits:
            raise AssertionError(f"line does not match any regexp in {golden}: {line}")
        if len(hits) > 1:
            raise AssertionError(f"line matches several regexps in {golden}: {line}")
        used[hits[0]] += 1
    for i, n in enumerate(used):
        if n != 1:
            raise AssertionError(f"regexp {regexes[i].pattern!r} in {golden} matched {n} lines (want 1)")


def check_byte_golden(output: str, golden: str | Path, update: bool = False) -> None:
    path = Path(golden)
    if update:
        path.write_text(output)
        return
    expected = path.read_text()
    if output != expected:
        import difflib
        diff = "".join(difflib.unified_diff(expected.splitlines(True), output.splitlines(True), str(path), "output"))
        raise AssertionError(f"output differs from {path}:\n{diff}")


# Kubernetes label syntax (apimachinery validation.IsQualifiedName /
# IsValidLabelValue), which NFD applies before publishing a feature label:
# an optional DNS-subdomain prefix (<= 253 chars) and '/', a name of <= 63
# chars, and a value of <= 63 chars; name and non-empty value start and end
# alphanumeric with [-_.A-Za-z0-9] in between.
_NAME = re.compile(r"[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?")
_DNS1123_SUBDOMAIN = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")


def k8s_label_problems(labels: dict[str, str]) -> list[str]:
    """Labels NFD / the API server would reject, with the reason."""
    problems = []
    for key, value in labels.items():
        prefix, _, name = key.rpartition("/")
        if "/" in prefix:
            problems.append(f"{key}: more than one '/'")
        if prefix and (len(prefix) > 253 or not _DNS1123_SUBDOMAIN.fullmatch(prefix)):
            problems.append(f"{key}: prefix is not a DNS-1123 subdomain")
        if len(name) > 63 or not _NAME.fullmatch(name):
            problems.append(f"{key}: invalid name")
        if value and (len(value) > 63 or not _NAME.fullmatch(value)):
            problems.append(f"{key}={value}: invalid value")
    return problems
