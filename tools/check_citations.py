"""Checks every `File.scala:N[-M]` / `File.java:N` citation in the repo against /root/reference.

A citation is flagged when no reference file of that name (narrowed by any path prefix written
before it) has at least M lines.  Line ranges written after a citation as `,A-B` or `, :A` are
checked against the same file.  Run from the repo root; exits 1 when something is flagged.
Used by tests/test_citations.py (skipped where /root/reference is absent, e.g. on the GPU box).
"""
import os
import re
import sys

REF = "/root/reference"
EXTS = (".py", ".c", ".h", ".hip", ".hpp", ".md", ".sh")
SKIP_FILES = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "PAPERS.md", "SNIPPETS.md", "BASELINE.md"}
# ambiguous basenames cited without a path in this repo
ALIASES = {"package.scala": "zorder/sfcurve"}
CITE = re.compile(r"((?:[\w\-.]+/|\.\.\./)*)([A-Za-z][\w]*\.(?:scala|java))((?::\d+(?:-\d+)?)(?:,\s*:?\d+(?:-\d+)?)*)")


def ref_index():
    idx = {}
    for root, _, files in os.walk(REF):
        for f in files:
            if f.endswith((".scala", ".java")):
                idx.setdefault(f, []).append(os.path.join(root, f))
    return idx


_lines = {}


def nlines(p):
    if p not in _lines:
        with open(p, "rb") as fh:
            _lines[p] = fh.read().count(b"\n") + 1
    return _lines[p]


def repo_files(root):
    for d, dirs, files in os.walk(root):
        dirs[:] = [x for x in dirs if not x.startswith(".") and x not in ("gpurun_out", "__pycache__", "_ref", "build")]
        for f in files:
            if f.endswith(EXTS) and f not in SKIP_FILES:
                yield os.path.join(d, f)


def check(root="."):
    idx = ref_index()
    bad = []
    for path in repo_files(root):
        if os.path.basename(path) == "check_citations.py":
            continue
        with open(path, encoding="utf-8", errors="replace") as fh:
            for ln, line in enumerate(fh, 1):
                for m in CITE.finditer(line):
                    prefix, name, spans = m.group(1), m.group(2), m.group(3)
                    cands = idx.get(name, [])
                    parts = [p for p in prefix.split("/") if p and p not in ("...", "..")]
                    if not parts and name in ALIASES:
                        parts = ALIASES[name].split("/")
                    for k in range(len(parts)):   # the longest suffix of the written path that matches
                        narrowed = [c for c in cands if "/" + "/".join(parts[k:]) + "/" + name in c]
                        if narrowed:
                            cands = narrowed
                            break
                    hi = max(int(x) for x in re.findall(r"\d+", spans))
                    if not cands:
                        bad.append((path, ln, m.group(0), "no such reference file"))
                    elif all(nlines(c) < hi for c in cands):
                        bad.append((path, ln, m.group(0), "file has %s lines" % "/".join(str(nlines(c)) for c in cands)))
    return bad


if __name__ == "__main__":
    out = check(sys.argv[1] if len(sys.argv) > 1 else ".")
    for p, ln, c, why in out:
        print("%s:%d: %s (%s)" % (p, ln, c, why))
    print("%d flagged" % len(out))
    sys.exit(1 if out else 0)
