"""Every `<file>.rs:N` / `<file>.rs:N-M` citation in the repository must point inside
the cited reference file (a restatement that cites line ranges that do
not exist cannot be audited).  Paths may be abbreviated to a suffix of the real path;
`lib/` = packages/ray-tracer-lib/src/, `app/` = packages/ray-tracer/src/ (DESIGN.md).
Skipped where /root/reference is absent (the GPU box)."""
import collections
import os
import re

import pytest

from helpers import ROOT

REF = "/root/reference"
PAT = re.compile(r"((?:[A-Za-z_]+/)*[A-Za-z_\-]+\.rs):(\d+)(?:-(\d+))?")
EXTS = (".py", ".cpp", ".hpp", ".hip", ".h", ".md", ".sh", "Makefile")
SKIP_DOCS = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "BASELINE.md", "PAPERS.md", "SNIPPETS.md"}  # not ours


def _reference_files():
    files = collections.defaultdict(list)
    for dp, _, fs in os.walk(REF):
        for f in fs:
            if f.endswith(".rs"):
                p = os.path.join(dp, f)
                with open(p, errors="replace") as fh:
                    files[f].append((p, sum(1 for _ in fh)))
    return files


def _expand(path):
    if path.startswith("lib/"):
        return "ray-tracer-lib/src/" + path[4:]
    if path.startswith("app/"):
        return "ray-tracer/src/" + path[4:]
    return path


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources not present")
def test_every_reference_citation_is_in_range():
    files = _reference_files()
    bad, seen = [], 0
    for dp, dns, fs in os.walk(ROOT):
        dns[:] = [d for d in dns if d not in (".git", "gpurun_out", "build", "__pycache__", "ab")]
        for f in fs:
            if not f.endswith(EXTS) or f in SKIP_DOCS:
                continue
            p = os.path.join(dp, f)
            with open(p, errors="replace") as fh:
                for i, line in enumerate(fh, 1):
                    for m in PAT.finditer(line):
                        path, a = m.group(1), int(m.group(2))
                        b = int(m.group(3) or a)
                        full = _expand(path)
                        base = full.split("/")[-1]
                        cands = [c for c in files.get(base, []) if c[0].endswith("/" + full)] or files.get(base, [])
                        seen += 1
                        if not cands:
                            bad.append(f"{os.path.relpath(p, ROOT)}:{i}: {m.group(0)} (no such file)")
                        elif not any(a <= b <= n for _, n in cands):
                            bad.append(f"{os.path.relpath(p, ROOT)}:{i}: {m.group(0)} "
                                       f"(file has {'/'.join(str(n) for _, n in cands)} lines)")
    assert seen > 100
    assert not bad, "\n".join(bad)
