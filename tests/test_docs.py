"""The measurements DESIGN.md / README.md / INTEGRATION.md cite are in the tree: every
`profiles/...` path (globs and {a,b} alternatives expanded; rNN placeholders skipped) names at
least one committed file, and the bench line's traffic sources parse."""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cited():
    for doc in ("DESIGN.md", "DESIGN_HISTORY.md", "README.md", "INTEGRATION.md"):
        text = open(os.path.join(ROOT, doc)).read()
        for path in re.findall(r"`(profiles/[^`\s]+)`", text):
            if "rNN" in path:
                continue
            if "{" in path:
                head, rest = path.split("{", 1)
                opts, tail = rest.split("}", 1)
                yield from ((doc, head + o + tail) for o in opts.split(","))
            else:
                yield doc, path


def test_cited_profiles_exist():
    missing = [(doc, p) for doc, p in _cited() if not glob.glob(os.path.join(ROOT, p))]
    assert not missing, missing


def test_traffic_files_parse():
    files = glob.glob(os.path.join(ROOT, "profiles", "r04_pmc_traffic_*.json"))
    assert files
    for f in files:
        d = json.load(open(f))
        assert d["kernels"], f
        for name, k in d["kernels"].items():
            assert k["bytes_per_launch"] >= 0, (f, name)
