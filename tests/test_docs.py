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


def test_r06_traffic_files_parse():
    """The same-build traffic every r06 bench line cites (tools/pmc_passes.sh output)."""
    files = glob.glob(os.path.join(ROOT, "profiles", "r06_pmc_traffic_*_final.json"))
    assert len(files) == 4
    for f in files:
        d = json.load(open(f))
        assert d["kernels"] and len(d["libmbls_sha256_16"]) == 16, f
        for name, k in d["kernels"].items():
            assert k["bytes_per_launch"] >= 0, (f, name)


def test_variant_builder_links_every_object():
    """tools/build_variant.sh links the same objects as the Makefile's libmbls.so (a TU missing
    from its list makes every A/B variant fail to link, or link a stale object)."""
    mk = open(os.path.join(ROOT, "lambda_ethereum_consensus_amd", "csrc", "Makefile")).read()
    objs = re.search(r"^OBJS := \$\(addprefix \$\(OBJ\)/,(.*?)\)$", mk, re.M | re.S).group(1)
    made = set(re.findall(r"(mbls_\w+)\.o", objs))
    sh = open(os.path.join(ROOT, "tools", "build_variant.sh")).read()
    listed = set(re.search(r"^for o in ([^;]*); do objs", sh, re.M).group(1).split())
    assert made and made == listed, (made ^ listed)


def test_lds_bank_model_reproduces_its_profile():
    """DESIGN.md section 9 quotes tools/lds_bank_model.py's figures from
    profiles/r06_lds_bank_model.json; the model still computes them."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("lds_bank_model", os.path.join(ROOT, "tools", "lds_bank_model.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.summary() == json.load(open(os.path.join(ROOT, "profiles", "r06_lds_bank_model.json")))


def test_every_library_knob_is_in_the_design_table():
    """Every environment variable libmbls reads (getenv in csrc/) has a row in DESIGN.md
    section 11's knob table."""
    csrc = os.path.join(ROOT, "lambda_ethereum_consensus_amd", "csrc")
    read = set()
    for f in glob.glob(os.path.join(csrc, "*")):
        if f.endswith((".cpp", ".hpp", ".hip", ".h")):
            read |= set(re.findall(r'getenv\("([A-Z_0-9]+)"\)', open(f).read()))
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    table = design[design.index("## 11."):]
    listed = set(re.findall(r"`([A-Z_0-9]+)`", table))
    assert read and read <= listed, sorted(read - listed)
