"""Every tracked file under profiles/ is listed in a round's index (profiles/R0x_INDEX.md), so
the evidence a document cites can be found and nothing unindexed accumulates.  Index entries are
backquoted names, with shell brace lists (`r04t_duo_ab_d{1,0}_{1,2}.json`) and `(+ _detail.json)`
for a bench line's detail file."""
import glob
import itertools
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(ROOT, "profiles")


def _expand(name):
    parts = re.split(r"\{([^}]*)\}", name)
    fixed, choices = parts[0::2], [p.split(",") for p in parts[1::2]]
    for pick in itertools.product(*choices):
        yield "".join(a + b for a, b in itertools.zip_longest(fixed, pick, fillvalue=""))


def _indexed():
    names = set()
    for path in glob.glob(os.path.join(PROFILES, "R0*_INDEX.md")):
        with open(path) as f:
            for raw in re.findall(r"`([^`]+)`", f.read()):
                names.update(_expand(raw.strip()))
    names |= {n[:-len(".json")] + "_detail.json" for n in names if n.endswith(".json")}
    return names


def _tracked():
    try:
        out = subprocess.run(["git", "ls-files", "profiles"], cwd=ROOT, capture_output=True, text=True,
                             check=True).stdout
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    return [os.path.relpath(os.path.join(ROOT, p), PROFILES) for p in out.split()]


def test_brace_expansion():
    assert sorted(_expand("a_{1,0}_{x,y}.json")) == ["a_0_x.json", "a_0_y.json", "a_1_x.json", "a_1_y.json"]
    assert list(_expand("plain.log")) == ["plain.log"]


def test_every_tracked_profile_is_indexed():
    names = _indexed()
    missing = []
    for rel in _tracked():
        if re.fullmatch(r"R0\d_INDEX\.md", rel):
            continue
        top = rel.split(os.sep)[0]
        if rel in names or top in names or top + "/" in names:
            continue
        missing.append(rel)
    assert not missing, f"tracked under profiles/ but listed in no R0x_INDEX.md: {missing}"
