"""Every measurement file the documentation cites is in the repository
(round-5 VERDICT item 8): DESIGN.md, INTEGRATION.md and README.md name
`profiles/...` paths (and bare `r05xx_name.txt`-style names inside profile
lists) as evidence, so each must be tracked by git, not only present in a
builder's working tree."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

DOCS = ["DESIGN.md", "INTEGRATION.md", "README.md"]


def tracked():
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    return set(out.split())


def cited(text):
    """Paths under profiles/ cited in backquotes or plain text; a trailing
    '*' or '{a,b}' pattern is expanded against the tracked files by the caller."""
    return set(re.findall(r"profiles/[A-Za-z0-9_./{},*-]+[A-Za-z0-9_*}]", text))


def test_cited_profiles_are_tracked():
    files = tracked()
    missing = []
    for doc in DOCS:
        path = os.path.join(ROOT, doc)
        if not os.path.exists(path):
            continue
        for ref in sorted(cited(open(path, encoding="utf-8").read())):
            ref = ref.rstrip(".,;:)")
            if "{" in ref:  # profiles/a_{x,y}.txt
                head, rest = ref.split("{", 1)
                alts, tail = rest.split("}", 1)
                refs = [head + a + tail for a in alts.split(",")]
            else:
                refs = [ref]
            for r in refs:
                if "*" in r:
                    pat = re.compile("^" + re.escape(r).replace(r"\*", ".*") + "$")
                    ok = any(pat.match(f) or f.startswith(r.split("*")[0]) for f in files)
                elif r.endswith("/"):
                    ok = any(f.startswith(r) for f in files)
                else:
                    ok = r in files or any(f.startswith(r + "/") for f in files)
                if not ok:
                    missing.append(f"{doc}: {r}")
    assert not missing, "cited but not tracked:\n" + "\n".join(missing)
