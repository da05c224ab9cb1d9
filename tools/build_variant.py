#!/usr/bin/env python3
"""Build libPhaseType.so from another git revision (or with extra -D flags)
into phasetype_amd/_variants/<name>.so, for tools/ab.py A/B runs.

usage: python3 tools/build_variant.py <name> [--ref GITREF] [-D FLAG ...]
--ref builds that revision's sources (git worktree in a temp dir); without it
the working tree's sources are built with the given defines (and --flag
hipcc flags)."""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--ref")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="extra hipcc flag for the .hip units")
    a = ap.parse_args()
    out = os.path.join(REPO, "phasetype_amd", "_variants", a.name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    src = REPO
    tmp = None
    if a.ref:
        tmp = tempfile.mkdtemp(prefix="pht_wt_")
        subprocess.run(["git", "-C", REPO, "worktree", "add", "--detach", tmp, a.ref], check=True,
                       stdout=subprocess.DEVNULL)
        src = tmp
    try:
        code = ("import sys; sys.path.insert(0, %r); from phasetype_amd import build as B; "
                "B.build(force=True, defines=%r, out=%r, flags=%r)" % (src, tuple(a.defines), out, tuple(a.flags)))
        subprocess.run([sys.executable, "-c", code], check=True)
    finally:
        if tmp:
            subprocess.run(["git", "-C", REPO, "worktree", "remove", "--force", tmp], check=True)
            shutil.rmtree(tmp, ignore_errors=True)
    print(out)


if __name__ == "__main__":
    main()
