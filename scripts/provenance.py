"""Which library a measurement belongs to: a content digest of the sources libdmt.so is built
from (diffusionmcmctools.jl_amd/csrc/*.hip, *.h, *.inc, Makefile and include/dmt.h).

The GPU box has no .git, so the profile summaries (kstats_summary.py, pmc_traffic.py,
issue_summary.py) record this digest of the tree they profiled, and bench.py quotes a
committed summary only when its digest equals the digest of the tree it runs from (VERDICT r04
"tie every roofline figure to the tree it measured")."""
import glob
import hashlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SRC_GLOBS = ("diffusionmcmctools.jl_amd/csrc/*.hip", "diffusionmcmctools.jl_amd/csrc/*.h",
              "diffusionmcmctools.jl_amd/csrc/*.inc", "diffusionmcmctools.jl_amd/csrc/Makefile",
              "include/dmt.h")


def csrc_digest(root=ROOT):
    """sha256 (16 hex digits) over the library's source files, by relative path and content."""
    h = hashlib.sha256()
    files = sorted({os.path.relpath(p, root) for g in _SRC_GLOBS
                    for p in glob.glob(os.path.join(root, g))})
    for rel in files:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def git_commit(root=ROOT):
    """HEAD's commit when a checkout is present (this container), else None (the GPU box)."""
    try:
        r = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"],
                           capture_output=True, text=True, timeout=10)
        return r.stdout.strip() or None if r.returncode == 0 else None
    except Exception:
        return None


def stamp(out, root=ROOT, digest=None):
    """Add the provenance fields to a summary dict (in place) and return it.  `digest`: the
    digest the GPU session recorded for the tree it ran (its tree.txt); default: this tree's."""
    out["csrc_sha16"] = digest or csrc_digest(root)
    out["git_commit"] = git_commit(root)
    return out


def read_digest(path):
    """The digest a GPU session wrote with `python scripts/provenance.py > <dir>/tree.txt`."""
    with open(path) as f:
        return f.read().split()[0]


if __name__ == "__main__":
    print(csrc_digest())
