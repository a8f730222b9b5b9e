"""Provenance of a measurement line: which sources and which built library produced it.

    head          the commit the measured tree was sent from (PST_HEAD, set by the gpurun command line:
                  the GPU box's snapshot has no .git), else `git rev-parse` where .git exists
    sources_sha16 SHA-256 (first 16 hex) over the product sources: csrc/*, include/pst.h, pst_amd/*.py,
                  bench.py — unchanged by documentation-only commits after the measurement
    libpst_sha16  SHA-256 of the libpst.so the process loaded
"""
import glob
import hashlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "protein-structure-tokenizer_amd")


def _sha16(paths):
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def sources():
    pats = ["csrc/*.hip", "csrc/*.cpp", "csrc/*.h", "csrc/Makefile", "pst_amd/*.py"]
    files = sorted(f for p in pats for f in glob.glob(os.path.join(PKG, p)))
    return files + [os.path.join(ROOT, "include", "pst.h"), os.path.join(ROOT, "bench.py")]


def provenance():
    head = os.environ.get("PST_HEAD")
    if not head:
        try:
            head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                  text=True, timeout=10).stdout.strip() or None
        except Exception:
            head = None
    lib = os.environ.get("PST_LIB", os.path.join(PKG, "pst_amd", "_lib", "libpst.so"))
    return {"head": head, "sources_sha16": _sha16(sources()),
            "libpst_sha16": _sha16([lib]) if os.path.exists(lib) else None}
