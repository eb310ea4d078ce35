"""Content hash of the HIP sources the library is built from (csrc/*.hip, csrc/*.h,
include/dgvcc.h).  build.py compiles it into libdgvcc_hip.so (`dg_source_hash`), and
_capi.py refuses a library whose hash differs from the sources next to it, so a stale
binary can never be the one a test or benchmark runs."""
from __future__ import annotations

import hashlib
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)


def source_files() -> list[str]:
    csrc = os.path.join(_PKG, "csrc")
    if not os.path.isdir(csrc):
        return []
    fs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".h")))
    return fs + [os.path.join(_ROOT, "include", "dgvcc.h")]


def source_hash() -> str | None:
    """16 hex digits of sha256 over (relative path, contents) of every source; None when
    the sources are not present (an installed library without its tree)."""
    fs = source_files()
    if not fs:
        return None
    h = hashlib.sha256()
    for f in fs:
        h.update(os.path.relpath(f, _ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
