"""Build libdgvcc_hip.so (all HIP kernels + the C-ABI) for gfx950, in-tree.

    python -m dgvcc_amd.build          # incremental
    python -m dgvcc_amd.build --force  # rebuild everything

Objects go to dgvcc_amd/build/, the library to dgvcc_amd/lib/libdgvcc_hip.so
(git-ignored, but shipped to the GPU box by gpurun with the snapshot).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

try:
    from .srchash import source_hash
except ImportError:  # run as a script
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dgvcc_amd.srchash import source_hash

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libdgvcc_hip.so")
ARCH = "gfx950"
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
          "-Wno-unused-result"]


def _hipcc() -> str:
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found: the DGVCC HIP library cannot be built")
    return h


def sources() -> list[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _deps_mtime() -> float:
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(ROOT, "include", "dgvcc.h"))
    return max(os.path.getmtime(h) for h in hdrs)


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hipcc = _hipcc()
    hdr_t = _deps_mtime()
    todo = []
    objs = []
    for src in sources():
        obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            todo.append((src, obj))

    def _compile(item):
        src, obj = item
        cmd = [hipcc, *CFLAGS, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {os.path.basename(src)}:\n{r.stderr}")
        return obj

    jobs = jobs or min(8, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    objs.append(_hash_object(force))
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


def _hash_object(force: bool) -> str:
    """srchash.o: `dg_source_hash` returning the content hash of the sources compiled above
    (regenerated whenever the hash changes, so a relink follows any source edit)."""
    h = source_hash()
    src = os.path.join(OBJ, "srchash.cpp")
    obj = os.path.join(OBJ, "srchash.o")
    code = ('#include <string.h>\n'
            f'static const char kHash[] = "{h}";\n'
            'extern "C" int dg_source_hash(char* out, int cap) {\n'
            '  const int n = (int)sizeof(kHash) - 1;\n'
            '  if (!out || cap <= n) return -1;\n'
            '  memcpy(out, kHash, n + 1);\n'
            '  return n;\n'
            '}\n')
    old = open(src).read() if os.path.exists(src) else None
    if force or old != code or not os.path.exists(obj):
        with open(src, "w") as f:
            f.write(code)
        r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"srchash compile failed:\n{r.stderr}")
    return obj


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))
    sys.exit(0)
