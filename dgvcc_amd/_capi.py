"""ctypes binding of libdgvcc_hip.so (the C-ABI declared in include/dgvcc.h).

The prototypes are parsed from the header itself, so the Python side can never
drift from the ABI.  `torch` is imported first so the library binds to the HIP
runtime torch already loaded (same SONAME `libamdhip64.so.7`): device pointers
from the caching allocator and `torch.cuda.current_stream()` handles are then
valid in our launches.

There is no CPU fallback: if the library is missing every op raises.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the dlopen of our HIP library)

from .srchash import source_hash

_PKG = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(_PKG), "include", "dgvcc.h")
LIB_PATH = os.path.join(_PKG, "lib", "libdgvcc_hip.so")

DG_F32, DG_BF16, DG_F16 = 0, 1, 2
_ERRORS = {-1: "invalid argument", -2: "unsupported shape/dtype", -3: "HIP error"}


class DGError(RuntimeError):
    pass


def _ctype(tok: str):
    tok = tok.strip()
    if "*" in tok:
        return ctypes.c_void_p
    base = tok.replace("const", "").split()
    base = base[0] if base else ""
    return {"int": ctypes.c_int, "int64_t": ctypes.c_int64, "float": ctypes.c_float, "double": ctypes.c_double,
            "void": None}[base]


def parse_header(path: str = HEADER) -> dict[str, tuple]:
    """Return {name: (restype, [argtypes])} for every prototype in dgvcc.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"^(int64_t|int)\s+(dg_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.M | re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        args = " ".join(args.split())
        argtypes = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                # drop the parameter name (last identifier), keep the type
                t = re.sub(r"\b\w+$", "", a).strip() if not a.endswith("*") else a
                argtypes.append(_ctype(t))
        protos[name] = (ctypes.c_int64 if ret == "int64_t" else ctypes.c_int, argtypes)
    return protos


def header_abi_version(path: str = HEADER) -> int:
    """DGVCC_ABI_VERSION as include/dgvcc.h declares it."""
    m = re.search(r"^#define\s+DGVCC_ABI_VERSION\s+(\d+)", open(path).read(), flags=re.M)
    if m is None:
        raise DGError(f"{path}: no DGVCC_ABI_VERSION")
    return int(m.group(1))


_lib = None
_protos = None


def lib():
    global _lib, _protos
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DGError(f"{LIB_PATH} not built: run `python -m dgvcc_amd.build` "
                          "(there is no CPU fallback for the DGVCC kernels)")
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        _protos = parse_header()
        for name, (res, args) in _protos.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        abi = header_abi_version()
        if l.dg_version() != abi:
            raise DGError(f"{LIB_PATH} implements ABI {l.dg_version()}, include/dgvcc.h declares {abi}: "
                          "rebuild with `python -m dgvcc_amd.build`")
        want = source_hash()
        got = library_hash(l)
        if want is not None and got != want:
            raise DGError(f"{LIB_PATH} was built from other sources (library {got}, sources {want}): "
                          "rebuild with `python -m dgvcc_amd.build`")
        _lib = l
    return _lib


def library_hash(l=None) -> str:
    """The source hash compiled into the library (dg_source_hash)."""
    l = l if l is not None else lib()
    buf = ctypes.create_string_buffer(64)
    n = l.dg_source_hash(buf, 64)
    return buf.value.decode() if n > 0 else ""


def exported_symbols() -> list[str]:
    lib()
    return sorted(_protos)


def call(name: str, *args) -> int:
    """Invoke a status-returning entry point; raise on a negative code."""
    r = getattr(lib(), name)(*args)
    if r < 0:
        raise DGError(f"{name} failed: {_ERRORS.get(r, r)} ({r})")
    return r


def lib_call_status(name: str, *args) -> int:
    """Invoke an entry point and return its status code unchecked (for callers that
    handle DG_ERR_UNSUPPORTED themselves)."""
    return int(getattr(lib(), name)(*args))


def query(name: str, *args) -> int:
    r = getattr(lib(), name)(*args)
    if r < 0:
        raise DGError(f"{name} failed: {_ERRORS.get(r, r)} ({r})")
    return int(r)


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DG_F32
    if dt == torch.bfloat16:
        return DG_BF16
    if dt == torch.float16:
        return DG_F16
    raise DGError(f"unsupported dtype {dt}")
