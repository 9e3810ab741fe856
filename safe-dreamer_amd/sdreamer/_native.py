"""ctypes binding of libsdhip.so (include/sdhip.h) — the only way the product reaches the GPU kernels.

There is no CPU fallback: if the library is missing or fails to load, importing this module raises.
Device pointers come from torch tensors (PyTorch is the allocator/stream provider only); every call is
enqueued on torch's current HIP stream, so the whole update can be captured into a HIP graph.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDHIP_LIB", os.path.join(_HERE, "_lib", "libsdhip.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libsdhip.so not found at {LIB_PATH}: build it with `make -C safe-dreamer_amd/csrc` "
        "(or __graft_entry__.build()). The HIP path has no fallback.")
lib = ctypes.CDLL(LIB_PATH)

c_float_p = ctypes.c_void_p
c_long = ctypes.c_long
c_int = ctypes.c_int
c_float = ctypes.c_float
c_ptr = ctypes.c_void_p


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("A", c_ptr), ("B", c_ptr), ("C", c_ptr), ("bias", c_ptr),
        ("lda", c_long), ("ldb", c_long), ("ldc", c_long),
        ("strideA", c_long), ("strideB", c_long), ("strideC", c_long), ("strideBias", c_long),
        ("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
        ("a_kcontig", c_int), ("b_kcontig", c_int),
        ("ksplit", c_int), ("tile", c_int),
        ("alpha", c_float), ("beta", c_float),
    ]


HEADER = os.environ.get("SDHIP_HEADER", os.path.join(_HERE, "..", "..", "include", "sdhip.h"))


def _parse_struct(path, name):
    """ctypes.Structure for `typedef struct <name> {...} <name>;` in the header (fields in declaration order)."""
    import re
    text = re.sub(r"/\*.*?\*/", " ", open(path).read(), flags=re.S)
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}\s*" + name + r"\s*;", text, flags=re.S).group(1)
    scalars = {"int": c_int, "long": c_long, "float": c_float, "double": ctypes.c_double, "uint64_t": ctypes.c_uint64}
    fields = []
    for decl in body.split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        is_ptr = "*" in decl
        toks = decl.replace("const ", "").replace("*", " ").replace(",", " , ").split()
        if toks[0] == "unsigned":
            toks = toks[1:]
        if toks[:2] == ["long", "long"]:  # one type of two words
            toks = ["long"] + toks[2:]
        base, names = toks[0], [t for t in toks[1:] if t != ","]
        for n in names:
            typ = c_ptr if is_ptr else scalars[base]
            m = re.match(r"(\w+)\[(\w+)\]$", n)
            if m:  # array length: a literal or a #define of the header
                ln = m.group(2)
                ln = int(ln) if ln.isdigit() else int(re.search(r"#define " + ln + r"\s+(\d+)", text).group(1))
                n, typ = m.group(1), typ * ln
            fields.append((n, typ))
    return type(name, (ctypes.Structure,), {"_fields_": fields})


ScanDesc = _parse_struct(HEADER, "sd_rssm_scan")
ImagineDesc = _parse_struct(HEADER, "sd_imagine")
SliceKey = _parse_struct(HEADER, "sd_slice_key")


def _define(path, name):
    import re
    return int(re.search(r"#define " + name + r"\s+(\d+)", open(path).read()).group(1))


class SliceKeys(ctypes.Structure):
    _fields_ = [("k", SliceKey * _define(HEADER, "SD_MAX_SLICE_KEYS")), ("n", c_int)]


StatReq = _parse_struct(HEADER, "sd_stat_req")
MlpExt = _parse_struct(HEADER, "sd_mlp_ext")


class Stats(ctypes.Structure):
    _fields_ = [("r", StatReq * _define(HEADER, "SD_MAX_STATS")), ("nreq", c_int)]


LossTerm = _parse_struct(HEADER, "sd_loss_term")


class LossTerms(ctypes.Structure):
    _fields_ = [("t", LossTerm * _define(HEADER, "SD_MAX_LOSS_TERMS")), ("n", c_int)]


WgradAcc = _parse_struct(HEADER, "sd_wgrad_acc")
LayoutCopy = _parse_struct(HEADER, "sd_layout_copy")


class LayoutCopies(ctypes.Structure):
    _fields_ = [("e", LayoutCopy * _define(HEADER, "SD_MAX_LAYOUT_COPIES")), ("n", c_int)]

_CTYPES = {
    "int": c_int, "long": c_long, "float": c_float, "double": ctypes.c_double, "uint64_t": ctypes.c_uint64,
    "uint32_t": ctypes.c_uint32, "sd_stream": c_ptr, "void": None,
}


def _parse_header(path):
    """name -> argtypes for every `int sd_*(...);` declaration in include/sdhip.h (the ABI's single source)."""
    import re
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    sigs = {}
    for m in re.finditer(r"\bint\s+(sd_\w+)\s*\(([^)]*)\)\s*;", text):
        name, args = m.group(1), m.group(2).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                if "*" in a:
                    types.append(ctypes.POINTER(GemmDesc) if "sd_gemm_desc" in a else c_ptr)
                else:
                    t = a.replace("const ", "").split()[0]
                    types.append(_CTYPES[t])
        sigs[name] = types
    return sigs


_SIGS = _parse_header(HEADER)


def _bind(name, argtypes):
    fn = getattr(lib, name)
    fn.argtypes = argtypes
    fn.restype = c_int
    return fn


fns = {}


def register(name, argtypes):
    fns[name] = _bind(name, argtypes)
    return fns[name]


for _n, _a in _SIGS.items():
    register(_n, _a)

ABI_VERSION = lib.sd_abi_version()


class NativeError(RuntimeError):
    pass


SD_ESHAPE = -2  # common.h


def check(rc, name=""):
    if rc != 0:
        raise NativeError(f"{name} failed with status {rc}")


PROBES = []  # active LaunchProbe objects (sdreamer.kernels); empty in normal runs


def call(name, *args):
    if PROBES:
        hit = [pr for pr in PROBES if pr.match(name, args)]
        for pr in hit:
            pr.begin()
        check(fns[name](*args), name)
        for pr in hit:
            pr.end(args)
        return
    check(fns[name](*args), name)


def call_shaped(name, *args):
    """Like call(), but returns False (nothing launched) when the entry point reports SD_ESHAPE, i.e. the shape is
    outside a specialised kernel and the caller runs its general path."""
    if PROBES:
        hit = [pr for pr in PROBES if pr.match(name, args)]
        for pr in hit:
            pr.begin()
        rc = fns[name](*args)
        if rc == SD_ESHAPE:
            return False
        check(rc, name)
        for pr in hit:
            pr.end(args)
        return True
    rc = fns[name](*args)
    if rc == SD_ESHAPE:
        return False
    check(rc, name)
    return True


def exported_symbols():
    return sorted(_SIGS)
