"""ctypes binding of libdfcsa.so (the C ABI declared in include/dfcsa.h).

The argument types of every entry point are derived from the header itself, so the header is
the single source of truth for the boundary.  Loading fails loudly (ImportError) when the
library is missing: there is no fallback path.  torch must be imported first so that the HIP
runtime torch ships (soname libamdhip64.so.7) is the one libdfcsa binds to.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (must precede the library load, see above)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("DFCSA_LIB", os.path.join(PKG_DIR, "libdfcsa.so"))
HEADER_PATH = os.path.join(REPO_DIR, "include", "dfcsa.h")

MAX_SEG = 32
DT_F32 = 0
DT_BF16 = 1
EINVAL = -10000


class DfcsaError(RuntimeError):
    pass


def parse_header(path=HEADER_PATH):
    """Return {name: (restype, [argtypes])} for every `dfcsa_*` prototype in the header."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(int64_t|int|const\s+char\s*\*)\s*(dfcsa_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        restype = ctypes.c_char_p if "char" in ret else (ctypes.c_int64 if ret == "int64_t" else ctypes.c_int)
        argtypes = []
        args = args.strip()
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                if "*" in a:
                    argtypes.append(ctypes.c_void_p)
                elif a.startswith("int64_t"):
                    argtypes.append(ctypes.c_int64)
                elif a.startswith("int"):
                    argtypes.append(ctypes.c_int)
                elif a.startswith("float"):
                    argtypes.append(ctypes.c_float)
                elif a.startswith("double"):
                    argtypes.append(ctypes.c_double)
                else:
                    raise DfcsaError(f"unparsed argument {a!r} of {name}")
        protos[name] = (restype, argtypes)
    return protos


class ConvDesc(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int), ("M", ctypes.c_int), ("N", ctypes.c_int), ("Kpad", ctypes.c_int),
                ("Cseg", ctypes.c_int), ("nseg", ctypes.c_int),
                ("seg_ptr", ctypes.c_void_p * MAX_SEG), ("seg_dh", ctypes.c_int * MAX_SEG),
                ("seg_dw", ctypes.c_int * MAX_SEG),
                ("Ho", ctypes.c_int), ("Wo", ctypes.c_int), ("Hi", ctypes.c_int), ("Wi", ctypes.c_int),
                ("stride", ctypes.c_int), ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p),
                ("mode", ctypes.c_int), ("ndest", ctypes.c_int), ("dest", ctypes.c_void_p * 3),
                ("Nd", ctypes.c_int), ("accumulate", ctypes.c_int), ("stats", ctypes.c_void_p),
                ("Hout", ctypes.c_int), ("Wout", ctypes.c_int), ("stats_floats", ctypes.c_int64),
                ("work", ctypes.c_void_p), ("work_floats", ctypes.c_int64)]


class BnFold(ctypes.Structure):
    """dfcsa_bn_fold: the train-mode BatchNorm finalisation dfcsa_conv_gemm_bn folds into a conv."""
    _fields_ = [("C", ctypes.c_int), ("count", ctypes.c_int), ("conv_bias", ctypes.c_void_p),
                ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("running_mean", ctypes.c_void_p),
                ("running_var", ctypes.c_void_p), ("num_batches_tracked", ctypes.c_void_p),
                ("momentum", ctypes.c_float), ("eps", ctypes.c_float), ("scale", ctypes.c_void_p),
                ("shift", ctypes.c_void_p), ("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p)]


class WgradDesc(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int), ("M", ctypes.c_int), ("ng", ctypes.c_int), ("Cg", ctypes.c_int),
                ("g_ptr", ctypes.c_void_p * 3), ("nseg", ctypes.c_int), ("Cseg", ctypes.c_int),
                ("seg_ptr", ctypes.c_void_p * MAX_SEG), ("seg_dh", ctypes.c_int * MAX_SEG),
                ("seg_dw", ctypes.c_int * MAX_SEG),
                ("Ho", ctypes.c_int), ("Wo", ctypes.c_int), ("Hi", ctypes.c_int), ("Wi", ctypes.c_int),
                ("stride", ctypes.c_int), ("slab", ctypes.c_void_p), ("splits", ctypes.c_int),
                ("mchunk", ctypes.c_int), ("layout", ctypes.c_int), ("ntaps", ctypes.c_int), ("Ctot", ctypes.c_int),
                ("Creal", ctypes.c_int), ("ndst", ctypes.c_int), ("dst", ctypes.c_void_p * 3),
                ("slab_floats", ctypes.c_int64), ("bias_dst", ctypes.c_void_p * 3)]


class PackEntry(ctypes.Structure):
    _fields_ = [("start", ctypes.c_int64), ("count", ctypes.c_int64), ("kind", ctypes.c_int), ("dtype", ctypes.c_int),
                ("w0", ctypes.c_void_p), ("w1", ctypes.c_void_p), ("w2", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("a", ctypes.c_int * 8)]


class WstdEntry(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("what", ctypes.c_void_p), ("rstd", ctypes.c_void_p), ("g", ctypes.c_void_p),
                ("dw", ctypes.c_void_p), ("K", ctypes.c_int), ("rows", ctypes.c_int), ("row0", ctypes.c_int),
                ("pad", ctypes.c_int)]


class ResampleDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("bounds", ctypes.c_void_p),
                ("kk", ctypes.c_void_p), ("n_out", ctypes.c_int), ("n_lines", ctypes.c_int), ("ksize", ctypes.c_int),
                ("axis", ctypes.c_int), ("src_pitch", ctypes.c_int), ("dst_pitch", ctypes.c_int),
                ("row0", ctypes.c_int), ("pad", ctypes.c_int)]


class PoolContract(ctypes.Structure):
    _fields_ = [("wsum", ctypes.c_void_p), ("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p),
                ("rows", ctypes.c_void_p), ("H", ctypes.c_int), ("W", ctypes.c_int), ("P", ctypes.c_int)]


class AugDesc(ctypes.Structure):
    _fields_ = [("img", ctypes.c_void_p), ("mask", ctypes.c_void_p), ("xtab", ctypes.c_void_p),
                ("ytab", ctypes.c_void_p), ("m", ctypes.c_double * 6), ("fix", ctypes.c_int * 6),
                ("rotate", ctypes.c_int), ("flip", ctypes.c_int), ("mask_w", ctypes.c_int), ("pad", ctypes.c_int)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libdfcsa.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (or `make -C dfc-sa-unet_amd/csrc`). The DFC-SA-UNet MI355X path has no fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    protos = parse_header()
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)  # AttributeError = exported symbol missing: fail loudly
        fn.restype = res
        fn.argtypes = args
    return lib, protos


LIB, PROTOS = _load()

# DFCSA_TUNE="knob=value,..." applies dfcsa_set_tuning knobs at load time (A/B experiments)
for _kv in filter(None, os.environ.get("DFCSA_TUNE", "").split(",")):
    _k, _v = _kv.split("=")
    LIB.dfcsa_set_tuning(int(_k), int(_v))


def call(name, *args):
    """Invoke an entry point; raise DfcsaError on a non-zero status."""
    rc = getattr(LIB, name)(*args)
    if rc != 0:
        what = "invalid argument/shape" if rc == EINVAL else f"HIP error {-rc}"
        raise DfcsaError(f"{name} failed: {what}")
    return rc


def version():
    return LIB.dfcsa_version().decode()
