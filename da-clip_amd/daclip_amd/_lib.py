"""ctypes binding of libdaclip_hip.so (C ABI: include/daclip_hip.h).

torch is imported BEFORE the library is loaded on purpose: the torch ROCm wheel bundles its
own libamdhip64.so.7 / libhsa-runtime64.so.1, and loading torch first makes the dynamic
linker resolve our library's NEEDED entries to those same objects (one HIP runtime per
process, so torch device pointers and streams are valid handles for the library).

There is no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# DAC_LIB_PATH: an alternative build of the same sources, for A/B measurements only. A stale
# value left in a shell would silently run another build, so setting it warns, and build_info()
# (printed by smoke() and carried in every bench line) names the library actually loaded.
DEFAULT_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdaclip_hip.so")
LIB_PATH = os.environ.get("DAC_LIB_PATH") or DEFAULT_LIB_PATH
if LIB_PATH != DEFAULT_LIB_PATH:
    import warnings
    warnings.warn(f"DAC_LIB_PATH is set: loading {LIB_PATH} instead of the in-tree {DEFAULT_LIB_PATH}",
                  RuntimeWarning, stacklevel=2)

DAC_F32, DAC_BF16, DAC_FP8, DAC_F16 = 0, 1, 2, 3
DAC_SRC_F32, DAC_SRC_F16, DAC_SRC_BF16 = 0, 1, 2
DAC_POSTERIOR, DAC_SDE = 0, 1
DAC_COSINE, DAC_LINEAR, DAC_CONSTANT = 0, 1, 2
DAC_E_MISSING, DAC_E_KEY = -3, -2
DAC_ATTN_Q_PRESCALED = 8

EXPORTS = ["dac_create", "dac_destroy", "dac_set_weight", "dac_finalize_weights",
           "dac_encode_image", "dac_encode_text", "dac_degradation_probs", "dac_unet_forward",
           "dac_sde_schedule", "dac_sde_set_time_scale", "dac_sde_reverse", "dac_build_id",
           "dac_set_noise_offset", "dac_posterior_step", "dac_unet_flops", "dac_encode_flops", "dac_profile_enable",
           "dac_profile_read", "dac_profile_mode", "dac_profile_launch", "dac_profile_graph_ms",
           "dac_op_attention", "dac_last_error"]


class DacConfig(ctypes.Structure):
    _fields_ = [("unet", ctypes.c_int), ("in_nc", ctypes.c_int), ("out_nc", ctypes.c_int),
                ("nf", ctypes.c_int), ("depth", ctypes.c_int), ("ch_mult", ctypes.c_int * 8),
                ("context_dim", ctypes.c_int), ("use_degra_context", ctypes.c_int),
                ("use_image_context", ctypes.c_int), ("vit", ctypes.c_int),
                ("image_size", ctypes.c_int), ("patch_size", ctypes.c_int),
                ("width", ctypes.c_int), ("layers", ctypes.c_int), ("head_width", ctypes.c_int),
                ("mlp_width", ctypes.c_int), ("embed_dim", ctypes.c_int),
                ("text", ctypes.c_int), ("context_length", ctypes.c_int), ("vocab_size", ctypes.c_int),
                ("text_width", ctypes.c_int), ("text_heads", ctypes.c_int), ("text_layers", ctypes.c_int),
                ("unet_scale_half", ctypes.c_int), ("unet_st_from", ctypes.c_int)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (or `make -C da-clip_amd`)")
    L = ctypes.CDLL(LIB_PATH)
    P, I, F, D, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_uint64
    sig = {
        "dac_create": (I, [I, I, ctypes.POINTER(DacConfig), ctypes.POINTER(P)]),
        "dac_destroy": (None, [P]),
        "dac_set_weight": (I, [P, ctypes.c_char_p, P, ctypes.POINTER(ctypes.c_int64), I, I]),
        "dac_finalize_weights": (I, [P]),
        "dac_encode_image": (I, [P, P, I, P, P, P]),
        "dac_encode_text": (I, [P, P, I, P, P]),
        "dac_degradation_probs": (I, [P, P, P, I, I, I, P, P, P]),
        "dac_unet_forward": (I, [P, P, P, F, P, P, I, I, I, P, P]),
        "dac_sde_schedule": (I, [P, F, I, I, F, P, F]),
        "dac_sde_set_time_scale": (I, [P, D]),
        "dac_sde_reverse": (I, [P, I, P, P, P, P, I, I, I, I, P, U64, P]),
        "dac_build_id": (ctypes.c_char_p, []),
        "dac_set_noise_offset": (I, [P, U64]),
        "dac_posterior_step": (I, [P, I, P, P, P, P, I, I, P]),
        "dac_unet_flops": (D, [P, I, I, I]),
        "dac_encode_flops": (D, [P, I]),
        "dac_profile_enable": (I, [P, I]),
        "dac_profile_read": (I, [P, ctypes.POINTER(D), ctypes.POINTER(D), ctypes.POINTER(D)]),
        "dac_profile_mode": (I, [P, I]),
        "dac_profile_launch": (I, [P, I, ctypes.POINTER(D), ctypes.POINTER(D), ctypes.POINTER(D),
                                   ctypes.POINTER(I), ctypes.POINTER(D), ctypes.POINTER(I),
                                   ctypes.c_char_p, I, ctypes.c_char_p, I]),
        "dac_profile_graph_ms": (I, [P, ctypes.POINTER(D)]),
        "dac_op_attention": (I, [P, P, I, I, I, I, I, P]),
        "dac_last_error": (ctypes.c_char_p, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Handle:
    """Owns one dac_handle (one network set on one GPU)."""

    def __init__(self, device: torch.device, dtype: str, cfg: DacConfig):
        if not torch.cuda.is_available():
            raise RuntimeError("daclip_amd needs a ROCm GPU (HIP path only, no CPU fallback)")
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.dtype = dtype
        self.cfg = cfg
        h = ctypes.c_void_p()
        code = {"fp32": DAC_F32, "bf16": DAC_BF16, "fp8": DAC_FP8, "fp16": DAC_F16}[dtype]
        with torch.cuda.device(idx):
            rc = lib().dac_create(idx, code, ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"dac_create failed ({rc})")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.dac_destroy(self.h)
            self.h = None

    def check(self, rc: int, what: str):
        if rc < 0:
            msg = lib().dac_last_error(self.h).decode()
            raise RuntimeError(f"{what}: {msg}")
        return rc

    def set_weight(self, key: str, t: torch.Tensor):
        t = t.detach().contiguous()
        src = {torch.float32: DAC_SRC_F32, torch.float16: DAC_SRC_F16,
               torch.bfloat16: DAC_SRC_BF16}.get(t.dtype)
        if src is None:
            t = t.float()
            src = DAC_SRC_F32
        shape = (ctypes.c_int64 * max(1, t.dim()))(*t.shape)
        with torch.cuda.device(self.device):
            self.check(lib().dac_set_weight(self.h, key.encode(), ctypes.c_void_p(t.data_ptr()),
                                            shape, t.dim(), src), f"set_weight({key})")

    def finalize(self):
        with torch.cuda.device(self.device):
            self.check(lib().dac_finalize_weights(self.h), "finalize_weights")

    def stream(self):
        return _stream(self.device)


def source_hash() -> str:
    """sha256 (first 16 hex digits) over csrc/* in byte order of the names, then the public
    header and the Makefile: the value the Makefile bakes into dac_build_id()."""
    import glob
    import hashlib
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*")), key=lambda p: os.path.basename(p).encode())
    files.append(os.path.join(os.path.dirname(pkg), "include", "daclip_hip.h"))
    files.append(os.path.join(pkg, "Makefile"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info() -> dict:
    """{"build_id": the loaded library's id, "source_hash": this tree's, "matches": bool,
    "lib_path": the file loaded, "lib_override": whether DAC_LIB_PATH chose it}."""
    bid = lib().dac_build_id().decode()
    src = source_hash()
    return {"build_id": bid, "source_hash": src, "matches": bid.split(" ")[0] == src,
            "lib_path": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(os.path.dirname(
                os.path.abspath(__file__))))), "lib_override": LIB_PATH != DEFAULT_LIB_PATH}


def exports_present(names: Sequence[str] = EXPORTS):
    L = ctypes.CDLL(LIB_PATH)
    return {n: hasattr(L, n) for n in names}
