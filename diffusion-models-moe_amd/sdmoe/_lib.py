"""ctypes binding of libsdmoe_hip.so (the C ABI declared in include/sdmoe.h).

The product path has exactly one compute backend: these HIP kernels. If the shared library is missing or
fails to load, every op raises -- there is no eager-PyTorch or CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsdmoe_hip.so")

_P = ctypes.c_void_p
_L = ctypes.c_long
_I = ctypes.c_int
_F = ctypes.c_float
_FP = ctypes.POINTER(ctypes.c_float)

# name -> argtypes, in the exact order of include/sdmoe.h
SIGNATURES = {
    "sdmoe_linear": [_P, _L, _P, _L, _P, _P, _L, _I, _P, _L, _P, _L, _I, _I, _I, _I, _P, _L, _P],
    "sdmoe_conv3x3": [_P, _L, _I, _I, _I, _I, _P, _P, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _P, _L, _P],
    "sdmoe_conv3x3_sc": [_P, _L, _I, _I, _I, _I, _P, _P, _P, _L, _P, _L, _I, _P, _L, _I, _I, _P, _L, _P],
    "sdmoe_conv3x3_gn": [_P, _L, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P, _L, _P, _L, _P, _L, _I, _P, _L, _I, _P, _L,
                         _P],
    "sdmoe_groupnorm_apply": [_P, _L, _I, _I, _I, _P, _P, _I, _P, _L, _P],
    "sdmoe_mask_weight": [_P, _P, _L, _L, _P, _P],
    "sdmoe_groupnorm_stats": [_P, _L, _I, _I, _I, _I, _P, _P, _F, _P, _P, _P, _L, _P],
    "sdmoe_groupnorm": [_P, _L, _I, _I, _I, _I, _P, _P, _F, _I, _P, _L, _P, _P, _P, _L, _P],
    "sdmoe_gn_fold": [_P, _L, _I, _I, _P, _P, _P, _I, _P, _P, _P],
    "sdmoe_linear_per_image": [_P, _L, _P, _L, _L, _P, _L, _I, _P, _L, _P, _L, _I, _I, _I, _P, _L, _P],
    "sdmoe_layernorm": [_P, _L, _P, _L, _I, _I, _P, _P, _F, _P],
    "sdmoe_ln_fold": [_P, _L, _I, _I, _P, _P, _P, _P, _L, _P, _P, _P],
    "sdmoe_linear_ln": [_P, _L, _P, _L, _P, _P, _F, _P, _L, _I, _I, _I, _P],
    "sdmoe_linear_geglu_ln": [_P, _L, _P, _L, _P, _P, _F, _P, _L, _I, _I, _I, _I, _P, _L, _I, _P],
    "sdmoe_attention": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _F, _P],
    "sdmoe_geglu_route": [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _L, _P, _L, _P, _P, _P],
    "sdmoe_linear_geglu": [_P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _P, _L, _I, _P],
    "sdmoe_moe_topk_mask": [_P, _L, _I, _I, _I, _I, _I, _P, _L, _P, _P, _P],
    "sdmoe_moe_topk_keep": [_I, _I, _I, _I, _I, _P, _L, _P, _P, _P, _P],
    "sdmoe_linear_keep": [_P, _L, _P, _P, _L, _P, _P, _L, _P, _L, _I, _I, _I, _P, _L, _P],
    "sdmoe_linear_masked": [_P, _L, _P, _P, _L, _P, _P, _P, _L, _P, _L, _I, _I, _I, _P, _L, _P],
    "sdmoe_gemm_plan": [_I, _I, _I, _I, _I, _I, _L, _P],
    "sdmoe_wmask_kmajor": [_P, _L, _I, _I, _P, _P, _P],
    "sdmoe_timestep_embedding": [_P, _P, _F, _I, _I, _F, _P],
    "sdmoe_cfg_multistep_step": [_P, _L, _P, _I, _I, _I, _F, _P, _P, _P, _P, _P, _L, _P],
    "sdmoe_sqdist_f32": [_P, _L, _P, _L, _I, _I, _I, _P, _L, _P],
    "sdmoe_balanced_assign": [_P, _I, _I, ctypes.c_double, _P, _I, _P],
    "sdmoe_expert_mean_topk": [_P, _L, _I, _I, _I, _P, _I, _I, _P, _P, _P, _L, _P],
    "sdmoe_colnorm_accum": [_P, _L, _I, _I, _P, _P, _L, _P],
    "sdmoe_wanda_mask": [_P, _L, _I, _I, _P, _P, _I, _P, _P],
    "sdmoe_union_over_time": [_P, _L, _I, _L, _F, _P, _P],
    "sdmoe_softmax_rows": [_P, _L, _P, _L, _I, _I, _P],
    "sdmoe_transpose": [_P, _L, _P, _L, _I, _I, _P],
    "sdmoe_gather_rows": [_P, _L, _P, _I, _I, _P, _L, _I, _P, _L, _P],
    "sdmoe_attention_short": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _F, _I, _P],
    "sdmoe_timestep_embedding_rows": [_P, _L, _P, _I, _I, _I, _I, _F, _P],
    "sdmoe_prepare_input": [_P, _P, _I, _I, _L, _I, _P],
    "sdmoe_cfg_ddim_step": [_P, _L, _P, _I, _I, _I, _F, _F, _F, _P, _L, _P],
    "sdmoe_add": [_P, _P, _P, _L, _P],
    "sdmoe_tune": [_I, _I],
    "sdmoe_set_gelu_table": [_P],
    "sdmoe_version": [],
}

ERRORS = {-1: "bad pointer/size", -2: "unsupported shape/alignment", -3: "unsupported mode"}

_lib = None


class SdmoeError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the library with typed entry points. Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("SDMOE_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise SdmoeError(
            f"libsdmoe_hip.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C diffusion-models-moe_amd/csrc`). There is no CPU fallback."
        )
    lib = ctypes.CDLL(p)
    # same-box A/B against an older build (SDMOE_AB=1, with SDMOE_LIB naming it): entry points it lacks stay unbound
    # and the callers that probe with has() take their older path; otherwise a missing symbol is an error
    ab_lib = os.environ.get("SDMOE_AB", "0") == "1"
    for name, argt in SIGNATURES.items():
        if ab_lib and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = ctypes.c_char_p if name == "sdmoe_version" else ctypes.c_int
    # A/B experiments without code changes: SDMOE_TUNE="knob=value,..." (sdmoe_tune, include/sdmoe.h)
    for k, v in parse_tune(os.environ.get("SDMOE_TUNE", "")):
        check(lib.sdmoe_tune(k, v), f"sdmoe_tune({k}={v})")
    _lib = lib
    return lib


def parse_tune(spec: str):
    """SDMOE_TUNE="knob=value,..." -> [(knob, value)]; malformed entries raise SdmoeError (not a bare ValueError)."""
    out = []
    for kv in filter(None, (s.strip() for s in spec.split(","))):
        parts = kv.split("=")
        if len(parts) != 2:
            raise SdmoeError(f"SDMOE_TUNE entry {kv!r}: expected knob=value")
        try:
            out.append((int(parts[0]), int(parts[1])))
        except ValueError:
            raise SdmoeError(f"SDMOE_TUNE entry {kv!r}: knob and value must be integers") from None
    return out


def has(lib, name: str) -> bool:
    """Whether the loaded library exports `name` (only an SDMOE_AB=1 build may lack one)."""
    return hasattr(lib, name)


def check(status: int, what: str):
    if status != 0:
        msg = ERRORS.get(status, f"hipError_t {status}")
        raise SdmoeError(f"{what} failed: {msg} ({status})")
