"""Torch-facing wrappers of the HIP kernels (libsdmoe_hip.so).

PyTorch is used only for device memory and streams: every op here validates its operands, hands raw device
pointers plus sizes to the C ABI (include/sdmoe.h) on the current HIP stream, and returns. Nothing falls back
to an eager or CPU implementation; a missing library or a non-GPU tensor raises.

Activations are 2-D row-major views [rows, channels] whose row stride may exceed the channel count (channel
slices of a concatenation buffer, fused QKV outputs); spatial tensors are NHWC flattened to [images*H*W, C].
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

ACT_NONE, ACT_SILU, ACT_GELU, ACT_RELU, ACT_QUICK_GELU = 0, 1, 2, 3, 4
ACT_BY_NAME = {"none": ACT_NONE, "silu": ACT_SILU, "gelu": ACT_GELU, "relu": ACT_RELU, "quick_gelu": ACT_QUICK_GELU}


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """hipStream_t of torch's current stream on the current device. The C accessors skip the Python Stream object
    and device-index resolution of torch.cuda.current_stream() (2.7 us -> ~0.3 us per launch; ~370 launches per
    U-Net evaluation)."""
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _rows(t: torch.Tensor, name: str):
    """(data_ptr, row stride) of a 2-D row-major fp16 device view."""
    if t.dim() != 2:
        raise ValueError(f"{name}: expected a 2-D [rows, channels] view, got shape {tuple(t.shape)}")
    if not t.is_cuda:
        raise _lib.SdmoeError(f"{name}: tensor is not on a GPU device; sdmoe has no CPU path")
    if t.dtype != torch.float16:
        raise TypeError(f"{name}: expected float16, got {t.dtype}")
    if t.stride(1) != 1 and t.shape[1] > 1:
        raise ValueError(f"{name}: inner dimension must be contiguous")
    return t.data_ptr(), t.stride(0)


def _dev(t: torch.Tensor, name: str, dtype=torch.float16):
    if not t.is_cuda:
        raise _lib.SdmoeError(f"{name}: tensor is not on a GPU device; sdmoe has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    return t.data_ptr()


_WS = {}
WS_FLOATS = 32 * 1024 * 1024  # split-K fp32 partial slabs (128 MB per device), reused stream-ordered


def _workspace(device):
    ws = _WS.get(device)
    if ws is None:
        ws = _WS[device] = torch.empty(WS_FLOATS, dtype=torch.float32, device=device)
    return ws


_GN_WS = {}


def _gn_workspace(device, floats):
    """GroupNorm partial-sum scratch (reused across calls; no allocation per call)."""
    ws = _GN_WS.get(device)
    if ws is None or ws.numel() < floats:
        ws = _GN_WS[device] = torch.zeros(max(floats, 1 << 16), dtype=torch.float32, device=device)
    return ws


def groupnorm_apply(x, nimg, HW, scale, shift, silu, out=None):
    """out = (SiLU?)(x * scale[img, c] + shift[img, c]) on [nimg*HW, C] views."""
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    C = x.shape[1]
    if out is None:
        out = torch.empty((x.shape[0], C), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    st = lib.sdmoe_groupnorm_apply(xp, ldx, nimg, HW, C, scale.data_ptr(), shift.data_ptr(), int(bool(silu)), op,
                                   ldy, _stream())
    _lib.check(st, "sdmoe_groupnorm_apply")
    return out


def mask_weight(w, bits, out=None):
    """Wanda-masked copy of w [N, K]: bit (n, k) of bits [N, K/8] set -> 0."""
    lib = _lib.load()
    N, K = w.shape
    if tuple(bits.shape) != (N, K // 8) or bits.dtype != torch.uint8:
        raise ValueError(f"mask bits {tuple(bits.shape)} {bits.dtype} do not match weight {tuple(w.shape)}")
    if out is None:
        out = torch.empty_like(w)
    st = lib.sdmoe_mask_weight(_dev(w, "w"), _dev(bits, "bits", torch.uint8), N, K, _dev(out, "out"), _stream())
    _lib.check(st, "sdmoe_mask_weight")
    return out


def wmask_kmajor(bits, perm=None, out=None):
    """Packed Wanda bits [N, K/8] (bit set = weight removed) -> the masked GEMM's K-step-major layout int64
    [K/64, N] (sdmoe_wmask_kmajor); perm (int32 [K], optional): column j of the result = column perm[j] of the
    mask (the routed FFN's expert-major neuron order). Made once per (t, l) mask, not per call."""
    lib = _lib.load()
    if bits.dim() != 2 or bits.dtype != torch.uint8:
        raise ValueError(f"wmask bits must be uint8 [N, K/8], got {bits.dtype} {tuple(bits.shape)}")
    N, K = bits.shape[0], bits.shape[1] * 8
    if out is None:
        out = torch.empty((K // 64, N), dtype=torch.int64, device=bits.device)
    pp = None
    if perm is not None:
        if perm.dtype != torch.int32 or perm.numel() != K:
            raise ValueError("perm must be int32 [K]")
        pp = _dev(perm, "perm", torch.int32)
    st = lib.sdmoe_wmask_kmajor(_dev(bits, "bits", torch.uint8), bits.stride(0), N, K, pp,
                                _dev(out, "out", torch.int64), _stream())
    _lib.check(st, "sdmoe_wmask_kmajor")
    return out


GEMM_PLAN_MODES = {"plain": 0, "keep": 4, "wmask": 5, "keepw": 6, "ln": 7}


def gemm_plan(mode, M, N, K, residual=False, act=ACT_NONE, workspace_floats=WS_FLOATS):
    """The launch sdmoe_linear / _linear_masked / _linear_ln would make for an M x N x K product (sdmoe_gemm_plan,
    host-only: no device needed): {"tile": (rows, cols), "waves": (along M, along N), "ksplit": k}."""
    lib = _lib.load()
    out = (ctypes.c_int * 5)()
    _lib.check(lib.sdmoe_gemm_plan(GEMM_PLAN_MODES[mode], M, N, K, int(bool(residual)), act, workspace_floats, out),
               "sdmoe_gemm_plan")
    return {"tile": (out[0], out[1]), "waves": (out[2], out[3]), "ksplit": out[4]}


def linear_masked(x, w, bias=None, *, keep=None, wmask=None, residual=None, out=None):
    """out = (x ⊙ keep) @ (w ⊙ (1 - M))^T + bias + residual (sdmoe_linear_masked): keep int64 [K/64, M] (A keep bits,
    sdmoe_moe_topk_keep), wmask int64 [K/64, N] (wmask_kmajor). Either may be None."""
    lib = _lib.load()
    xp, lda = _rows(x, "x")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear_masked: weight {tuple(w.shape)} does not match input K={K}")
    if keep is not None and (tuple(keep.shape) != (K // 64, M) or keep.dtype != torch.int64):
        raise ValueError(f"keep must be int64 [{K // 64}, {M}], got {keep.dtype} {tuple(keep.shape)}")
    if wmask is not None and (tuple(wmask.shape) != (K // 64, N) or wmask.dtype != torch.int64):
        raise ValueError(f"wmask must be int64 [{K // 64}, {N}], got {wmask.dtype} {tuple(wmask.shape)}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=x.device)
    op, ldc = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    ws = _workspace(x.device)
    st = lib.sdmoe_linear_masked(xp, lda, None if keep is None else _dev(keep, "keep", torch.int64), _dev(w, "w"),
                                 w.stride(0), None if wmask is None else _dev(wmask, "wmask", torch.int64),
                                 _ptr(bias), rp, ldr, op, ldc, M, N, K, ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_linear_masked")
    return out


def linear(x, w, bias=None, *, out=None, residual=None, act=ACT_NONE, coladd=None, coladd_bstride=0,
           rows_per_batch=0, gn=None, wmask=None, wmask_bits=None):
    """out = act(GN?(x) @ w.T + bias + coladd) + residual.  w: [N, K] fp16 (nn.Linear layout).
    gn = (scale, shift, silu): per-(image, channel) GroupNorm apply on x first (rows_per_batch rows/image).
    wmask: Wanda mask in the GEMM's layout (wmask_kmajor) applied to the W fragments in the GEMM
    (remove_wanda_neurons_fast.py:69-83); wmask_bits: the same mask packed [N, K/8], converted on this call."""
    lib = _lib.load()
    if gn is not None:
        x = groupnorm_apply(x, x.shape[0] // rows_per_batch, rows_per_batch, gn[0], gn[1], gn[2])
    if wmask_bits is not None:
        if tuple(wmask_bits.shape) != (w.shape[0], w.shape[1] // 8):
            raise ValueError(f"mask bits {tuple(wmask_bits.shape)} do not match weight {tuple(w.shape)}")
        wmask = wmask_kmajor(wmask_bits)
    if wmask is not None:
        if act != ACT_NONE or coladd is not None:
            raise ValueError("linear: a Wanda weight mask combines with bias/residual only")
        return linear_masked(x, w, bias, wmask=wmask, residual=residual, out=out)
    xp, lda = _rows(x, "x")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: weight {tuple(w.shape)} does not match input K={K}")
    wp = _dev(w, "w")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=x.device)
    op, ldc = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    ws = _workspace(x.device)
    st = lib.sdmoe_linear(xp, lda, wp, w.stride(0), _ptr(bias), _ptr(coladd), coladd_bstride, rows_per_batch,
                          rp, ldr, op, ldc, M, N, K, act, ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_linear")
    return out


def conv_weight(w):
    """Conv weight in the kernel's layout [Cout, Cin/64, 3, 3, 64] from [Cout, 3, 3, Cin] (taps-last NHWC filter)
    or a torch [Cout, Cin, 3, 3] filter (pass nchw=True-shaped tensors through conv_weight_from_torch). K runs over
    (64-channel slice, tap, channel): the 9 taps of one slice are consecutive K-steps of the implicit GEMM."""
    Cout, kh, kw, Cin = w.shape
    if (kh, kw) != (3, 3) or Cin % 64:
        raise ValueError(f"conv_weight: expected [Cout, 3, 3, Cin] with Cin % 64 == 0, got {tuple(w.shape)}")
    return w.reshape(Cout, 9, Cin // 64, 64).permute(0, 2, 1, 3).reshape(Cout, Cin // 64, 3, 3, 64).contiguous()


def conv_weight_from_torch(w):
    """torch.nn.Conv2d weight [Cout, Cin, 3, 3] -> conv_weight layout."""
    return conv_weight(w.permute(0, 2, 3, 1))


def conv_weight_with_shortcut(w, w_sc):
    """[Cout, 9*Cin + Cin2]: the conv3x3 weight (conv_weight layout) with a 1x1 shortcut's [Cout, Cin2] columns
    appended — the operand of conv3x3(..., shortcut=x2) (sdmoe_conv3x3_sc)."""
    return torch.cat([w.reshape(w.shape[0], -1), w_sc.reshape(w.shape[0], -1)], 1).contiguous()


def conv3x3(x, nimg, H, W, w, bias=None, *, stride=1, upsample=False, out=None, residual=None, act=ACT_NONE,
            coladd=None, coladd_bstride=0, gn=None, shortcut=None):
    """3x3 conv (pad 1) on NHWC x viewed as [nimg*H*W, Cin]; w: [Cout, Cin/64, 3, 3, 64] fp16 (conv_weight).
    gn = (scale, shift, silu): GroupNorm(+SiLU) applied to x once (one read + write of x) before the conv.
    shortcut = x2 [nimg*H*W, Cin2]: a 1x1 projection of x2 folded in as extra K-steps (stride 1, no residual);
    w is then conv_weight_with_shortcut(...) [Cout, 9*Cin + Cin2]."""
    lib = _lib.load()
    if gn is not None:
        if stride == 1 and not upsample and act == ACT_NONE and conv_gn_fusable(H, W, x.shape[1], w.shape[0]):
            y = _conv3x3_gn(lib, x, nimg, H, W, w, bias, out, residual, coladd, coladd_bstride, gn, shortcut)
            if y is not None:
                return y
        x = groupnorm_apply(x, nimg, H * W, gn[0], gn[1], gn[2])
    xp, ldx = _rows(x, "x")
    Cin = x.shape[1]
    Cout = w.shape[0]
    if shortcut is not None:
        x2p, ldx2 = _rows(shortcut, "shortcut")
        Cin2 = shortcut.shape[1]
        if w.dim() != 2 or w.shape[1] != 9 * Cin + Cin2 or Cin % 64 or Cin2 % 64:
            raise ValueError(f"conv3x3: weight {tuple(w.shape)} is not [Cout, 9*{Cin} + {Cin2}] "
                             "(ops.conv_weight_with_shortcut)")
        if stride != 1 or upsample or residual is not None or shortcut.shape[0] != x.shape[0]:
            raise ValueError("conv3x3: a folded shortcut needs stride 1, no upsample, no residual, same rows")
        if x.shape[0] != nimg * H * W:
            raise ValueError("conv3x3: rows != nimg*H*W")
        if out is None:
            out = torch.empty((nimg * H * W, Cout), dtype=torch.float16, device=x.device)
        op, ldy = _rows(out, "out")
        return conv3x3_launch(xp, ldx, nimg, H, W, Cin, w, bias, coladd, coladd_bstride, None, 0, out, op, ldy, Cout,
                              1, False, act, sc=(x2p, ldx2, Cin2))
    if w.dim() != 5 or tuple(w.shape[1:]) != (Cin // 64, 3, 3, 64) or Cin % 64:
        raise ValueError(f"conv3x3: weight {tuple(w.shape)} is not the [Cout, Cin/64, 3, 3, 64] layout for "
                         f"Cin={Cin} (ops.conv_weight)")
    if x.shape[0] != nimg * H * W:
        raise ValueError("conv3x3: rows != nimg*H*W")
    if upsample:
        OH, OW = 2 * H, 2 * W
    else:
        OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    if out is None:
        out = torch.empty((nimg * OH * OW, Cout), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    return conv3x3_launch(xp, ldx, nimg, H, W, Cin, w, bias, coladd, coladd_bstride, rp, ldr, out, op, ldy, Cout,
                          stride, upsample, act)


FUSED_GN = os.environ.get("SDMOE_FUSED_GN", "1") != "0"  # GroupNorm(+SiLU) inside the halo conv (0: apply pass)


def conv_gn_fusable(H, W, Cin, Cout):
    """Shapes whose conv applies a GroupNorm in the kernel (sdmoe_conv3x3_gn: the 64-wide halo tiles)."""
    return (FUSED_GN and W == 64 and (H * W) % 256 == 0 and Cin <= 1280 and Cin % 64 == 0 and Cout % 320 == 0
            and _lib.has(_lib.load(), "sdmoe_conv3x3_gn"))


def _conv3x3_gn(lib, x, nimg, H, W, w, bias, out, residual, coladd, coladd_bstride, gn, shortcut):
    """conv3x3(act(GroupNorm(x))) with the norm applied to the staged input inside the conv; None if unsupported."""
    xp, ldx = _rows(x, "x")
    Cin, Cout = x.shape[1], w.shape[0]
    if x.shape[0] != nimg * H * W:
        raise ValueError("conv3x3: rows != nimg*H*W")
    x2p, ldx2, Cin2 = None, 0, 0
    if shortcut is not None:
        x2p, ldx2 = _rows(shortcut, "shortcut")
        Cin2 = shortcut.shape[1]
        if w.dim() != 2 or w.shape[1] != 9 * Cin + Cin2 or residual is not None:
            raise ValueError(f"conv3x3: weight {tuple(w.shape)} is not [Cout, 9*{Cin} + {Cin2}] or a residual was given")
    elif w.dim() != 5 or tuple(w.shape[1:]) != (Cin // 64, 3, 3, 64):
        raise ValueError(f"conv3x3: weight {tuple(w.shape)} is not the [Cout, Cin/64, 3, 3, 64] layout for Cin={Cin}")
    sc, sh, silu = gn
    if tuple(sc.shape) != (nimg, Cin) or sc.dtype != torch.float32 or tuple(sh.shape) != (nimg, Cin):
        raise ValueError("conv3x3: gn scale / shift must be fp32 [nimg, Cin]")
    if out is None:
        out = torch.empty((nimg * H * W, Cout), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    return conv3x3_gn_launch(xp, ldx, nimg, H, W, Cin, w, bias, coladd, coladd_bstride, rp, ldr, out, op, ldy, Cout,
                             (sc, sh, silu), sc=(x2p, ldx2, Cin2) if shortcut is not None else None)


def conv3x3_gn_launch(xp, ldx, nimg, H, W, Cin, w, bias, coladd, coladd_bstride, rp, ldr, out, op, ldy, Cout, gn,
                      sc=None):
    """The sdmoe_conv3x3_gn launch alone (argument order of conv3x3_launch: bench.py times both families); None when
    the shape is not one the kernel normalises itself."""
    lib = _lib.load()
    ws = _workspace(out.device)
    x2p, ldx2, Cin2 = sc if sc is not None else (None, 0, 0)
    st = lib.sdmoe_conv3x3_gn(xp, ldx, nimg, H, W, Cin, gn[0].data_ptr(), gn[1].data_ptr(), int(bool(gn[2])),
                              _dev(w, "w"), _ptr(bias), _ptr(coladd), coladd_bstride, rp, ldr, x2p, ldx2, Cin2, op, ldy,
                              Cout, ws.data_ptr(), ws.numel(), _stream())
    if st == -3:
        return None
    _lib.check(st, "sdmoe_conv3x3_gn")
    return out


def conv3x3_launch(xp, ldx, nimg, H, W, Cin, w, bias, coladd, coladd_bstride, rp, ldr, out, op, ldy, Cout, stride,
                   upsample, act, sc=None):
    """The sdmoe_conv3x3 launch alone (bench.py times exactly this with HIP events); sc = (x2 ptr, ldx2, Cin2):
    sdmoe_conv3x3_sc with the folded 1x1 shortcut."""
    lib = _lib.load()
    ws = _workspace(out.device)
    if sc is not None:
        st = lib.sdmoe_conv3x3_sc(xp, ldx, nimg, H, W, Cin, _dev(w, "w"), _ptr(bias), _ptr(coladd), coladd_bstride,
                                  sc[0], sc[1], sc[2], op, ldy, Cout, act, ws.data_ptr(), ws.numel(), _stream())
        _lib.check(st, "sdmoe_conv3x3_sc")
        return out
    st = lib.sdmoe_conv3x3(xp, ldx, nimg, H, W, Cin, _dev(w, "w"), _ptr(bias), _ptr(coladd), coladd_bstride, rp, ldr,
                           op, ldy, Cout, stride, int(bool(upsample)), act, ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_conv3x3")
    return out


def groupnorm_stats(x, nimg, HW, gamma, beta, eps, groups=32):
    """Per-(image, channel) fp32 (scale, shift) of GroupNorm(groups) over x viewed as [nimg*HW, C]."""
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    C = x.shape[1]
    scale = torch.empty((nimg, C), dtype=torch.float32, device=x.device)
    shift = torch.empty((nimg, C), dtype=torch.float32, device=x.device)
    ws = _gn_workspace(x.device, nimg * groups * 64 * 2)
    st = lib.sdmoe_groupnorm_stats(xp, ldx, nimg, HW, C, groups, _dev(gamma, "gamma"), _dev(beta, "beta"),
                                   float(eps), scale.data_ptr(), shift.data_ptr(), ws.data_ptr(), ws.numel(),
                                   _stream())
    _lib.check(st, "sdmoe_groupnorm_stats")
    return scale, shift


def groupnorm(x, nimg, HW, gamma, beta, eps, groups=32, silu=False, out=None):
    """act(GroupNorm(x)) as a new [nimg*HW, C] fp16 tensor (sdmoe_groupnorm: statistics + apply)."""
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    C = x.shape[1]
    scale = torch.empty((nimg, C), dtype=torch.float32, device=x.device)
    shift = torch.empty((nimg, C), dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty((x.shape[0], C), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    ws = _gn_workspace(x.device, nimg * groups * 64 * 2)
    st = lib.sdmoe_groupnorm(xp, ldx, nimg, HW, C, groups, _dev(gamma, "gamma"), _dev(beta, "beta"), float(eps),
                             int(bool(silu)), op, ldy, scale.data_ptr(), shift.data_ptr(), ws.data_ptr(), ws.numel(),
                             _stream())
    _lib.check(st, "sdmoe_groupnorm")
    return out


def gn_fold(w, bias, scale, shift):
    """Per-image GroupNorm-folded weights of a linear (sdmoe_gn_fold): Wf [nimg, N, K] fp16 and colbias [nimg, N]
    fp32 with x . Wf[i]^T + colbias[i] = GN(x) . w^T + bias on the rows of image i (scale / shift from
    groupnorm_stats)."""
    lib = _lib.load()
    N, K = w.shape
    nimg = scale.shape[0]
    if tuple(scale.shape) != (nimg, K) or tuple(shift.shape) != (nimg, K):
        raise ValueError(f"gn_fold: scale/shift {tuple(scale.shape)} do not match weight {tuple(w.shape)}")
    wf = torch.empty((nimg, N, K), dtype=torch.float16, device=w.device)
    cb = torch.empty((nimg, N), dtype=torch.float32, device=w.device)
    st = lib.sdmoe_gn_fold(_dev(w, "w"), w.stride(0), N, K, _ptr(bias), _dev(scale, "scale", torch.float32),
                           _dev(shift, "shift", torch.float32), nimg, wf.data_ptr(), cb.data_ptr(), _stream())
    _lib.check(st, "sdmoe_gn_fold")
    return wf, cb


def linear_per_image(x, wf, colbias, rows_per_batch, *, residual=None, out=None):
    """out[m] = x[m] . wf[m // rows_per_batch]^T + colbias[m // rows_per_batch] (+ residual): the GEMM behind a folded
    GroupNorm (sdmoe_linear_per_image; rows_per_batch % 256 == 0)."""
    lib = _lib.load()
    xp, lda = _rows(x, "x")
    M, K = x.shape
    nimg, N, Kw = wf.shape
    if Kw != K or M != nimg * rows_per_batch or tuple(colbias.shape) != (nimg, N):
        raise ValueError(f"linear_per_image: x {tuple(x.shape)}, wf {tuple(wf.shape)}, colbias "
                         f"{tuple(colbias.shape)}, rows_per_batch {rows_per_batch}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=x.device)
    op, ldc = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    ws = _workspace(x.device)
    st = lib.sdmoe_linear_per_image(xp, lda, _dev(wf, "wf"), wf.stride(1), wf.stride(0),
                                    _dev(colbias, "colbias", torch.float32), colbias.stride(0), rows_per_batch, rp,
                                    ldr, op, ldc, M, N, K, ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_linear_per_image")
    return out


def layernorm(x, gamma, beta, eps=1e-5, out=None):
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    M, C = x.shape
    if out is None:
        out = torch.empty((M, C), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    st = lib.sdmoe_layernorm(xp, ldx, op, ldy, M, C, _dev(gamma, "gamma"), _dev(beta, "beta"), float(eps), _stream())
    _lib.check(st, "sdmoe_layernorm")
    return out


class LNFold:
    """LayerNorm(gamma, beta) folded into a following linear W [N, K] (+ bias): wf = fp16(W diag(gamma)), bias_f =
    bias + W beta and wsum = rowsum(wf) in fp32 (sdmoe_ln_fold) — the operands of sdmoe_linear_ln /
    sdmoe_linear_geglu_ln. Built once per (weight, norm) version by the owning module."""

    def __init__(self, w, gamma, beta, eps, bias=None):
        lib = _lib.load()
        N, K = w.shape
        self.eps = float(eps)
        self.w = torch.empty((N, K), dtype=torch.float16, device=w.device)
        self.bias = torch.empty(N, dtype=torch.float32, device=w.device)
        self.wsum = torch.empty(N, dtype=torch.float32, device=w.device)
        if bias is not None:
            _dev(bias, "bias")
        st = lib.sdmoe_ln_fold(_dev(w, "w"), w.stride(0), N, K, _dev(gamma, "gamma"), _dev(beta, "beta"), _ptr(bias),
                               self.w.data_ptr(), K, self.bias.data_ptr(), self.wsum.data_ptr(), _stream())
        _lib.check(st, "sdmoe_ln_fold")

    def rows(self, idx):
        """The fold with its rows reordered (torch index tensor): a view-free copy for permuted layouts."""
        f = LNFold.__new__(LNFold)
        f.eps, f.w, f.bias, f.wsum = self.eps, self.w[idx].contiguous(), self.bias[idx].contiguous(), \
            self.wsum[idx].contiguous()
        return f


def linear_ln(x, fold: LNFold, out=None):
    """out = LayerNorm(x) @ W^T + bias with the norm folded into the GEMM (sdmoe_linear_ln): x is the
    un-normalised [M, K] input; no normalised copy of x is written."""
    lib = _lib.load()
    xp, lda = _rows(x, "x")
    M, K = x.shape
    N = fold.w.shape[0]
    if fold.w.shape[1] != K:
        raise ValueError(f"linear_ln: folded weight {tuple(fold.w.shape)} does not match input K={K}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=x.device)
    op, ldc = _rows(out, "out")
    st = lib.sdmoe_linear_ln(xp, lda, fold.w.data_ptr(), fold.w.stride(0), fold.bias.data_ptr(), fold.wsum.data_ptr(),
                             fold.eps, op, ldc, M, N, K, _stream())
    _lib.check(st, "sdmoe_linear_ln")
    return out


def attention(q, k, v, nimg, Nq, Nk, heads, out=None, scale=None):
    """softmax(q k^T * scale) v per (image, head); q [nimg*Nq, heads*d], k/v [nimg*Nk, heads*d] views."""
    lib = _lib.load()
    qp, ldq = _rows(q, "q")
    kp, ldk = _rows(k, "k")
    vp, ldv = _rows(v, "v")
    C = q.shape[1]
    d = C // heads
    if out is None:
        out = torch.empty((nimg * Nq, C), dtype=torch.float16, device=q.device)
    op, ldo = _rows(out, "out")
    if scale is None:
        scale = d ** -0.5
    st = lib.sdmoe_attention(qp, ldq, kp, ldk, vp, ldv, op, ldo, nimg, Nq, Nk, heads, d, float(scale), _stream())
    _lib.check(st, "sdmoe_attention")
    return out


class Routing:
    """Device-side expert layout of one MoE-fied GEGLU: labels [F] int32 and the per-expert neuron lists
    (CSR), built once from the reference's `module.patterns` [E, F] (helper.py:48-62) or its label file."""

    def __init__(self, labels: torch.Tensor, num_experts: int, k: int, device):
        labels = labels.to(torch.int64).cpu()
        F = labels.numel()
        if labels.min() < 0 or labels.max() >= num_experts:
            raise ValueError("expert labels out of range")
        order = torch.argsort(labels, stable=True)
        counts = torch.bincount(labels, minlength=num_experts)
        off = torch.zeros(num_experts + 1, dtype=torch.int64)
        off[1:] = torch.cumsum(counts, 0)
        self.F, self.E, self.k = F, int(num_experts), int(k)
        self.labels = labels.to(torch.int32).to(device)
        self.e_off = off.to(torch.int32).to(device)
        self.e_nid = order.to(torch.int32).to(device)
        # fused path (sdmoe_linear_geglu + sdmoe_moe_topk_mask): balanced experts (the reference's
        # KMeansConstrained split), permuted expert-major so every expert is a contiguous neuron slice
        sizes = set(counts.tolist())
        self.esize = sizes.pop() if len(sizes) == 1 else 0
        self.perm = order  # new neuron position -> original neuron id (cpu int64)
        self.perm_dev = order.to(torch.int32).to(device)  # the same on the device (Wanda mask column permutation)
        self.fusable = bool(self.esize and 40 % self.esize == 0 and F % 80 == 0 and self.E <= 256)

    @classmethod
    def from_patterns(cls, patterns: torch.Tensor, k: int, device=None):
        p = patterns.detach().float().cpu()
        E, F = p.shape
        if not torch.all((p == 0) | (p == 1)) or not torch.all(p.sum(0) == 1):
            raise ValueError("patterns must be a 0/1 [E, F] matrix with exactly one expert per neuron")
        labels = p.argmax(0)
        return cls(labels, E, k, device or patterns.device)


def geglu_rows(F: int, perm: torch.Tensor | None, device) -> torch.Tensor:
    """Source row of proj.weight [2F, K] (value rows, then gate rows) for every row of the layout sdmoe_linear_geglu
    reads (include/sdmoe.h): neurons permuted by `perm`, value and gate rows interleaved per neuron pair [v 2 | g 2]
    (rows 4 q .. 4 q + 3 = value 2 q, value 2 q + 1, gate 2 q, gate 2 q + 1), so each lane of the kernel's swapped
    MFMA fragments holds both halves of two neurons."""
    if F % 2:
        raise ValueError(f"GEGLU layout: F = {F} is odd")
    idx = torch.arange(F, device=device) if perm is None else perm.to(device)
    r = torch.arange(2 * F, device=device)
    q, e = r // 4, r % 4
    c = 2 * q + (e & 1)
    return torch.where(e < 2, idx[c], F + idx[c])


def interleave_geglu(weight: torch.Tensor, bias: torch.Tensor | None, perm: torch.Tensor | None):
    """proj.weight [2F, K] -> rows in geglu_rows' order (neurons permuted by `perm`), the layout sdmoe_linear_geglu
    reads; bias likewise (zeros if None)."""
    F2, K = weight.shape
    rows = geglu_rows(F2 // 2, perm, weight.device)
    b = torch.zeros(F2, dtype=weight.dtype, device=weight.device) if bias is None else bias
    return weight[rows].contiguous(), b[rows].contiguous()


def interleave_ln_fold(fold: LNFold, perm: torch.Tensor | None) -> LNFold:
    """An LNFold of proj.weight [2F, K] with its rows in interleave_geglu's order."""
    F = fold.w.shape[0] // 2
    return fold.rows(geglu_rows(F, perm, fold.w.device))


_GELU_TABLES = {}


def gelu_table_values() -> torch.Tensor:
    """The 16384 fp16 inputs x with 2^-5 <= |x| < 8 in sdmoe_set_gelu_table's index order (int16 bit patterns:
    index i -> |x| bits 0x2800 + (i & 8191), sign i >> 13), as an fp16 CPU tensor."""
    i = torch.arange(16384, dtype=torch.int32)
    bits = (0x2800 + (i & 8191)) | ((i >> 13) << 15)
    return bits.to(torch.int16).view(torch.float16)


def ensure_gelu_table(device) -> torch.Tensor:
    """Register (once per device) the GELU table the GEGLU kernels apply for act == GELU: the reference module's
    activation itself -- diffusers GEGLU.gelu is F.gelu, which the hook applies to the fp16 gate (moefy.py:13,
    remove_skilled_experts.py:27) -- evaluated on every fp16 input of the table's range, so the device gates equal
    the reference's fp16 gates bit for bit (sdmoe_set_gelu_table, include/sdmoe.h). Must run outside graph capture
    (one host->device copy); the first GELU call on a device does it."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _GELU_TABLES.get(idx)
    if t is None:
        # F.gelu on the DEVICE fp16 tensor: the reference hook applies module.gelu to the gate on the GPU the model
        # sits on (base_receiver.py model.to(args.gpu); moefy.py:13, remove_skilled_experts.py:27)
        t = torch.nn.functional.gelu(gelu_table_values().to(torch.device("cuda", idx))).contiguous()
        lib = _lib.load()
        if _lib.has(lib, "sdmoe_set_gelu_table"):  # (an older A/B build evaluates GELU itself)
            with torch.cuda.device(idx):
                _lib.check(lib.sdmoe_set_gelu_table(t.data_ptr()), "sdmoe_set_gelu_table")
        _GELU_TABLES[idx] = t
    return t


def linear_geglu(x, w_il, b_il, act=ACT_GELU, *, score=None, esize=0, out=None, ln: LNFold | None = None):
    """P = value * act(gate) from the interleaved projection (interleave_geglu), plus per-expert gate sums
    into score [M, E] (experts = contiguous esize-neuron slices) when given. ln (interleave_ln_fold): x is the
    un-normalised input and the LayerNorm is folded into the GEMM (w_il / b_il are then ignored)."""
    lib = _lib.load()
    if act == ACT_GELU:
        ensure_gelu_table(x.device)
    if ln is not None:
        xp, lda = _rows(x, "x")
        M, K = x.shape
        F = ln.w.shape[0] // 2
        if out is None:
            out = torch.empty((M, F), dtype=torch.float16, device=x.device)
        op, ldp = _rows(out, "out")
        sp, lds = (None, 0) if score is None else _rows(score, "score")
        st = lib.sdmoe_linear_geglu_ln(xp, lda, ln.w.data_ptr(), ln.w.stride(0), ln.bias.data_ptr(),
                                       ln.wsum.data_ptr(), ln.eps, op, ldp, M, F, K, act, sp, lds, int(esize),
                                       _stream())
        _lib.check(st, "sdmoe_linear_geglu_ln")
        return out
    xp, lda = _rows(x, "x")
    M, K = x.shape
    F = w_il.shape[0] // 2
    if w_il.shape[1] != K:
        raise ValueError(f"linear_geglu: weight {tuple(w_il.shape)} does not match input K={K}")
    if out is None:
        out = torch.empty((M, F), dtype=torch.float16, device=x.device)
    op, ldp = _rows(out, "out")
    sp, lds = (None, 0) if score is None else _rows(score, "score")
    st = lib.sdmoe_linear_geglu(xp, lda, _dev(w_il, "w"), w_il.stride(0), _dev(b_il, "bias"), op, ldp, M, F, K,
                                act, sp, lds, int(esize), _stream())
    _lib.check(st, "sdmoe_linear_geglu")
    return out


def moe_topk_mask(P, score, routing: "Routing", removed=None, sel_out=None):
    """In place on the fused product P [M, F]: zero the neurons of experts outside each token's top-k."""
    lib = _lib.load()
    pp, ldp = _rows(P, "P")
    sp, lds = _rows(score, "score")
    st = lib.sdmoe_moe_topk_mask(pp, ldp, P.shape[0], P.shape[1], routing.E, routing.esize, routing.k, sp, lds,
                                 _ptr(removed), _ptr(sel_out), _stream())
    _lib.check(st, "sdmoe_moe_topk_mask")
    return P


def moe_topk_keep(score, routing: "Routing", M: int, removed=None, sel_out=None, keep=None):
    """Top-k selection of sdmoe_moe_topk_mask as keep bits for sdmoe_linear_keep: int64 [F/64, M] words, bit j of
    word (s, m) = expert-major neuron 64 s + j of token m kept."""
    lib = _lib.load()
    sp, lds = _rows(score, "score")
    F = routing.E * routing.esize
    if keep is None:
        keep = torch.empty((F // 64, M), dtype=torch.int64, device=score.device)
    if tuple(keep.shape) != (F // 64, M) or keep.dtype != torch.int64:
        raise ValueError(f"keep must be int64 [{F // 64}, {M}], got {keep.dtype} {tuple(keep.shape)}")
    st = lib.sdmoe_moe_topk_keep(M, F, routing.E, routing.esize, routing.k, sp, lds, _ptr(removed),
                                 _dev(keep, "keep", torch.int64), _ptr(sel_out), _stream())
    _lib.check(st, "sdmoe_moe_topk_keep")
    return keep


def linear_keep(x, keep, w, bias=None, *, residual=None, out=None, wmask=None):
    """out = (x with the neurons whose keep bit is clear zeroed) @ w.T + bias + residual (sdmoe_linear_keep);
    with wmask (wmask_kmajor layout) the Wanda weight mask too (sdmoe_linear_masked)."""
    if wmask is not None:
        return linear_masked(x, w, bias, keep=keep, wmask=wmask, residual=residual, out=out)
    lib = _lib.load()
    xp, lda = _rows(x, "x")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K or tuple(keep.shape) != (K // 64, M) or keep.dtype != torch.int64:
        raise ValueError(f"linear_keep: x {tuple(x.shape)}, keep {tuple(keep.shape)}, w {tuple(w.shape)} mismatch")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=x.device)
    op, ldc = _rows(out, "out")
    rp, ldr = (None, 0) if residual is None else _rows(residual, "residual")
    ws = _workspace(x.device)
    st = lib.sdmoe_linear_keep(xp, lda, _dev(keep, "keep", torch.int64), _dev(w, "w"), w.stride(0), _ptr(bias), rp,
                               ldr, op, ldc, M, N, K, ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_linear_keep")
    return out


def removed_bits(expert_ids, num_experts: int, device) -> torch.Tensor:
    """uint32-packed (as int32) bitmask of removed experts."""
    nw = (num_experts + 31) // 32
    words = [0] * nw
    for e in expert_ids:
        e = int(e)
        if not 0 <= e < num_experts:
            raise IndexError(f"expert id {e} out of range [0, {num_experts})")
        words[e >> 5] |= 1 << (e & 31)
    words = [w - (1 << 32) if w >= (1 << 31) else w for w in words]
    return torch.tensor(words, dtype=torch.int32, device=device)


def geglu_route(y, routing: Routing | None, act=ACT_GELU, removed=None, out=None, gate_out=None, sel_out=None,
                score_out=None, k=None):
    """Routed GEGLU over y = proj(x) [M, 2F]; routing None -> dense value*act(gate). k overrides routing.k
    (k = E: every expert kept, i.e. the dense product plus the per-token expert scores)."""
    lib = _lib.load()
    if act == ACT_GELU:
        ensure_gelu_table(y.device)
    yp, ldy = _rows(y, "y")
    M = y.shape[0]
    F = y.shape[1] // 2
    if out is None:
        out = torch.empty((M, F), dtype=torch.float16, device=y.device)
    op, ldo = _rows(out, "out")
    gp, ldg = (None, 0) if gate_out is None else _rows(gate_out, "gate_out")
    if routing is None:
        E, k, lab, off, nid = 0, 0, None, None, None
    else:
        if routing.F != F:
            raise ValueError(f"routing has F={routing.F}, projection gives F={F}")
        E, k = routing.E, (routing.k if k is None else int(k))
        lab, off, nid = routing.labels.data_ptr(), routing.e_off.data_ptr(), routing.e_nid.data_ptr()
    st = lib.sdmoe_geglu_route(yp, ldy, M, F, E, k, act, lab, off, nid, _ptr(removed), op, ldo, gp, ldg,
                               _ptr(sel_out), _ptr(score_out), _stream())
    _lib.check(st, "sdmoe_geglu_route")
    return out


def expert_mean_topk(score, k: int, rows_per_img: int = 0, row_idx=None, mean_out=None, topk_out=None):
    """GetExperts statistic (get_experts.py:72-80): mean of the fp16 expert scores [M, E] over all tokens, or
    over positions row_idx (int32 device tensor) of every rows_per_img-row image, then the top-k expert ids
    (descending, ties -> lowest id) as int32 [k]."""
    lib = _lib.load()
    sp, lds = _rows(score, "score")
    M, E = score.shape
    if topk_out is None:
        topk_out = torch.empty(int(k), dtype=torch.int32, device=score.device)
    rp, n_idx = (None, 0) if row_idx is None else (_dev(row_idx, "row_idx", torch.int32), row_idx.numel())
    ws = _workspace(score.device)
    st = lib.sdmoe_expert_mean_topk(sp, lds, M, E, int(rows_per_img), rp, n_idx, int(k),
                                    None if mean_out is None else _dev(mean_out, "mean_out"),
                                    _dev(topk_out, "topk_out", torch.int32), ws.data_ptr(), ws.numel(), _stream())
    _lib.check(st, "sdmoe_expert_mean_topk")
    return topk_out


def colnorm_accum(P, sumsq):
    """Wanda column statistic (wanda_receiver.py:37-57): sumsq[f] += sum_m (P[m,f] / ||P[m,:]||_2)^2."""
    lib = _lib.load()
    pp, ldp = _rows(P, "P")
    M, F = P.shape
    if sumsq.numel() != F:
        raise ValueError(f"colnorm_accum: sumsq has {sumsq.numel()} entries, P has {F} columns")
    ws = _workspace(P.device)
    st = lib.sdmoe_colnorm_accum(pp, ldp, M, F, _dev(sumsq, "sumsq", torch.float32), ws.data_ptr(), ws.numel(),
                                 _stream())
    _lib.check(st, "sdmoe_colnorm_accum")
    return sumsq


def wanda_mask(W, norm_base, norm_adj, kprune: int, out=None):
    """modularity/wanda.py:140-160 on device: bit-packed [C, F/8] mask of (top-kprune of |W|*norm_adj per row)
    AND (|W|*norm_adj > |W|*norm_base); norms fp16 [F]."""
    lib = _lib.load()
    wp, ldw = _rows(W, "W")
    C, F = W.shape
    if out is None:
        out = torch.empty((C, F // 8), dtype=torch.uint8, device=W.device)
    st = lib.sdmoe_wanda_mask(wp, ldw, C, F, _dev(norm_base, "norm_base"), _dev(norm_adj, "norm_adj"), int(kprune),
                              _dev(out, "bits", torch.uint8), _stream())
    _lib.check(st, "sdmoe_wanda_mask")
    return out


def timestep_embedding(t: float, dim: int, device, flip_sin_to_cos=True, freq_shift=0.0, out=None, t_dev=None):
    lib = _lib.load()
    if out is None:
        out = torch.empty((1, dim), dtype=torch.float16, device=device)
    st = lib.sdmoe_timestep_embedding(out.data_ptr(), _ptr(t_dev), float(t), dim, int(flip_sin_to_cos),
                                      float(freq_shift), _stream())
    _lib.check(st, "sdmoe_timestep_embedding")
    return out


def timestep_embedding_rows(t_dev: torch.Tensor, dim: int, out: torch.Tensor, group: int = 1,
                            flip_sin_to_cos=True, freq_shift=0.0):
    """Sinusoids of t_dev (fp32 [n]) into `out` (2-D fp16 view): row r at out[r // group, (r % group)*dim:]."""
    lib = _lib.load()
    op, ldo = _rows(out, "out")
    n = t_dev.numel()
    if out.shape[0] * group < n or out.shape[1] < group * dim:
        raise ValueError("timestep_embedding_rows: output view too small")
    st = lib.sdmoe_timestep_embedding_rows(op, ldo, _dev(t_dev, "t_dev", torch.float32), n, group, dim,
                                           int(bool(flip_sin_to_cos)), float(freq_shift), _stream())
    _lib.check(st, "sdmoe_timestep_embedding_rows")
    return out


def prepare_input(lat: torch.Tensor, out: torch.Tensor, ncopy: int):
    lib = _lib.load()
    B, C, H, W = lat.shape
    op, ldo = _rows(out, "out")
    st = lib.sdmoe_prepare_input(_dev(lat, "lat", torch.float32), op, B, H * W, ldo, ncopy, _stream())
    _lib.check(st, "sdmoe_prepare_input")
    return out


def cfg_ddim_step(eps: torch.Tensor, lat: torch.Tensor, do_cfg: bool, guidance: float, alpha_t: float,
                  alpha_prev: float, next_in: torch.Tensor | None = None):
    lib = _lib.load()
    B, C, H, W = lat.shape
    ep, lde = _rows(eps, "eps")
    np_, ldn = (None, 0) if next_in is None else _rows(next_in, "next_in")
    st = lib.sdmoe_cfg_ddim_step(ep, lde, _dev(lat, "lat", torch.float32), B, H * W, int(bool(do_cfg)),
                                 float(guidance), float(alpha_t), float(alpha_prev), np_, ldn, _stream())
    _lib.check(st, "sdmoe_cfg_ddim_step")
    return lat


def cfg_multistep_step(eps: torch.Tensor, lat: torch.Tensor, do_cfg: bool, guidance: float, hist: torch.Tensor,
                       cur: torch.Tensor, coef, flags, next_in: torch.Tensor | None = None):
    """CFG + one PLMS (PNDM) update in place (pipeline.pndm_schedule gives coef[7] / flags[3] per call)."""
    import ctypes
    lib = _lib.load()
    B, C, H, W = lat.shape
    if tuple(hist.shape) != (4, B, C, H, W) or tuple(cur.shape) != (B, C, H, W):
        raise ValueError("cfg_multistep_step: history [4, B, 4, H, W] and cur [B, 4, H, W] expected")
    ep, lde = _rows(eps, "eps")
    np_, ldn = (None, 0) if next_in is None else _rows(next_in, "next_in")
    cf = (ctypes.c_float * 7)(*[float(v) for v in coef])
    fl = (ctypes.c_int * 3)(*[int(v) for v in flags])
    st = lib.sdmoe_cfg_multistep_step(ep, lde, _dev(lat, "lat", torch.float32), B, H * W, int(bool(do_cfg)),
                                      float(guidance), _dev(hist, "hist", torch.float32),
                                      _dev(cur, "cur", torch.float32), ctypes.cast(cf, ctypes.c_void_p),
                                      ctypes.cast(fl, ctypes.c_void_p), np_, ldn, _stream())
    _lib.check(st, "sdmoe_cfg_multistep_step")
    return lat


def softmax_rows(x, out=None):
    """Row softmax of a 2-D fp16 view (fp32 max / sum), sdmoe_softmax_rows."""
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    R, N = x.shape
    if out is None:
        out = torch.empty((R, N), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    _lib.check(lib.sdmoe_softmax_rows(xp, ldx, op, ldy, R, N, _stream()), "sdmoe_softmax_rows")
    return out


def transpose(x, out=None):
    """[R, C] fp16 view -> contiguous [C, R] (sdmoe_transpose)."""
    lib = _lib.load()
    xp, ldx = _rows(x, "x")
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), dtype=torch.float16, device=x.device)
    op, ldy = _rows(out, "out")
    _lib.check(lib.sdmoe_transpose(xp, ldx, op, ldy, R, C, _stream()), "sdmoe_transpose")
    return out


def add(a, b, out=None):
    lib = _lib.load()
    if out is None:
        out = torch.empty_like(a)
    st = lib.sdmoe_add(_dev(a, "a"), _dev(b, "b"), _dev(out, "out"), a.numel(), _stream())
    _lib.check(st, "sdmoe_add")
    return out


def gather_rows(table, idx, *, add=None, period=0, out=None):
    """out[r] = table[idx[r]] (+ add[r % period]) — token + position embedding, pooled-row gather
    (sdmoe_gather_rows). idx: int32 device tensor [R]."""
    lib = _lib.load()
    tp, ldt = _rows(table, "table")
    C = table.shape[1]
    R = idx.numel()
    if out is None:
        out = torch.empty((R, C), dtype=torch.float16, device=table.device)
    op, ldo = _rows(out, "out")
    ap, lda = (None, 0) if add is None else _rows(add, "add")
    if add is not None and period <= 0:
        period = add.shape[0]
    st = lib.sdmoe_gather_rows(tp, ldt, _dev(idx, "idx", torch.int32), R, C, ap, lda, int(period), op, ldo,
                               _stream())
    _lib.check(st, "sdmoe_gather_rows")
    return out


def attention_short(q, k, v, nseq, N, heads, out=None, scale=None, causal=True):
    """Short-sequence (N <= 128) attention per (sequence, head), optional causal mask (sdmoe_attention_short)."""
    lib = _lib.load()
    qp, ldq = _rows(q, "q")
    kp, ldk = _rows(k, "k")
    vp, ldv = _rows(v, "v")
    C = q.shape[1]
    d = C // heads
    if out is None:
        out = torch.empty((nseq * N, C), dtype=torch.float16, device=q.device)
    op, ldo = _rows(out, "out")
    if scale is None:
        scale = d ** -0.5
    st = lib.sdmoe_attention_short(qp, ldq, kp, ldk, vp, ldv, op, ldo, nseq, N, heads, d, float(scale),
                                   int(bool(causal)), _stream())
    _lib.check(st, "sdmoe_attention_short")
    return out
