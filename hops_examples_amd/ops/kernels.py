"""Typed, validated launchers for the gfx950 kernels (no autograd here).

Conventions: activations are bf16 row-major (NHWC for images), weights used by
the MFMA kernels are the bf16 *shadow* of the fp32 master parameters, gradient
buffers are fp32 and are ACCUMULATED into (atomics) so they must be zeroed by
the caller (the fused optimizers zero them after consuming them).
"""
from __future__ import annotations

import os

import torch

from . import _C
from ._C import ACT, EPI_ATOMIC_F32, EPI_DACT_BF16, EPI_STORE_BF16, EPI_STORE_F32, check, debug_errors, ptr, stream  # noqa: F401

BF16 = torch.bfloat16
F32 = torch.float32


def _req(t: torch.Tensor, dtype, name: str, contiguous=True):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a GPU tensor")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")


def act_id(act) -> int:
    return act if isinstance(act, int) else ACT[act]


# ---------------------------------------------------------------- dense GEMM
def gemm_raw(a, lda, a_kc, b, ldb, b_kc, M, N, K, epi, out, ldo, bias=None, alpha=1.0, beta=0.0, act=0, aux=None,
             ldaux=0, colsum=None, ws=None, a_mask_y=None, a_mask_act=0, a_rowsum=None):
    """ws: optional fp32 workspace (>= M*N) enabling split-K for small-M/long-K store epilogues.
    a_mask_y/a_mask_act: multiply the A operand by act'(y) while staging it (prologue fusion).
    a_rowsum: accumulate the row sums of the (masked) A operand (RC-A only; bias gradients)."""
    rc = _C.ext().gemm(ptr(a), lda, int(a_kc), ptr(b), ldb, int(b_kc), M, N, K, epi, ptr(out), ldo, ptr(bias),
                       float(alpha), float(beta), act_id(act), ptr(aux), ldaux, ptr(colsum), ptr(ws),
                       0 if ws is None else ws.numel(), ptr(a_mask_y), act_id(a_mask_act), ptr(a_rowsum),
                       ptr(ticket(a.device)) if ws is not None else 0, stream())
    check(rc, "gemm")


_SPLITK_WS: dict = {}


def _splitk_ws(M, N, K, device):
    """fp32 split-K accumulator: a persistent per-device buffer that is zero at rest (the
    in-launch finish of each split-K GEMM re-zeroes the tiles it consumed), so no memset
    node or finishing kernel runs per call.  Grown only outside graph capture."""
    # split-K pays when the output has few tiles but the reduction is long
    if not (M * N <= (1 << 22) and K >= 1024 and (M <= 128 or N <= 128)):
        return None
    buf = _SPLITK_WS.get(device)
    if buf is None or buf.numel() < M * N:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("split-K workspace must be sized before graph capture (run an eager step first)")
        buf = torch.zeros(max(M * N, 1 << 16), device=device, dtype=F32)
        _SPLITK_WS[device] = buf
    return buf[: M * N]


def linear_fwd(x, w, bias=None, act=0, out=None, out_f32=False, colsum=None):
    """y[M,N] = act(x[M,K] @ w[N,K]^T + bias)."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K, (x.shape, w.shape)
    _req(x, BF16, "x")
    _req(w, BF16, "w")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=F32 if out_f32 else BF16)
    epi = EPI_STORE_F32 if out.dtype == F32 else EPI_STORE_BF16
    gemm_raw(x, K, True, w, K, True, M, N, K, epi, out, N, bias=bias, act=act, colsum=colsum,
             ws=_splitk_ws(M, N, K, x.device))
    return out


def linear_dgrad(dy, w, yprev=None, act_prev=0, out=None, colsum=None, y=None, act=0):
    """dx[M,K] = ((dy * act'(y)) [M,N] @ w[N,K]) * act'(yprev)  (+ column sum -> previous layer's bias grad).
    y/act: this layer's own activation output (mask fused into the A-operand staging)."""
    M, N = dy.shape
    K = w.shape[1]
    _req(dy, BF16, "dy")
    _req(w, BF16, "w")
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=BF16)
    gemm_raw(dy, N, True, w, K, False, M, K, N, EPI_DACT_BF16, out, K, act=act_prev if yprev is not None else 0,
             aux=yprev, ldaux=K, colsum=colsum, ws=_splitk_ws(M, K, N, dy.device), a_mask_y=y, a_mask_act=act)
    return out


def linear_wgrad(dy, x, dw, alpha=1.0, y=None, act=0, dbias=None):
    """dw[N,K] += (dy * act'(y))[M,N]^T @ x[M,K]  (fp32 atomics, split-K over the batch);
    dbias[N] += column sums of the masked dy, computed while dy^T is staged."""
    M, N = dy.shape
    K = x.shape[1]
    _req(dy, BF16, "dy")
    _req(x, BF16, "x")
    _req(dw, F32, "dw")
    gemm_raw(dy, N, False, x, K, False, N, K, M, EPI_ATOMIC_F32, dw, K, alpha=alpha, a_mask_y=y, a_mask_act=act,
             a_rowsum=dbias)
    return dw


def linear_bwd_pair(dy, w, x, dw, y=None, act=0, dbias=None, pool=None, dw_store=False):
    """dX and dW (+ dbias) of a Linear layer in ONE launch (gemm.hip linear_bwd_pair_k); returns
    dX [M, K] bf16, or False when the shape goes to the separate launches (small-M split-K dgrad).
    ``pool`` = (am, premask, in_shape, (KH, KW), act, rng, salt, p): the Linear's input is the
    flattened output of a non-overlapping max-pool; the returned tensor is then the gradient of the
    POOL INPUT (shape in_shape), scattered by the dgrad epilogue (the pool backward fused away).
    ``premask``: also apply ReLU' of the pool input (read off the pooled value = this layer's input).
    ``dw_store``: dW is the only contribution to a zeroed buffer — stored, not atomically added."""
    M, N = dy.shape
    K = x.shape[1]
    _req(dy, BF16, "dy")
    _req(x, BF16, "x")
    _req(w, BF16, "w")
    _req(dw, F32, "dw")
    pl, pam, px, prng, psalt, pp = [], 0, 0, 0, 0, 0.0
    if pool is not None:
        am, xin, in_shape, (kh, kw), pact, rng, salt, p = pool[:8]
        B, H, W, C = in_shape
        pl = [C, H // kh, W // kw, kh, kw, act_id(pact) if xin else 0, H, W]
        pam, px, prng, psalt, pp = ptr(am), (ptr(x) if xin else 0), ptr(rng), int(salt) & 0xFFFFFFFF, float(p)
        dx = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
    else:
        dx = torch.empty(M, K, device=dy.device, dtype=BF16)
    rc = _C.ext().linear_bwd_pair(ptr(dy), ptr(w), ptr(x), ptr(dx), 0, 0, 0, ptr(y), act_id(act), ptr(dw),
                                  ptr(dbias), M, N, K, pl, pam, px, prng, psalt, pp, int(bool(dw_store)), stream())
    if rc == -2:
        return False
    check(rc, "linear_bwd_pair")
    return dx


def colsum(x, out):
    """out[N] += sum_m x[M,N]."""
    _req(x, BF16, "x")
    M, N = x.reshape(-1, x.shape[-1]).shape
    check(_C.ext().colsum_bf16(ptr(x), ptr(out), M, N, stream()), "colsum")
    return out


# -------------------------------------------------------------- conv2d NHWC
def conv_geom(x_shape, w_shape, stride, padding, dilation):
    """The kernels' geometry vector.  ``padding`` = (ph, pw), symmetric, or (ph, pw, eh, ew): ph / pw
    rows / columns of zeros before the input and eh / ew after it (TF 'same' with an even kernel pads
    one more at the end).  The kernels only see the leading pad and the output size: every gather
    bounds-checks against H / W, so the trailing pad needs no data."""
    B, H, W, C = x_shape
    CO, KH, KW, CI = w_shape
    assert CI == C, (x_shape, w_shape)
    sh, sw = stride
    ph, pw = padding[:2]
    eh, ew = (padding[2], padding[3]) if len(padding) == 4 else (ph, pw)
    dh, dw = dilation
    OH = (H + ph + eh - dh * (KH - 1) - 1) // sh + 1
    OW = (W + pw + ew - dw * (KW - 1) - 1) // sw + 1
    return [B, H, W, C, OH, OW, CO, KH, KW, sh, sw, ph, pw, dh, dw]


_TICKETS: dict = {}


def ticket(device) -> torch.Tensor:
    """Per-device in-launch-reduction ticket counter (uint32, zero at rest: every kernel that
    draws tickets has its last workgroup re-arm it, so it stays valid across graph replays).
    Allocated outside any capture on first use (the eager warm-up steps)."""
    t = _TICKETS.get(device)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("ticket counter must be created before graph capture (run an eager step first)")
        t = torch.zeros(8192, device=device, dtype=torch.int32)
        _TICKETS[device] = t
    return t


def conv_u8_fusable(geom) -> bool:
    """The uint8 input layer can skip its normalisation pass: the direct forward kernel and the
    small-K weight-gradient kernel both read raw pixels (x * scale + shift) themselves."""
    K = geom[7] * geom[8] * geom[3]
    CO = geom[6]
    return K in (4, 9, 16) and CO % 8 == 0 and CO <= 256 and K * CO <= 1024 and \
        "u8_fuse" not in os.environ.get("HOPSX_DISABLE", "")


def conv2d_fwd(x, w, geom, bias=None, act=0, out=None, colsum=None, in_affine=None):
    """in_affine=(scale, shift): x is raw uint8 and is normalised inside the kernel."""
    _req(x, torch.uint8 if in_affine else BF16, "x")
    _req(w, BF16, "w")
    B, OH, OW, CO = geom[0], geom[4], geom[5], geom[6]
    if out is None:
        out = torch.empty(B, OH, OW, CO, device=x.device, dtype=BF16)
    epi = EPI_STORE_F32 if out.dtype == F32 else EPI_STORE_BF16
    sc, sh = (float(in_affine[0]), float(in_affine[1])) if in_affine else (0.0, 0.0)
    check(_C.ext().conv2d_fwd(ptr(x), ptr(w), geom, epi, ptr(out), ptr(bias), act_id(act), ptr(colsum), sc, sh,
                              stream()), "conv2d_fwd")
    return out


def conv_fwd_pool_ok(geom, act, pk: int = 2) -> bool:
    """conv(geom, act) -> pk x pk / stride-pk max-pool (pk 2 or 4, floor windows) can run as one launch
    (conv_mfma.hip POOL epilogue)."""
    return bool(_C.ext().conv2d_fwd_pool_ok(list(geom), act_id(act), int(pk)))


def conv2d_fwd_pool(x, w, geom, bias=None, act=0, drop_p=0.0, rng=None, salt=0, pk: int = 2):
    """Conv + act + pk x pk / stride-pk max-pool (+ dropout) in one launch: returns (pooled [B, OH//pk,
    OW//pk, CO] bf16, argmax uint8 = the window tap kh*pk+kw).  With a ReLU an all-zero window's argmax
    is 0xFF (no gradient), so the pool backward applies ReLU' and the conv output itself is never
    stored."""
    _req(x, BF16, "x")
    _req(w, BF16, "w")
    B, OH, OW, CO = geom[0], geom[4], geom[5], geom[6]
    y = torch.empty(B, OH // pk, OW // pk, CO, device=x.device, dtype=BF16)
    am = torch.empty(B, OH // pk, OW // pk, CO, device=x.device, dtype=torch.uint8)
    check(_C.ext().conv2d_fwd_pool(ptr(x), ptr(w), list(geom), ptr(y), ptr(am), ptr(bias), act_id(act),
                                   float(drop_p), ptr(rng), int(salt) & 0xFFFFFFFF, int(pk), stream()),
          "conv2d_fwd_pool")
    return y, am


def conv_fwd_pool_in_ok(geom0, geom, act) -> bool:
    """input layer (geom0) -> conv(geom, act) -> 2x2/2 max-pool can run as ONE launch
    (conv_mfma.hip IN0: the input layer is evaluated inside the conv's operand gather)."""
    return bool(_C.ext().conv2d_fwd_pool_in_ok(list(geom0), list(geom), act_id(act)))


def conv2d_fwd_pool_in(x0, w0, b0, act0, geom0, w, geom, bias=None, act=0, drop_p=0.0, rng=None, salt=0,
                       in_affine=None, keep_y1=True):
    """pool(conv(input_layer(x0))) in one launch.  x0: raw uint8 pixels [B, H0, W0, 1], normalised
    as ``x * scale + shift`` (``in_affine``) inside the kernel.  Returns (pooled, argmax, y1): y1 is the input layer's
    output [B, H, W, C] bf16 (stored by the same launch for the backward; None if not ``keep_y1``)."""
    _req(w0, BF16, "w0")
    _req(w, BF16, "w")
    _req(x0, torch.uint8, "x0")
    if in_affine is None or float(in_affine[0]) == 0.0:
        raise ValueError("conv2d_fwd_pool_in: uint8 pixels need in_affine=(scale != 0, shift)")
    xs, xh = float(in_affine[0]), float(in_affine[1])
    B, OH, OW, CO = geom[0], geom[4], geom[5], geom[6]
    y = torch.empty(B, OH // 2, OW // 2, CO, device=x0.device, dtype=BF16)
    am = torch.empty(B, OH // 2, OW // 2, CO, device=x0.device, dtype=torch.uint8)
    y1 = torch.empty(B, geom[1], geom[2], geom[3], device=x0.device, dtype=BF16) if keep_y1 else None
    check(_C.ext().conv2d_fwd_pool_in(ptr(x0), xs, xh, ptr(w0), ptr(b0), act_id(act0), list(geom0), ptr(y1), ptr(w),
                                      list(geom), ptr(y), ptr(am), ptr(bias), act_id(act), float(drop_p), ptr(rng),
                                      int(salt) & 0xFFFFFFFF, stream()), "conv2d_fwd_pool_in")
    return y, am, y1


def conv2d_dgrad(dy, w, geom, yprev=None, act_prev=0, out=None, colsum=None, y=None, act=0, addend=None):
    """dX = conv_transpose(dY, W) (* act'(yprev)) (+ addend: a gradient of x from another consumer,
    added in the epilogue; bf16, x's layout)."""
    _req(dy, BF16, "dy")
    B, H, W, C = geom[:4]
    if out is None:
        out = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
    if addend is not None:
        _req(addend, BF16, "addend")
        if addend.shape != out.shape:
            raise ValueError("conv2d_dgrad: addend must have the input gradient's shape")
    check(_C.ext().conv2d_dgrad(ptr(dy), ptr(w), geom, ptr(out), ptr(yprev), act_id(act_prev) if yprev is not None
                                else 0, ptr(colsum), ptr(y), act_id(act), ptr(addend), stream()), "conv2d_dgrad")
    return out


def conv2d_dgrad_bn(dy, w, geom, bn, addend=None):
    """dX of a conv whose input is a sole-consumed training BN output, ``bn`` = (z, mean, rstd, yprev,
    act_prev): the epilogue adds ``addend``, applies act_prev'(yprev), stores g and reduces the BN's backward
    column sums into its accumulator (finish with ``bn_bwd_pre``).  False: shape not covered (nothing
    launched)."""
    _req(dy, BF16, "dy")
    z, mean, rstd, yprev, act_prev, acc = bn
    _req(z, BF16, "bn z")
    B, H, W, C = geom[:4]
    if addend is not None:
        _req(addend, BF16, "addend")
    out = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
    rc = _C.ext().conv2d_dgrad_bn(ptr(dy), ptr(w), list(geom), ptr(out), ptr(yprev),
                                  act_id(act_prev) if yprev is not None else 0, ptr(addend), ptr(z), ptr(mean),
                                  ptr(rstd), ptr(acc), stream())
    if rc == -2:
        return False
    check(rc, "conv2d_dgrad_bn")
    return out


def conv_dgrad_fused_wgrad_ok(geom, geom0) -> bool:
    """conv(geom)'s dgrad can carry the weight gradient of the input layer conv(geom0) feeding it."""
    return bool(_C.ext().conv2d_dgrad_fused_wgrad_ok(list(geom), list(geom0)))


def conv2d_dgrad_fused_wgrad(dy, w, geom, yprev, act_prev, y, act, x0, geom0, dw0, db0, in_affine=None):
    """Backward of conv(geom) when its input came from the network's input layer conv(geom0):
    instead of dX (which only that layer's wgrad would read) the kernel accumulates
    dw0 += (dX * act_prev'(yprev))^T . im2col(x0) and db0 += column sums, in one launch."""
    _req(dy, BF16, "dy")
    _req(yprev, BF16, "yprev")
    _req(x0, torch.uint8 if in_affine else BF16, "x0")
    _req(dw0, F32, "dw0")
    _req(db0, F32, "db0")
    sc, sh = (float(in_affine[0]), float(in_affine[1])) if in_affine else (0.0, 0.0)
    check(_C.ext().conv2d_dgrad_fused_wgrad(ptr(dy), ptr(w), list(geom), ptr(yprev), act_id(act_prev), ptr(db0),
                                            ptr(y), act_id(act), list(geom0), ptr(x0), sc, sh, ptr(dw0), stream()),
          "conv2d_dgrad_fused_wgrad")


def conv2d_bwd_pair_bn_ok(geom) -> bool:
    """conv2d_bwd_pair(bn=...) covers this conv: its dgrad epilogue can reduce the input BN's backward
    column sums."""
    return bool(_C.ext().conv2d_bwd_pair_bn_ok(list(geom)))


def conv2d_bwd_pair(dy, w, geom, x, dw, dbias=None, y=None, act=0, prev=None, addend=None, opt_slice=None, bn=None):
    """A conv layer's dgrad and wgrad in ONE launch (conv_mfma.hip conv_bwd_pair_k).  ``prev`` =
    (x0, geom0, dw0, db0, yprev, act_prev, in_affine) fuses the input layer's weight gradient into the
    dgrad (no dX).  ``addend``: another consumer's gradient of the same input, added to dX in the
    epilogue where the kernel has it (else added afterwards).  ``bn`` = (z, mean, rstd, yprev, act_prev):
    x is the output of a training BatchNorm (input z [M, C], batch mean / rstd) consumed only by this
    conv — dX is masked by act_prev'(yprev) and the BN's backward column sums go into its accumulator
    (``bn_bwd_pre`` then finishes that BN's backward in one launch).  Returns dX (None when fused), or
    False when the shapes are not covered."""
    B, H, W, C = geom[:4]
    bnargs = (0, 0, 0, 0)
    if bn is not None:
        if prev is not None or opt_slice is not None or dbias is not None:
            raise ValueError("conv2d_bwd_pair: bn excludes prev / opt_slice / dbias")
        z, mean, rstd, yprev, act_prev, acc = bn
        _req(z, BF16, "bn z")
        bnargs = (ptr(z), ptr(mean), ptr(rstd), ptr(acc))
        dx = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
        args = (ptr(dx), ptr(yprev), act_id(act_prev) if yprev is not None else 0, 0, ptr(y), act_id(act), [], 0, 0.0,
                0.0, 0)
    elif prev is None:
        dx = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
        args = (ptr(dx), 0, 0, 0, ptr(y), act_id(act), [], 0, 0.0, 0.0, 0)
    else:
        x0, g0, dw0, db0, yprev, act_prev, aff = prev
        dx = None
        sc, sh = (float(aff[0]), float(aff[1])) if aff else (0.0, 0.0)
        args = (0, ptr(yprev), act_id(act_prev), ptr(db0), ptr(y), act_id(act), list(g0), ptr(x0), sc, sh, ptr(dw0))
    dxp, yp, ap, cs, yy, ya, g0l, x0p, sc_, sh_, dw0p = args
    if addend is not None:
        _req(addend, BF16, "addend")
    if opt_slice is not None:
        # + a fused optimizer's update of an arena slice whose gradients are final (optim_slice.h):
        # opt_slice = (kind, master, grad, s1, s2, s3, shadow, hp list, hp_dev, step_dev)
        kind, p_, g_, s1, s2, s3, shd, hp, hp_dev, step_dev = opt_slice
        nblk = int(os.environ.get("HOPSX_OPT_SLICE_BLK", "256"))
        first = int(os.environ.get("HOPSX_OPT_SLICE_FIRST", "0"))
        rc = _C.ext().conv2d_bwd_pair_opt(ptr(dy), ptr(w), list(geom), dxp, yp, ap, cs, yy, ya, g0l, x0p, sc_, sh_,
                                          dw0p, ptr(x), ptr(dw), ptr(dbias), ptr(addend), int(kind), ptr(p_),
                                          ptr(g_), ptr(s1), ptr(s2), ptr(s3), ptr(shd), int(p_.numel()),
                                          [float(v) for v in (list(hp) + [0.0] * 8)[:8]], ptr(hp_dev), ptr(step_dev),
                                          nblk, first, stream())
        if rc in (-2, -3):
            return False
        check(rc, "conv2d_bwd_pair_opt")
        return dx
    rc = _C.ext().conv2d_bwd_pair(ptr(dy), ptr(w), list(geom), dxp, yp, ap, cs, yy, ya, g0l, x0p, sc_, sh_, dw0p,
                                  ptr(x), ptr(dw), ptr(dbias), ptr(addend), *bnargs, stream())
    if rc == -3:  # no epilogue addend for this shape: nothing launched; pair without it, then add
        if bn is not None:
            return False  # (the sums would miss the addend)
        rc = _C.ext().conv2d_bwd_pair(ptr(dy), ptr(w), list(geom), dxp, yp, ap, cs, yy, ya, g0l, x0p, sc_, sh_,
                                      dw0p, ptr(x), ptr(dw), ptr(dbias), 0, 0, 0, 0, 0, stream())
        if rc == 0 and dx is not None:
            dx.add_(addend.view(dx.shape))
    if rc == -2:
        return False
    check(rc, "conv2d_bwd_pair")
    return dx


def conv_wgrad_uses_ticket(geom, in_affine=None) -> bool:
    """True when conv2d_wgrad would take the small-K kernel, whose in-launch combine draws from the
    shared per-device ticket counter (so it must not run concurrently with another such kernel)."""
    return _c1_wgrad(geom) or _smallk_wgrad(geom)


def _c1_wgrad(geom) -> bool:
    """conv.hip conv_wgrad_c1_k: a one-channel input layer (K <= 25 taps, CO in 8/16/32/64)."""
    K = geom[7] * geom[8] * geom[3]
    return geom[3] == 1 and K <= 25 and geom[6] in (8, 16, 32, 64) and "c1_wgrad" not in os.environ.get("HOPSX_DISABLE", "")


def _smallk_wgrad(geom) -> bool:
    K = geom[7] * geom[8] * geom[3]
    return K in (4, 9, 16) and geom[6] % 8 == 0 and geom[6] <= 256 and \
        "smallk_wgrad" not in os.environ.get("HOPSX_DISABLE", "")


def conv2d_wgrad(dy, x, geom, dw, dbias=None, y=None, act=0, in_affine=None):
    """dw += (dy * act'(y))^T . im2col(x); dbias += per-channel sums of the masked dy.
    in_affine=(scale, shift): x is the raw uint8 input (see conv_u8_fusable)."""
    _req(dy, BF16, "dy")
    _req(x, torch.uint8 if in_affine else BF16, "x")
    _req(dw, F32, "dw")
    K = geom[7] * geom[8] * geom[3]
    KC = K * geom[6]
    ws = None
    smallk = _c1_wgrad(geom) or _smallk_wgrad(geom)
    if smallk:  # per-workgroup partial rows (<= 256: workgroups + group rows), combined in-launch
        # (c1: rows padded to 128-B lines)
        row = (geom[6] * (K + 1) + 31) // 32 * 32 if _c1_wgrad(geom) else geom[6] * (K + 1)
        ws = torch.empty((256 if _c1_wgrad(geom) else 128) * row, device=dy.device, dtype=F32)
    elif K <= 64 and KC <= 1024:  # older direct kernel: slab workspace
        ws = torch.empty(1024 * (KC + geom[6]), device=dy.device, dtype=F32)
    sc, sh = (float(in_affine[0]), float(in_affine[1])) if in_affine else (0.0, 0.0)
    check(_C.ext().conv2d_wgrad(ptr(dy), ptr(x), geom, ptr(dw), ptr(dbias), ptr(y), act_id(act), ptr(ws),
                                0 if ws is None else ws.numel(), sc, sh, ptr(ticket(dy.device)), stream()),
          "conv2d_wgrad")
    return dw


# ------------------------------------------------------------------ pooling
def pool_out(H, W, k, s, p):
    return (H + 2 * p[0] - k[0]) // s[0] + 1, (W + 2 * p[1] - k[1]) // s[1] + 1


def maxpool2d_fwd(x, k, s, p, out=None, argmax=None, drop_p=0.0, rng=None, salt=0):
    """Max-pool (NHWC) with an optional fused dropout on the pooled output."""
    B, H, W, C = x.shape
    OH, OW = pool_out(H, W, k, s, p)
    if out is None:
        out = torch.empty(B, OH, OW, C, device=x.device, dtype=BF16)
    if argmax is None:
        argmax = torch.empty(B, OH, OW, C, device=x.device, dtype=torch.uint8)
    check(_C.ext().maxpool2d_fwd(ptr(x), ptr(out), ptr(argmax), B, H, W, C, OH, OW, k[0], k[1], s[0], s[1], p[0],
                                 p[1], float(drop_p), ptr(rng), int(salt) & 0xFFFFFFFF, stream()), "maxpool_fwd")
    return out, argmax


def maxpool2d_bwd(dy, argmax, x_shape, k, s, p, x=None, act=0, out=None, colsum=None, drop_p=0.0, rng=None, salt=0):
    """Gather backward of max-pool; optionally re-applies the fused dropout mask, multiplies by
    act'(x) (x = pool input = previous activation output) and emits that layer's bias gradient."""
    B, H, W, C = x_shape
    OH, OW = dy.shape[1], dy.shape[2]
    if out is None:
        out = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
    check(_C.ext().maxpool2d_bwd(ptr(dy), ptr(argmax), ptr(x), ptr(out), B, H, W, C, OH, OW, k[0], k[1], s[0], s[1],
                                 p[0], p[1], act_id(act), ptr(colsum), float(drop_p), ptr(rng),
                                 int(salt) & 0xFFFFFFFF, stream()), "maxpool_bwd")
    return out


def gap_fwd(x, out=None):
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty(B, C, device=x.device, dtype=BF16)
    check(_C.ext().avgpool_global_fwd(ptr(x), ptr(out), B, H * W, C, stream()), "gap_fwd")
    return out


def gap_bwd(dy, x_shape, out=None):
    B, H, W, C = x_shape
    if out is None:
        out = torch.empty(B, H, W, C, device=dy.device, dtype=BF16)
    check(_C.ext().avgpool_global_bwd(ptr(dy), ptr(out), B, H * W, C, stream()), "gap_bwd")
    return out


# ------------------------------------------------------------------- losses
def loss_fwd_bwd(kind: int, logits, target, grad_scale, loss_sum, correct, dlogits=None):
    B, C = logits.shape
    check(_C.ext().loss_fwd_bwd(kind, ptr(logits), int(logits.dtype == F32), ptr(target), B, C, float(grad_scale),
                                ptr(loss_sum), ptr(correct), ptr(dlogits),
                                int(dlogits is not None and dlogits.dtype == F32), stream()), "loss")
    return dlogits


# --------------------------------------------------------------- optimizers
def optim_step(kind: int, param, grad, s1, s2, s3, shadow, hp, step_dev, zero_grad=True, arrive=None, rng=None,
               prefetch=None, hp_dev=None):
    """One fused update over flat buffers.  ``step_dev`` (f32[1]) counts completed steps and,
    with ``arrive`` (int32[288], zero-initialised), is bumped in-kernel by the last workgroup,
    together with the dropout RNG counter ``rng[1]`` when given.
    ``prefetch`` = (pairs, cursor): pairs of (resident [nbatch, ...] tensor, static input buffer);
    the kernel copies batch (cursor+1) % nbatch into the buffers and advances the int64 cursor.
    ``hp_dev`` (f32[8] on the device): the kernel reads the hyper-parameters from it at run time
    instead of ``hp`` (so a replayed hipGraph sees learning-rate changes)."""
    n = param.numel()
    if step_dev is not None and arrive is None:
        arrive = torch.zeros(9 * 32, device=param.device, dtype=torch.int32)  # optim_core.h kArriveWords
    srcs, dsts, nbytes, cur, nb = [], [], [], 0, 0
    if prefetch is not None:
        pairs, cursor = prefetch
        for src, dst in pairs:
            per = dst.numel() * dst.element_size()
            assert src.is_contiguous() and dst.is_contiguous() and src.numel() == src.shape[0] * dst.numel(), \
                "prefetch: src must be [nbatch, *dst.shape] contiguous"
            srcs.append(ptr(src))
            dsts.append(ptr(dst))
            nbytes.append(per)
            nb = src.shape[0]
        cur = ptr(cursor)
    check(_C.ext().optim_step(kind, ptr(param), ptr(grad), ptr(s1), ptr(s2), ptr(s3), ptr(shadow), n,
                              [float(v) for v in hp], ptr(step_dev), ptr(arrive), ptr(rng), int(zero_grad), srcs,
                              dsts, nbytes, cur, nb, ptr(hp_dev), stream()),
          "optim")


# ------------------------------------------------------------- misc / RNG
def dropout(x, p, rng, salt, out=None):
    if out is None:
        out = torch.empty_like(x)
    check(_C.ext().dropout_fwd(ptr(x), ptr(out), x.numel(), float(p), ptr(rng), int(salt) & 0xFFFFFFFF, stream()),
          "dropout")
    return out


def rng_advance(rng):
    check(_C.ext().rng_advance(ptr(rng), stream()), "rng_advance")


def cast_f32_bf16(x, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=BF16)
    check(_C.ext().cast_f32_bf16(ptr(x), ptr(out), x.numel(), stream()), "cast")
    return out


def pad_cin(w, cp, out=None, out16=None):
    """w fp32 [..., C] -> (fp32 [..., cp], bf16 [..., cp]) with channels C..cp-1 zero, one launch."""
    _req(w, F32, "w")
    shp = tuple(w.shape[:-1]) + (int(cp),)
    out = torch.empty(shp, device=w.device, dtype=F32) if out is None else out
    out16 = torch.empty(shp, device=w.device, dtype=BF16) if out16 is None else out16
    R = w.numel() // w.shape[-1]
    check(_C.ext().pad_cin(ptr(w), R, w.shape[-1], int(cp), ptr(out), ptr(out16), stream()), "pad_cin")
    return out, out16


def unpad_cin_add(gpad, C, tgt):
    """tgt[..., :C] += gpad[..., :C] (tgt: [..., C] fp32, may be None), then gpad = 0; one launch."""
    _req(gpad, F32, "gpad")
    R = gpad.numel() // gpad.shape[-1]
    check(_C.ext().unpad_cin_add(ptr(gpad), R, int(C), gpad.shape[-1], 0 if tgt is None else ptr(tgt), stream()),
          "unpad_cin_add")


_COL_DT = {torch.float32: 0, torch.float64: 1, torch.int64: 2, torch.int32: 3, torch.int16: 4, torch.int8: 5,
           torch.uint8: 6, torch.float16: 7}


def cols_to_f32(cols, out):
    """Interleave 1-D device columns (any of int8..int64 / f16 / f32 / f64, equal length) into the
    fp32 matrix ``out`` [rows, >= len(cols)] (row stride out.stride(0)) in ONE launch."""
    rows = out.shape[0]
    if any(c.numel() != rows or c.device != out.device for c in cols):
        raise ValueError("cols_to_f32: every column must have out.shape[0] elements on out's device")
    _req(out, F32, "out", contiguous=False)
    if out.stride(1) != 1:
        raise ValueError("cols_to_f32: out must have unit column stride")
    dts = [_COL_DT[c.dtype] for c in cols]
    check(_C.ext().cols_to_f32([ptr(c) for c in cols], dts, rows, ptr(out), out.stride(0), stream()), "cols_to_f32")
    return out


def u8_normalize_chan(x, scale, shift, reverse=False, out=None, cout=None):
    """uint8 NHWC [..., C] -> bf16, per channel x * scale[c] + shift[c] (channel order reversed first
    with ``reverse``: RGB -> BGR).  ``cout=8``: the output has 8 channels, C..7 zero (a stem conv's
    input padded for the C % 8 == 0 MFMA paths, nn.Conv2d)."""
    C = x.shape[-1]
    cout = C if cout is None else int(cout)
    if out is None:
        out = torch.empty((*x.shape[:-1], cout), device=x.device, dtype=torch.bfloat16)
    check(_C.ext().u8_normalize_chan(ptr(x), ptr(out), x.numel() // C, C, [float(v) for v in scale],
                                     [float(v) for v in shift], int(bool(reverse)), cout, stream()),
          "u8_normalize_chan")
    return out


def u8_normalize(x, scale, shift, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=BF16)
    check(_C.ext().u8_normalize(ptr(x), ptr(out), x.numel(), float(scale), float(shift), stream()), "u8_normalize")
    return out


def act_bwd(dy, y, act, out=None):
    if out is None:
        out = torch.empty_like(dy)
    check(_C.ext().act_bwd(ptr(dy), ptr(y), ptr(out), dy.numel(), act_id(act), stream()), "act_bwd")
    return out


def act_bwd_colsum(dy, y, act, colsum, out=None):
    """dx = dy * act'(y) (y may be None = identity) and colsum += sum over rows of dx."""
    if out is None:
        out = torch.empty_like(dy)
    N = dy.shape[-1]
    M = dy.numel() // N
    check(_C.ext().act_bwd_colsum(ptr(dy), ptr(y), ptr(out), M, N, act_id(act), ptr(colsum), stream()),
          "act_bwd_colsum")
    return out


def add(a, b, act=0, out=None):
    if out is None:
        out = torch.empty_like(a)
    check(_C.ext().add_bf16(ptr(a), ptr(b), ptr(out), a.numel(), act_id(act), stream()), "add")
    return out


# ---------------------------------------------------------------- batchnorm
_BN_ACC: dict = {}
BN_NREP = 8  # replica rows of the BN column-reduction accumulators (norm.hip BN_NREP)


def bn_acc(device, C, alt: bool = False) -> torch.Tensor:
    """Zero-at-rest [BN_NREP, 2C] fp32 accumulator (+ arrival counter) for the vectorized BN
    reductions: the reduction's last workgroup finalizes and re-zeroes it, so one buffer per
    (device, C) serves every BN layer of that width in stream order, with no memset or finalize
    launches.  Created outside graph capture (warm-up).  ``alt``: the second buffer of the width, for a
    conv that reads one BN's statistics (its folded input BN, conv2d_fwd_bnstats_inbn) while producing
    the next one's."""
    key = (str(device), int(C)) + ((1,) if alt else ())
    t = _BN_ACC.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("BN accumulator must be created before graph capture (run an eager step first)")
        # + the 9 x 32 arrival words of the in-launch finalize (common.h grid_arrive_last) + the
        # one-launch backward's grid barrier (count, generation, timeout flag; norm.hip bn_bwd_coop8_k)
        t = torch.zeros(BN_NREP * 2 * C + 9 * 32 + 3 * 32, device=device, dtype=F32)
        _BN_ACC[key] = t
    return t


def bn_sums_acc(owner, device, C) -> torch.Tensor:
    """A zero-at-rest accumulator (bn_acc's layout) private to ONE BatchNorm (kept on ``owner``, its gamma):
    the backward column sums that a consumer conv's dgrad epilogue reduces (conv2d_bwd_pair /
    conv2d_dgrad_bn bn=...) wait there until that BN's apply (bn_bwd_pre) folds and re-zeroes them, so no
    other BN reduction of the same width that autograd schedules in between can mix into them."""
    t = getattr(owner, "_hx_bnsum_acc", None) if owner is not None else None
    if t is None or t.numel() != BN_NREP * 2 * C + 12 * 32 or t.device != torch.device(device):
        if owner is None:
            return bn_acc(device, C)
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("BN accumulator must be created before graph capture (run an eager step first)")
        t = torch.zeros(BN_NREP * 2 * C + 12 * 32, device=device, dtype=F32)
        owner._hx_bnsum_acc = t
    return t


def bn_fwd_train(x2d, gamma, beta, mean, rstd, rmean, rvar, momentum, eps, residual=None, act=0, out=None):
    M, C = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    check(_C.ext().bn_fwd_train(ptr(x2d), ptr(out), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd), ptr(rmean),
                                ptr(rvar), float(momentum), float(eps), M, C, ptr(residual), act_id(act),
                                ptr(bn_acc(x2d.device, C)), stream()),
          "bn_fwd_train")
    return out


def conv2d_fwd_bnstats(x, w, geom, out=None):
    """Conv forward (bf16 out, no bias / activation) whose epilogue also accumulates the BatchNorm
    statistics of its output into the per-width accumulator ``bn_acc`` (norm.hip layout).  Returns
    None — nothing launched — when the shape has no such epilogue; otherwise the output, and the
    next op on the stream MUST be ``bn_fwd_apply_fin`` on it (it consumes and re-zeroes acc)."""
    _req(x, BF16, "x")
    _req(w, BF16, "w")
    B, OH, OW, CO = geom[0], geom[4], geom[5], geom[6]
    if out is None:
        out = torch.empty(B, OH, OW, CO, device=x.device, dtype=BF16)
    rc = _C.ext().conv2d_fwd_bnstats(ptr(x), ptr(w), list(geom), ptr(out), ptr(bn_acc(x.device, CO)), stream())
    if rc == -2:
        return None
    check(rc, "conv2d_fwd_bnstats")
    return out


def conv2d_fwd_bnstats_inbn(z, a, w, geom, fold, out=None):
    """conv2d_fwd_bnstats whose input a = act(bn(z)) is a training BatchNorm's output that no apply launch
    produced (functional.batch_norm fold_next): the conv applies the BN inside its operand gather and
    writes ``a`` itself (conv_mfma.hip InBn).  ``fold`` = (gamma, beta, mean, rstd, rmean, rvar, momentum,
    eps, act) of that BN; its statistics are in bn_acc(C), this conv's output statistics go to
    bn_acc(CO, alt=True).  None — nothing launched — when the shape has no such path."""
    _req(z, BF16, "z")
    _req(w, BF16, "w")
    gamma, beta, mean, rstd, rm, rv, momentum, eps, act = fold
    B, OH, OW, CO, C = geom[0], geom[4], geom[5], geom[6], geom[3]
    if out is None:
        out = torch.empty(B, OH, OW, CO, device=z.device, dtype=BF16)
    rc = _C.ext().conv2d_fwd_bnstats_inbn(ptr(z), ptr(a), ptr(w), list(geom), ptr(out),
                                          ptr(bn_acc(z.device, CO, alt=True)), ptr(bn_acc(z.device, C)), ptr(gamma),
                                          ptr(beta), ptr(mean), ptr(rstd), ptr(rm), ptr(rv), float(momentum),
                                          float(eps), act_id(act), stream())
    if rc == -2:
        return None
    check(rc, "conv2d_fwd_bnstats_inbn")
    return out


def bn_coop_timeouts(device, C) -> int:
    """Nonzero if a one-launch BN backward barrier of width C ever timed out (never expected)."""
    return int(_C.ext().bn_coop_timeouts(ptr(bn_acc(device, C)), int(C)))


def bn_prestats_ok(C) -> bool:
    return bool(_C.ext().bn_prestats_ok(int(C)))


def bn_fwd_apply_fin(x2d, gamma, beta, mean, rstd, rmean, rvar, momentum, eps, residual=None, act=0, out=None,
                     alt=False):
    """Training BN forward whose statistics the producing conv already accumulated
    (conv2d_fwd_bnstats; into bn_acc(C, alt) for conv2d_fwd_bnstats_inbn): one launch that finalizes them,
    applies act(bn(x) + residual) and re-zeroes the accumulator."""
    M, C = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    check(_C.ext().bn_fwd_apply_fin(ptr(x2d), ptr(out), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd), ptr(rmean),
                                    ptr(rvar), float(momentum), float(eps), M, C, ptr(residual), act_id(act),
                                    ptr(bn_acc(x2d.device, C, alt=alt)), stream()),
          "bn_fwd_apply_fin")
    return out


def bn_fwd_infer(x2d, gamma, beta, rmean, rvar, eps, residual=None, act=0, out=None):
    M, C = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    check(_C.ext().bn_fwd_infer(ptr(x2d), ptr(out), ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), float(eps), M, C,
                                ptr(residual), act_id(act), stream()), "bn_fwd_infer")
    return out


def bn_bwd(dy, x, y, gamma, mean, rstd, dgamma, dbeta, ws, act=0, dresidual=None, out=None, zbeta=None):
    """``zbeta``: the BN's beta when its forward had NO residual: a ReLU's act' is then recomputed from
    x (the forward's exact z * scale + shift > 0 test) instead of reading y (norm.hip bn_shift)."""
    M, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(_C.ext().bn_bwd(ptr(dy), ptr(x), ptr(y), ptr(gamma), ptr(mean), ptr(rstd), ptr(out), ptr(dgamma),
                          ptr(dbeta), ptr(ws), M, C, act_id(act), ptr(dresidual), ptr(bn_acc(dy.device, C)),
                          ptr(zbeta), stream()), "bn_bwd")
    return out


def bn_bwd_pre(g, x, gamma, mean, rstd, dgamma, dbeta, ws, acc, out=None):
    """BN backward whose column sums a consumer conv's dgrad epilogue already reduced into ``acc`` (the BN's
    own accumulator, bn_sums_acc; conv2d_bwd_pair bn=...); ``g`` is the act'-masked output gradient.  One
    apply launch, which also re-zeroes ``acc``."""
    M, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(_C.ext().bn_bwd_pre(ptr(g), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), ptr(out), ptr(dgamma), ptr(dbeta),
                              ptr(ws), M, C, ptr(acc), stream()), "bn_bwd_pre")
    return out


# ------------------------------------------------------------ embedding bag
def embedding_bag_fwd(table, idx, offsets, mode, out, ldo=None, bag_len=1):
    """Bags are given by ``offsets`` or, without offsets, by a fixed ``bag_len`` (idx [bags, bag_len])."""
    nb = out.shape[0] if offsets is None else offsets.numel()
    dim = table.shape[1]
    assert offsets is not None or idx.numel() == nb * bag_len, "idx / bag_len / out shape mismatch"
    check(_C.ext().embedding_bag_fwd(ptr(table), ptr(idx), ptr(offsets), nb, dim, idx.numel(), bag_len, mode, ptr(out),
                                     int(out.dtype == F32), ldo if ldo is not None else out.stride(0), table.shape[0],
                                     stream()),
          "embedding_bag_fwd")
    return out


def embedding_bag_bwd(dout, idx, offsets, mode, dtable, nbags, ldo=None, bag_len=1):
    dim = dtable.shape[1]
    assert offsets is not None or idx.numel() == nbags * bag_len, "idx / bag_len mismatch"
    check(_C.ext().embedding_bag_bwd(ptr(dout), int(dout.dtype == F32), ldo if ldo is not None else dout.stride(0),
                                     ptr(idx), ptr(offsets), nbags, dim, idx.numel(), bag_len, mode, ptr(dtable),
                                     dtable.shape[0], stream()),
          "embedding_bag_bwd")
    return dtable


# --------------------------------------------------------- TFX transform (transform.hip)
def taxi_transform(raw, vids, ints, flts, offs, nd, nc, with_label=True):
    """Apply an analyzed Chicago-taxi transform to raw fp32 rows [n, F] on the GPU (one launch):
    returns (dense fp32 [n, nd], cat int64 [n, nc] global wide ids, label fp32 [n, 1] | None)."""
    n = raw.shape[0]
    dense = torch.empty(n, nd, device=raw.device, dtype=F32)
    cat = torch.empty(n, nc, device=raw.device, dtype=torch.int64)
    label = torch.empty(n, 1, device=raw.device, dtype=F32) if with_label else None
    check(_C.ext().taxi_transform(ptr(raw), ptr(vids), n, [int(v) for v in ints], [float(v) for v in flts],
                                  [int(v) for v in offs], ptr(dense), ptr(cat), ptr(label), stream()),
          "taxi_transform")
    return dense, cat, label


# --------------------------------------------------------- range windows (window.hip)
def prefix_sum_f64(v):
    """Exclusive fp64 prefix sum P[0..n] of a 1-D fp64 tensor (P[n] = total)."""
    n = v.numel()
    P = torch.empty(n + 1, device=v.device, dtype=torch.float64)
    work = torch.empty(max(1, -(-n // 4096)), device=v.device, dtype=torch.float64)
    check(_C.ext().prefix_sum_f64(ptr(v), n, ptr(P), ptr(work), stream()), "prefix_sum_f64")
    return P


def range_window(ts, seg, seg_off, v, lo, hi, want_count=False):
    """Range-window sums (Spark rangeBetween) of rows sorted by (partition, ts): returns fp64 [n, W]
    (NaN where the range is empty) and, with ``want_count``, int32 [n, W] row counts."""
    n, W = ts.numel(), lo.numel()
    P = prefix_sum_f64(v)
    out = torch.empty(n, W, device=ts.device, dtype=torch.float64)
    cnt = torch.empty(n, W, device=ts.device, dtype=torch.int32) if want_count else None
    check(_C.ext().range_window(ptr(ts), ptr(seg), ptr(seg_off), ptr(P), n, ptr(lo), ptr(hi), W, ptr(out), ptr(cnt),
                                stream()), "range_window")
    return (out, cnt) if want_count else out


# --------------------------------------------------------- column statistics
def column_stats(x):
    """x [rows, cols] f32 on GPU -> [cols, 5] = count, sum, sumsq, min, max (NaN = missing)."""
    rows, cols = x.shape
    out = torch.zeros(cols, 5, device=x.device, dtype=F32)
    out[:, 3] = float("inf")
    out[:, 4] = float("-inf")
    check(_C.ext().column_stats(ptr(x), rows, cols, ptr(out), stream()), "column_stats")
    return out


def column_stats64(x):
    """x [rows, cols] f64 on GPU -> [cols, 7] f64 = count, sum, sumsq, min, max, #(>= 0), #(> 0)."""
    rows, cols = x.shape
    out = torch.zeros(cols, 7, device=x.device, dtype=torch.float64)
    out[:, 3] = float("inf")
    out[:, 4] = float("-inf")
    check(_C.ext().column_stats64(ptr(x), rows, cols, ptr(out), stream()), "column_stats64")
    return out


def column_hist(x, mins, maxs, bins):
    rows, cols = x.shape
    hist = torch.zeros(cols, bins, device=x.device, dtype=torch.int32)
    check(_C.ext().column_hist(ptr(x), rows, cols, ptr(mins), ptr(maxs), bins, ptr(hist), stream()), "column_hist")
    return hist


def gram(x, mean):
    rows, cols = x.shape
    g = torch.zeros(cols, cols, device=x.device, dtype=F32)
    check(_C.ext().gram(ptr(x), ptr(mean), rows, cols, ptr(g), stream()), "gram")
    return g


# ------------------------------------------------------------- health checks
def zero_(t):
    """Graph-safe zero fill (a kernel node, not a hipMemsetAsync blit node)."""
    check(_C.ext().zero(ptr(t), t.numel() * t.element_size(), stream()), "zero")
    return t


def nonfinite_counts(x, out=None):
    """int32[2] = (#NaN, #Inf) of an fp32 / bf16 GPU tensor; one fused read pass, no host sync."""
    if x.dtype not in (F32, BF16):
        raise TypeError(f"nonfinite_counts: fp32 or bf16 expected, got {x.dtype}")
    x = x.contiguous()
    if out is None:
        out = torch.empty(2, device=x.device, dtype=torch.int32)
    zero_(out)
    check(_C.ext().nonfinite(ptr(x), x.numel(), int(x.dtype == BF16), ptr(out), stream()), "nonfinite")
    return out


# --------------------------------------------------------- fused classifier head
_MLP_WS: dict = {}


def _mlp_ws(device, n: int):
    """Persistent zero-at-rest workspace + arrival counter of the fused Dense->head kernel (one per
    device; every launch leaves them zeroed, so graph replays reuse them)."""
    cur = _MLP_WS.get(device)
    if cur is None or cur[0].numel() < n:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("mlp_head workspace must exist before graph capture (run an eager step first)")
        cur = (torch.zeros(max(n, 4096), device=device, dtype=F32), torch.zeros(9 * 32, device=device, dtype=torch.int32))
        _MLP_WS[device] = cur
    return cur


def mlp_head(x, w1, b1, act1, y, kind: int, logits, target, w2, b2, dw2, db2, grad_scale: float, loss_sum, correct,
             drop=None):
    """Last hidden Dense layer + classifier head in ONE launch (loss.hip mlp_head_k): fills ``y`` =
    act(x W1^T + b1) (bf16 [B, N1]) and ``logits``, and does what head_ce does (loss, dW2/db2
    accumulation); returns dh [B, N1] bf16, or False when the shape is not supported.  ``drop`` =
    (p, rng, salt): a Dropout between the two (applied to the head's input, dh is then the gradient of y)."""
    B, K = x.shape
    N1 = w1.shape[0]
    C = w2.shape[0]
    _req(x, BF16, "x")
    _req(w1, BF16, "w1")
    _req(w2, BF16, "w2")
    _req(y, BF16, "y")
    ws, arrive = _mlp_ws(x.device, B * N1)
    dh = torch.empty(B, N1, device=x.device, dtype=BF16)
    rc = _C.ext().mlp_head(ptr(x), ptr(w1), ptr(b1), act_id(act1), ptr(y), ptr(ws), ptr(arrive), B, K, N1, int(kind),
                           ptr(target), C, float(grad_scale), ptr(w2), ptr(b2), ptr(dw2), ptr(db2), ptr(dh),
                           ptr(loss_sum), ptr(correct), ptr(logits), int(logits.dtype == F32),
                           float(drop[0]) if drop else 0.0, ptr(drop[1]) if drop else 0,
                           (int(drop[2]) & 0xFFFFFFFF) if drop else 0, stream())
    if rc == -2:
        return False
    check(rc, "mlp_head")
    return dh


def head_ce_ok(C: int, KD: int) -> bool:
    return bool(_C.ext().head_ce_ok(int(C), int(KD)))


def head_ce(kind: int, logits, target, h, w, dw, db, grad_scale: float, loss_sum, correct, bias=None,
            forward: bool = False, drop=None):
    """Loss + dlogits (never materialised) + dW += dl^T h + db += sum dl + returns dh = dl W, in one
    launch (loss.hip head_ce_k).  logits [B, C<=32] fp32/bf16, h [B, KD] bf16, w [C, KD] bf16.
    ``forward``: the layer's forward runs in the same launch — logits = h W^T + bias are computed
    from the staged operands and WRITTEN into ``logits`` (which is only an output then).
    ``drop`` = (p, rng, salt): ``h`` is the input of a Dropout feeding the head; the head applies it
    (dropout_k's mask and rounding) and dh is the gradient of that input."""
    B, C = logits.shape
    KD = h.shape[1]
    _req(h, BF16, "h")
    _req(w, BF16, "w")
    _req(dw, F32, "dw")
    dh = torch.empty(B, KD, device=h.device, dtype=BF16)
    check(_C.ext().head_ce(kind, ptr(logits), int(logits.dtype == F32), ptr(target), B, C, KD, float(grad_scale),
                           ptr(h), ptr(w), ptr(dw), ptr(db), ptr(dh), ptr(loss_sum), ptr(correct), ptr(bias),
                           ptr(logits) if forward else 0, float(drop[0]) if drop else 0.0,
                           ptr(drop[1]) if drop else 0, (int(drop[2]) & 0xFFFFFFFF) if drop else 0, stream()),
          "head_ce")
    return dh
