"""Thin torch-tensor front end of the C ABI (``include/rp_api.h``).

Every function validates device / dtype / layout on the host, then enqueues the HIP kernel on the
current torch stream through ``_native.call``.  Outputs are allocated with the torch caching
allocator; the library itself never allocates.  There is no CPU path: CPU tensors raise.
"""
import ctypes
import os

import torch

from . import _native as N

_DT = {torch.float32: N.RP_F32, torch.bfloat16: N.RP_BF16}
RP_ATTN_Q_PRESCALED = 0x100  # include/rp_api.h: q holds Q * scale * log2(e)
LOG2E = 1.4426950408889634


def _adt(t, q_prescaled):
    """dtype argument of the attention entry points (with the Q-prescaled flag)."""
    return _dt(t) | (RP_ATTN_Q_PRESCALED if q_prescaled else 0)

# Live per-kernel timing with HIP events recorded on the launch stream (bench.py roofline).
_timer = {"names": (), "ev": {}}


def timer_start(*names):
    _timer["names"] = tuple(names)
    _timer["ev"] = {n: [] for n in names}


def timer_stop(detail=False):
    """{name: average duration (ms) of that kernel's launches since timer_start, or None}; with
    detail, {name: (average ms, launches, total ms, total algorithmic FLOPs or None, [ms per launch])}."""
    ev = _timer["ev"]
    _timer["names"] = ()
    _timer["ev"] = {}
    torch.cuda.synchronize()
    out = {}
    for n, v in ev.items():
        if not v:
            out[n] = None if not detail else (None, 0, 0.0, None, [])
            continue
        each = [a.elapsed_time(b) for a, b, _ in v]
        tot = sum(each)
        fl = sum(f for _, _, f in v) if all(f is not None for _, _, f in v) else None
        out[n] = tot / len(v) if not detail else (tot / len(v), len(v), tot, fl, each)
    return out


def _tick(name):
    if name not in _timer["names"]:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return (name, e)


def _tock(t0, flops=None):
    if t0 is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        _timer["ev"][t0[0]].append((t0[1], e1, flops))


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"repurpose_amd: unsupported dtype {t.dtype} (float32 / bfloat16)") from None


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("repurpose_amd: HIP kernels need tensors on a ROCm device "
                               f"(got {t.device}); there is no CPU path")


def _contig(*ts):
    for t in ts:
        if t is not None and not t.is_contiguous():
            raise ValueError("repurpose_amd: tensor must be contiguous")


# ------------------------------------------------------------------------------------- K1, casts
def concat_rows(v, a, t, out_dtype):
    """[v | a | t] along the last dim; inputs [..., d] fp32 -> [rows, dv+da+dt] of out_dtype."""
    _gpu(v, a, t)
    v, a, t = (x.contiguous().float() for x in (v, a, t))
    rows = v.numel() // max(v.shape[-1], 1) if v.shape[-1] else a.numel() // max(a.shape[-1], 1)
    dv, da, dt = v.shape[-1], a.shape[-1], t.shape[-1]
    out = torch.empty(rows, dv + da + dt, device=v.device, dtype=out_dtype)
    N.call("rp_concat_rows", _p(v), dv, _p(a), da, _p(t), dt, rows, _p(out), _DT[out_dtype], _stream(v))
    return out


def cast_bf16(src, dst):
    _gpu(src, dst)
    _contig(src, dst)
    assert src.dtype == torch.float32 and dst.dtype == torch.bfloat16 and src.numel() == dst.numel()
    N.call("rp_cast_f32_to_bf16", _p(src), _p(dst), src.numel(), _stream(src))
    return dst


# ------------------------------------------------------------------------------------- GEMM
def gemm(A, B, C, M, Nn, K, lda, a_kmajor, ldb, b_kmajor, ldc, alpha=1.0, bias=None, relu=False,
         dropout_p=0.0, seed=0, residual=None, ldr=0, gate=None, ldg=0, gate_scale=1.0,
         accumulate=False, col_scale_n=0, col_scale=1.0, seed_base=None):
    """Raw rp_gemm (see include/rp_api.h for the operand conventions).  ``seed_base``: optional int32
    device word; the dropout then draws with rp_hash(*seed_base, seed), read when the kernel runs."""
    _gpu(A, B, C, bias, residual, gate)
    _seed_word(seed_base)
    if A.dtype != B.dtype:
        raise TypeError("rp_gemm: A and B must share a dtype")
    ep = N.GemmEpilogue(_p(bias).value, int(relu), float(dropout_p), int(seed) & 0xFFFFFFFF,
                        _p(residual).value, int(ldr), _p(gate).value,
                        _dt(gate) if gate is not None else 0, int(ldg), float(gate_scale),
                        int(accumulate), int(col_scale_n), float(col_scale), _p(seed_base).value)
    N.call("rp_gemm", _dt(A), int(M), int(Nn), int(K), _p(A), int(lda), int(a_kmajor), _p(B), int(ldb),
           int(b_kmajor), _p(C), int(ldc), _dt(C), float(alpha), ctypes.byref(ep), _stream(A))
    return C


def linear_fwd(x, W, b=None, out_dtype=None, relu=False, dropout_p=0.0, seed=0, residual=None, tag=None,
               col_scale_n=0, col_scale=1.0, seed_base=None):
    """y = epilogue(x W^T + b); x [M, K], W [N, K] (same dtype), residual fp32 [M, N]; columns
    < col_scale_n are multiplied by col_scale after the bias (the attention's Q prescale)."""
    M, K = x.shape
    Nn = W.shape[0]
    out = torch.empty(M, Nn, device=x.device, dtype=out_dtype or x.dtype)
    e0 = _tick(tag) if tag else None
    gemm(x, W, out, M, Nn, K, K, True, K, True, Nn, bias=b, relu=relu, dropout_p=dropout_p,
         seed=seed, residual=residual, ldr=Nn, col_scale_n=col_scale_n, col_scale=col_scale, seed_base=seed_base)
    _tock(e0)
    return out


def linear_dgrad(dy, W, out_dtype, gate=None, gate_scale=1.0):
    """dx = (dy W) [* gate_scale * (gate > 0)]; dy [M, N], W [N, K] -> [M, K]."""
    M, Nn = dy.shape
    K = W.shape[1]
    out = torch.empty(M, K, device=dy.device, dtype=out_dtype)
    return gemm(dy, W, out, M, K, Nn, Nn, True, K, False, K, gate=gate, ldg=K, gate_scale=gate_scale)


def linear_wgrad(dy, x, dW, db=None, accumulate=True, ws=None):
    """dW (+)= dy^T x and db (+)= colsum(dy); dy [T, N], x [T, K], dW fp32 [N, K] (split-K over T)."""
    _gpu(dy, x, dW, db)
    T, Nn = dy.shape
    K = x.shape[1]
    if dy.dtype != x.dtype:
        raise TypeError("rp_gemm_wgrad: dy and x must share a dtype")
    need = N.load().rp_gemm_wgrad_workspace(Nn, K, T)
    if ws is None or ws.numel() * ws.element_size() < need:
        ws = torch.empty(max(need // 4, 4), device=dy.device, dtype=torch.float32)
    e0 = _tick("gemm_wgrad")
    N.call("rp_gemm_wgrad", _dt(dy), Nn, K, T, _p(dy), dy.stride(0), _p(x), x.stride(0), _p(dW), _p(db),
           int(accumulate), _p(ws), ws.numel() * ws.element_size(), _stream(dy))
    _tock(e0, 2.0 * Nn * K * T)
    return dW


WGRAD_GROUP_MAX = 64  # items per rp_gemm_wgrad_grouped launch


def linear_wgrad_grouped(items, accumulate=True):
    """dW_i (+)= dy_i^T x_i, db_i (+)= colsum(dy_i) for items [(dy, x, dW, db)], all bf16 operands over
    the same token count T (a multiple of 64): whole-K tiles, no split-K workspace (rp_gemm_wgrad_grouped).
    Launches ceil(len / 64) kernels."""
    if not items:
        return
    T = items[0][0].shape[0]
    for dy, x, dW, db in items:
        _gpu(dy, x, dW, db)
        if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16:
            raise TypeError("rp_gemm_wgrad_grouped: bf16 operands")
        if dy.shape[0] != T or x.shape[0] != T:
            raise ValueError("rp_gemm_wgrad_grouped: every item needs the same token count")
        if dW.dtype != torch.float32 or not dW.is_contiguous() or tuple(dW.shape) != (dy.shape[1], x.shape[1]):
            raise ValueError("rp_gemm_wgrad_grouped: dW must be fp32 contiguous [N_out, N_in]")
    for c in range(0, len(items), WGRAD_GROUP_MAX):
        chunk = items[c:c + WGRAD_GROUP_MAX]
        arr = (N.WgradItem * len(chunk))()
        fl = 0.0
        for i, (dy, x, dW, db) in enumerate(chunk):
            arr[i] = N.WgradItem(_p(dy).value, _p(x).value, _p(dW).value, _p(db).value, dy.shape[1], x.shape[1],
                                 dy.stride(0), x.stride(0))
            fl += 2.0 * dy.shape[1] * x.shape[1] * T
        e0 = _tick("gemm_wgrad")
        N.call("rp_gemm_wgrad_grouped", T, ctypes.cast(arr, ctypes.c_void_p), len(chunk), int(accumulate),
               _stream(chunk[0][0]))
        _tock(e0, fl)


# ----------------------------------------------------------------------- GEMM + LayerNorm seams
_LNX = {}        # device -> [workspace (uint8), rows it serves, last stream that used it]
_LNX_KEEP = []   # every workspace ever handed out: a captured graph holds their raw pointers
_LNX_MIN_ROWS = 65536  # first allocation: 2.2 MB, enough for B * T up to 65,536 rows


def _lnx_ws(dev, M):
    """The exchange workspace of the GEMM + LayerNorm exchange kernels (rp_gemm_ln_xchg_bytes, zero-filled
    once; every launch leaves it zeroed), one per device.  It is never freed: a workspace that is too small
    is replaced by a larger one but kept alive, because a captured step's graph holds the raw pointer of
    the workspace it was captured with.  Launches sharing it must be ordered: when the current stream
    differs from the one that used it last (and no capture is running), the current stream waits for the
    other's work so far.  RP_GEMM_LNX=0 (A/B): None, i.e. the 64-row full-row kernels."""
    if M % 64 or os.environ.get("RP_GEMM_LNX", "1") != "1":
        return None
    ent = _LNX.get(dev)
    if ent is None or ent[1] < M:
        rows = max(M, _LNX_MIN_ROWS if ent is None else 2 * ent[1])
        ws = torch.zeros(int(N.load().rp_gemm_ln_xchg_bytes(rows)), device=dev, dtype=torch.uint8)
        _LNX_KEEP.append(ws)
        ent = [ws, rows, None]
        _LNX[dev] = ent
    cur = torch.cuda.current_stream(dev)
    last = ent[2]
    if last is not None and last != cur and not torch.cuda.is_current_stream_capturing():
        ev = torch.cuda.Event()
        ev.record(last)
        cur.wait_event(ev)
    ent[2] = cur
    return ent[0]


def lnx_status():
    """Raise RuntimeError if an exchange wait has given up since the last reset (rp_gemm_ln_status: a
    host-mapped word, no synchronisation); the workspaces are then re-zeroed and the fault cleared, so the
    next launch starts clean."""
    if N.load().rp_gemm_ln_status() != N.RP_OK:
        msg = N.last_error()
        lnx_reset()
        raise RuntimeError(f"rp_gemm_ln_status: {msg}")


def lnx_reset():
    """rp_gemm_ln_reset on every device's exchange workspace (synchronises their streams)."""
    for dev, (ws, rows, last) in _LNX.items():
        st = last if last is not None else torch.cuda.current_stream(dev)
        N.call("rp_gemm_ln_reset", _p(ws), int(rows), ctypes.c_void_p(st.cuda_stream))
    if not _LNX:
        N.call("rp_gemm_ln_reset", ctypes.c_void_p(0), 0, ctypes.c_void_p(0))


def _lnx_call(name, M, K, args, stream):
    """rp_gemm_ln_fwd / bwd; a fault reported by the call resets the workspaces before it raises."""
    rc = getattr(N.load(), name)(M, K, ctypes.byref(args), stream)
    if rc != N.RP_OK:
        msg = N.last_error()
        if N.load().rp_gemm_ln_status() != N.RP_OK:
            lnx_reset()
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def linear_ln_fwd(x, W, b, residual, gamma, beta, eps=1e-5, dropout_p=0.0, seed=0, seed_base=None):
    """One launch (rp_gemm_ln_fwd) for ``y = dropout(x W^T + b) + residual`` (fp32, returned) and
    ``h = LayerNorm(y)`` (bf16) with its mean / rstd — linear_fwd(..., residual=...) followed by
    layernorm_fwd(y, out_f32=False, lp_dtype=bf16): y bitwise; h / mean / rstd bitwise on the 64-row
    kernels, to fp32 rounding of the row sums on the exchange kernels (the default; RP_GEMM_LNX=0 A/B).  x [M, K] bf16, W [512, K] bf16, M % 64 == 0.  Returns (y, h, mean, rstd)."""
    a, outs = ln_fwd_args(x, W, b, residual, gamma, beta, eps, dropout_p, seed, seed_base)
    M, K = x.shape
    e0 = _tick("gemm_ln_fwd")
    _lnx_call("rp_gemm_ln_fwd", M, K, a, _stream(x))
    _tock(e0, 2.0 * M * 512 * K)
    return outs


def ln_fwd_args(x, W, b, residual, gamma, beta, eps=1e-5, dropout_p=0.0, seed=0, seed_base=None):
    """(rp_gemm_ln_args, (y, h, mean, rstd)) of linear_ln_fwd, outputs allocated, nothing launched."""
    _gpu(x, W, b, residual, gamma, beta)
    _seed_word(seed_base)
    M, K = x.shape
    dev = x.device
    y = torch.empty(M, 512, device=dev, dtype=torch.float32)
    h = torch.empty(M, 512, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(M, device=dev, dtype=torch.float32)
    rstd = torch.empty(M, device=dev, dtype=torch.float32)
    a = N.GemmLnArgs(A=_p(x).value, lda=x.stride(0), W=_p(W).value, ldw=W.stride(0), bias=_p(b).value,
                     dropout_p=float(dropout_p), dropout_seed=int(seed) & 0xFFFFFFFF, seed_base=_p(seed_base).value,
                     residual=_p(residual).value, ldr=residual.stride(0), x_out=_p(y).value, ldx_out=512,
                     gamma=_p(gamma).value, beta=_p(beta).value, eps=float(eps), h_out=_p(h).value, ldh=512,
                     mean=_p(mean).value, rstd=_p(rstd).value, xchg=_p(_lnx_ws(dev, M)).value)
    return a, (y, h, mean, rstd)


def linear_ln_bwd(dy, W, x, mean, rstd, gamma, dres=None, lp_dtype=None, lp_dropout_p=0.0, lp_seed=0, dgamma=None,
                  dbeta=None, defer=None, ws=None, seed_base=None):
    """One launch (rp_gemm_ln_bwd) for ``dh = dy W`` (dy [M, K] bf16, W [K, 512] bf16) followed by the
    LayerNorm backward of the LayerNorm whose input was x — linear_dgrad(dy, W, fp32) then
    layernorm_bwd(dh, x, mean, rstd, gamma, dres=..., lp_dtype=..., ...), bitwise on the 64-row kernels and
    to fp32 rounding of the row sums on the exchange kernels (as linear_ln_fwd); dh is never written.
    Returns (dx fp32, dx_lp or None); gamma / beta partials as layernorm_bwd (``defer`` / ``ws``)."""
    a, (dx, dxl, jobs) = ln_bwd_args(dy, W, x, mean, rstd, gamma, dres, lp_dtype, lp_dropout_p, lp_seed, dgamma,
                                     dbeta, seed_base)
    M, K = dy.shape
    e0 = _tick("gemm_ln_bwd")
    _lnx_call("rp_gemm_ln_bwd", M, K, a, _stream(dy))
    _tock(e0, 2.0 * M * 512 * K)
    if defer is not None:
        defer.extend(jobs)
    else:
        for p, o in jobs:
            colsum(p, out=o, accumulate=True, ws=ws)
    return dx, dxl


def ln_bwd_args(dy, W, x, mean, rstd, gamma, dres=None, lp_dtype=None, lp_dropout_p=0.0, lp_seed=0, dgamma=None,
                dbeta=None, seed_base=None):
    """(rp_gemm_ln_args, (dx, dx_lp, gamma / beta partial jobs)) of linear_ln_bwd, nothing launched."""
    _gpu(dy, W, x, mean, rstd, gamma, dres)
    _seed_word(seed_base)
    M, K = dy.shape
    dev = dy.device
    D = 512
    dx = torch.empty(M, D, device=dev, dtype=torch.float32)
    dxl = torch.empty(M, D, device=dev, dtype=lp_dtype) if lp_dtype is not None else None
    nb = M // 32
    both = (dgamma is not None and dbeta is not None and dgamma.is_contiguous() and dbeta.is_contiguous()
            and dbeta.data_ptr() == dgamma.data_ptr() + 4 * D and dgamma.dtype == dbeta.dtype == torch.float32
            and dgamma.untyped_storage().data_ptr() == dbeta.untyped_storage().data_ptr())
    ld_part = 2 * D if both else D
    if both:
        part = torch.empty(nb, 2 * D, device=dev, dtype=torch.float32)
        pg, pb = part[:, :D], part[:, D:]
    else:
        pg = torch.empty(nb, D, device=dev, dtype=torch.float32) if dgamma is not None else None
        pb = torch.empty(nb, D, device=dev, dtype=torch.float32) if dbeta is not None else None
    a = N.GemmLnArgs(A=_p(dy).value, lda=dy.stride(0), W=_p(W).value, ldw=W.stride(0), gamma=_p(gamma).value,
                     seed_base=_p(seed_base).value, mean=_p(mean).value, rstd=_p(rstd).value, x=_p(x).value,
                     ldx=x.stride(0), dres=_p(dres).value, lddres=dres.stride(0) if dres is not None else 0,
                     dx=_p(dx).value, lddx=D, dx_lp=_p(dxl).value, lddx_lp=D, lp_dropout_p=float(lp_dropout_p),
                     lp_seed=int(lp_seed) & 0xFFFFFFFF, dgamma_part=_p(pg).value, dbeta_part=_p(pb).value,
                     ld_part=ld_part, xchg=_p(_lnx_ws(dev, M)).value)
    jobs = [(part, dgamma.as_strided((2 * D,), (1,)))] if both else \
        [(p, o) for p, o in ((pg, dgamma), (pb, dbeta)) if o is not None]
    return a, (dx, dxl, jobs)


# ------------------------------------------------------------------------------------- LayerNorm
def layernorm_fwd(x, gamma, beta, eps=1e-5, pe=None, pe_period=1, relu=False, dropout_p=0.0, seed=0,
                  out_f32=True, lp_dtype=None, save_stats=True, seed_base=None):
    _gpu(x, gamma, beta, pe)
    _seed_word(seed_base)
    rows, D = x.shape
    of = torch.empty(rows, D, device=x.device, dtype=torch.float32) if out_f32 else None
    ol = torch.empty(rows, D, device=x.device, dtype=lp_dtype) if lp_dtype is not None else None
    mean = torch.empty(rows, device=x.device, dtype=torch.float32) if save_stats else None
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32) if save_stats else None
    a = N.LnFwdArgs(_p(x).value, _dt(x), x.stride(0), _p(gamma).value, _p(beta).value, float(eps),
                    _p(pe).value, int(pe_period), int(relu), float(dropout_p), int(seed) & 0xFFFFFFFF,
                    _p(of).value, D, _p(ol).value, _dt(ol) if ol is not None else 0, D, _p(mean).value,
                    _p(rstd).value, _p(seed_base).value)
    N.call("rp_layernorm_fwd", rows, D, ctypes.byref(a), _stream(x))
    return of, ol, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, y=None, dropout_p=0.0, seed=0, dres=None, want_f32=True,
                  lp_dtype=None, lp_dropout_p=0.0, lp_seed=0, dgamma=None, dbeta=None, ws=None, defer=None,
                  seed_base=None):
    """Returns (dx_f32, dx_lp); accumulates dgamma / dbeta (fp32 [D]) when given.  With ``defer`` (a
    list), the gamma / beta partial reductions are appended to it as (partials, out) pairs for one
    ``colsum_batched`` call later instead of being launched here."""
    _gpu(dy, x, mean, rstd, gamma, y, dres)
    _seed_word(seed_base)
    rows, D = x.shape
    dev = x.device
    dx = torch.empty(rows, D, device=dev, dtype=torch.float32) if want_f32 else None
    dxl = torch.empty(rows, D, device=dev, dtype=lp_dtype) if lp_dtype is not None else None
    nb = N.load().rp_layernorm_bwd_blocks(rows)
    # gamma / beta gradients adjacent in memory (a LayerNorm's weight and bias in the flat
    # gradient buffer): interleave the partial rows [nb, 2D] and reduce both in one launch
    both = (dgamma is not None and dbeta is not None and dgamma.is_contiguous() and dbeta.is_contiguous()
            and dbeta.data_ptr() == dgamma.data_ptr() + 4 * D and dgamma.dtype == dbeta.dtype == torch.float32
            and dgamma.untyped_storage().data_ptr() == dbeta.untyped_storage().data_ptr())
    ld_part = 2 * D if both else D
    if both:
        part = torch.empty(nb, 2 * D, device=dev, dtype=torch.float32)
        pg, pb = part[:, :D], part[:, D:]
    else:
        pg = torch.empty(nb, D, device=dev, dtype=torch.float32) if dgamma is not None else None
        pb = torch.empty(nb, D, device=dev, dtype=torch.float32) if dbeta is not None else None
    a = N.LnBwdArgs(_p(dy).value, _dt(dy), dy.stride(0), _p(x).value, _dt(x), x.stride(0),
                    _p(mean).value, _p(rstd).value, _p(gamma).value, _p(y).value,
                    _dt(y) if y is not None else 0, y.stride(0) if y is not None else 0,
                    float(dropout_p), int(seed) & 0xFFFFFFFF, _p(dres).value, D, _p(dx).value, D,
                    _p(dxl).value, _dt(dxl) if dxl is not None else 0, D, float(lp_dropout_p),
                    int(lp_seed) & 0xFFFFFFFF, _p(pg).value, _p(pb).value, ld_part, _p(seed_base).value)
    N.call("rp_layernorm_bwd", rows, D, ctypes.byref(a), _stream(x))
    jobs = [(part, dgamma.as_strided((2 * D,), (1,)))] if both else \
        [(p, o) for p, o in ((pg, dgamma), (pb, dbeta)) if o is not None]
    if defer is not None:
        defer.extend(jobs)
    else:
        for p, o in jobs:
            colsum(p, out=o, accumulate=True, ws=ws)
    return dx, dxl


COLSUM_BATCH_MAX = 64


def colsum_batched(jobs, accumulate=True):
    """out (+)= column sums of X for every (X fp32 [rows, cols] with unit column stride, out fp32 [cols])
    in ``jobs``, ceil(len / 64) launches (rp_colsum_batched)."""
    for c in range(0, len(jobs), COLSUM_BATCH_MAX):
        chunk = jobs[c:c + COLSUM_BATCH_MAX]
        arr = (N.ColsumItem * len(chunk))()
        for i, (X, out) in enumerate(chunk):
            _gpu(X, out)
            if X.dtype != torch.float32 or out.dtype != torch.float32 or X.stride(1) != 1 or out.stride(0) != 1 \
                    or out.shape[0] != X.shape[1]:
                raise ValueError("colsum_batched: fp32 X with unit column stride and a matching fp32 out")
            arr[i] = N.ColsumItem(_p(X).value, _p(out).value, X.shape[0], X.shape[1], X.stride(0), int(accumulate))
        N.call("rp_colsum_batched", ctypes.cast(arr, ctypes.c_void_p), len(chunk), _stream(chunk[0][0]))


SUMSQ_BATCH_MAX = 64


def sumsq_batched(tensors):
    """fp64 device tensor [len(tensors)]: the sum of squares of every (contiguous fp32) tensor,
    ceil(len / 64) launches (rp_sumsq_batched); no host synchronisation."""
    if not tensors:
        return torch.zeros(0, dtype=torch.float64)
    _gpu(*tensors)
    out = torch.empty(len(tensors), dtype=torch.float64, device=tensors[0].device)
    for c in range(0, len(tensors), SUMSQ_BATCH_MAX):
        chunk = tensors[c:c + SUMSQ_BATCH_MAX]
        arr = (N.SumsqItem * len(chunk))()
        for i, t in enumerate(chunk):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != out.device:
                raise ValueError("sumsq_batched: contiguous fp32 tensors on one device")
            arr[i] = N.SumsqItem(_p(t).value, t.numel(), out.data_ptr() + 8 * (c + i))
        N.call("rp_sumsq_batched", ctypes.cast(arr, ctypes.c_void_p), len(chunk), _stream(chunk[0]))
    return out


# ------------------------------------------------------------------------------------- reductions
def colsum(X, w=None, out=None, accumulate=False, ws=None):
    """out[c] (+)= sum_r w[r] X[r, c] (deterministic)."""
    _gpu(X, w, out)
    rows, cols = X.shape
    if out is None:
        out = torch.empty(cols, device=X.device, dtype=torch.float32)
    need = N.load().rp_colsum_workspace(rows, cols)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 1), device=X.device, dtype=torch.float32)
    N.call("rp_colsum", _p(X), _dt(X), rows, cols, X.stride(0), _p(w), _p(out), int(accumulate), _p(ws),
           _stream(X))
    return out


# ------------------------------------------------------------------------------------- attention
def attn_fwd(qkv, key_valid, B, T, H, scale, dropout_p=0.0, seed=0, q_prescaled=False, out_lo=None, seed_base=None):
    """-> (out [B*T, H*dk], lse [B, H, T], dropmask or None).  The dropout keep bits drawn by the
    forward are returned and must be handed to attn_bwd.  q_prescaled: the Q columns of qkv hold
    Q * scale * log2(e) (linear_fwd's col_scale); the same flag must go to attn_bwd.  out_lo (bf16,
    optional, out's shape): filled with the output's rounding residual; hand it to attn_bwd too."""
    _gpu(qkv, key_valid)
    _contig(qkv, key_valid)
    _seed_word(seed_base)
    dk = qkv.shape[1] // (3 * H)
    out = torch.empty(B * T, H * dk, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(B, H, T, device=qkv.device, dtype=torch.float32)
    mask = None
    if dropout_p > 0:
        mask = torch.empty(N.load().rp_attn_dropmask_elems(B, T, H), device=qkv.device, dtype=torch.int16)
    e0 = _tick("attn_fwd")
    if out_lo is not None:
        _gpu(out_lo)
        if out_lo.shape != out.shape or out_lo.dtype != out.dtype or not out_lo.is_contiguous():
            raise ValueError("attn_fwd: out_lo must be a contiguous tensor like out")
    N.call("rp_attn_fwd", _adt(qkv, q_prescaled), _p(qkv), _p(key_valid), B, T, H, dk, float(scale), float(dropout_p),
           int(seed) & 0xFFFFFFFF, _p(seed_base), _p(out), _p(out_lo), _p(lse), _p(mask), _stream(qkv))
    _tock(e0)
    return out, lse, mask


def attn_bwd_uses_roles(qkv, B, T, H, q_prescaled=False):
    """True where attn_bwd runs the delta pass + ONE two-role launch (dK/dV and dQ workgroups side by
    side: grids that fill the CUs once, e.g. config 4) instead of the fused-delta dQ kernel + dK/dV."""
    return bool(N.load().rp_attn_bwd_uses_roles(_adt(qkv, q_prescaled), B, T, H, qkv.shape[1] // (3 * H)))


def attn_dout_delta(dy, W, out, out_lo, lse, B, T, H, dropout_p=0.0):
    """dO = dy W (bf16, the attention output's gradient through out_proj) with the attention backward's
    delta planes formed in the same launch (rp_gemm_attn_dout_delta).  -> (dO [M, H*64], delta
    [3, B, H, T]); hand delta to attn_bwd(delta=...).  bf16 operands, M = B*T and H*64 multiples of 128."""
    _gpu(dy, W, out, out_lo, lse)
    M, K = dy.shape
    D = H * 64
    if dy.dtype != torch.bfloat16 or W.dtype != torch.bfloat16 or out.dtype != torch.bfloat16:
        raise TypeError("attn_dout_delta: bf16 operands")
    if W.shape != (K, D) or out.shape != (M, D) or M != B * T or dy.stride(1) != 1 or W.stride(1) != 1:
        raise ValueError("attn_dout_delta: dy [B*T, K], W [K, H*64], out [B*T, H*64] with unit column strides")
    if out_lo is not None and (out_lo.shape != out.shape or out_lo.stride(0) != out.stride(0)):
        raise ValueError("attn_dout_delta: out_lo must be laid out as out")
    _contig(lse)
    dO = torch.empty(M, D, device=dy.device, dtype=torch.bfloat16)
    delta = torch.empty(3, B, H, T, device=dy.device, dtype=torch.float32)
    N.call("rp_gemm_attn_dout_delta", _p(dy), dy.stride(0), _p(W), W.stride(0), M, K, _p(dO), D, _p(out), _p(out_lo),
           out.stride(0), _p(lse), B, T, H, float(dropout_p), _p(delta), _stream(dy))
    return dO, delta


def attn_delta(out, out_lo, dout, lse, B, T, H, dropout_p=0.0):
    """The attention backward's delta pre-pass alone (rp_attn_bwd_delta): [3, B, H, T] planes
    (delta, -delta / (1 / (1 - p)), -lse log2 e + log2 (1 / (1 - p)))."""
    _gpu(out, out_lo, dout, lse)
    _contig(out, dout, lse)
    delta = torch.empty(3, B, H, T, device=out.device, dtype=torch.float32)
    N.call("rp_attn_bwd_delta", _dt(out), _p(out), _p(out_lo), _p(dout), _p(lse), B, T, H, out.shape[1] // H,
           float(dropout_p), _p(delta), _stream(out))
    return delta


def attn_dout_delta_ok(M, H, K, dtype):
    """Whether the fused dO + delta launch serves a shape (else linear_dgrad + attn_bwd's own pass);
    RP_DOUT_DELTA=0 turns it off (A/B)."""
    if os.environ.get("RP_DOUT_DELTA", "1") == "0":
        return False
    return dtype == torch.bfloat16 and M % 128 == 0 and (H * 64) % 128 == 0 and K % 64 == 0


def attn_bwd(qkv, out, dout, lse, key_valid, B, T, H, scale, dropout_p=0.0, seed=0, dropmask=None,
             q_prescaled=False, out_lo=None, delta=None):
    """-> dqkv.  delta (optional): the [3, B, H, T] planes already formed (attn_dout_delta); the
    backward then skips its own delta pass."""
    _gpu(qkv, out, dout, lse, key_valid, dropmask, delta)
    _contig(qkv, out, dout, lse, key_valid)
    if dropout_p > 0 and dropmask is None:
        raise ValueError("attn_bwd: dropout needs the forward's dropmask")
    dk = qkv.shape[1] // (3 * H)
    dqkv = torch.empty_like(qkv)
    st, dt = _stream(qkv), _adt(qkv, q_prescaled)
    e0 = _tick("attn_bwd")
    timed = {"attn_bwd_dq", "attn_bwd_dkdv", "attn_bwd_roles"} & set(_timer["names"])
    roles = bool(timed) and attn_bwd_uses_roles(qkv, B, T, H, q_prescaled)
    if delta is not None:
        _contig(delta)
        if tuple(delta.shape) != (3, B, H, T) or delta.dtype != torch.float32:
            raise ValueError("attn_bwd: delta must be fp32 [3, B, H, T]")
        if not timed or roles:
            e3 = _tick("attn_bwd_roles") if roles else None
            N.call("rp_attn_bwd_given_delta", dt, _p(qkv), _p(dout), _p(lse), _p(delta), _p(key_valid), B, T, H, dk,
                   float(scale), float(dropout_p), _p(dropmask), _p(dqkv), st)
            _tock(e3)
            _tock(e0)
            return dqkv
        e2 = _tick("attn_bwd_dq")
        N.call("rp_attn_bwd_dq", dt, _p(qkv), _p(dout), _p(lse), _p(delta), _p(key_valid), B, T, H, dk,
               float(scale), float(dropout_p), _p(dropmask), _p(dqkv), st)
        _tock(e2)
        e1 = _tick("attn_bwd_dkdv")
        N.call("rp_attn_bwd_dkdv", dt, _p(qkv), _p(dout), _p(lse), _p(delta), _p(key_valid), B, T, H, dk,
               float(scale), float(dropout_p), _p(dropmask), _p(dqkv), st)
        _tock(e1)
        _tock(e0)
        return dqkv
    delta = torch.empty(3, B, H, T, device=qkv.device, dtype=torch.float32)  # delta + 2 row-constant planes
    if not timed or roles:
        # one entry: the library launches the fused-delta dQ kernel then dK/dV, or, where each grid
        # fills the CUs once but not twice (config 4), the delta pass and ONE two-role launch (timed
        # whole as "attn_bwd_roles": the per-kernel timers must time what the step runs)
        e3 = _tick("attn_bwd_roles") if roles else None
        N.call("rp_attn_bwd", dt, _p(qkv), _p(out), _p(out_lo), _p(dout), _p(lse), _p(key_valid), B, T, H, dk,
               float(scale), float(dropout_p), _p(dropmask), _p(dqkv), _p(delta), st)
        _tock(e3)
        _tock(e0)
        return dqkv
    # per-kernel timing (bench.py roofline): the two kernels of rp_attn_bwd as separate calls — dQ
    # first, with the delta = rowsum(dO * O) pre-pass fused in; dK/dV reads it
    e2 = _tick("attn_bwd_dq")
    N.call("rp_attn_bwd_dq_delta", dt, _p(qkv), _p(out), _p(out_lo), _p(dout), _p(lse), _p(delta), _p(key_valid), B, T,
           H, dk, float(scale), float(dropout_p), _p(dropmask), _p(dqkv), st)
    _tock(e2)
    e1 = _tick("attn_bwd_dkdv")
    N.call("rp_attn_bwd_dkdv", dt, _p(qkv), _p(dout), _p(lse), _p(delta), _p(key_valid), B, T, H, dk,
           float(scale), float(dropout_p), _p(dropmask), _p(dqkv), st)
    _tock(e1)
    _tock(e0)
    return dqkv


def _rows(t, H, dk):
    """(data pointer, row stride) of a [rows, >= H*dk] activation view with unit column stride."""
    if t.dim() != 2 or t.stride(1) != 1 or t.shape[1] < H * dk:
        raise ValueError("mha: operands are [rows, H*dk] views with unit column stride")
    return t.data_ptr(), t.stride(0)


def mha_fwd(q, k, v, key_valid, B, Tq, Tk, H, scale, dropout_p=0.0, seed=0, q_prescaled=False,
            empty_uniform=False, seed_base=None):
    """General (self / cross) attention core.  q [B*Tq, >=H*dk], k/v [B*Tk, >=H*dk] row views (any row
    stride), key_valid [B, Tk] uint8.  -> (out [B*Tq, H*dk], lse [B, H, Tq], dropmask or None)."""
    _gpu(q, k, v, key_valid)
    _contig(key_valid)
    if not (q.dtype == k.dtype == v.dtype):
        raise TypeError("mha_fwd: q, k, v must share a dtype")
    dk = 64
    out = torch.empty(B * Tq, H * dk, device=q.device, dtype=q.dtype)
    lse = torch.empty(B, H, Tq, device=q.device, dtype=torch.float32)
    mask = None
    if dropout_p > 0:
        mask = torch.empty(N.load().rp_mha_dropmask_elems(B, Tq, Tk, H), device=q.device, dtype=torch.int16)
    a = N.MhaArgs()
    a.q, a.ldq = _rows(q, H, dk)
    a.k, a.ldk = _rows(k, H, dk)
    a.v, a.ldv = _rows(v, H, dk)
    a.key_valid = key_valid.data_ptr()
    a.B, a.Tq, a.Tk, a.H, a.head_dim = B, Tq, Tk, H, dk
    a.scale, a.dropout_p, a.seed = float(scale), float(dropout_p), int(seed) & 0xFFFFFFFF
    a.out, a.ldo = out.data_ptr(), out.stride(0)
    a.lse = lse.data_ptr()
    a.dropmask = mask.data_ptr() if mask is not None else None
    a.empty_rows_uniform = int(empty_uniform)
    _seed_word(seed_base)
    a.seed_base = _p(seed_base).value
    N.call("rp_mha_fwd", _adt(q, q_prescaled), ctypes.byref(a), _stream(q))
    return out, lse, mask


def mha_bwd(q, k, v, out, dout, lse, key_valid, B, Tq, Tk, H, scale, dropout_p=0.0, dropmask=None,
            q_prescaled=False, empty_uniform=False):
    """-> (dq [B*Tq, H*dk], dk [B*Tk, H*dk], dv [B*Tk, H*dk]) for mha_fwd's inputs."""
    _gpu(q, k, v, out, dout, lse, key_valid, dropmask)
    _contig(out, dout, lse, key_valid)
    if dropout_p > 0 and dropmask is None:
        raise ValueError("mha_bwd: dropout needs the forward's dropmask")
    dk = 64
    dq = torch.empty(B * Tq, H * dk, device=q.device, dtype=q.dtype)
    dkk = torch.empty(B * Tk, H * dk, device=q.device, dtype=q.dtype)
    dv = torch.empty(B * Tk, H * dk, device=q.device, dtype=q.dtype)
    delta = torch.empty(3, B, H, Tq, device=q.device, dtype=torch.float32)
    a = N.MhaArgs()
    a.q, a.ldq = _rows(q, H, dk)
    a.k, a.ldk = _rows(k, H, dk)
    a.v, a.ldv = _rows(v, H, dk)
    a.key_valid = key_valid.data_ptr()
    a.B, a.Tq, a.Tk, a.H, a.head_dim = B, Tq, Tk, H, dk
    a.scale, a.dropout_p = float(scale), float(dropout_p)
    a.out, a.ldo = out.data_ptr(), out.stride(0)
    a.lse = lse.data_ptr()
    a.dropmask = dropmask.data_ptr() if dropmask is not None else None
    a.dout, a.lddo = dout.data_ptr(), dout.stride(0)
    a.dq, a.lddq = dq.data_ptr(), dq.stride(0)
    a.dk, a.lddk = dkk.data_ptr(), dkk.stride(0)
    a.dv, a.lddv = dv.data_ptr(), dv.stride(0)
    a.delta_ws = delta.data_ptr()
    a.empty_rows_uniform = int(empty_uniform)
    N.call("rp_mha_bwd", _adt(q, q_prescaled), ctypes.byref(a), 7, _stream(q))
    return dq, dkk, dv


# ------------------------------------------------------------------------------------- focal loss
def mha_general_fwd(q, k, v, mask4, B, Tq, Tk, H, dk, scale):
    """General attention core (rp_mha_general_fwd, fp32): q [B*Tq, >= H*dk], k / v [B*Tk, >= H*dk] row
    views, mask4 None or a uint8 view broadcast to [B, H, Tq, Tk] (any strides).  Returns (out
    [B*Tq, H*dk], probs [B, H, Tq, Tk]) — probs is the backward's input."""
    _gpu(q, k, v, mask4)
    for t in (q, k, v):
        if t.dtype != torch.float32 or t.stride(1) != 1:
            raise TypeError("mha_general: fp32 row views with unit column stride")
    out = torch.empty(B * Tq, H * dk, device=q.device, dtype=torch.float32)
    probs = torch.empty(B, H, Tq, Tk, device=q.device, dtype=torch.float32)
    if B * Tq == 0:
        return out, probs
    a = _general_args(q, k, v, mask4, B, Tq, Tk, H, dk, scale, probs)
    a.out, a.ldo = _p(out).value, out.stride(0)
    N.call("rp_mha_general_fwd", ctypes.byref(a), _stream(q))
    return out, probs


def mha_general_bwd(q, k, v, dout, probs, mask4, B, Tq, Tk, H, dk, scale):
    """Backward of mha_general_fwd -> (dq, dk, dv) [rows, H*dk] fp32."""
    _gpu(q, k, v, dout, probs, mask4)
    dev = q.device
    dq = torch.empty(B * Tq, H * dk, device=dev, dtype=torch.float32)
    if B * Tq == 0:  # no queries: dK = dV = 0, as the reference's autograd gives (never uninitialised)
        z = torch.zeros(B * Tk, H * dk, device=dev, dtype=torch.float32)
        return dq, z, z.clone()
    dkk = torch.empty(B * Tk, H * dk, device=dev, dtype=torch.float32)
    dv = torch.empty(B * Tk, H * dk, device=dev, dtype=torch.float32)
    ds = torch.empty_like(probs)
    a = _general_args(q, k, v, mask4, B, Tq, Tk, H, dk, scale, probs)
    a.dout, a.lddo, a.dscores = _p(dout).value, dout.stride(0), _p(ds).value
    a.dq, a.lddq, a.dk, a.lddk, a.dv, a.lddv = _p(dq).value, dq.stride(0), _p(dkk).value, dkk.stride(0), \
        _p(dv).value, dv.stride(0)
    N.call("rp_mha_general_bwd", ctypes.byref(a), _stream(q))
    return dq, dkk, dv


def _general_args(q, k, v, mask4, B, Tq, Tk, H, dk, scale, probs):
    a = N.MhaGeneralArgs(q=_p(q).value, ldq=q.stride(0), k=_p(k).value, ldk=k.stride(0), v=_p(v).value,
                         ldv=v.stride(0), B=B, Tq=Tq, Tk=Tk, H=H, head_dim=dk, scale=float(scale), probs=_p(probs).value)
    if mask4 is not None:
        if mask4.dtype != torch.uint8 or tuple(mask4.shape) != (B, H, Tq, Tk):
            raise ValueError("mha_general: mask4 must be a uint8 view of shape [B, H, Tq, Tk]")
        a.mask = _p(mask4).value
        a.mask_sb, a.mask_sh, a.mask_sq, a.mask_sk = mask4.stride()
    return a


def focal_fwd_sum(x, t, mask=None, alpha=0.7, gamma=2.0):
    """sum_i mask_i * focal(x_i, t_i) on the device: per-chunk partials over many workgroups, then one
    wave sums them in order (rp_focal_fwd_sum_ws; deterministic for a given n)."""
    _gpu(x, t, mask)
    x, t = x.contiguous().float(), t.contiguous().float()
    m = mask.contiguous().view(torch.uint8) if mask is not None else None
    loss = torch.empty((), device=x.device, dtype=torch.float32)
    nw = int(N.load().rp_focal_ws_elems(x.numel()))
    ws = torch.empty(nw, device=x.device, dtype=torch.float32)
    N.call("rp_focal_fwd_sum_ws", _p(x), _p(t), _p(m), x.numel(), float(alpha), float(gamma), _p(ws), nw, _p(loss),
           _stream(x))
    return loss


def focal_elementwise(x, t, alpha=0.7, gamma=2.0):
    _gpu(x, t)
    x, t = x.contiguous().float(), t.contiguous().float()
    out = torch.empty_like(x)
    N.call("rp_focal_elementwise", _p(x), _p(t), x.numel(), float(alpha), float(gamma), _p(out),
           _stream(x))
    return out


def focal_bwd(x, t, mask, grad_out, alpha=0.7, gamma=2.0, per_elem=False):
    _gpu(x, t, mask, grad_out)
    x, t = x.contiguous().float(), t.contiguous().float()
    m = mask.contiguous().view(torch.uint8) if mask is not None else None
    g = grad_out.contiguous().float()
    dx = torch.empty_like(x)
    N.call("rp_focal_bwd", _p(x), _p(t), _p(m), x.numel(), float(alpha), float(gamma), _p(g),
           int(per_elem), _p(dx), _stream(x))
    return dx


# ------------------------------------------------------------------------------------- small heads
def rowdot_fwd(X, W, b=None, relu=False):
    _gpu(X, W, b)
    rows, K = X.shape
    nout = W.shape[0]
    out = torch.empty(rows, nout, device=X.device, dtype=torch.float32)
    N.call("rp_rowdot_fwd", _dt(X), _p(X), X.stride(0), rows, K, _p(W), _p(b), nout, int(relu), _p(out),
           nout, _stream(X))
    return out


def rowdot_bwd_dx(dout, W, gate=None, gate_scale=1.0, out_dtype=torch.float32):
    _gpu(dout, W, gate)
    rows, nout = dout.shape
    K = W.shape[1]
    dX = torch.empty(rows, K, device=dout.device, dtype=out_dtype)
    N.call("rp_rowdot_bwd_dx", _p(dout), dout.stride(0), rows, K, _p(W), nout, _p(gate),
           _dt(gate) if gate is not None else 0, gate.stride(0) if gate is not None else 0,
           float(gate_scale), _p(dX), _DT[out_dtype], K, _stream(dout))
    return dX


# ------------------------------------------------------------------------------------- optimizer
def adam_step(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, p_lp=None, coef_dev=None):
    """One Adam update; with ``coef_dev`` (fp32 device tensor of 6, see ``adam_coefficients``) the
    kernel reads its coefficients from device memory when it runs (graph replay) and the host
    hyper-parameters are not used."""
    _gpu(p, g, m, v, p_lp, coef_dev)
    e0 = _tick("adam")
    if coef_dev is not None:
        N.call("rp_adam_step_dev", _p(p), _p(g), _p(m), _p(v), p.numel(), _p(coef_dev), _p(p_lp), _stream(p))
    else:
        N.call("rp_adam_step", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2),
               float(eps), float(weight_decay), int(step), _p(p_lp), _stream(p))
    _tock(e0)


def adam_coefficients(lr, beta1, beta2, eps, weight_decay, step):
    """The six fp32 kernel coefficients of an Adam step (computed by the library, as rp_adam_step does)."""
    buf = (ctypes.c_float * 6)()
    N.call("rp_adam_coefficients", float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), int(step),
           ctypes.cast(buf, ctypes.c_void_p))
    return list(buf)


def _seed_word(t):
    """Validate an optional graph-replayable dropout base: an int32 device word (see include/rp_api.h,
    "Graph-replayable dropout"); it is passed per launch, the library holds no dropout state."""
    if t is not None:
        _gpu(t)
        if t.dtype not in (torch.int32, torch.uint32) or t.numel() < 1 or t.data_ptr() % 4:
            raise TypeError("seed_base: needs an aligned int32 device word")


# ------------------------------------------------------------------------------------- inference
def infer_select(logits, mask, offsets, thresh, topk, dur_min, dur_max):
    """logits [B, T] fp32, mask [B, T] bool, offsets [B, T, 2] -> (count, idx, score, seg)."""
    _gpu(logits, mask, offsets)
    B, T = logits.shape
    logits = logits.contiguous().float()
    offsets = offsets.contiguous().float()
    m = mask.contiguous().view(torch.uint8)
    dev = logits.device
    count = torch.empty(B, device=dev, dtype=torch.int32)
    idx = torch.empty(B, max(topk, 1), device=dev, dtype=torch.int64)
    score = torch.empty(B, max(topk, 1), device=dev, dtype=torch.float32)
    seg = torch.empty(B, max(topk, 1), 2, device=dev, dtype=torch.float32)
    N.call("rp_infer_select", _p(logits), _p(m), _p(offsets), B, T, float(thresh), int(topk),
           float(dur_min), float(dur_max), _p(count), _p(idx), _p(score), _p(seg), _stream(logits))
    return count, idx, score, seg


def softnms(scores, segs, count, sigma, thresh, max_seg, want_final_scores=False):
    """scores [B, cap], segs [B, cap, 2], count/max_seg int32 [B] -> (keep [B, cap], keep_count)."""
    _gpu(scores, segs, count, max_seg)
    B, cap = scores.shape
    scores, segs = scores.contiguous().float(), segs.contiguous().float()
    count = count.contiguous().to(torch.int32)
    max_seg = max_seg.contiguous().to(torch.int32)
    keep = torch.empty(B, max(cap, 1), device=scores.device, dtype=torch.int32)
    keep_count = torch.empty(B, device=scores.device, dtype=torch.int32)
    final = torch.empty_like(scores) if want_final_scores else None
    nws = N.load().rp_softnms_workspace(B, cap)
    ws = torch.empty(max(nws // 4, 1), device=scores.device, dtype=torch.float32) if nws else None
    N.call("rp_softnms", _p(scores), _p(segs), _p(count), B, cap, float(sigma), float(thresh), _p(max_seg),
           _p(keep), _p(keep_count), _p(final), _p(ws), int(nws), _stream(scores))
    return keep, keep_count, final


# ------------------------------------------------------------------------------------- metric, DIoU
def tiou_hits(pred, pred_count, ref, ref_count, thresholds):
    """pred [V, P, 2] fp32, ref [V, R, 2] fp64, counts [V] int32, thresholds fp64 [n] -> hits [V, n] int32."""
    _gpu(pred, pred_count, ref, ref_count, thresholds)
    _contig(pred, pred_count, ref, ref_count, thresholds)
    V, P = pred.shape[0], pred.shape[1]
    R = ref.shape[1]
    hits = torch.empty(V, thresholds.numel(), device=pred.device, dtype=torch.int32)
    N.call("rp_tiou_hits", _p(pred), _p(pred_count), P, _p(ref), _p(ref_count), R, _p(thresholds),
           thresholds.numel(), V, _p(hits), _stream(pred))
    return hits


def diou_fwd(pred, gt, eps, reduction):
    """pred, gt [n, 2] fp32 contiguous; reduction 0 none / 1 mean / 2 sum."""
    _gpu(pred, gt)
    _contig(pred, gt)
    n = pred.shape[0]
    out = torch.empty(n if reduction == 0 else (), device=pred.device, dtype=torch.float32)
    N.call("rp_diou_fwd", _p(pred), _p(gt), n, float(eps), int(reduction), _p(out), _stream(pred))
    return out


def diou_bwd(pred, gt, eps, grad_out, per_elem, grad_scale, want_pred=True, want_gt=False):
    _gpu(pred, gt, grad_out)
    _contig(pred, gt, grad_out)
    n = pred.shape[0]
    dp = torch.empty_like(pred) if want_pred else None
    dg = torch.empty_like(gt) if want_gt else None
    N.call("rp_diou_bwd", _p(pred), _p(gt), n, float(eps), _p(grad_out), int(per_elem), float(grad_scale),
           _p(dp), _p(dg), _stream(pred))
    return dp, dg
