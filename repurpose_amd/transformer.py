"""Drop-in for the reference's ``models/transformer.py`` on the same HIP kernels.

Same classes, constructor arguments, submodule names (so ``state_dict`` keys and shapes match) and
``torch.manual_seed`` initialisation order as models/transformer.py:6-190:

  PositionalEncoding (:6-21)   seq-first ``pe`` buffer [max_len, 1, d]; ``forward`` adds
                               ``pe[:x.size(0)]`` — on batch-first input that is pe[b] added to every
                               timestep of sample b.  The reference behaves this way and so does this
                               module (preserve the bug).
  MLP (:24-35)                 fc1 -> ReLU -> fc2
  MultiHeadAttention (:37-81)  q/k/v/out projections, ``scale`` buffer = sqrt(d_k); scores
                               QK^T / scale, key mask (mask == 0 -> excluded), softmax, PV, out
  EncoderLayer (:84-102)       pre-LN self attention + FFN, dropout on both residual branches
  CrossAttentionEncoderLayer (:105-130), CrossSelfEncoderLayer (:133-176), UniModalEncoder (:179-190)

Every projection is rp_gemm (bias and, where the residual branch has no dropout, the residual add
fused in the epilogue), every LayerNorm rp_layernorm_fwd/bwd, the attention core rp_mha_fwd/bwd
(independent q/k/v row strides, Tq != Tk for cross attention; q/k/v of one input come from ONE
GEMM into a [rows, 3d] buffer).  Arithmetic is fp32 (exact-f32 MFMA), like the reference.

Masks follow the reference exactly: ``mask.unsqueeze(1)`` broadcast against the scores [B, H, Tq, Tk]
(:69-71; a mask that does not broadcast raises, as masked_fill does), a score is replaced by -1e9 iff
mask == 0.  Two HIP paths:
  * per-key masks (the [B, 1, Tk] padding mask the reference passes, a [B, Tq, Tk] mask whose rows are
    equal, no mask) with head dims d_k <= 64: the flash kernels rp_mha_fwd/bwd (heads below 64 are
    zero-padded to 64 — zero columns add nothing to QK^T, the scale stays 1/sqrt(d_k)); a sequence with
    no valid key averages all values, the -1e9 result (rp_mha empty_rows_uniform);
  * everything else — d_k > 64, masks that differ between queries (causal) or heads (a [B, Tk] mask,
    which the reference's unsqueeze(1) broadcasts as [1, B, 1, Tk], i.e. per HEAD when B == H):
    rp_mha_general_fwd/bwd, the same formula with the probabilities materialised.
Residual-branch dropout (p > 0, training) is torch's nn.Dropout on the branch, as in the reference.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K

_F32 = torch.float32


def _flat(x):
    return x.reshape(-1, x.shape[-1])


# --------------------------------------------------------------------------------- autograd pieces
class _LinearFn(torch.autograd.Function):
    """y = x W^T + b [+ residual] (bias and residual add in the GEMM epilogue)."""

    @staticmethod
    def forward(ctx, x, W, b, residual):
        x2 = _flat(x).contiguous().float()
        M, Kd = x2.shape
        Nn = W.shape[0]
        out = torch.empty(M, Nn, device=x.device, dtype=_F32)
        res = _flat(residual).contiguous().float() if residual is not None else None
        K.gemm(x2, W.detach().contiguous(), out, M, Nn, Kd, Kd, True, Kd, True, Nn,
               bias=b.detach() if b is not None else None, residual=res, ldr=Nn)
        ctx.save_for_backward(x2, W)
        ctx.has_b, ctx.has_res, ctx.shape = b is not None, residual is not None, x.shape
        return out.view(*x.shape[:-1], Nn)

    @staticmethod
    def backward(ctx, dy):
        x2, W = ctx.saved_tensors
        dy2 = _flat(dy).contiguous().float()
        dx = K.linear_dgrad(dy2, W.detach().contiguous(), out_dtype=_F32).view(ctx.shape)
        dW = torch.zeros_like(W, dtype=_F32)
        db = torch.zeros(W.shape[0], device=W.device, dtype=_F32) if ctx.has_b else None
        K.linear_wgrad(dy2, x2, dW, db=db, accumulate=True)
        return dx, dW, db, (dy if ctx.has_res else None)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        x2 = _flat(x).contiguous().float()
        y, _, mean, rstd = K.layernorm_fwd(x2, gamma.detach(), beta.detach(), eps=eps)
        ctx.save_for_backward(x2, mean, rstd, gamma)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, gamma = ctx.saved_tensors
        dg = torch.zeros_like(gamma, dtype=_F32)
        dbt = torch.zeros_like(gamma, dtype=_F32)
        dx, _ = K.layernorm_bwd(_flat(dy).contiguous().float(), x2, mean, rstd, gamma.detach(), dgamma=dg, dbeta=dbt)
        return dx.view(ctx.shape), dg, dbt, None


class _AttentionCoreFn(torch.autograd.Function):
    """softmax(scale * Q K^T + key mask) V on [rows, H*64] row views of q, k, v; a sequence without
    any valid key averages all values (masked_fill(-1e9) semantics)."""

    @staticmethod
    def forward(ctx, q, k, v, kv, B, Tq, Tk, H, scale):
        out, lse, _ = K.mha_fwd(q, k, v, kv, B, Tq, Tk, H, scale, empty_uniform=True)
        ctx.save_for_backward(q, k, v, out, lse, kv)
        ctx.dims = (B, Tq, Tk, H, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse, kv = ctx.saved_tensors
        B, Tq, Tk, H, scale = ctx.dims
        dq, dk, dv = K.mha_bwd(q, k, v, out, dout.contiguous(), lse, kv, B, Tq, Tk, H, scale, empty_uniform=True)
        return dq, dk, dv, None, None, None, None, None, None


def _linear(lin, x, residual=None):
    return _LinearFn.apply(x, lin.weight, lin.bias, residual)


def _layernorm(ln, x):
    return _LayerNormFn.apply(x, ln.weight, ln.bias, float(ln.eps))


def _mask4(mask, B, H, Tq, Tk):
    """The reference's ``mask.unsqueeze(1)`` broadcast to the scores [B, H, Tq, Tk] (models/transformer.py
    :69-71) as a uint8 keep view (strides 0 on broadcast dimensions), or None."""
    if mask is None:
        return None
    m = mask.unsqueeze(1)
    shape = torch.broadcast_shapes(m.shape, (B, H, Tq, Tk))  # raises where masked_fill would
    if tuple(shape) != (B, H, Tq, Tk):
        raise RuntimeError(f"MultiHeadAttention: mask {tuple(mask.shape)} broadcasts the scores ({B}, {H}, {Tq}, "
                           f"{Tk}) to {tuple(shape)}")
    return (m != 0).to(torch.uint8).expand(B, H, Tq, Tk)


def _key_valid(m4, B, Tk, device):
    """[B, Tk] uint8 key mask if the broadcast mask depends only on (batch, key), else None."""
    if m4 is None:
        return torch.ones(B, Tk, device=device, dtype=torch.uint8)
    if m4.stride(1) == 0 and m4.stride(2) == 0:
        return m4[:, 0, 0, :].contiguous()
    if bool((m4 == m4[:, :1, :1, :]).all()):
        return m4[:, 0, 0, :].contiguous()
    return None


class _GeneralAttnFn(torch.autograd.Function):
    """softmax(scale * Q K^T, masked with -1e9) V for any head dim and any broadcast mask
    (rp_mha_general_fwd/bwd)."""

    @staticmethod
    def forward(ctx, q, k, v, m4, B, Tq, Tk, H, dk, scale):
        out, probs = K.mha_general_fwd(q, k, v, m4, B, Tq, Tk, H, dk, scale)
        ctx.save_for_backward(q, k, v, probs)
        ctx.m4 = m4
        ctx.dims = (B, Tq, Tk, H, dk, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, probs = ctx.saved_tensors
        B, Tq, Tk, H, dk, scale = ctx.dims
        dq, dkk, dv = K.mha_general_bwd(q, k, v, dout.contiguous(), probs, ctx.m4, B, Tq, Tk, H, dk, scale)
        return dq, dkk, dv, None, None, None, None, None, None, None


# --------------------------------------------------------------------------------- modules
class PositionalEncoding(nn.Module):
    """models/transformer.py:6-21 (sequence-first table; see the module docstring)."""

    def __init__(self, d_model, max_len=5000):
        super().__init__()
        position = torch.arange(max_len, dtype=torch.float).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        pe = torch.zeros(max_len, d_model)
        pe[:, 0::2] = torch.sin(position * div_term)
        pe[:, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe", pe.unsqueeze(1))

    def forward(self, x):
        return x + self.pe[:x.size(0)]


class MLP(nn.Module):
    """models/transformer.py:24-35."""

    def __init__(self, input_dim, hidden_dim, output_dim):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, hidden_dim)
        self.relu = nn.ReLU()
        self.fc2 = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        h = _LinearReluFn.apply(x, self.fc1.weight, self.fc1.bias)
        return _linear(self.fc2, h)


class _LinearReluFn(torch.autograd.Function):
    """relu(x W^T + b) with the bias and ReLU in the GEMM epilogue."""

    @staticmethod
    def forward(ctx, x, W, b):
        x2 = _flat(x).contiguous().float()
        y = K.linear_fwd(x2, W.detach().contiguous(), b.detach(), out_dtype=_F32, relu=True)
        ctx.save_for_backward(x2, W, y)
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, W, y = ctx.saved_tensors
        dz = _flat(dy).contiguous().float() * (y > 0)
        dx = K.linear_dgrad(dz, W.detach().contiguous(), out_dtype=_F32).view(ctx.shape)
        dW = torch.zeros_like(W, dtype=_F32)
        db = torch.zeros(W.shape[0], device=W.device, dtype=_F32)
        K.linear_wgrad(dz, x2, dW, db=db, accumulate=True)
        return dx, dW, db


class MultiHeadAttention(nn.Module):
    """models/transformer.py:37-81 with the score/softmax/PV core in rp_mha_fwd/bwd."""

    def __init__(self, d_model, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.d_model = d_model
        self.d_k = d_model // num_heads
        if self.d_k * num_heads != d_model:
            raise ValueError(f"MultiHeadAttention: d_model {d_model} is not divisible by {num_heads} heads "
                             "(the reference's view(bs, -1, num_heads, d_k) needs it)")
        self.q_linear = nn.Linear(d_model, d_model)
        self.k_linear = nn.Linear(d_model, d_model)
        self.v_linear = nn.Linear(d_model, d_model)
        self.out = nn.Linear(d_model, d_model)
        self.register_buffer("scale", torch.sqrt(torch.FloatTensor([self.d_k])))
        self._inv_scale = 1.0 / math.sqrt(self.d_k)  # host copy of 1/scale (no device sync per call)

    def _project(self, x, lins):
        """One GEMM for all projections of the same input: rows of [q | k | v] (views)."""
        W = torch.cat([l.weight for l in lins], 0)
        b = torch.cat([l.bias for l in lins], 0)
        y = _LinearFn.apply(x, W, b, None)
        y2 = y.reshape(-1, y.shape[-1])
        d = self.d_model
        return [y2[:, j * d:(j + 1) * d] for j in range(len(lins))]

    def forward(self, q, k, v, mask=None, residual=None):
        B, Tq, Tk = q.size(0), q.size(1), k.size(1)
        if q is k and k is v:
            qp, kp, vp = self._project(q, [self.q_linear, self.k_linear, self.v_linear])
        elif k is v:
            (qp,) = self._project(q, [self.q_linear])
            kp, vp = self._project(k, [self.k_linear, self.v_linear])
        else:
            (qp,) = self._project(q, [self.q_linear])
            (kp,) = self._project(k, [self.k_linear])
            (vp,) = self._project(v, [self.v_linear])
        H, dk = self.num_heads, self.d_k
        m4 = _mask4(mask, B, H, Tq, Tk)
        kv = _key_valid(m4, B, Tk, q.device) if dk <= 64 else None
        if kv is None:  # head dims above 64 or masks varying per query / head: the general core
            att = _GeneralAttnFn.apply(qp, kp, vp, m4, B, Tq, Tk, H, dk, self._inv_scale)
            return _linear(self.out, att.reshape(B, Tq, self.d_model), residual=residual)
        if dk < 64:  # zero-pad every head to the kernels' 64 columns
            qp, kp, vp = (F.pad(t.reshape(t.shape[0], H, dk), (0, 64 - dk)).reshape(t.shape[0], H * 64)
                          for t in (qp, kp, vp))
        att = _AttentionCoreFn.apply(qp, kp, vp, kv, B, Tq, Tk, H, self._inv_scale)
        if dk < 64:
            att = att.view(-1, H, 64)[:, :, :dk].reshape(-1, H * dk)
        return _linear(self.out, att.reshape(B, Tq, self.d_model), residual=residual)


def _attend_residual(attn, x, q, k, v, mask, drop):
    """x + dropout(attn(q, k, v, mask)): the residual add fused into the out-projection epilogue
    when the branch has no dropout."""
    if drop.p == 0.0 or not drop.training:
        return attn(q, k, v, mask, residual=x)
    a = attn(q, k, v, mask)
    return x + drop(a)


def _ffn_residual(ff, x, h, drop, inner_drop=None):
    """x + dropout(ff(h)) for ff = Sequential(Linear, ReLU, [Dropout,] Linear)."""
    lin1, lin2 = ff[0], ff[-1]
    z = _LinearReluFn.apply(h, lin1.weight, lin1.bias)
    if inner_drop is not None and inner_drop.p > 0 and inner_drop.training:
        z = inner_drop(z)
    if drop.p == 0.0 or not drop.training:
        return _linear(lin2, z, residual=x)
    return x + drop(_linear(lin2, z))


class EncoderLayer(nn.Module):
    """models/transformer.py:84-102 (pre-LN)."""

    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.ff = nn.Sequential(nn.Linear(d_model, d_ff), nn.ReLU(), nn.Linear(d_ff, d_model))
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, mask):
        x2 = _layernorm(self.norm_1, x)
        x = _attend_residual(self.attention, x, x2, x2, x2, mask, self.dropout_1)
        x2 = _layernorm(self.norm_2, x)
        return _ffn_residual(self.ff, x, x2, self.dropout_2)


class CrossAttentionEncoderLayer(nn.Module):
    """models/transformer.py:105-130: queries from x, keys/values from ``context``."""

    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.cross_attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.ff = nn.Sequential(nn.Linear(d_model, d_ff), nn.ReLU(), nn.Linear(d_ff, d_model))
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, context, mask=None):
        x2 = _layernorm(self.norm_1, x)
        x = _attend_residual(self.cross_attention, x, x2, context, context, mask, self.dropout_1)
        x2 = _layernorm(self.norm_2, x)
        return _ffn_residual(self.ff, x, x2, self.dropout_2)


class CrossSelfEncoderLayer(nn.Module):
    """models/transformer.py:133-176 (self attention -> cross attention -> FFN; LN before each;
    note the reference's residuals: the cross-attention and FFN residuals add to the NORMALISED
    input, and dropout_2 serves both of them)."""

    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.self_attention = MultiHeadAttention(d_model, num_heads)
        self.cross_attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.norm_3 = nn.LayerNorm(d_model)
        self.ff = nn.Sequential(nn.Linear(d_model, d_ff), nn.ReLU(), nn.Dropout(dropout), nn.Linear(d_ff, d_model))
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, context, mask=None):
        h = _layernorm(self.norm_1, x)
        x = _attend_residual(self.self_attention, x, h, h, h, mask, self.dropout_1)
        x = _layernorm(self.norm_2, x)
        x = _attend_residual(self.cross_attention, x, x, context, context, mask, self.dropout_2)
        x = _layernorm(self.norm_3, x)
        return _ffn_residual(self.ff, x, x, self.dropout_2, inner_drop=self.ff[2])


class UniModalEncoder(nn.Module):
    """models/transformer.py:179-190: MLP -> positional encoding (seq-first quirk) -> layers."""

    def __init__(self, input_dim, d_model, num_layers, num_heads, d_ff=2048):
        super().__init__()
        self.mlp = MLP(input_dim, d_ff, d_model)
        self.positional_encoding = PositionalEncoding(d_model)
        self.layers = nn.ModuleList([EncoderLayer(d_model, num_heads, d_ff) for _ in range(num_layers)])

    def forward(self, x, mask=None):
        x = self.mlp(x)
        x = self.positional_encoding(x)
        for layer in self.layers:
            x = layer(x, mask)
        return x
