"""Drop-in ``MMCTransformer`` whose forward, backward and inference run on hand-written HIP
kernels for MI355X (reference: ``models/MMCTransformer.py``).

Same constructor signature (``:26``), same ``forward(batch) -> 6-tuple`` (``:109-151``), same
``losses`` (``:159-179``), ``inference_single_video`` (``:181-229``), ``inference_`` (``:231-275``),
``device`` property (``:153-157``) and an identical ``state_dict`` (keys, shapes, the persistent
``positional_encoding.pe`` buffer), so reference checkpoints load unchanged and vice versa.
Initialisation consumes the torch RNG in the reference's order, so ``torch.manual_seed`` gives the
reference's initial weights bit for bit (tests/test_model_host.py).

Execution model (MI355X-first, not a port of the nn.Module graph):

* parameters live in ONE flat fp32 buffer (named ``nn.Parameter`` views into it), gradients in one
  flat fp32 buffer: gradient all-reduce is a handful of large RCCL calls over contiguous buckets,
  Adam is one kernel, the bf16 operand copy of the weights is one cast kernel;
* the whole model (16 encoder layers + heads) is ONE ``torch.autograd.Function``: the forward
  schedule saves exactly the tensors the hand-written backward needs; dropout masks are never
  stored (regenerated from a counter hash in the backward kernels);
* ``compute_dtype='bf16'`` keeps the residual stream, LayerNorm statistics, softmax and every
  accumulator in fp32 and feeds bf16 operands to MFMA; ``'fp32'`` (default, the reference's
  precision) runs exact-f32 MFMA for the 1e-3 parity gate.

There is no CPU execution path: forward on CPU tensors raises ``RuntimeError``.  The module can
be constructed on CPU (as ``main.py:139`` does) and moved with ``.to(device)``.
"""
import copy
import math
import os
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _native
from . import kernels as K
from .losses import focal_loss_masked_sum
from .softnms import soft_nms_intervals_cpu  # noqa: F401  (re-exported, reference import site)

_F32 = torch.float32
_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
           "bfloat16": torch.bfloat16}

# Parameter -> owning model (weak), so FusedAdam(model.parameters()) finds the flat buffers
_OWNERS = weakref.WeakValueDictionary()


def owner_of(param):
    """The MMCTransformer that ``param`` belongs to, or None."""
    m = _OWNERS.get(id(param))
    if m is not None and any(q is param for q in m.parameters()):
        return m
    return None


class PositionalEncoding(nn.Module):
    """Holds the persistent ``pe`` buffer [1, max_len, d] (reference ``:9-22``).  The add itself is
    fused into the input LayerNorm kernel (rp_layernorm_fwd, pe_period = T)."""

    def __init__(self, d_model, max_len=5000):
        super().__init__()
        pos = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
        freq = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        table = torch.zeros(max_len, d_model)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", table.unsqueeze(0))


class _SelfAttention(nn.Module):
    """Parameter container with ``nn.MultiheadAttention``'s key names and init order."""

    def __init__(self, d_model):
        super().__init__()
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d_model, d_model))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d_model))
        self.out_proj = nn.Linear(d_model, d_model)  # default init consumes the RNG first
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.constant_(self.in_proj_bias, 0.0)
        nn.init.constant_(self.out_proj.bias, 0.0)


class _EncoderLayer(nn.Module):
    """Parameter container with ``nn.TransformerEncoderLayer``'s key names and init order."""

    def __init__(self, d_model, d_ff):
        super().__init__()
        self.self_attn = _SelfAttention(d_model)
        self.linear1 = nn.Linear(d_model, d_ff)
        self.linear2 = nn.Linear(d_ff, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)


class _Encoder(nn.Module):
    def __init__(self, layer, num_layers):
        super().__init__()
        # deep copies of one prototype, like nn.TransformerEncoder's _get_clones
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(num_layers)])


def _head(d_model, hidden, n_out, final_relu):
    mods = [nn.LayerNorm(d_model), nn.Linear(d_model, hidden), nn.ReLU(), nn.Dropout(0.1),
            nn.Linear(hidden, hidden), nn.ReLU(), nn.Dropout(0.1), nn.Linear(hidden, n_out)]
    if final_relu:
        mods.append(nn.ReLU())
    return nn.Sequential(*mods)


class MMCTransformer(nn.Module):
    DROPOUT = 0.1

    def __init__(self, vis_dim, aud_dim, text_dim, d_model, self_num_layers, text_num_layers,
                 cross_num_layers, num_heads, d_ff=2048, compute_dtype=None):
        super().__init__()
        self.vis_dim, self.aud_dim, self.text_dim = vis_dim, aud_dim, text_dim
        self.d_model, self.num_heads, self.num_layers, self.d_ff = d_model, num_heads, self_num_layers, d_ff
        # text_num_layers / cross_num_layers are accepted and unused, as in the reference (:26)
        self.input_projection = nn.Linear(vis_dim + aud_dim + text_dim, d_model)
        self.input_norm = nn.LayerNorm(d_model)
        self.positional_encoding = PositionalEncoding(d_model)
        self.multimodal_encoder = _Encoder(_EncoderLayer(d_model, d_ff), self_num_layers)
        self.encoder_norm = nn.LayerNorm(d_model)
        self.feature_map = nn.Sequential(nn.Linear(d_model, d_model), nn.LayerNorm(d_model), nn.ReLU(),
                                         nn.Dropout(0.1))
        self.cls_head = _head(d_model, 256, 1, final_relu=False)
        self.reg_head = _head(d_model, 256, 2, final_relu=True)
        self._init_weights()
        dt = compute_dtype or os.environ.get("REPURPOSE_AMD_DTYPE", "fp32")
        self.compute_dtype = _DTYPES[dt] if isinstance(dt, str) else dt
        self._flat = None
        self._gflat = None
        self._lp = None
        self._lp_version = None
        self._layout = None
        self._grad_ready_hooks = []   # called with (lo, hi) flat ranges whose gradients are final
        self._grad_done_hooks = []    # called once at the end of backward
        # set by CapturedTrainStep in place of zero_grad(): the next backward WRITES every trained
        # gradient (each has exactly one producer) instead of accumulating into a zeroed buffer
        self._grad_fresh = False
        self._seed_base = None        # int32 device word while a step is captured (graph.py), else None
        self._build_flat()
        for p in self.parameters():
            _OWNERS[id(p)] = self

    # ---------------------------------------------------------------- init / storage -----------
    def _init_weights(self):
        """Reference ``_init_weights`` (``:98-107``)."""
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.LayerNorm):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _ordered_params(self):
        named = list(self.named_parameters())
        live = [(n, p) for n, p in named if not n.startswith("reg_head.")]
        frozen = [(n, p) for n, p in named if n.startswith("reg_head.")]
        return live + frozen

    def _build_flat(self, device=None):
        """(Re)pack every parameter into one flat fp32 buffer and rebind the Parameters as views.
        reg_head (never trained by the reference: no loss reaches it) sits at the end so the
        trainable range is contiguous."""
        params = self._ordered_params()
        device = device or params[0][1].device
        total = sum(p.numel() for _, p in params)
        # align every tensor to 8 elements: 16-byte aligned in the fp32 master AND the bf16 copy
        layout, off = {}, 0
        for n, p in params:
            layout[n] = (off, tuple(p.shape))
            off += (p.numel() + 7) // 8 * 8
        flat = torch.zeros(off, device=device, dtype=_F32)
        with torch.no_grad():
            for n, p in params:
                o, shp = layout[n]
                flat[o:o + p.numel()].copy_(p.detach().reshape(-1).to(device=device, dtype=_F32))
        for n, p in params:
            o, shp = layout[n]
            p.data = flat[o:o + p.numel()].view(shp)
        self._flat = flat
        # host-side parameter table (the per-step checks walk this list, not named_parameters():
        # the module-tree walk costs ~0.6 ms per call at L = 16, several calls per step)
        self._ptable = [(n, p, layout[n][0]) for n, p in params]
        self._plist = [p for n, p in self.named_parameters()]
        self._trained_params = [p for n, p, _ in self._ptable if not n.startswith("reg_head.")]
        self._flat_dirty = False
        self._bound_grads = None
        self._layout = layout
        self._trainable = layout[next(n for n, _ in params if n.startswith("reg_head."))][0] \
            if any(n.startswith("reg_head.") for n, _ in params) else off
        self._names = [n for n, _ in params]
        self._gflat = None
        self._lp = None
        self._lp_version = None
        assert total <= off

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cuda() / .float() rebind every Parameter's storage: repack on the next use
        out = super()._apply(fn, *args, **kwargs)
        self._flat_dirty = True
        return out

    def _flat_ok(self):
        f = self._flat
        if f is None or self._flat_dirty:
            if f is None or not self._flat_walk_ok():
                return False
            self._flat_dirty = False
            return True
        # fast path: the table's first and last Parameters still view the flat buffer (catches a
        # direct ``p.data = ...`` on them; module conversions go through _apply above)
        base = f.data_ptr()
        for n, p, o in (self._ptable[0], self._ptable[-1]):
            if p.data_ptr() != base + 4 * o:
                return False
        return True

    def _flat_walk_ok(self):
        f = self._flat
        base = f.data_ptr()
        for n, p in self.named_parameters():
            o, _ = self._layout[n]
            if p.data_ptr() != base + 4 * o or p.device != f.device or p.dtype != _F32:
                return False
        return True

    def flat_params(self):
        if not self._flat_ok():
            self._build_flat(next(self.parameters()).device)
        return self._flat

    def flat_grads(self):
        """Flat fp32 gradient buffer; the Parameters' ``.grad`` are views into it."""
        f = self.flat_params()
        if self._gflat is None or self._gflat.device != f.device or self._gflat.numel() != f.numel():
            self._gflat = torch.zeros_like(f)
        return self._gflat

    def _bind_grads(self):
        """Make every trained Parameter's .grad a view of the flat gradient buffer.  If the trainer
        set grads to None (optimizer.zero_grad()), the buffer is zeroed first (grad semantics)."""
        g = self.flat_grads()
        bound = self._bound_grads
        rebind = bound is None or bound[0] is not g or any(
            p.grad is not v for p, v in zip(self._trained_params, bound[1]))
        if rebind:
            g.zero_()
            views = []
            for n, p, o in self._ptable:
                if n.startswith("reg_head."):
                    continue
                p.grad = g[o:o + p.numel()].view(p.shape)
                views.append(p.grad)
            self._bound_grads = (g, views)
        return g

    def trainable_numel(self):
        return self._trainable

    def flat_range(self, prefixes):
        """[lo, hi) of the flat buffer covering every parameter whose name starts with a prefix."""
        lo, hi = None, None
        for n in self._names:
            if any(n.startswith(p) for p in prefixes):
                o, shp = self._layout[n]
                e = o + (int(np.prod(shp)) + 7) // 8 * 8  # include the alignment pad: ranges tile
                lo = o if lo is None else min(lo, o)
                hi = e if hi is None else max(hi, e)
        return lo, hi

    def _grads_ready(self, prefixes):
        if self._grad_ready_hooks:
            lo, hi = self.flat_range(prefixes)
            for h in self._grad_ready_hooks:
                h(lo, hi)

    def _master_version(self):
        """Version key of the fp32 master.  ``_build_flat`` rebinds every Parameter with
        ``p.data = view``, which gives the Parameter a version counter of its own: in-place updates
        through the Parameters (torch.optim.Adam, ``load_state_dict``'s copy_) bump only those, writes
        through the flat buffer bump only ``flat._version`` — the key covers both."""
        return (self._flat._version,) + tuple(p._version for p in self._plist)

    def lowp_weights(self):
        """bf16 operand copy of the flat weights, refreshed when the fp32 master changed."""
        f = self.flat_params()
        if self._lp is None or self._lp.device != f.device:
            self._lp = torch.empty(f.numel(), device=f.device, dtype=torch.bfloat16)
            self._lp_version = None
        key = self._master_version()
        if self._lp_version != key:
            K.cast_bf16(f, self._lp)
            self._lp_version = key
        return self._lp

    def mark_lowp_fresh(self):
        """Called by FusedAdam after its kernel rewrote both the fp32 master and the bf16 copy
        through raw pointers (no version counter moves)."""
        self._lp_version = self._master_version()

    @property
    def device(self):
        if self._flat is not None and self._flat_ok():
            return self._flat.device
        return list(set(p.device for p in self.parameters()))[0]

    # ---------------------------------------------------------------- forward -------------------
    def forward(self, batch):
        v, a, t = batch["visual_feats"], batch["audio_feats"], batch["text_feats"]
        masks = batch["masks"]
        if not v.is_cuda:
            raise RuntimeError("repurpose_amd.MMCTransformer: forward needs the model and batch on a ROCm "
                               "device (HIP kernels only; there is no CPU path)")
        flat = self.flat_params()
        if flat.device != v.device:
            raise RuntimeError(f"model on {flat.device}, batch on {v.device}")
        run = _Schedule(self, v, a, t, masks, train=self.training)
        params = self._trained_params
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            logits, offsets, feats = _ModelFunction.apply(run, *params)
        else:
            logits, offsets, feats = run.forward(save=False)
        return masks, logits, offsets, batch["labels"], batch["segments"], feats

    def losses(self, masks, out_cls_logits, out_offsets, gt_cls_labels, gt_offsets, feats):
        """Reference ``:159-179``: sum over frames of mask * sigmoid_focal_loss (alpha .7, gamma 2)."""
        return {"cls_loss": focal_loss_masked_sum(out_cls_logits, gt_cls_labels, masks)}

    # ---------------------------------------------------------------- inference -----------------
    @torch.no_grad()
    def inference_single_video(self, masks, out_cls_logits, out_offsets, inference_settings):
        """Reference ``:181-229`` on one video (GPU rp_infer_select)."""
        cfg = inference_settings
        T = out_cls_logits.numel()
        logit = out_cls_logits.reshape(1, T).float()
        mask = (masks.reshape(1, T) != 0)
        off = out_offsets.reshape(1, T, 2)
        count, idx, score, seg = K.infer_select(logit, mask, off, cfg["pre_nms_thresh"], cfg["pre_nms_topk"],
                                                cfg["duration_thresh"], cfg["duration_thresh_max"])
        n = int(count[0].item())
        return {"segments": seg[0, :n], "scores": score[0, :n], "labels": idx[0, :n]}

    @torch.no_grad()
    def inference_(self, batch, inference_settings):
        """Reference ``:231-275``: forward, then per-video selection + Soft-NMS — here one batched
        launch each (rp_infer_select, rp_softnms) and a single device->host copy of the counts.

        Length buckets: a batch padded to its longest video (the collate of ``main.py`` / config 5)
        runs as up to four sub-batches of similar valid length, each cut to its own longest video
        (``RP_INFER_BUCKETS``, default 4; 1 = one padded forward).  Every video's valid frames see the
        same computation either way (row-wise GEMMs / LayerNorm, key-padding-masked attention, the
        positional table indexed by the frame), so the proposals are those of the padded forward;
        the padded frames' work is what is skipped."""
        cfg = inference_settings
        out = [None] * batch["visual_feats"].shape[0]
        for rows, tg in self._length_groups(batch["masks"]):
            sub = batch if rows is None else _sub_batch(batch, rows, tg)
            res = self._infer_batch(sub, cfg)
            for j, b in enumerate(rows if rows is not None else range(len(out))):
                out[b] = res[j]
        return out

    def _length_groups(self, masks):
        """[(row indices or None for the whole batch, padded length)] of the inference buckets."""
        B = masks.shape[0]
        T = masks.shape[-1]
        nb = int(os.environ.get("RP_INFER_BUCKETS", "4"))
        if nb <= 1 or B < 2 * nb:
            return [(None, T)]
        mk = masks.reshape(B, T) != 0
        pos = torch.arange(1, T + 1, device=mk.device)
        lens = (mk * pos).amax(1).cpu().tolist()  # last valid frame + 1 (0: no valid frame)
        if min(lens) * 10 >= T * 9:
            return [(None, T)]
        order = sorted(range(B), key=lambda b: lens[b])
        groups = []
        for g in range(nb):
            rows = order[g * B // nb:(g + 1) * B // nb]
            tg = min(T, max(16, (max(lens[b] for b in rows) + 15) // 16 * 16))
            groups.append((rows, tg))
        return groups

    def _infer_batch(self, batch, cfg):
        masks, logits, offsets, _, _, _ = self.forward(batch)
        B, T = logits.shape[0], logits.shape[1]
        lg = logits.reshape(B, T)
        mk = masks.reshape(B, T) != 0
        count, idx, score, seg = K.infer_select(lg, mk, offsets, cfg["pre_nms_thresh"], cfg["pre_nms_topk"],
                                                cfg["duration_thresh"], cfg["duration_thresh_max"])
        ms = [int(np.ceil((int(vlen) // 60) * cfg["max_seg_per_min"])) for vlen in batch["duration"]]
        max_seg = torch.tensor(ms, dtype=torch.int32).to(lg.device, non_blocking=True)
        keep, keep_count, _ = K.softnms(score, seg, count, cfg["nms_sigma"], cfg["min_score"], max_seg)
        kc = keep_count.cpu().tolist()
        out = []
        for b, (vid, vlen) in enumerate(zip(batch["video_id"], batch["duration"])):
            sel = keep[b, :kc[b]].long()
            out.append({"segments": seg[b].index_select(0, sel), "scores": score[b].index_select(0, sel),
                        "labels": idx[b].index_select(0, sel), "video_id": vid, "duration": vlen})
        return out


def _mask_u8(masks, B, T):
    """[B, T] uint8 key-valid bytes of a [B, 1, T] mask: a zero-copy view of a contiguous bool mask
    (torch stores bool as 0 / 1 bytes), otherwise one conversion."""
    if masks.dtype == torch.bool and masks.is_contiguous():
        return masks.reshape(B, T).view(torch.uint8)
    return (masks.reshape(B, T) != 0).to(torch.uint8).contiguous()


def _sub_batch(batch, rows, tg):
    """Rows ``rows`` of a padded batch, its frame axis cut to ``tg``: tensors whose first dim is the
    batch are row-selected (and cut on the axis that has the padded length), lists are picked."""
    B = batch["visual_feats"].shape[0]
    T = batch["visual_feats"].shape[1]
    out = {}
    for k, v in batch.items():
        if torch.is_tensor(v) and v.dim() >= 1 and v.shape[0] == B:
            v = v.index_select(0, torch.tensor(rows, device=v.device))
            if v.dim() >= 2 and v.shape[1] == T:
                v = v[:, :tg]
            elif v.dim() >= 3 and v.shape[2] == T:
                v = v[:, :, :tg]
            out[k] = v.contiguous()
        elif isinstance(v, (list, tuple)) and len(v) == B:
            out[k] = [v[b] for b in rows]
        else:
            out[k] = v
    return out


def _mix(base, site):
    x = (base * 0x9E3779B1 + site * 0x85EBCA77 + 0x165667B1) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x2C1B3C6D) & 0xFFFFFFFF
    x ^= x >> 12
    return x


class _Schedule:
    """Kernel schedule of one forward (and its backward) — the hot path."""

    def __init__(self, model, v, a, t, masks, train):
        self.m = model
        self.v, self.a, self.t = v, a, t
        self.B, self.T = v.shape[0], v.shape[1]
        self.M = self.B * self.T
        self.masks = masks
        self.train = train
        self.p = model.DROPOUT if train else 0.0
        self.scale_drop = 1.0 / (1.0 - self.p) if self.p > 0 else 1.0
        self.dt = model.compute_dtype
        self.base_seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if train else 0
        # graph capture (graph.py): the model's device seed word, passed to every dropout launch
        self.sb = model._seed_base
        self.saved = None
        # bf16 at d_model 512: GEMM + LayerNorm seams as single launches (rp_gemm_ln_*).  On 128 x 128 (or
        # 64 x 128) tiles whose four column tiles exchange the row statistics (kernels._lnx_ws); with
        # RP_GEMM_LNX=0 the 64 x 512 full-row kernels (bitwise the unfused pairs, but streaming the whole
        # weight per 64 rows at one workgroup per CU: +0.17 ms per step at the bench shape).  RP_GEMM_LN:
        # auto (default: the exchange kernels where their grid gives every CU a workgroup — bench shape
        # 14.93 -> 14.39 ms per step, config 2 7.40 -> 7.10 ms, config 4 on 64-row tiles, DESIGN.md §8
        # round 5), 1 both directions, fwd / bwd one, 0 none
        ln = os.environ.get("RP_GEMM_LN", "auto")
        ok = self.dt == torch.bfloat16 and self.M % 64 == 0 and model.d_model == 512
        if ln == "auto":
            dev = model._flat.device
            cus = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 0
            ln = "1" if (self.M % 64 == 0 and cus > 0 and (self.M // 64) * 4 >= cus
                         and os.environ.get("RP_GEMM_LNX", "1") == "1") else "0"
        self.fused_ln_fwd = ok and ln in ("1", "fwd")
        self.fused_ln = ok and ln in ("1", "bwd")

    # ---- parameter access ----
    def P(self, name):  # fp32 master tensor
        o, shp = self.m._layout[name]
        n = int(np.prod(shp))
        return self.m._flat[o:o + n].view(shp)

    def W(self, name):  # GEMM operand (compute dtype)
        if self.dt == _F32:
            return self.P(name)
        o, shp = self.m._layout[name]
        n = int(np.prod(shp))
        return self._lp[o:o + n].view(shp)

    def G(self, name):
        o, shp = self.m._layout[name]
        n = int(np.prod(shp))
        return self._g[o:o + n].view(shp)

    def seed(self, site):
        if not self.train:
            return 0
        # graph-replayable mode (graph.py): the kernels mix the site with the device base word
        return site if self.sb is not None else _mix(self.base_seed, site)

    # ---- forward ----
    def forward(self, save):
        m, B, T, M, dt, p = self.m, self.B, self.T, self.M, self.dt, self.p
        H, L = m.num_heads, m.num_layers
        d = m.d_model
        if T > m.positional_encoding.pe.shape[1]:
            raise ValueError(f"sequence length {T} exceeds the positional table "
                             f"({m.positional_encoding.pe.shape[1]})")
        self._lp = m.lowp_weights() if dt != _F32 else None
        kv = _mask_u8(self.masks, B, T)
        self.kv = kv
        scale = 1.0 / math.sqrt(d // H)
        self.scale = scale
        xin = K.concat_rows(self.v, self.a, self.t, dt)
        proj = K.linear_fwd(xin, self.W("input_projection.weight"), self.P("input_projection.bias"), out_dtype=_F32)
        pe = m.positional_encoding.pe
        if pe.device != xin.device:
            raise RuntimeError("positional_encoding.pe is not on the model device")
        x, _, mu0, rs0 = K.layernorm_fwd(proj, self.P("input_norm.weight"), self.P("input_norm.bias"),
                                         pe=pe, pe_period=T, save_stats=save)
        layers = []
        # bf16 at d_model 512: every "Linear + residual -> LayerNorm" seam is one rp_gemm_ln_fwd launch
        # (out_proj -> norm2, linear2 -> the next norm1 / encoder_norm), bitwise the unfused pair
        fused = self.fused_ln_fwd
        _, h1, mu1, rs1 = K.layernorm_fwd(x, self.P("multimodal_encoder.layers.0.norm1.weight"),
                                          self.P("multimodal_encoder.layers.0.norm1.bias"),
                                          out_f32=False, lp_dtype=dt, save_stats=save)
        for l in range(L):
            pre = f"multimodal_encoder.layers.{l}."
            # the Q columns leave the GEMM as Q * scale * log2(e) (rounded once, read by the attention
            # forward and both backward kernels: the backward recomputes the forward's exact scores)
            qkv = K.linear_fwd(h1, self.W(pre + "self_attn.in_proj_weight"), self.P(pre + "self_attn.in_proj_bias"),
                               col_scale_n=d, col_scale=scale * K.LOG2E)
            # bf16 training: the output's rounding residual too, so the backward's rowsum(dO * O) is
            # that of the unrounded output
            olo = torch.empty(M, d, device=qkv.device, dtype=dt) if (save and dt != _F32) else None
            o, lse, dmask = K.attn_fwd(qkv, kv, B, T, H, scale, p, self.seed(100 + 4 * l), seed_base=self.sb, q_prescaled=True,
                                       out_lo=olo)
            nxt = f"multimodal_encoder.layers.{l + 1}.norm1." if l + 1 < L else "encoder_norm."
            if fused:
                x1, h2, mu2, rs2 = K.linear_ln_fwd(o, self.W(pre + "self_attn.out_proj.weight"),
                                                   self.P(pre + "self_attn.out_proj.bias"), x,
                                                   self.P(pre + "norm2.weight"), self.P(pre + "norm2.bias"),
                                                   dropout_p=p, seed=self.seed(101 + 4 * l), seed_base=self.sb)
            else:
                x1 = K.linear_fwd(o, self.W(pre + "self_attn.out_proj.weight"), self.P(pre + "self_attn.out_proj.bias"),
                                  out_dtype=_F32, dropout_p=p, seed=self.seed(101 + 4 * l), seed_base=self.sb, residual=x)
                _, h2, mu2, rs2 = K.layernorm_fwd(x1, self.P(pre + "norm2.weight"), self.P(pre + "norm2.bias"),
                                                  out_f32=False, lp_dtype=dt, save_stats=save)
            f = K.linear_fwd(h2, self.W(pre + "linear1.weight"), self.P(pre + "linear1.bias"), relu=True,
                             dropout_p=p, seed=self.seed(102 + 4 * l), seed_base=self.sb)
            if fused:
                x2, hn, mun, rsn = K.linear_ln_fwd(f, self.W(pre + "linear2.weight"), self.P(pre + "linear2.bias"), x1,
                                                   self.P(nxt + "weight"), self.P(nxt + "bias"), dropout_p=p,
                                                   seed=self.seed(103 + 4 * l), seed_base=self.sb)
            else:
                x2 = K.linear_fwd(f, self.W(pre + "linear2.weight"), self.P(pre + "linear2.bias"), out_dtype=_F32,
                                  dropout_p=p, seed=self.seed(103 + 4 * l), seed_base=self.sb, residual=x1)
                _, hn, mun, rsn = K.layernorm_fwd(x2, self.P(nxt + "weight"), self.P(nxt + "bias"),
                                                  out_f32=False, lp_dtype=dt, save_stats=save)
            if save:
                layers.append((x, h1, mu1, rs1, qkv, o, olo, lse, dmask, x1, h2, mu2, rs2, f))
            x = x2
            h1, mu1, rs1 = hn, mun, rsn
        e, muE, rsE = h1, mu1, rs1  # the last seam normalised with encoder_norm
        z = K.linear_fwd(e, self.W("feature_map.0.weight"), self.P("feature_map.0.bias"), out_dtype=_F32)
        feats, _, muF, rsF = K.layernorm_fwd(z, self.P("feature_map.1.weight"), self.P("feature_map.1.bias"),
                                             relu=True, dropout_p=p, seed=self.seed(1), seed_base=self.sb, save_stats=save)
        # cls head
        _, c0, muC, rsC = K.layernorm_fwd(feats, self.P("cls_head.0.weight"), self.P("cls_head.0.bias"),
                                          out_f32=False, lp_dtype=dt, save_stats=save)
        c1 = K.linear_fwd(c0, self.W("cls_head.1.weight"), self.P("cls_head.1.bias"), relu=True, dropout_p=p,
                          seed=self.seed(2), seed_base=self.sb)
        c2 = K.linear_fwd(c1, self.W("cls_head.4.weight"), self.P("cls_head.4.bias"), relu=True, dropout_p=p,
                          seed=self.seed(3), seed_base=self.sb)
        logits = K.rowdot_fwd(c2, self.P("cls_head.7.weight"), self.P("cls_head.7.bias"))
        # reg head (forward only: no loss reaches it in the reference trainer)
        _, r0, _, _ = K.layernorm_fwd(feats, self.P("reg_head.0.weight"), self.P("reg_head.0.bias"),
                                      out_f32=False, lp_dtype=dt, save_stats=False)
        r1 = K.linear_fwd(r0, self.W("reg_head.1.weight"), self.P("reg_head.1.bias"), relu=True, dropout_p=p,
                          seed=self.seed(4), seed_base=self.sb)
        r2 = K.linear_fwd(r1, self.W("reg_head.4.weight"), self.P("reg_head.4.bias"), relu=True, dropout_p=p,
                          seed=self.seed(5), seed_base=self.sb)
        offsets = K.rowdot_fwd(r2, self.P("reg_head.7.weight"), self.P("reg_head.7.bias"), relu=True)
        if save:
            self.saved = dict(xin=xin, proj=proj, mu0=mu0, rs0=rs0, layers=layers, xL=x, e=e, muE=muE, rsE=rsE,
                              z=z, feats=feats, muF=muF, rsF=rsF, c0=c0, muC=muC, rsC=rsC, c1=c1, c2=c2)
        return (logits.view(B, T, 1), offsets.view(B, T, 2), feats.view(B, T, d))

    # ---- backward ----
    def backward(self, dlogits, dfeats):
        m, B, T, M, dt, p = self.m, self.B, self.T, self.M, self.dt, self.p
        H, L = m.num_heads, m.num_layers
        sd = self.scale_drop
        S = self.saved
        self._g = m._bind_grads()
        acc = not m._grad_fresh  # False: write the gradients (the captured step's zero_grad)
        m._grad_fresh = False
        lib = _native.load()
        ws = torch.empty(max(lib.rp_colsum_workspace(M, 256), 1), device=dlogits.device, dtype=_F32)
        d, dff = m.d_model, m.d_ff
        din = m.vis_dim + m.aud_dim + m.text_dim
        shapes = [(3 * d, d), (d, d), (dff, d), (d, dff), (d, din), (256, d), (256, 256), (d, d)]
        wws = torch.empty(max(lib.rp_gemm_wgrad_workspace(a, b, M) for a, b in shapes) // 4 + 4,
                          device=dlogits.device, dtype=_F32)
        G = self.G
        # Weight gradients (dW = dY^T X + bias) run on the step's one stream (a side stream beside the
        # dgrad chain measured 1.4 % slower, rounds 1-2); a layer's flat-gradient range is announced to
        # the all-reduce hooks once its weight-gradient GEMMs are launched.

        # bf16 training: the encoder layers' weight gradients are deferred and computed by grouped
        # whole-K launches (all 16 layers x 4 GEMMs = 768 256x256 tiles, three per CU: no split-K
        # slabs and no reduce pass).  Under DP a layer's gradient range is announced to the all-reduce
        # hooks once all its GEMMs have been launched, so the first launch's exchange overlaps the
        # backward of the remaining layers.
        deferred = [] if (dt == torch.bfloat16 and M % 64 == 0
                          and os.environ.get("RP_WGRAD_GROUPED", "1") != "0") else None
        held = []  # layer prefixes whose gradients wait for their group launch
        # one launch for the whole encoder on one GPU.  With gradient hooks (DP all-reduce) the launch is
        # cut so that each part's exchange overlaps the backward after it: every time the tiles gathered
        # since the last cut fill a whole round of the CUs (768 tiles at the metric shape: layers 15..11
        # plus layer 10's linear2 = 256 tiles = one round, then layer 10's rest .. layer 5's linear1 =
        # 256, then the last 256 — three launches; a 256-tile launch runs at the per-tile rate of the
        # 768-tile one, 455 vs 450 us per 256 tiles, so the cuts cost no GEMM time; eight-layer groups
        # were 384 + 384, a half-idle round each: 0.25 ms per step more).  Only the last part's exchange
        # is exposed after the backward.  RP_WGRAD_GROUP_LAYERS=n cuts every n whole layers instead
        env_layers = os.environ.get("RP_WGRAD_GROUP_LAYERS")
        per_launch = 4 * int(env_layers or "16")
        tile_cut = deferred is not None and bool(m._grad_ready_hooks) and env_layers is None
        ncu = torch.cuda.get_device_properties(dlogits.device).multi_processor_count if tile_cut else 0
        cut = {"tiles": 0}  # 256 x 256 tiles gathered since the last cut

        # LayerNorm gamma / beta partials: reduced together by one rp_colsum_batched launch per flush
        # (before the gradients they finish are announced, and at the end) instead of one per LayerNorm
        cs = []

        def flush_cs():
            if cs:
                K.colsum_batched(cs, accumulate=acc)
                cs.clear()

        def flush_group():
            if deferred:
                K.linear_wgrad_grouped(deferred, accumulate=acc)
                deferred.clear()
            flush_cs()
            for pf in held:
                m._grads_ready(pf)
            held.clear()

        def wgrad(dy, x, wname, bname):
            if deferred is not None and wname.startswith("multimodal_encoder."):
                deferred.append((dy, x, G(wname), G(bname)))
                if tile_cut:
                    cut["tiles"] += -(-dy.shape[1] // 256) * -(-x.shape[1] // 256)
                    if cut["tiles"] >= ncu and (cut["tiles"] % ncu == 0 or cut["tiles"] >= 2 * ncu):
                        cut["tiles"] = 0
                        flush_group()  # announces the layers already complete (held), not this one
                return
            K.linear_wgrad(dy, x, G(wname), db=G(bname), accumulate=acc, ws=wws)

        def ready(prefixes):
            if deferred is not None and prefixes[0].startswith("multimodal_encoder."):
                held.append(prefixes)
                if not tile_cut and len(deferred) >= per_launch:
                    flush_group()
                return
            if m._grad_ready_hooks:
                flush_cs()
            m._grads_ready(prefixes)

        dl = dlogits.reshape(M, 1).contiguous().float()
        # cls_head[7]  (N = 1)
        K.colsum(S["c2"], w=dl.view(M), out=G("cls_head.7.weight").view(-1), accumulate=acc, ws=ws)
        K.colsum(dl, out=G("cls_head.7.bias"), accumulate=acc, ws=ws)
        dz2 = K.rowdot_bwd_dx(dl, self.P("cls_head.7.weight"), gate=S["c2"], gate_scale=sd, out_dtype=dt)
        # cls_head[4]
        wgrad(dz2, S["c1"], "cls_head.4.weight", "cls_head.4.bias")
        dz1 = K.linear_dgrad(dz2, self.W("cls_head.4.weight"), out_dtype=dt, gate=S["c1"], gate_scale=sd)
        # cls_head[1]
        wgrad(dz1, S["c0"], "cls_head.1.weight", "cls_head.1.bias")
        dc0 = K.linear_dgrad(dz1, self.W("cls_head.1.weight"), out_dtype=_F32)
        # cls_head[0] LayerNorm (+ any external gradient on feats)
        dres = dfeats.reshape(M, -1).contiguous().float() if dfeats is not None else None
        dfe, _ = K.layernorm_bwd(dc0, S["feats"], S["muC"], S["rsC"], self.P("cls_head.0.weight"), dres=dres,
                                 dgamma=G("cls_head.0.weight"), dbeta=G("cls_head.0.bias"), ws=ws, defer=cs)
        # feature_map: LN + ReLU + dropout, then Linear
        _, dz = K.layernorm_bwd(dfe, S["z"], S["muF"], S["rsF"], self.P("feature_map.1.weight"), y=S["feats"],
                                dropout_p=p, seed=self.seed(1), seed_base=self.sb, want_f32=False, lp_dtype=dt,
                                dgamma=G("feature_map.1.weight"), dbeta=G("feature_map.1.bias"), ws=ws, defer=cs)
        wgrad(dz, S["e"], "feature_map.0.weight", "feature_map.0.bias")
        # encoder_norm; emit the masked lp gradient for the last layer's dropout2
        if self.fused_ln:
            dx, g2 = K.linear_ln_bwd(dz, self.W("feature_map.0.weight"), S["xL"], S["muE"], S["rsE"],
                                     self.P("encoder_norm.weight"), lp_dtype=dt, lp_dropout_p=p,
                                     lp_seed=self.seed(103 + 4 * (L - 1)), seed_base=self.sb,
                                     dgamma=G("encoder_norm.weight"), dbeta=G("encoder_norm.bias"), ws=ws, defer=cs)
        else:
            de = K.linear_dgrad(dz, self.W("feature_map.0.weight"), out_dtype=_F32)
            dx, g2 = K.layernorm_bwd(de, S["xL"], S["muE"], S["rsE"], self.P("encoder_norm.weight"), lp_dtype=dt,
                                     lp_dropout_p=p, lp_seed=self.seed(103 + 4 * (L - 1)), seed_base=self.sb,
                                     dgamma=G("encoder_norm.weight"), dbeta=G("encoder_norm.bias"), ws=ws, defer=cs)
        ready(["encoder_norm.", "feature_map.", "cls_head."])
        for l in reversed(range(L)):
            pre = f"multimodal_encoder.layers.{l}."
            x, h1, mu1, rs1, qkv, o, olo, lse, dmask, x1, h2, mu2, rs2, f = S["layers"][l]
            # linear2 (+dropout2 handled by g2's mask)
            wgrad(g2, f, pre + "linear2.weight", pre + "linear2.bias")
            dzf = K.linear_dgrad(g2, self.W(pre + "linear2.weight"), out_dtype=dt, gate=f, gate_scale=sd)
            # linear1 (ReLU + dropout folded into the gate above)
            wgrad(dzf, h2, pre + "linear1.weight", pre + "linear1.bias")
            # norm2 + residual; masked lp gradient for dropout1 (bf16: one rp_gemm_ln_bwd launch)
            if self.fused_ln:
                dx1, g1 = K.linear_ln_bwd(dzf, self.W(pre + "linear1.weight"), x1, mu2, rs2, self.P(pre + "norm2.weight"),
                                          dres=dx, lp_dtype=dt, lp_dropout_p=p, lp_seed=self.seed(101 + 4 * l),
                                          seed_base=self.sb, dgamma=G(pre + "norm2.weight"),
                                          dbeta=G(pre + "norm2.bias"), ws=ws, defer=cs)
            else:
                dh2 = K.linear_dgrad(dzf, self.W(pre + "linear1.weight"), out_dtype=_F32)
                dx1, g1 = K.layernorm_bwd(dh2, x1, mu2, rs2, self.P(pre + "norm2.weight"), dres=dx, lp_dtype=dt,
                                          lp_dropout_p=p, lp_seed=self.seed(101 + 4 * l), seed_base=self.sb,
                                          dgamma=G(pre + "norm2.weight"), dbeta=G(pre + "norm2.bias"), ws=ws, defer=cs)
            # out_proj
            wgrad(g1, o, pre + "self_attn.out_proj.weight", pre + "self_attn.out_proj.bias")
            # attention (bf16: the delta = rowsum(dO * O) pre-pass rides in the out_proj dgrad's epilogue)
            if K.attn_dout_delta_ok(M, H, d, dt):
                do, delta = K.attn_dout_delta(g1, self.W(pre + "self_attn.out_proj.weight"), o, olo, lse, B, T, H, p)
            else:
                do = K.linear_dgrad(g1, self.W(pre + "self_attn.out_proj.weight"), out_dtype=dt)
                delta = None
            dqkv = K.attn_bwd(qkv, o, do, lse, self.kv, B, T, H, self.scale, p, dropmask=dmask, q_prescaled=True,
                              out_lo=olo, delta=delta)
            # in_proj
            wgrad(dqkv, h1, pre + "self_attn.in_proj_weight", pre + "self_attn.in_proj_bias")
            # norm1 + residual; masked lp gradient for the previous layer's dropout2
            last = l == 0
            if self.fused_ln:
                dx, g2 = K.linear_ln_bwd(dqkv, self.W(pre + "self_attn.in_proj_weight"), x, mu1, rs1,
                                         self.P(pre + "norm1.weight"), dres=dx1, lp_dtype=None if last else dt,
                                         lp_dropout_p=0.0 if last else p,
                                         lp_seed=0 if last else self.seed(103 + 4 * (l - 1)), seed_base=self.sb,
                                         dgamma=G(pre + "norm1.weight"), dbeta=G(pre + "norm1.bias"), ws=ws, defer=cs)
            else:
                dh1 = K.linear_dgrad(dqkv, self.W(pre + "self_attn.in_proj_weight"), out_dtype=_F32)
                dx, g2 = K.layernorm_bwd(dh1, x, mu1, rs1, self.P(pre + "norm1.weight"), dres=dx1,
                                         lp_dtype=None if last else dt, lp_dropout_p=0.0 if last else p,
                                         lp_seed=0 if last else self.seed(103 + 4 * (l - 1)), seed_base=self.sb,
                                         dgamma=G(pre + "norm1.weight"), dbeta=G(pre + "norm1.bias"), ws=ws, defer=cs)
            ready([pre])
        if deferred is not None and (deferred or held):
            # the rest of the grouped launch, and the layers it completes (a tile cut can fall on the
            # last layer's last GEMM: then nothing is left to launch, but layer 0 is still to announce)
            flush_group()
        # input LayerNorm (+PE, no grad) and input projection (weight/bias grads only)
        _, dproj = K.layernorm_bwd(dx, S["proj"], S["mu0"], S["rs0"], self.P("input_norm.weight"), want_f32=False,
                                   lp_dtype=dt, dgamma=G("input_norm.weight"), dbeta=G("input_norm.bias"), ws=ws, defer=cs)
        wgrad(dproj, S["xin"], "input_projection.weight", "input_projection.bias")
        ready(["input_projection.", "input_norm."])
        flush_cs()
        for h in m._grad_done_hooks:
            h()
        self.saved = None


class _ModelFunction(torch.autograd.Function):
    """The whole model as one autograd node.  Gradients are written straight into the flat gradient
    buffer (the Parameters' .grad views), so backward returns None for every parameter input."""

    @staticmethod
    def forward(ctx, run, *params):
        ctx.set_materialize_grads(False)
        ctx.run = run
        return run.forward(save=True)

    @staticmethod
    def backward(ctx, dlogits, doffsets, dfeats):
        run = ctx.run
        if doffsets is not None:
            raise NotImplementedError("repurpose_amd: gradient through out_offsets (reg_head) is not part of "
                                      "the reference training path (losses() uses cls_loss only)")
        if dlogits is None:
            dlogits = torch.zeros(run.M, device=run.v.device, dtype=_F32)
        if run.saved is None:
            raise RuntimeError("repurpose_amd: backward called twice on one forward")
        run.backward(dlogits, dfeats)
        ctx.run = None
        return (None,) * (1 + _ModelFunction._nparams(run))

    @staticmethod
    def _nparams(run):
        return len(run.m._trained_params)
