"""TEST INFRASTRUCTURE ONLY — fp32 CPU restatement of ``models/MMCTransformer.py``.

Used by tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of bench.py as the
checker.  Never imported by ``repurpose_amd``.

It restates the reference module graph with *stock* ``torch.nn`` building blocks (third-party
code, not reference code), created in the same order as the reference constructor so that
``torch.manual_seed`` reproduces the reference initialisation:

* ``MMCTransformer.__init__``        -> reference ``models/MMCTransformer.py:26-96``
* ``_init_weights``                  -> ``:98-107`` (xavier-uniform Linear, zero bias, LN 1/0;
  MHA ``in_proj_weight`` is *not* an ``nn.Linear`` and keeps MHA's own init, identical across the
  deep-copied layers)
* ``PositionalEncoding``             -> ``:9-22``
* ``forward``                        -> ``:109-151``
* ``losses``                         -> ``:159-179``
* ``inference_single_video``         -> ``:181-229``
* ``inference_``                     -> ``:231-275``

Pin: with the SURVEY §8c recipe the 2-layer tri-modal model has 8,475,395 parameters and
``cls_loss`` = 32.2317 (tests/test_oracle.py::test_known_answer_cls_loss).
"""
import math

import numpy as np
import torch
import torch.nn as nn

from .focal_oracle import sigmoid_focal_loss
from .softnms_oracle import soft_nms_intervals_cpu


class PositionalEncoding(nn.Module):
    """Sinusoidal table, batch-first add (reference ``MMCTransformer.py:9-22``)."""

    def __init__(self, d_model, max_len=5000):
        super().__init__()
        pos = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
        freq = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        table = torch.zeros(max_len, d_model)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", table.unsqueeze(0))

    def forward(self, x):
        return x + self.pe[:, : x.size(1)]


def _head(d_model, hidden, n_out, final_relu):
    layers = [nn.LayerNorm(d_model), nn.Linear(d_model, hidden), nn.ReLU(), nn.Dropout(0.1),
              nn.Linear(hidden, hidden), nn.ReLU(), nn.Dropout(0.1), nn.Linear(hidden, n_out)]
    if final_relu:
        layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class MMCTransformer(nn.Module):
    """Oracle restatement; same constructor signature as the reference (``:26``)."""

    def __init__(self, vis_dim, aud_dim, text_dim, d_model, self_num_layers, text_num_layers,
                 cross_num_layers, num_heads, d_ff=2048):
        super().__init__()
        self.input_projection = nn.Linear(vis_dim + aud_dim + text_dim, d_model)
        self.input_norm = nn.LayerNorm(d_model)
        self.positional_encoding = PositionalEncoding(d_model)
        proto = nn.TransformerEncoderLayer(d_model=d_model, nhead=num_heads, dim_feedforward=d_ff,
                                           dropout=0.1, activation="relu", batch_first=True,
                                           norm_first=True)
        self.multimodal_encoder = nn.TransformerEncoder(proto, num_layers=self_num_layers,
                                                        enable_nested_tensor=False)
        self.encoder_norm = nn.LayerNorm(d_model)
        self.feature_map = nn.Sequential(nn.Linear(d_model, d_model), nn.LayerNorm(d_model),
                                         nn.ReLU(), nn.Dropout(0.1))
        self.cls_head = _head(d_model, 256, 1, final_relu=False)
        self.reg_head = _head(d_model, 256, 2, final_relu=True)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.LayerNorm):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    @property
    def device(self):
        return next(self.parameters()).device

    def forward(self, batch):
        x = torch.cat([batch["visual_feats"], batch["audio_feats"], batch["text_feats"]], dim=-1)
        x = self.positional_encoding(self.input_norm(self.input_projection(x)))
        pad = (batch["masks"] == 0).squeeze(1)
        x = self.encoder_norm(self.multimodal_encoder(x, src_key_padding_mask=pad))
        feats = self.feature_map(x)
        return (batch["masks"], self.cls_head(feats), self.reg_head(feats), batch["labels"],
                batch["segments"], feats)

    def losses(self, masks, out_cls_logits, out_offsets, gt_cls_labels, gt_offsets, feats):
        per_frame = sigmoid_focal_loss(out_cls_logits, gt_cls_labels.unsqueeze(-1))
        return {"cls_loss": (per_frame * masks.transpose(1, 2).contiguous()).sum()}

    @torch.no_grad()
    def inference_single_video(self, masks, out_cls_logits, out_offsets, inference_settings):
        return select_candidates(masks, out_cls_logits, out_offsets, inference_settings)

    @torch.no_grad()
    def inference_(self, batch, inference_settings):
        masks, logits, offsets, _, _, _ = self.forward(batch)
        return postprocess(masks, logits.squeeze(-1), offsets, batch["video_id"], batch["duration"],
                           inference_settings)


def select_candidates(masks, logits, offsets, cfg):
    """Reference ``inference_single_video`` (``MMCTransformer.py:181-229``).

    The reference sorts with the unstable ``torch.sort(descending=True)``; this restatement uses a
    stable (score desc, index asc) order, which is what the HIP kernel reproduces.
    """
    prob = (logits.sigmoid().squeeze() * masks).flatten()
    keep = prob > cfg["pre_nms_thresh"]
    cand = keep.nonzero(as_tuple=True)[0]
    prob = prob[keep]
    k = min(cfg["pre_nms_topk"], cand.size(0))
    order = torch.sort(prob, descending=True, stable=True).indices
    prob = prob[order[:k]].clone()
    cand = cand[order[:k]].clone()
    off = offsets[cand]
    left = cand - off[:, 0]
    right = cand + off[:, 1]
    segs = torch.stack((left, right), -1)
    dur = right - left
    ok = (dur > cfg["duration_thresh"]) & (dur < cfg["duration_thresh_max"])
    return {"segments": segs[ok], "scores": prob[ok], "labels": cand[ok]}


def max_segments_for(duration, per_min):
    """``int(np.ceil((vlen // 60) * max_seg_per_min))`` in float64 (``MMCTransformer.py:255-257``)."""
    return int(np.ceil((duration // 60) * per_min))


def postprocess(masks, prob_logits, offsets, video_ids, durations, cfg):
    """Per-video loop of ``inference_`` (``MMCTransformer.py:248-273``)."""
    out = []
    for i, (vid, vlen) in enumerate(zip(video_ids, durations)):
        res = select_candidates(masks[i], prob_logits[i], offsets[i], cfg)
        keep = soft_nms_intervals_cpu(res["scores"], res["segments"], sigma=cfg["nms_sigma"],
                                      thresh=cfg["min_score"],
                                      max_seg_num=max_segments_for(vlen, cfg["max_seg_per_min"]))
        keep = torch.as_tensor(keep, dtype=torch.long)
        res = {k: v[keep] for k, v in res.items()}
        res["video_id"] = vid
        res["duration"] = vlen
        out.append(res)
    return out
