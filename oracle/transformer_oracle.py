"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's models/transformer.py (:6-190),
the checker for repurpose_amd.transformer.  Written from the reference's behaviour with stock torch
ops; imported only by tests/.

Restated semantics (file:line of the reference):
  * PositionalEncoding :6-21 — table pe[pos, 2i] = sin(pos * 10000^(-2i/d)), pe[pos, 2i+1] = cos(...),
    stored [max_len, 1, d]; forward adds pe[:x.size(0)] (the batch index on batch-first input).
  * MLP :24-35 — fc1, ReLU, fc2.
  * MultiHeadAttention :37-81 — q/k/v projections (construction order q, k, v, out), heads of
    d_k = d/h, scores = QK^T / sqrt(d_k), masked_fill(mask.unsqueeze(1) == 0, -1e9), softmax, PV,
    heads concatenated, out projection.
  * EncoderLayer :84-102, CrossAttentionEncoderLayer :105-130, CrossSelfEncoderLayer :133-176,
    UniModalEncoder :179-190 — the layer compositions (pre-LN; residual placements as in the reference,
    including CrossSelf's residuals onto the normalised input).
Parity status: no reference fixtures exist for this file — parity unpinned beyond this
restatement; state_dict keys and parameter counts are checked structurally.
"""
import math

import torch
import torch.nn as nn


class PositionalEncoding(nn.Module):
    def __init__(self, d_model, max_len=5000):
        super().__init__()
        pos = torch.arange(max_len, dtype=torch.float).unsqueeze(1)
        freq = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        table = torch.zeros(max_len, d_model)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", table.unsqueeze(1))

    def forward(self, x):
        return x + self.pe[:x.size(0)]


class MLP(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, hidden_dim)
        self.relu = nn.ReLU()
        self.fc2 = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        return self.fc2(self.relu(self.fc1(x)))


class MultiHeadAttention(nn.Module):
    def __init__(self, d_model, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.d_model = d_model
        self.d_k = d_model // num_heads
        self.q_linear = nn.Linear(d_model, d_model)
        self.k_linear = nn.Linear(d_model, d_model)
        self.v_linear = nn.Linear(d_model, d_model)
        self.out = nn.Linear(d_model, d_model)
        self.register_buffer("scale", torch.sqrt(torch.FloatTensor([self.d_k])))

    def forward(self, q, k, v, mask=None):
        B = q.size(0)

        def heads(t):
            return t.view(B, -1, self.num_heads, self.d_k).transpose(1, 2)

        kh, qh, vh = heads(self.k_linear(k)), heads(self.q_linear(q)), heads(self.v_linear(v))
        s = qh @ kh.transpose(-2, -1) / self.scale
        if mask is not None:
            s = s.masked_fill(mask.unsqueeze(1) == 0, -1e9)
        o = torch.softmax(s, dim=-1) @ vh
        return self.out(o.transpose(1, 2).contiguous().view(B, -1, self.d_model))


def _ff(d_model, d_ff, dropout=None):
    mods = [nn.Linear(d_model, d_ff), nn.ReLU()]
    if dropout is not None:
        mods.append(nn.Dropout(dropout))
    return nn.Sequential(*mods, nn.Linear(d_ff, d_model))


class EncoderLayer(nn.Module):
    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.ff = _ff(d_model, d_ff)
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, mask):
        h = self.norm_1(x)
        x = x + self.dropout_1(self.attention(h, h, h, mask))
        return x + self.dropout_2(self.ff(self.norm_2(x)))


class CrossAttentionEncoderLayer(nn.Module):
    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.cross_attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.ff = _ff(d_model, d_ff)
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, context, mask=None):
        x = x + self.dropout_1(self.cross_attention(self.norm_1(x), context, context, mask))
        return x + self.dropout_2(self.ff(self.norm_2(x)))


class CrossSelfEncoderLayer(nn.Module):
    def __init__(self, d_model, num_heads, d_ff=2048, dropout=0.0):
        super().__init__()
        self.self_attention = MultiHeadAttention(d_model, num_heads)
        self.cross_attention = MultiHeadAttention(d_model, num_heads)
        self.norm_1 = nn.LayerNorm(d_model)
        self.norm_2 = nn.LayerNorm(d_model)
        self.norm_3 = nn.LayerNorm(d_model)
        self.ff = _ff(d_model, d_ff, dropout)
        self.dropout_1 = nn.Dropout(dropout)
        self.dropout_2 = nn.Dropout(dropout)

    def forward(self, x, context, mask=None):
        h = self.norm_1(x)
        x = x + self.dropout_1(self.self_attention(h, h, h, mask))
        x = self.norm_2(x)
        x = x + self.dropout_2(self.cross_attention(x, context, context, mask))
        x = self.norm_3(x)
        return x + self.dropout_2(self.ff(x))


class UniModalEncoder(nn.Module):
    def __init__(self, input_dim, d_model, num_layers, num_heads, d_ff=2048):
        super().__init__()
        self.mlp = MLP(input_dim, d_ff, d_model)
        self.positional_encoding = PositionalEncoding(d_model)
        self.layers = nn.ModuleList([EncoderLayer(d_model, num_heads, d_ff) for _ in range(num_layers)])

    def forward(self, x, mask=None):
        x = self.positional_encoding(self.mlp(x))
        for layer in self.layers:
            x = layer(x, mask)
        return x
