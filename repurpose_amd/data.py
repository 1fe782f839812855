"""Batch collation for the Repurpose trainer: drop-ins for
``dataset/RepurposeClip.py`` ``preprocessing`` (:449-533), ``collate_fn`` (:536-567) and
``collate_fn_test`` (:997-1030), plus a device-side path.

Reference semantics kept exactly (fp32 outputs, ``padding_val`` fill, masks from the VISUAL lengths
only — SURVEY hazard 9: text may be shorter and is then zero inside the valid region — and the
same ValueErrors).

Device path: the DataLoader workers only concatenate each modality's ragged rows into one array
(``collate_ragged`` -> ``RaggedBatch``; no per-item padding loops, no torch.full of the padded
batch on the host); the main process then moves the concatenated rows through pinned memory in one
copy per modality and pads / converts on the GPU with ``rp_pad_rows`` (fp16 CLIP, fp32 PANNs, fp64
text rows as stored in the .npy files).  ``RaggedBatch.to_device`` returns the same dict as
``collate_fn`` with the tensors already on the device.

``load_features`` reads the feature files with ``numpy.load(allow_pickle=False, mmap_mode='r')``
(the reference uses allow_pickle=True).
"""
import ctypes
from dataclasses import dataclass, field
from typing import List

import numpy as np
import torch

from . import _native as N
from . import kernels as K

_NP_DT = {np.dtype(np.float16): N.RP_F16, np.dtype(np.float32): N.RP_F32, np.dtype(np.float64): N.RP_F64,
          np.dtype(np.int64): N.RP_I64}
_TORCH_DT = {torch.float16: N.RP_F16, torch.float32: N.RP_F32, torch.float64: N.RP_F64, torch.int64: N.RP_I64}


def load_features(path):
    """[seq_len, dim] feature array of one video (memory-mapped, no pickle)."""
    return np.load(path, mmap_mode="r", allow_pickle=False)


# ----------------------------------------------------------------------------- host drop-ins
@torch.no_grad()
def preprocessing(vis_feats, aud_feats, text_feats, labels, segments, padding_val=0.0):
    """dataset/RepurposeClip.py:449-533: pad the per-video tensors to the longest VISUAL sequence."""
    lens = torch.as_tensor([v.shape[0] for v in vis_feats])
    T = int(lens.max().item()) if len(vis_feats) else 0
    if T == 0:
        raise ValueError("All sequences in the batch have zero length")

    def pad(seqs, tail):
        out = torch.full((len(seqs), T) + tail, padding_val)
        for i, s in enumerate(seqs):
            if s.shape[0] > 0:
                out[i, :s.shape[0], ...] = s
        return out

    v = pad(vis_feats, (vis_feats[0].shape[1],))
    a = pad(aud_feats, (aud_feats[0].shape[1],))
    t = pad(text_feats, (text_feats[0].shape[1],))
    lab = pad(labels, ())
    if len(segments) == 0:
        raise ValueError("No segments provided to preprocessing function")
    if all(s.shape[0] == 0 for s in segments):
        raise ValueError("All segments in the batch have zero length")
    seg_dim = next(s.shape[1] if s.dim() > 1 else 1 for s in segments if s.shape[0] > 0)
    seg = torch.full((len(segments), T, seg_dim), padding_val)
    for i, s in enumerate(segments):
        if s.shape[0] > 0:
            s = s.unsqueeze(1) if s.dim() == 1 else s
            if s.shape[1] != seg_dim:
                continue  # the reference logs a warning and skips the item
            seg[i, :s.shape[0], ...] = s
    masks = (torch.arange(T).expand(len(lens), T) < lens.unsqueeze(1)).unsqueeze(1)
    return v, a, t, masks, lab, seg


def _items(batch):
    vis = [torch.tensor(np.asarray(it["feats"]["visual"])) for it in batch]
    aud = [torch.tensor(np.asarray(it["feats"]["audio"])) for it in batch]
    txt = [torch.tensor(np.asarray(it["feats"]["text"])) for it in batch]
    lab = [torch.tensor(it["labels"]) for it in batch]
    seg = [torch.tensor(it["segments"]) for it in batch]
    return vis, aud, txt, lab, seg


def collate_fn(batch):
    """dataset/RepurposeClip.py:536-567."""
    v, a, t, m, lab, seg = preprocessing(*_items(batch))
    return {"video_id": [it["video_id"] for it in batch], "duration": [it["duration"] for it in batch],
            "visual_feats": v, "audio_feats": a, "text_feats": t, "masks": m, "labels": lab, "segments": seg}


def collate_fn_test(batch):
    """dataset/RepurposeClip.py:997-1030 (adds the reference segments used by the metric)."""
    out = collate_fn(batch)
    out["gt_segments"] = [it["gt_segments"] for it in batch]
    return out


# ----------------------------------------------------------------------------- device path
def _dma_rows(src, offs, dst, padding_val):
    """fp32 pinned rows [sum len, D] -> padded dst [B, T, D] by DMA (current stream): one copy when every
    sequence fills T (the rows are then dst's layout), else one per sequence and a fill of its padding."""
    B, T, _ = dst.shape
    lens = np.diff(offs)
    if np.all(lens == T):
        dst.view(-1, dst.shape[2]).copy_(src[:B * T], non_blocking=True)
        return
    for b in range(B):
        n = int(lens[b])
        if n:
            dst[b, :n].copy_(src[int(offs[b]):int(offs[b]) + n], non_blocking=True)
        if n < T:
            dst[b, n:].fill_(padding_val)


@dataclass
class RaggedBatch:
    """One modality per entry: rows of all videos concatenated + prefix offsets (int64 [B+1])."""
    video_id: list
    duration: list
    rows: dict                      # name -> np.ndarray [sum len, D] (labels: [sum len, 1])
    offsets: dict                   # name -> np.ndarray int64 [B+1]
    extra: dict = field(default_factory=dict)

    def pin(self):
        """This batch with every row array in page-locked host memory (what a DataLoader's pin_memory
        thread does off the training loop); ``to_device`` then issues the H2D copies straight away."""
        rows = {k: (v if torch.is_tensor(v) and v.is_pinned() else torch.from_numpy(np.ascontiguousarray(v)).pin_memory())
                for k, v in self.rows.items()}
        offs = {k: (v if torch.is_tensor(v) and v.is_pinned() else torch.from_numpy(np.asarray(v, dtype=np.int64)).pin_memory())
                for k, v in self.offsets.items()}
        return RaggedBatch(self.video_id, self.duration, rows, offs, dict(self.extra))

    def to_device(self, device, padding_val=0.0, out=None):
        """collate_fn's dict with every tensor on ``device``: one pinned H2D copy per modality, then
        rp_pad_rows pads and converts on the GPU (all enqueued on the current stream).  fp32 rows (PANNs
        audio, labels, segments) need no conversion: from pinned memory they are copied by DMA straight
        into their padded places (one copy when no sequence is short, else one per sequence plus a fill
        of the padding).  ``out``: an existing dict of device tensors of the padded shapes (e.g. a
        captured training step's static inputs, ``CapturedTrainStep.input_set``) written in place."""
        if not torch.device(device).type == "cuda":
            raise RuntimeError("RaggedBatch.to_device: the device path needs a ROCm device (use collate_fn on CPU)")
        B = len(self.video_id)
        host_offs = {k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in self.offsets.items()}
        vlens = np.diff(host_offs["visual"])
        T = int(vlens.max()) if B else 0
        if T == 0:
            raise ValueError("All sequences in the batch have zero length")
        if int(np.diff(host_offs["segments"]).max()) == 0:
            raise ValueError("All segments in the batch have zero length")
        res = {"video_id": self.video_id, "duration": self.duration}
        names = {"visual": "visual_feats", "audio": "audio_feats", "text": "text_feats", "labels": "labels",
                 "segments": "segments"}
        for name, key in names.items():
            rows = self.rows[name]
            offs = host_offs[name]
            if np.any(np.diff(offs) > T):
                raise ValueError(f"{name}: a sequence is longer than the visual padding length {T}")
            if torch.is_tensor(rows) and rows.is_pinned():
                hsrc, code = rows, _TORCH_DT[rows.dtype]
            else:
                rows = np.ascontiguousarray(rows)
                hsrc, code = torch.from_numpy(rows).pin_memory(), _NP_DT[rows.dtype]
            D = rows.shape[1] if rows.ndim > 1 else 1
            if out is not None:
                dst = out[key]
                if dst.device != torch.device(device) or dst.dtype != torch.float32 or not dst.is_contiguous() \
                        or dst.numel() != B * T * D:
                    raise ValueError(f"RaggedBatch.to_device: out[{key!r}] must be a contiguous fp32 tensor of "
                                     f"{B} x {T} x {D} on {device}")
                dst = dst.view(B, T, D)
            else:
                dst = torch.empty(B, T, D, device=device, dtype=torch.float32)
            if code == N.RP_F32:
                _dma_rows(hsrc.view(-1, D), offs, dst, padding_val)
            else:
                hoff = self.offsets[name]
                if not (torch.is_tensor(hoff) and hoff.is_pinned()):
                    hoff = torch.from_numpy(offs.astype(np.int64)).pin_memory()
                src = hsrc.to(device, non_blocking=True)
                off = hoff.to(device, non_blocking=True)
                N.call("rp_pad_rows", ctypes.c_void_p(src.data_ptr()), code, ctypes.c_void_p(off.data_ptr()),
                       B, T, D, float(padding_val), ctypes.c_void_p(dst.data_ptr()), K._stream(dst))
            res[key] = dst.view(B, T) if name == "labels" else dst
        # the lengths from pinned memory: a pageable H2D copy would hold the host until the stream reached
        # it (e.g. behind a wait for the step that last read ``out``)
        # the padding masks from the host lengths (collate's arange(T) < len, dataset/RepurposeClip.py:449-567):
        # one pinned copy, no device kernels beside a running step
        mh = torch.from_numpy(np.arange(T)[None, :] < vlens[:, None]).unsqueeze(1).pin_memory()
        if out is not None:
            out["masks"].copy_(mh, non_blocking=True)
            m = out["masks"]
        else:
            m = mh.to(device, non_blocking=True)
        res["masks"] = m
        res.update(self.extra)
        return res


def collate_ragged(batch, test=False, f32=False):
    """Worker-side collate: concatenation only (no padding, no torch tensors).  ``f32``: the rows also
    converted to float32 in the worker, as the reference's collate does while padding
    (dataset/RepurposeClip.py:449-567 builds fp32 batches) — ``to_device`` then moves every modality by
    DMA into its padded place and runs no conversion kernel beside the training step."""
    def cat(arrs, D=None):
        arrs = [np.asarray(a, dtype=np.float32) if f32 else np.asarray(a) for a in arrs]
        lens = [a.shape[0] for a in arrs]
        offs = np.zeros(len(arrs) + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        dt = np.result_type(*[a.dtype for a in arrs])
        dt = np.dtype(np.float32) if dt not in _NP_DT else dt
        shape = (int(offs[-1]),) + (arrs[0].shape[1:] if arrs[0].ndim > 1 else (1,))
        rows = np.empty(shape, dtype=dt)
        for a, o, n in zip(arrs, offs[:-1], lens):
            if n:
                rows[o:o + n] = a.reshape(n, -1)
        return rows, offs

    rows, offs = {}, {}
    for name in ("visual", "audio", "text"):
        rows[name], offs[name] = cat([it["feats"][name] for it in batch])
    rows["labels"], offs["labels"] = cat([np.asarray(it["labels"], dtype=np.int64 if np.asarray(it["labels"]).dtype.kind in "iub" else np.float32) for it in batch])
    rows["segments"], offs["segments"] = cat([np.asarray(it["segments"], dtype=np.float32).reshape(-1, 2) for it in batch])
    extra = {"gt_segments": [it["gt_segments"] for it in batch]} if test else {}
    return RaggedBatch([it["video_id"] for it in batch], [it["duration"] for it in batch], rows, offs, extra)
