"""TEST INFRASTRUCTURE ONLY — restatement of dataset/RepurposeClip.py ``preprocessing`` (:449-533)
and ``collate_fn`` (:536-567): every modality padded with ``padding_val`` to the longest VISUAL
sequence of the batch in fp32 (torch copy conversion), masks [B, 1, T] from the visual lengths,
labels [B, T], segments [B, T, seg_dim]; ValueError for an all-empty batch or all-empty segments."""
import torch


def preprocessing(vis, aud, txt, labels, segments, padding_val=0.0):
    lens = [v.shape[0] for v in vis]
    T = max(lens)
    if T == 0:
        raise ValueError("All sequences in the batch have zero length")
    outs = []
    for seqs in (vis, aud, txt):
        o = torch.full((len(seqs), T, seqs[0].shape[1]), padding_val)
        for i, s in enumerate(seqs):
            if s.shape[0]:
                o[i, :s.shape[0]] = s
        outs.append(o)
    lab = torch.full((len(labels), T), padding_val)
    for i, s in enumerate(labels):
        if s.shape[0]:
            lab[i, :s.shape[0]] = s
    if not segments or all(s.shape[0] == 0 for s in segments):
        raise ValueError("All segments in the batch have zero length")
    first = [s for s in segments if s.shape[0]][0]
    sd = first.shape[1] if first.dim() > 1 else 1
    seg = torch.full((len(segments), T, sd), padding_val)
    for i, s in enumerate(segments):
        if s.shape[0]:
            s = s.unsqueeze(1) if s.dim() == 1 else s
            if s.shape[1] == sd:
                seg[i, :s.shape[0]] = s
    masks = torch.stack([torch.arange(T) < n for n in lens]).unsqueeze(1)
    return outs[0], outs[1], outs[2], masks, lab, seg


def collate_fn(batch):
    v, a, t, m, lab, seg = preprocessing([torch.tensor(b["feats"]["visual"]) for b in batch],
                                         [torch.tensor(b["feats"]["audio"]) for b in batch],
                                         [torch.tensor(b["feats"]["text"]) for b in batch],
                                         [torch.tensor(b["labels"]) for b in batch],
                                         [torch.tensor(b["segments"]) for b in batch])
    return {"video_id": [b["video_id"] for b in batch], "duration": [b["duration"] for b in batch],
            "visual_feats": v, "audio_feats": a, "text_feats": t, "masks": m, "labels": lab, "segments": seg}
