"""Generates the golden fixtures under tests/golden/ from the CPU oracle (oracle/).

The reference cannot be imported in this pipeline (SURVEY §8c denial), so these vectors pin the
oracle restatement (itself pinned by the SURVEY known-answer point) against regressions and give
the GPU tests fixed expected values.  Run:  python -m tests.golden.make_golden
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
CFG = dict(vis_dim=512, aud_dim=2048, text_dim=384, d_model=512, self_num_layers=2, text_num_layers=3,
           cross_num_layers=3, num_heads=8)


def model_inputs(B=2, T=48, seed=7):
    g = torch.Generator().manual_seed(seed)
    lens = torch.tensor([T, T - 17])[:B]
    return {"visual_feats": torch.randn(B, T, 512, generator=g),
            "audio_feats": torch.relu(torch.randn(B, T, 2048, generator=g)),
            "text_feats": torch.randn(B, T, 384, generator=g),
            "masks": (torch.arange(T)[None] < lens[:, None]).unsqueeze(1),
            "labels": torch.randint(0, 2, (B, T), generator=g).float(),
            "segments": torch.rand(B, T, 2, generator=g) * 10}


def model_case():
    from oracle.mmct_oracle import MMCTransformer
    torch.manual_seed(0)
    m = MMCTransformer(**CFG).eval()
    b = model_inputs()
    with torch.no_grad():
        out = m(b)
        loss = m.losses(*out)["cls_loss"]
    return {"logits": out[1].numpy(), "offsets": out[2].numpy(), "loss": np.float32(loss.item())}


def softnms_cases(ncases=12, seed=11):
    rs = np.random.RandomState(seed)
    cases = []
    for c in range(ncases):
        n = [0, 1, 2, 7, 50, 300, 1000][c % 7]
        sc = np.sort(rs.uniform(0.5, 1.0, n).astype(np.float32))[::-1].copy()
        ctr = rs.uniform(0, 1800, n).astype(np.float32)
        segs = np.stack([ctr - rs.uniform(5.5, 45, n), ctr + rs.uniform(5.5, 45, n)], 1).astype(np.float32)
        thresh = [0.01, 0.001, 0.3][c % 3]
        maxseg = int([0, 1, 3, 9, 27, 60][c % 6])
        cases.append((sc, segs, thresh, maxseg))
    return cases


def main():
    from oracle.softnms_oracle import soft_nms_intervals_cpu
    np.savez(os.path.join(HERE, "golden_model_L2.npz"), **model_case())
    out = {"ncases": np.int64(0), "sigma": np.float32(0.5)}
    cases = softnms_cases()
    for c, (sc, segs, thresh, maxseg) in enumerate(cases):
        keep = soft_nms_intervals_cpu(torch.from_numpy(sc.copy()), torch.from_numpy(segs), 0.5, thresh, maxseg)
        out[f"n{c}"] = np.int64(len(sc))
        out[f"scores{c}"] = sc
        out[f"segs{c}"] = segs
        out[f"thresh{c}"] = np.float32(thresh)
        out[f"maxseg{c}"] = np.int64(maxseg)
        out[f"keep{c}"] = np.asarray(keep, dtype=np.int64)
    out["ncases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "golden_softnms.npz"), **out)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
