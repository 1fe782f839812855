"""Writes tests/golden/val_labels_64.json: the labels of the first 64 videos of the reference's
validation split (data/val.json of the reference repository: youtube_id, timeRangeOffset,
segmentsOffset — the ground truth that main.py:685-703 scores with calculate_tiou).  Data only; the
GPU box has no /root/reference, so the AtIoU parity run (scripts/val_atiou.py,
tests/test_infer_gpu.py) reads this fixture.

    python tests/golden/make_val_fixture.py [/root/reference/data/val.json]
"""
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/val.json"
items = json.load(open(src))[:64]
out = [{"youtube_id": it["youtube_id"], "timeRangeOffset": it["timeRangeOffset"],
        "segmentsOffset": it["segmentsOffset"]} for it in items]
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "val_labels_64.json")
with open(dst, "w") as f:
    json.dump({"source": "reference data/val.json, first 64 entries", "videos": out}, f, indent=0)
print(f"wrote {dst}: {len(out)} videos")
