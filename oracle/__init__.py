"""TEST INFRASTRUCTURE ONLY — CPU restatement ("oracle") of the Repurpose hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything under ``oracle/``; the product package ``repurpose_amd`` never does.
The oracle is the *checker*, never the thing measured or shipped.

Pinning status: the reference cannot be imported in this
pipeline (denial recorded in SURVEY.md §8c). The restatement is pinned by the one
known-answer point recorded there (2-layer tri-modal model: 8,475,395 parameters,
``cls_loss`` 32.2317 under the recorded seed recipe) plus hand-derived Soft-NMS
known-answer cases. Everything beyond that is "parity unpinned" against the reference
itself and pinned only against this restatement.
"""
