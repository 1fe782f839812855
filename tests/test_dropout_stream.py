"""Statistics of the element-dropout keep stream (csrc/rp_common.h rp_keep8) on its bitwise restatement
(tests/test_kernels_gpu.py keep_mask, pinned to the kernels' bits by the GPU tests): each group of 8
elements draws one rp_hash word w0 and three MWC64X words seeded x = w0, c = w0 >> 1.  Over 2^22
elements the keep rate of every slot (idx & 7) is 1 - p within 4.5 sigma, and no two slots of a group
are correlated beyond 4.5 sigma — the seeding makes words 1..3 functions of w0, this checks that it
leaves them independent-looking decisions."""
import pytest
import torch

from tests.test_kernels_gpu import keep_mask


@pytest.mark.parametrize("p", [0.1, 0.5])
@pytest.mark.parametrize("seed", [12345, 0x9E3779B1])
def test_keep_rate_per_slot_and_pairwise_independence(p, seed):
    n = 1 << 22
    k = keep_mask(seed, torch.arange(n, dtype=torch.int64), p).view(-1, 8).float()
    g = k.shape[0]
    sigma = ((1 - p) * p / g) ** 0.5
    dev = ((k.mean(0) - (1 - p)) / sigma).abs()
    assert dev.max().item() < 4.5, dev.tolist()
    c = torch.corrcoef(k.T)
    off = c[~torch.eye(8, dtype=torch.bool)].abs() * g ** 0.5  # ~N(0, 1) under independence
    assert off.max().item() < 4.5, off.max().item()
