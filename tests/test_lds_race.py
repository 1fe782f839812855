"""CPU check of the built gfx950 code for the "fill overtakes read" LDS hazard (tests/lds_race.py).

Round 5 found it in the GEMM + LayerNorm exchange main loop: the compiler left a step's last ds_reads in
flight across a raw s_barrier, and another wave's untracked LDS-DMA fill of that stage could land first
(wrong dx in the repeat tests, one or two cases per run).  This test fails on the disassembly of that
build (tests/golden/lds_race_prefix_lnx.dis.gz, made by tests/golden/make_lds_race_fixture.sh) and passes
on the library built from HEAD, where every LDS-DMA kernel drains its reads before such a barrier — the
8-wave phased GEMMs to depth 2 (their stages are refilled two barriers after the last read)."""
import gzip
import os

import pytest

from . import lds_race

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "repurpose_amd", "_native", "librepurpose_amd.so")
FIXTURE = os.path.join(ROOT, "tests", "golden", "lds_race_prefix_lnx.dis.gz")


def test_checker_flags_the_prefix_exchange_kernels():
    text = gzip.open(FIXTURE, "rt").read()
    found = lds_race.scan(text)
    names = set(found)
    # all six exchange kernels of that build: the 128-row forward / backward and the 64- / 32-row ones
    assert any("gemm_lnx_fwd_kernel" in n for n in names), found
    assert any("gemm_lnx_bwd_kernel" in n for n in names), found
    assert sum("gemm_lnx64_kernel" in n for n in names) == 4, found
    assert all(len(v) >= 1 for v in found.values())


def test_checker_understands_waits_and_branches():
    """Hand-made listings: a drained read passes, an undrained one is flagged, a loop back-edge carries
    the state, a barrier with no LDS-DMA after it is not a hazard, depth 2 tolerates one barrier."""
    def lst(body):
        lines = ["0000000000001000 <k>:"]
        for i, ins in enumerate(body):
            lines.append(f"\t{ins:50s} // {0x1000 + 4 * i:012X}: 00000000")
        return "\n".join(lines)

    dma = "global_load_lds_dwordx4 v[0:1], off"
    ok = lst([dma, "ds_read_b128 v[2:5], v6", "s_waitcnt lgkmcnt(0)", "s_barrier", dma, "s_endpgm"])
    bad = lst([dma, "ds_read_b128 v[2:5], v6", "s_waitcnt lgkmcnt(1)", "s_barrier", dma, "s_endpgm"])
    assert lds_race.scan(ok) == {}
    assert lds_race.scan(bad) == {"k": [0xc]}
    # the read at the end of the loop body reaches the barrier at its top through the back-edge
    loop = lst([dma, "s_barrier", dma, "ds_read_b128 v[2:5], v6", "s_cbranch_scc1 -4 <k+0x4>", "s_endpgm"])
    assert lds_race.scan(loop) == {"k": [0x4]}
    # epilogue: no LDS-DMA reachable after the barrier
    epi = lst([dma, "s_waitcnt lgkmcnt(0)", "ds_read_b128 v[2:5], v6", "s_barrier", "ds_write_b32 v1, v2",
               "s_endpgm"])
    assert lds_race.scan(epi) == {}
    insns = lds_race.kernels(bad)["k"]
    assert lds_race.barriers_with_reads_in_flight(insns, depth=2) == []
    two = lst([dma, "ds_read_b128 v[2:5], v6", "s_barrier", "s_barrier", dma, "s_endpgm"])
    assert lds_race.barriers_with_reads_in_flight(lds_race.kernels(two)["k"], depth=2) == [0xc]


def test_built_library_has_no_lds_read_in_flight_at_a_refill_barrier():
    if not os.path.exists(LIB):
        pytest.skip("librepurpose_amd.so not built (make)")
    text = lds_race.disassemble(LIB)
    ks = lds_race.kernels(text)
    assert len(ks) > 100 and sum(lds_race.uses_lds_dma(v) for v in ks.values()) > 30
    assert lds_race.scan(text) == {}
