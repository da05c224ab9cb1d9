"""CPU: register budget of the hot kernels, read from the built library's
gfx950 code objects (tools/kernel_regs.py; no GPU).

The ECS kernels sit at the 256-VGPR edge of two waves per SIMD: a harmless
looking source change once pushed ecs_exact_kernel<10> over it and cost 40 %
at cfg4.  Bar: the single-chain and chains ECS kernels for
n = 3, 5, 10, 15 keep 2 waves per SIMD with no VGPR spills; the MHRS search
keeps at least 4.  (n = 15 may spill 2 VGPRs: r06, measured faster.)
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.fixture(scope="module")
def regs(lib):
    import kernel_regs
    import phasetype_amd.build as B

    return kernel_regs.kernels(B.LIB)


@pytest.mark.parametrize("nt", [3, 5, 10, 15])
@pytest.mark.parametrize("kind", ["ecs_exact_kernelILi{nt}ELb0ELb0EE", "ecs_exact_kernelILi{nt}ELb0ELb1EE",
                                  "ecs_chains_kernelILi{nt}EE"])
def test_ecs_two_waves_no_spill(regs, nt, kind):
    key = kind.format(nt=nt)
    hits = {k: v for k, v in regs.items() if key in k}
    assert len(hits) == 1, (key, list(hits))
    (name, d), = hits.items()
    assert d["waves_per_simd"] >= 2, (name, d)
    # n = 15: two spilled VGPRs since r06's moveMass without register arrays,
    # which is faster anyway (cfg5 kernel -3.0 %, profiles/r06/movemass/)
    assert d["vgpr_spill"] <= (2 if nt == 15 else 0), (name, d)


@pytest.mark.parametrize("kind,ceiling", [("ecs_exact_kernelILi20ELb0ELb0EE", 43),
                                          ("ecs_exact_kernelILi20ELb0ELb1EE", 145),
                                          ("ecs_chains_kernelILi20EE", 43)])
def test_ecs_n20_spill_ceiling(regs, kind, ceiling):
    """n = 20 runs two waves per SIMD with some VGPRs spilled (faster than one
    wave without spills: cfg3 kernel 0.812 vs 0.865 ms, profiles/r05/cfg3/
    w1_ab_*.jsonl); the r04 counts are the ceiling, so the spills cannot grow
    unnoticed.  (The row kernel's 130 -> 145 in r06: its unit's Philox rounds
    unrolled, 142 spilled, cfg3 -1.4 % per sweep, profiles/r06/unroll/.)"""
    hits = {k: v for k, v in regs.items() if kind in k}
    assert len(hits) == 1, (kind, list(hits))
    (name, d), = hits.items()
    assert d["waves_per_simd"] >= 2 and d["vgpr_spill"] <= ceiling, (name, d)


def test_mhrs_search_occupancy(regs):
    hits = {k: v for k, v in regs.items() if "mhrs_search" in k}
    assert len(hits) >= 6 * 6  # 6 round widths x 6 compiled n
    for name, d in hits.items():
        assert d["waves_per_simd"] >= 4 and d["vgpr_spill"] == 0, (name, d)


@pytest.mark.parametrize("nt", [3, 5, 10, 15, 20])
def test_ecs_debug_instantiations(regs, nt):
    """Informational bound on the DEBUG=true ECS kernels (per-observation
    outputs; the parity tests run them, nothing times them): they may spill
    a few VGPRs (n = 15: 6, n = 20: 18 at r01, 51 at r03 after the absorb
    test moved to U den < exp(.)) but must not blow up."""
    key = f"ecs_exact_kernelILi{nt}ELb1ELb{int(0 < nt <= 16)}EE"
    hits = {k: v for k, v in regs.items() if key in k}
    assert len(hits) == 1, (key, list(hits))
    (name, d), = hits.items()
    assert d["vgpr_spill"] <= 96, (name, d)


def _ecs_dynamic_lds(n, env_k):
    """phasetype_amd/csrc/pht_kernels_impl.h smem_bytes_ecs: the parameter
    block's ECS prefix (Layout::necs doubles) + P's successor lists, the
    statistics and cursor, then the lane-interleaved envelope (x, y)."""
    nn = n * n
    necs = 7 * n + 4 * nn + 6 * n
    necs += necs & 1
    pbytes = necs * 8 + (((n + nn) * 4 + 15) & ~15)
    return ((pbytes + (n + 16) * 8 + (n + nn) * 4 + 4 + 4 + 15) & ~15) + 2 * env_k * 8 * 256


@pytest.mark.parametrize("nt,env_k", [(10, 15), (15, 13), (20, 13)])
def test_ecs_two_blocks_per_cu(regs, nt, env_k):
    """Two ECS blocks (two waves per SIMD) must fit one CU's 160 KB of LDS:
    until r04 the n = 15 and 20 kernels staged the whole parameter block with
    a 15-point envelope and ran ONE block per CU (DESIGN.md §0c,
    profiles/r04/ecs_lds/)."""
    key = f"ecs_exact_kernelILi{nt}ELb0ELb0EE"
    (name, d), = {k: v for k, v in regs.items() if key in k}.items()
    per_block = _ecs_dynamic_lds(nt, env_k) + int(d["lds_static"])
    assert 2 * per_block <= 160 * 1024, (name, per_block)
    assert d["waves_per_simd"] >= 2, (name, d)
