"""Host-side properties of clean_divergence's skewed (diagonal-major) layout
(fields2d.hip: skew_at, lex_skew_groups, lex_skew_floats, k_lex_gs_skew's
step count), restated here; no GPU.

Layout: rows in blocks of 64 (block m: rows 1 + 64 m + l), element
(m, d = j + l, l) at ((m DG + d // 4) 64 + l) 4 + d % 4, DG = ceil((nx + 63) / 4).
"""
import numpy as np
import pytest


def groups(nx):
    return (nx + 63 + 3) >> 2


def blocks(ny):
    return (ny - 2 + 63) >> 6


def skew_at(i, j, dg):
    m, l = (i - 1) >> 6, (i - 1) & 63
    d = j + l
    return ((m * dg + (d >> 2)) * 64 + l) * 4 + (d & 3)


@pytest.mark.parametrize("ny,nx", [(3, 3), (3, 50), (66, 30), (67, 64), (130, 66), (180, 600), (300, 67),
                                   (1030, 40), (2060, 66)])
def test_skew_layout_is_a_bijection_onto_its_slots(ny, nx):
    dg, nb = groups(nx), blocks(ny)
    n = nb * dg * 256  # lex_skew_floats
    i = np.arange(1, ny - 1)[:, None]
    j = np.arange(0, nx)[None, :]
    idx = skew_at(i, j, dg)
    assert idx.min() >= 0 and idx.max() < n
    assert np.unique(idx).size == idx.size  # injective: no two cells share a slot
    # a block's slots hold exactly its rows (the row beyond the last interior
    # row, zeroed by k_divergence_skew, stays inside the last block or past it)
    if (ny - 2) & 63:
        assert skew_at(ny - 1, nx - 1, dg) < n


@pytest.mark.parametrize("nx", [3, 4, 50, 61, 64, 65, 66, 67, 97, 100, 600, 1023, 1200, 4093])
def test_sweep_steps_cover_every_slot_of_a_block(nx):
    """k_lex_gs_skew stores its groups 0 .. DG - 1 in steps d = 0 .. 16 nq - 1;
    nq = ceil(DG / 4) chunks must reach lane 63's zero side column
    (d = nx + 62) and the whole last group (the r05 bug at nx = 50, 66: the
    earlier nq = ceil((nx + 62) / 16) stopped a group short)."""
    dg = groups(nx)
    nq = (dg + 3) >> 2
    assert 16 * nq >= 4 * dg >= nx + 63
    # lane 63's last interior column jmax = nx - 2 is at step jmax + 63
    assert 16 * nq > nx - 2 + 63

