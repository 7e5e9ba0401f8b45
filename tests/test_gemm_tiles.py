"""Tile list of the persistent phase-interleaved GEMM (``ops/csrc/gemm.hip::gemm8p_kernel``): a
line-for-line model of the kernel's (base, step, n_my) formula must hand every 256 x 256 output
tile to exactly one workgroup for any tile count and grid size (``grid = min(tiles, CUs)``), and in
the XCD-contiguous form (both multiples of 8) the tiles of XCD x (``blockIdx & 7``) must be exactly
the x-th eighth of the tile range, so the column tiles of a row block share an L2. CPU only; the
GPU twin is ``tests/test_wide_mlp.py::test_persistent_*`` (bit identity with one tile per
workgroup)."""

import pytest


def tile_lists(total: int, grid: int):
    """gemm8p_kernel's per-workgroup tile lists."""
    out = []
    for b in range(grid):
        if total % 8 == 0 and grid % 8 == 0:
            t8, g8, s = total >> 3, grid >> 3, b >> 3
            base, step = (b & 7) * t8 + s, g8
            n_my = (t8 - s + g8 - 1) // g8 if s < t8 else 0
        else:
            base, step = b, grid
            n_my = (total - b + grid - 1) // grid if b < total else 0
        out.append([base + j * step for j in range(max(n_my, 0))])
    return out


@pytest.mark.parametrize("total", [1, 3, 7, 8, 12, 64, 255, 256, 257, 822, 4096, 16384, 16388])
@pytest.mark.parametrize("cus", [256, 304, 80])
def test_every_tile_exactly_once(total, cus):
    grid = min(total, cus)
    lists = tile_lists(total, grid)
    flat = sorted(t for l in lists for t in l)
    assert flat == list(range(total))
    # balanced: workgroups differ by at most one tile
    sizes = [len(l) for l in lists]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("total,cus", [(16384, 256), (4096, 256), (1024, 304), (64, 256)])
def test_xcd_contiguous_ranges(total, cus):
    grid = min(total, cus)
    assert total % 8 == 0 and grid % 8 == 0
    lists = tile_lists(total, grid)
    t8 = total // 8
    for x in range(8):
        tiles = sorted(t for b, l in enumerate(lists) if b % 8 == x for t in l)
        assert tiles == list(range(x * t8, (x + 1) * t8))
    # the workgroups of one XCD walk its range in lock-step rounds of grid / 8 consecutive tiles
    g8 = grid // 8
    first_round = sorted(lists[b][0] for b in range(grid) if b % 8 == 0 and lists[b])
    assert first_round == list(range(0, min(g8, t8)))
