"""The static agent layout of the exchange added in the final diffusion pass
(lens_amd.lattice.exchange_image, read by vk_stencil_ps.h ex_stage / ex_apply),
checked on CPU against a direct restatement: for every wave region (64 rows x one
96-column tile of the line-aligned pass) its agents in bin order, and per row the
lane masks by level, the second-cell bits and the first entry, so that a lane's
entries start after those of the lanes below it."""

import numpy as np
import pytest
import torch

from lens_amd.lattice import EX_CAP, EX_HALO, EX_LEVELS, EX_TILE_W, exchange_image


def _layout(rows, ny, n, seed, crowd=0):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, rows * ny, n)
    if crowd:
        b[:crowd] = (rows // 2) * ny + 17 + (np.arange(crowd) % 3)
    return np.sort(b, kind='stable').astype(np.int32)


@pytest.mark.parametrize('rows,ny,n,crowd', [(200, 300, 4000, 0), (128, 390, 9000, 0), (64, 50, 300, 0),
                                             (130, 200, 2000, 9)])
def test_exchange_image_matches_restatement(rows, ny, n, crowd):
    bins = _layout(rows, ny, n, 3, crowd)
    img = exchange_image(torch.from_numpy(bins), n, rows, ny, 2)
    tiles = (ny + EX_TILE_W - 1) // EX_TILE_W
    chunks = (rows + 63) // 64
    assert (img.tiles, img.rows) == (tiles, 64)
    inv = img.inv.numpy()
    xoff = img.xoff.numpy()
    hdr = img.xhdr.numpy().view(np.uint64).reshape(-1, 6)
    bad = img.xbad.numpy()
    assert sorted(a for a in inv.tolist() if a >= 0) == list(range(n))
    assert np.all(xoff % 2 == 0) and img.ximg.shape == (2, int(xoff[-1]) + 128)
    groups = {}
    for a, bb in enumerate(bins.tolist()):
        r, c = divmod(bb, ny)
        g = (r // 64) * tiles + c // EX_TILE_W
        groups.setdefault(g, []).append((a, r % 64, c - (c // EX_TILE_W) * EX_TILE_W + EX_HALO))
    for g in range(tiles * chunks):
        members = groups.get(g, [])
        assert xoff[g + 1] - xoff[g] == len(members) + (len(members) & 1)
        # bin order within the region, then padding
        assert inv[xoff[g]:xoff[g + 1]].tolist() == [a for a, _, _ in members] + [-1] * (len(members) & 1)
        expect_bad = len(members) > EX_CAP
        for lr in range(64):
            row = [(k, colt) for k, (a, rr, colt) in enumerate(members) if rr == lr]
            h = hdr[g * 64 + lr]
            if not row:
                assert all(int(x) == 0 for x in h[:5])
                continue
            e0 = row[0][0]
            assert int(h[5]) == e0
            masks = [0] * EX_LEVELS
            qbits = 0
            count = {}
            for kr, (k, colt) in enumerate(row):
                lane = colt // 2
                lvl = count.get(lane, 0)
                count[lane] = lvl + 1
                if lvl >= EX_LEVELS or kr >= 64:
                    expect_bad = True
                    continue
                masks[lvl] |= 1 << lane
                if colt % 2:
                    qbits |= 1 << kr
            if not expect_bad:
                assert [int(x) for x in h[:4]] == masks + [0] * (4 - EX_LEVELS)
                assert int(h[4]) == qbits
                # a lane's first entry = e0 + the entries of the lanes below it
                for lane in count:
                    below = sum(bin(m & ((1 << lane) - 1)).count('1') for m in masks)
                    first = next(kr for kr, (k, colt) in enumerate(row) if colt // 2 == lane)
                    assert below == first
        assert bool(bad[g]) == expect_bad, g
