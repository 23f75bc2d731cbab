

def _tile_coords(b, nwg, tiles_m, tiles_n, xmap, xcds=8):
    """Python twin of loadgen.hip tile_coords (the device-side block -> tile map)."""
    xcd = b % xcds
    q, rem = divmod(nwg, xcds)
    wgid = (xcd * (q + 1) if xcd < rem else rem * (q + 1) + (xcd - rem) * q) + b // xcds
    if xmap & 0xFF:
        px, gm = xmap & 0xFF, (xmap >> 8) & 0xFF
        py = xcds // px
        bm, bn = tiles_m // px, tiles_n // py
        per = bm * bn
        x, l = divmod(wgid, per)
        g, r = divmod(l, gm * bn)
        gsize = min(bm - g * gm, gm)
        return (x // py) * bm + g * gm + r % gsize, (x % py) * bn + r // gsize, x
    per_group = 8 * tiles_n
    group = wgid // per_group
    first = group * 8
    gsize = min(tiles_m - first, 8)
    return first + (wgid % per_group) % gsize, (wgid % per_group) // gsize, None


def test_gemm_xcd_block_tile_map_is_a_bijection():
    """Every GEMM grid of the workload catalog (256x256 and 128x128 tiles) plus big lone shapes:
    the XCD-block order visits each output tile exactly once, keeps each XCD inside its own
    rectangle, and needs no more A + B strips per XCD than the GROUP_M order."""
    import pytest
    from k8s_gpu_scheduler_amd import _native
    h = _native.hip()
    if h is None:
        pytest.skip("HIP extension not built")
    from k8s_gpu_scheduler_amd.models import workloads as W
    shapes = {(o.M, o.N) for w in W.CATALOG.values() for o in w.ops if o.kind == "gemm"}
    shapes |= {(4096, 4096), (8192, 8192), (8192, 2048)}
    for M, N in sorted(shapes):
        for bt in (256, 128):
            tm_, tn_ = M // bt, N // bt
            nwg = tm_ * tn_
            xmap = h.pick_xcd_map(tm_, tn_)
            assert xmap == 0 or xmap >> 8 == 4
            seen, strips_new, strips_old = set(), {}, {}
            for b in range(nwg):
                m, n, x = _tile_coords(b, nwg, tm_, tn_, xmap)
                assert 0 <= m < tm_ and 0 <= n < tn_
                seen.add((m, n))
                if x is not None:
                    assert x == b % 8                     # each XCD stays in its rectangle
                s = strips_new.setdefault(b % 8, (set(), set()))
                s[0].add(m), s[1].add(n)
                m0, n0, _ = _tile_coords(b, nwg, tm_, tn_, 0)
                s = strips_old.setdefault(b % 8, (set(), set()))
                s[0].add(m0), s[1].add(n0)
            assert len(seen) == nwg, (M, N, bt)
            new = max(len(a) + len(c) for a, c in strips_new.values())
            old = max(len(a) + len(c) for a, c in strips_old.values())
            assert new <= old, (M, N, bt, new, old)
