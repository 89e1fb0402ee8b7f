"""Support tables (avr_hulltab.cpp): for every large hull of the FeedingJaco scene, the table
lookup returns the same vertex as the full scan (first strictly largest projection, the
btConvexHullShape / oracle rule) for random, axis-aligned, cube-edge and cell-border directions.
Host-only: calls the C-ABI builder, emulates the device cell lookup (avr_kernel.hip `support`)
in float32 numpy."""
import numpy as np
import pytest

G = 16


def full_scan(V, D):
    """First index of the largest float32 projection, per direction (rows of D)."""
    P = (D[:, None, 0] * V[None, :, 0] + D[:, None, 1] * V[None, :, 1]) + D[:, None, 2] * V[None, :, 2]
    return np.argmax(P, axis=1)          # argmax returns the first maximum


def table_scan(V, cell, idx, D):
    out = np.empty(len(D), dtype=np.int64)
    for n, l in enumerate(D.astype(np.float32)):
        a = np.abs(l)
        mx = a.max()
        if not mx > 0:
            out[n] = 0
            continue
        if a[0] >= a[1] and a[0] >= a[2]:
            f, u, w = int(l[0] < 0), l[1], l[2]
        elif a[1] >= a[2]:
            f, u, w = 2 + int(l[1] < 0), l[0], l[2]
        else:
            f, u, w = 4 + int(l[2] < 0), l[0], l[1]
        sc = np.float32(0.5 * G) / mx
        i = min(G - 1, max(0, int(np.float32(u + mx) * sc)))
        j = min(G - 1, max(0, int(np.float32(w + mx) * sc)))
        o, c = cell[(f * G + i) * G + j]
        cand = idx[o:o + c]
        Vc = V[cand]
        p = (l[0] * Vc[:, 0] + l[1] * Vc[:, 1]) + l[2] * Vc[:, 2]
        out[n] = cand[int(np.argmax(p))]
    return out


def directions(rng, n):
    D = [rng.normal(size=(n, 3))]
    axes = np.eye(3)
    D.append(np.concatenate([axes, -axes]))
    e = []
    for sx in (-1, 1):
        for sy in (-1, 1):
            e += [[sx, sy, 0], [sx, 0, sy], [0, sx, sy], [sx, sy, 1], [sx, sy, -1]]
    D.append(np.array(e, dtype=np.float64))
    # points on cell borders of every face: u or v at a grid line
    g = -1 + 2 * np.arange(G + 1) / G
    uv = rng.uniform(-1, 1, size=(n // 4, 2))
    uv[: n // 8, 0] = rng.choice(g, n // 8)
    uv[n // 8:, 1] = rng.choice(g, n // 4 - n // 8)
    for ax in range(3):
        for s in (-1, 1):
            B = np.zeros((len(uv), 3))
            o = [a for a in range(3) if a != ax]
            B[:, ax] = s
            B[:, o[0]], B[:, o[1]] = uv[:, 0], uv[:, 1]
            D.append(B)
    return np.concatenate(D).astype(np.float32)


def big_hulls(A):
    sh = A['shape_hull'].reshape(-1, 4)
    for s in range(len(sh)):
        if A['shape_kind'][s] == 3 and sh[s, 1] > 64:
            yield s, A['hull_verts'][sh[s, 0]:sh[s, 0] + sh[s, 1]].astype(np.float32)


def test_tables_cover_every_large_hull(scene):
    A, _ = scene
    from avr import _lib
    hulls = list(big_hulls(A))
    assert len(hulls) == 13
    for s, V in hulls[:3]:
        cell, idx = _lib.hull_support_table(V, G)
        assert cell.shape == (6 * G * G, 2) and cell[:, 1].min() >= 1
        assert np.all(cell[:, 0] + cell[:, 1] <= len(idx))
        for o, c in cell:                 # ascending vertex order per cell
            assert np.all(np.diff(idx[o:o + c]) > 0)
        assert cell[:, 1].mean() < 0.05 * len(V)


@pytest.mark.parametrize('which', range(13))
def test_table_support_equals_full_scan(scene, which):
    A, _ = scene
    from avr import _lib
    s, V = list(big_hulls(A))[which]
    cell, idx = _lib.hull_support_table(V, G)
    rng = np.random.default_rng(100 + which)
    D = directions(rng, 2000)
    # also the directions the hull's own vertices define (flat-face ties)
    D = np.concatenate([D, V[rng.choice(len(V), 200)] - V.mean(0)]).astype(np.float32)
    ref = full_scan(V, D)
    got = table_scan(V, cell, idx, D)
    bad = np.nonzero(ref != got)[0]
    assert len(bad) == 0, (s, bad[:5], D[bad[:5]], ref[bad[:5]], got[bad[:5]])


def small_hulls(A, lo=8, hi=64):
    sh = A['shape_hull'].reshape(-1, 4)
    for s in range(len(sh)):
        if A['shape_kind'][s] == 3 and lo < sh[s, 1] <= hi:
            yield s, A['hull_verts'][sh[s, 0]:sh[s, 0] + sh[s, 1]].astype(np.float32)


def test_table_support_equals_full_scan_small_hulls(scene):
    """Every hull above AVR_TAB_MIN_NV (8) vertices gets a table (spoon, bowl, wheelchair and head
    VHACD pieces too): the lookup equals the full scan on each of them."""
    A, _ = scene
    from avr import _lib
    hulls = list(small_hulls(A))
    assert len(hulls) > 100
    rng = np.random.default_rng(7)
    for s, V in hulls:
        cell, idx = _lib.hull_support_table(V, G)
        assert cell[:, 1].min() >= 1
        D = np.concatenate([directions(rng, 160), V[rng.choice(len(V), 20)] - V.mean(0)]).astype(np.float32)
        ref = full_scan(V, D)
        got = table_scan(V, cell, idx, D)
        bad = np.nonzero(ref != got)[0]
        assert len(bad) == 0, (s, bad[:5], D[bad[:5]], ref[bad[:5]], got[bad[:5]])
