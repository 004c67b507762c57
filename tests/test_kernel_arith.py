"""Host checks of the integer identities round 5's kernels rely on (CPU, numpy): each device formula,
restated here operation for operation, against the plain test it replaced.  They pin the arithmetic
(overflow, the none label, negative 'seen', zero operands); the kernels themselves are pinned by the GPU
parity suites.

  * the candidate mask in integer arithmetic (sweep_sparse.hpp SP_VMASK, sweep_tile.hpp ST_GVMASK):
    d = min over {none, own, earlier slots} of (label ^ that); keep = bit 31 of (d | -d) and of
    (seen - lc) | ~interior -- against sweep_sparse.hpp's compare form;
  * the quad tiles' per-lane split of the same test (ST_QVMASK: lane r decides slots r and r + 4);
  * the Jacobi scan's list decision (sweep_sparse.hpp sp_any_scan): the seven keep words
    ~(d - 1) & ((seen - lc) | ~interior) OR-ed together, bit 31 = "the mask is non-zero";
  * the band's box coordinates by float reciprocal plus one correction (sdfgen_hip.hip BAND_FDIV);
  * the band's wave-wide search for a pair's triangle (sdfgen_hip.hip band_wq) against find_q.
"""
import numpy as np
import pytest

LBL_BITS = 27
LBL_MASK = (1 << LBL_BITS) - 1
U32 = np.uint32


def _rand_words(rng, n):
    """Low words of 7 upwind neighbours and the own cell: labels from a small pool (duplicates and the
    own label are common), the none label, stamps 0..16."""
    pool = rng.integers(0, 40, size=n)
    lab = rng.integers(0, 6, size=(n, 8)) + pool[:, None]
    lab = np.where(rng.random((n, 8)) < 0.12, LBL_MASK, lab).astype(np.int64)   # none
    lc = rng.integers(0, 17, size=(n, 8)).astype(np.int64)
    return ((lc << LBL_BITS) | lab).astype(U32)   # [:, :7] neighbours, [:, 7] own


def _mask_compare(w, seen, interior):
    """sweep_sparse.hpp sp_mask_w, compare form."""
    lab = np.where((w & LBL_MASK) == LBL_MASK, -1, (w & LBL_MASK).astype(np.int64))
    lc = (w >> LBL_BITS).astype(np.int64)
    ct0 = lab[:, 7]
    f = np.zeros(len(w), dtype=np.int64)
    for q in range(7):
        t = lab[:, q]
        skip = (t < 0) | (t == ct0)
        for r in range(q):
            skip |= lab[:, r] == t
        skip |= interior & (lc[:, q] <= seen[q])
        f |= (~skip).astype(np.int64) << q
    return f


def _keep_bit31(d, seen_q, lc_q, itr):
    d = d.astype(U32)
    nz = d | (U32(0) - d)
    s = (np.int64(seen_q) - lc_q.astype(np.int64)).astype(np.int64).astype(U32)   # two's complement, as the kernel
    return ((nz & (s | ~itr)) >> U32(31)).astype(np.int64)


def _mask_arith(w, seen, interior):
    """SP_VMASK / ST_GVMASK."""
    rl = (w & U32(LBL_MASK)).astype(U32)
    lc = (w >> U32(LBL_BITS)).astype(np.int64)
    itr = np.where(interior, U32(0xFFFFFFFF), U32(0)).astype(U32)
    f = np.zeros(len(w), dtype=np.int64)
    for q in range(7):
        x = rl[:, q]
        d = np.minimum(x ^ U32(LBL_MASK), x ^ rl[:, 7])
        for r in range(q):
            d = np.minimum(d, x ^ rl[:, r])
        f |= _keep_bit31(d, seen[q], lc[:, q], itr) << q
    return f


def _mask_quad(w, seen, interior):
    """ST_QVMASK: lane r of the quad decides slots r and r + 4 (lane 3: slot 3 only), OR over the quad."""
    rl = (w & U32(LBL_MASK)).astype(U32)
    lc = (w >> U32(LBL_BITS)).astype(np.int64)
    itr = np.where(interior, U32(0xFFFFFFFF), U32(0)).astype(U32)
    own = rl[:, 7]
    ones, zero = U32(0xFFFFFFFF), U32(0)
    f = np.zeros(len(w), dtype=np.int64)
    for qr in range(4):
        m1, m2, m3 = (ones if qr < 1 else zero), (ones if qr < 2 else zero), (ones if qr < 3 else zero)
        xa, xb = rl[:, qr], rl[:, qr + 4 if qr < 3 else 6]
        la, lb = lc[:, qr], lc[:, qr + 4 if qr < 3 else 6]
        sa, sb = seen[qr], seen[qr + 4 if qr < 3 else 6]
        da = np.minimum(np.minimum(xa ^ U32(LBL_MASK), xa ^ own), (xa ^ rl[:, 0]) | m1)
        da = np.minimum(da, np.minimum((xa ^ rl[:, 1]) | m2, (xa ^ rl[:, 2]) | m3))
        db = np.minimum(np.minimum(xb ^ U32(LBL_MASK), xb ^ own), np.minimum(xb ^ rl[:, 0], xb ^ rl[:, 1]))
        db = np.minimum(db, np.minimum(np.minimum(xb ^ rl[:, 2], xb ^ rl[:, 3]),
                                       np.minimum((xb ^ rl[:, 4]) | m1, (xb ^ rl[:, 5]) | m2)))
        ka = _keep_bit31(da, sa, la, itr)
        kb = _keep_bit31(db, sb, lb, itr) & (1 if qr < 3 else 0)
        f |= (ka << qr) | (kb << (qr + 4))
    return f


def _any_scan(w, seen, interior):
    """sp_any_scan: on the raw words, d from (x ^ y) & LBL_MASK, keep = ~(d - 1) & (s | ~itr), OR over q."""
    M = U32(LBL_MASK)
    itr = np.where(interior, U32(0xFFFFFFFF), U32(0)).astype(U32)
    acc = np.zeros(len(w), U32)
    for q in range(7):
        x = w[:, q]
        d = np.minimum((x ^ M) & M, (x ^ w[:, 7]) & M)
        for r in range(q):
            d = np.minimum(d, (x ^ w[:, r]) & M)
        s = (np.int64(seen[q]) - (x >> U32(LBL_BITS)).astype(np.int64)).astype(U32)
        acc |= ~(d - U32(1)) & (s | ~itr)
    return (acc >> U32(31)).astype(bool)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_candidate_mask_integer_form_equals_compare_form(seed):
    rng = np.random.default_rng(seed)
    w = _rand_words(rng, 20000)
    interior = rng.random(len(w)) < 0.8
    for seen in ([-1] * 7, [0, 3, 8, 16, 2, -1, 5], list(rng.integers(-1, 17, size=7))):
        ref = _mask_compare(w, seen, interior)
        assert np.array_equal(_mask_arith(w, seen, interior), ref)
        assert np.array_equal(_mask_quad(w, seen, interior), ref)
        assert np.array_equal(_any_scan(w, seen, interior), ref != 0)


def test_band_float_reciprocal_division_is_exact():
    """(int)((float)x * rcp(d)) with one signed correction equals x / d, x % d for every x, d <= 4096
    (a small triangle's band box), with rcp anywhere within 1 ulp of 1/d (v_rcp_f32)."""
    x = np.arange(0, 4097, dtype=np.int64)
    xf = x.astype(np.float32)
    for d in range(1, 4097):
        r = np.float32(1.0) / np.float32(d)
        for rc in (np.nextafter(r, np.float32(0)), r, np.nextafter(r, np.float32(1))):
            q = (xf * np.float32(rc)).astype(np.int64)   # float product rounded to nearest, truncated
            rem = x - q * d
            q = np.where(rem < 0, q - 1, np.where(rem >= d, q + 1, q))
            rem = np.where(rem < 0, rem + d, np.where(rem >= d, rem - d, rem))
            assert np.array_equal(q, x // d) and np.array_equal(rem, x % d), d


def _find_q(pre, nb, fl):
    """sdfgen_hip.hip find_q: last q in [0, nb) with pre[q] <= fl (binary search from BAND_BT / 2)."""
    q, step = 0, 32
    while step >= 1:
        if q + step < nb and pre[q + step] <= fl:
            q += step
        step >>= 1
    return q


def _band_wq(pl, F):
    """sdfgen_hip.hip band_wq for the 64 lanes of a wave at first pair F."""
    q0 = sum(1 for p in pl if p <= F) - 1
    bounds = [pl[x] for x in range(64) if pl[x] > F and pl[x] - F <= 63]
    return [q0 + sum(1 for b in bounds if F + lane >= b) for lane in range(64)]


def test_band_wave_search_equals_binary_search():
    rng = np.random.default_rng(7)
    for _ in range(400):
        nb = int(rng.integers(1, 65))
        vols = rng.choice([0, 0, 1, 2, 5, 27, 64, 90, 300, 4096], size=nb)
        pre = np.concatenate([[0], np.cumsum(vols)]).tolist()
        total = pre[nb]
        pl = [pre[x] if x < nb else 0xFFFFFFFF for x in range(64)]
        for F in range(0, total, 64 if total < 3000 else 509):
            got = _band_wq(pl, F)
            for lane in range(64):
                if F + lane < total:
                    assert got[lane] == _find_q(pre, nb, F + lane)
