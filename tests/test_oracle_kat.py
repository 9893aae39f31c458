"""Known-answer tests for the oracle's scalar rules.

These pin the CPU restatement against values derived by reading
CommonOptFunction.cpp:1548-1627 and NITI_Conv_Int8.cpp:255-307 -- the reference
holds no fixture for them (parity unpinned).
"""
import numpy as np
import pytest


@pytest.mark.parametrize("a,s,want", [
    (1000, 3, 125), (1001, 3, 125), (1002, 3, 126), (1004, 3, 126), (1007, 3, 126),
    (-1007, 3, -126), (101, 2, 25), (102, 2, 26), (103, 2, 25), (40000, 9, 79),
    (65536, 9, 127), (-200, 0, -127),
])
def test_psto_appendix_a(oracle, a, s, want):
    assert int(oracle.psto(np.array([a]), s)[0]) == want


@pytest.mark.parametrize("vals,want", [
    ([0], 0), ([1], 0), ([2], 1), ([3], 2), ([-128], 7), ([129], 8), ([65536], 16), ([65537], 17),
])
def test_range_estimate_appendix_a(oracle, vals, want):
    assert oracle.range_estimate(vals) == want
    assert oracle.range_estimate_libm(vals) == want


def test_range_estimate_int_equals_libm(oracle):
    rng = np.random.default_rng(17)
    for _ in range(200):
        e = int(rng.integers(0, 31))
        v = rng.integers(-(1 << e), (1 << e) + 1, size=int(rng.integers(1, 64)), dtype=np.int64)
        v = np.clip(v, -(2**31 - 1), 2**31 - 1).astype(np.int32)
        assert oracle.range_estimate(v) == oracle.range_estimate_libm(v)
    for k in range(1, 31):
        for d in (-1, 0, 1):
            v = np.array([(1 << k) + d], np.int32)
            assert oracle.range_estimate(v) == oracle.range_estimate_libm(v)


def test_fwd_shift_branches(oracle):
    # max|acc| = 128 -> bw 7, shift 0: raw cast, 128 wraps to -128
    y, inc = oracle.requant_fwd(np.array([128, -5, 3], np.int32))
    assert inc == 0 and y.tolist() == [-128, -5, 3]
    # max|acc| = 200 -> bw 8, shift 1: PSTO(2), exponent + 2
    acc = np.array([200, -103, 101], np.int32)
    y, inc = oracle.requant_fwd(acc)
    assert inc == 2 and y.tolist() == oracle.psto(acc, 2).tolist() == [50, -25, 25]
    # shift > 1
    acc = np.array([40000, -1007, 0], np.int32)
    y, inc = oracle.requant_fwd(acc)
    assert inc == 16 - 7 and y.tolist() == oracle.psto(acc, 9).tolist()


def test_wgrad_rule(oracle):
    q, bw = oracle.requant_wgrad(np.zeros(5, np.int32))
    assert bw == 0 and not q.any()
    # bw 2 -> shift 0 -> identity (clip)
    q, bw = oracle.requant_wgrad(np.array([4, -3, 1], np.int32))
    assert bw == 2 and q.tolist() == [4, -3, 1]
    # max|acc| == 2 -> bw 1 -> shift -1: the reference's 1<<-1; executed on x86
    # (count & 31 -> 1<<31) the quotient is 0 and the rounding term gives sign(acc)
    q, bw = oracle.requant_wgrad(np.array([2, -1, 0], np.int32))
    assert bw == 1 and q.tolist() == [1, -1, 0]
    # max|acc| == 1 -> bw 0 -> zeros
    q, bw = oracle.requant_wgrad(np.array([1, -1, 0], np.int32))
    assert bw == 0 and q.tolist() == [0, 0, 0]
    # |g| <= 4 in general
    acc = np.random.default_rng(1).integers(-10**6, 10**6, 1000).astype(np.int32)
    q, bw = oracle.requant_wgrad(acc)
    assert np.abs(q.astype(int)).max() <= 4


def test_matmul_rule_negative_shifts(oracle):
    # bw 2 -> shift -1 -> sign(acc); bw 1 -> shift -2 -> zeros (x86 execution of the UB)
    q, bw = oracle.requant_matmul(np.array([3, -2, 1], np.int32))
    assert bw == 2 and q.tolist() == [1, -1, 1]
    q, bw = oracle.requant_matmul(np.array([2, -1, 0], np.int32))
    assert bw == 1 and q.tolist() == [0, 0, 0]


def test_psto_matches_formula(oracle):
    """Vectorised numpy restatement of :1595-1627 for shift >= 1."""
    rng = np.random.default_rng(3)
    a = rng.integers(-(1 << 24), 1 << 24, 5000).astype(np.int64)
    for s in range(1, 20):
        q = np.trunc(a / (1 << s)).astype(np.int64)
        prob = np.abs(a - q * (1 << s))
        h = s // 2
        qp = prob // (1 << h)
        pr = prob - qp * (1 << h)
        if s % 2 == 1:
            pr = pr * 2
        out = np.clip(q + (qp > pr) * np.sign(a), -127, 127)
        assert (oracle.psto(a.astype(np.int32), s) == out).all(), s


def test_maxpool_grad_ref806_walk(oracle):
    """NITI_DSPMaxPoolGradRef_Int8.cpp:36-88 on one 2x2 window over a 128-byte plane: dy goes to the
    first position (ky outer, kx inner) whose x equals y; the window's other positions get 0."""
    x = np.zeros((2, 2, 1, 128), np.int8)
    x[1, 0, 0, :] = 5
    x[0, 1, 0, 3] = 5
    y = np.full(128, 5, np.int8)
    dy = np.arange(128, dtype=np.int8)
    r = oracle.maxpool_grad_ref806(x, y, dy, np.full((2, 2, 1, 128), 9, np.int8)).reshape(4, 128)
    assert (r[0] == 0).all() and r[1][3] == 3 and (np.delete(r[1], 3) == 0).all()
    assert r[2][3] == 0 and (np.delete(r[2], 3) == np.delete(dy, 3)).all() and (r[3] == 0).all()
    # a plane tail (bc % 128) is never visited: those bytes keep their value
    x2 = np.zeros((2, 2, 1, 130), np.int8)
    r2 = oracle.maxpool_grad_ref806(x2, np.zeros(200, np.int8), np.ones(200, np.int8),
                                    np.full((2, 2, 1, 130), 9, np.int8)).reshape(-1)
    assert (r2[128:130] == 9).all() and r2[0] == 1


def test_residual_rule(oracle):
    """The residual add / gradient sum rule of oracle/niti_resnet_ref.py (this library's: the
    reference's NITI_Eltwise_Int8.cpp:20-28 is a stub)."""
    import niti_resnet_ref as RR
    a = np.array([100, -100, 1, -1], np.int8)
    b = np.array([3, -3, 127, -128], np.int8)
    z, e = RR.residual_add(a, 2, b, 0)          # a has the larger exponent: a * 4 + b, exponent 0
    assert e == 0 and z.tolist() == [403, -403, 131, -132]
    z, e = RR.residual_add(a, 0, b, 30)         # gap 30: b * 2^23 + (a >> 7) (floor), exponent 7
    assert e == 7 and z.tolist() == [3 * 2**23 + 0, -3 * 2**23 - 1, 127 * 2**23 + 0, -128 * 2**23 - 1]
    z, e = RR.residual_add(a, -4, b, -4)        # ties: a is hi, exponent unchanged
    assert e == -4 and z.tolist() == [103, -103, 128, -129]
