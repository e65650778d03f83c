"""Statistics of the tower dropout counter hash (csrc/common.h ``row_key`` / ``pair_hash``,
replicated in numpy): keep rate, and no correlation between neighbouring units, unit pairs, rows
or steps. The kernels' bits are checked against this replica on the GPU
(tests/test_dropout_gpu.py); the reference draws independent Bernoulli masks per (t, stock, unit)
(`/root/reference/src/model.py:208-219`, nn.Dropout)."""
import numpy as np

M32 = 0xFFFFFFFF


def fmix32(h):
    h = np.asarray(h, dtype=np.uint64) & M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def dropout_key(seed, step, layer):
    inner = fmix32((step * 0x632BE59B + layer * 0x1B873593 + 0x5BD1E995) & M32)
    return int(fmix32(((seed * 0x9E3779B1) & M32) ^ int(inner)))


def keep(key, rows, width, p):
    r = np.asarray(rows, dtype=np.uint64)[:, None]
    rowmix = ((r * 0xCC9E2D51) & M32) ^ (r >> 16)
    n = np.arange(width, dtype=np.uint64)[None, :]
    rk = fmix32(np.uint64(key) ^ rowmix)
    h = (rk + (n >> 1) * 0x9E3779B9) & M32
    h ^= h >> 16
    h = (h * 0x7FEB352D) & M32
    h ^= h >> 15
    half = (h >> (16 * (n & 1))) & 0xFFFF
    return half >= int(p * 65536.0 + 0.5)


def _corr(a, b):
    a = a.astype(np.float64).ravel() - a.mean()
    b = b.astype(np.float64).ravel() - b.mean()
    return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))


def test_keep_rate_and_independence():
    p = 0.05
    rows = np.arange(200_000)
    k = keep(dropout_key(7, 3, 0), rows, 64, p)
    n = k.size
    rate = 1.0 - k.mean()
    assert abs(rate - p) < 4 * np.sqrt(p * (1 - p) / n), rate
    # per unit: every unit drops at the rate (no stuck or biased unit)
    per_unit = 1.0 - k.mean(axis=0)
    assert np.all(np.abs(per_unit - p) < 5 * np.sqrt(p * (1 - p) / k.shape[0])), per_unit
    bound = 5 / np.sqrt(k.shape[0])
    # the two halves of one pair hash, neighbouring pairs, neighbouring rows
    assert abs(_corr(k[:, 0::2], k[:, 1::2])) < bound
    assert abs(_corr(k[:, 0:-2:2], k[:, 2::2])) < bound
    assert abs(_corr(k[:-1], k[1:])) < bound
    # consecutive steps and layers draw independent masks
    k2 = keep(dropout_key(7, 4, 0), rows, 64, p)
    k3 = keep(dropout_key(7, 3, 1), rows, 64, p)
    assert abs(_corr(k, k2)) < bound and abs(_corr(k, k3)) < bound
