"""The pixel-pool claim maps a launch-local pixel index q to (row, column) with an fp32 reciprocal
instead of an integer division (bdpt_kernels.hip pool_pixel): lr = (int)((float)q * rcp(W)),
then one correction step.  That is exact only if the estimate is never off by more than one row.
Check the bound here on the CPU, in fp32, with the reciprocal taken 1 ulp low, exact and 1 ulp
high (v_rcp_f32 is accurate to 1 ulp), for widths up to 2^16 - 1 and indices up to 2^28 (a launch
holds at most 2^28 samples, bdpt_host.cpp)."""
import numpy as np


def _rows(q, W, rcp):
    est = (q.astype(np.float32) * np.float32(rcp)).astype(np.float32)
    lr = est.astype(np.int64)                      # (int) truncation, est >= 0
    px = q - lr * W
    lr = np.where(px < 0, lr - 1, np.where(px >= W, lr + 1, lr))
    return lr


def test_reciprocal_row_estimate_needs_one_correction():
    rng = np.random.default_rng(7)
    widths = np.unique(np.concatenate([np.arange(1, 300), rng.integers(300, 65536, 400),
                                       [1921, 4097, 65535]]))
    for W in widths:
        W = int(W)
        top = min(1 << 28, W * 65535)
        q = np.unique(np.concatenate([rng.integers(0, top, 4000), np.arange(0, min(top, 4 * W)),
                                      (np.arange(1, min(65535, top // W)) * W)[-2000:] - 1,
                                      (np.arange(1, min(65535, top // W)) * W)[-2000:]]))
        q = q[(q >= 0) & (q < top)].astype(np.int64)
        r = np.float32(1.0) / np.float32(W)
        for rcp in (np.nextafter(r, np.float32(0)), r, np.nextafter(r, np.float32(1))):
            lr = _rows(q, W, rcp)
            assert np.array_equal(lr, q // W), W
