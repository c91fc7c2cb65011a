"""numpy restatement of prim.SSIM (internal/prim/ssim.go:27-182) -- TEST
INFRASTRUCTURE (checker for rt_ssim_rgba8; only tests/ import it).

Per window the ops follow ssim.go's order exactly (k1 = x offset outer, k2 = y
offset inner; means as sum(v * w); variances as sum(w * d^2) and
sum(w * d1 * d2)), vectorised over all windows at once, so per-window values
are bit-identical to a scalar restatement. Window sums: columns (x) summed in
y order, then columns in x order (the reference adds columns in goroutine
completion order). Gaussian weights use math.exp (Go's math.Exp may differ in
the last bit; parity tolerance 1e-12 relative).
"""
import math

import numpy as np

K = 11


def gaussian_kernel():
    """makeGaussianKernel (ssim.go:147-164)."""
    w = [0.0] * (K * K)
    center = (K - 1) / 2.0
    total = 0.0
    for i in range(K):
        for j in range(K):
            x = float(i) - center
            y = float(j) - center
            v = math.exp(-(x * x + y * y) / (2 * 1.5 * 1.5))
            w[i * K + j] = v
            total += v
    return [v / total for v in w]


def ssim(img1, img2):
    """SSIM of two uint8 [H, W, 3|4] frames; raises ValueError like the reference's errors."""
    a = np.asarray(img1)
    b = np.asarray(img2)
    if a.shape[:2] != b.shape[:2]:
        raise ValueError("images are not the same size")
    h, w = a.shape[:2]
    if w < K or h < K:
        raise ValueError("images are too small")
    nx, ny = w - K, h - K
    if nx == 0 or ny == 0:
        return float("nan")
    # [x][y] layout as convertImageToRGB builds it; RGBA() = v8 * 257 (0x101)
    A = [a[:, :, c].T.astype(np.float64) * 257.0 for c in range(3)]
    B = [b[:, :, c].T.astype(np.float64) * 257.0 for c in range(3)]
    kw = gaussian_kernel()
    m1 = [np.zeros((nx, ny)) for _ in range(3)]
    m2 = [np.zeros((nx, ny)) for _ in range(3)]
    for k1 in range(K):
        for k2 in range(K):
            wt = kw[k1 * K + k2]
            for c in range(3):
                m1[c] += A[c][k1:k1 + nx, k2:k2 + ny] * wt
                m2[c] += B[c][k1:k1 + nx, k2:k2 + ny] * wt
    v1 = [np.zeros((nx, ny)) for _ in range(3)]
    v2 = [np.zeros((nx, ny)) for _ in range(3)]
    v12 = [np.zeros((nx, ny)) for _ in range(3)]
    for k1 in range(K):
        for k2 in range(K):
            wt = kw[k1 * K + k2]
            for c in range(3):
                d1 = A[c][k1:k1 + nx, k2:k2 + ny] - m1[c]
                d2 = B[c][k1:k1 + nx, k2:k2 + ny] - m2[c]
                v1[c] += wt * (d1 * d1)
                v2[c] += wt * (d2 * d2)
                v12[c] += wt * d1 * d2
    c1, c2 = 429483.6225, 3865352.6025
    ch = []
    for c in range(3):
        num = (2 * m1[c] * m2[c] + c1) * (2 * v12[c] + c2)
        den = (m1[c] * m1[c] + m2[c] * m2[c] + c1) * (v1[c] + v2[c] + c2)
        ch.append(num / den)
    per_window = (ch[0] + ch[1] + ch[2]) / 3.0
    total = 0.0
    for x in range(nx):
        col = 0.0
        for v in per_window[x]:
            col += float(v)
        total += col
    return total / float(nx * ny)
