"""Non-local-means checker for nori_denoise (TEST INFRASTRUCTURE ONLY: only
tests/ may import it; the product path never calls it).

The filter of denoiser/denoiser.py:22-66, written here per pixel p = (i, j)
of an H x W image I with grey variance V, offsets s = (a, b) in [-r, r]^2
and box half-width h = f - 1:
  q_s(p)     = ((i - a) mod H, (j - b) mod W)               periodic neighbour
  dist_s(p)  = (|I(q) - I(p)|^2 - v1) / (1e-3 + k^2 v2)
                 script (mode 0): v1 = v2 = 2 V(q)  -- its d2() receives the
                 shifted variance and also reads the global one
                 textbook (mode 1): v1 = V(p) + min(V(p), V(q)), v2 = V(p) + V(q)
  patch_s(p) = window mean of dist_s over (2h+1)^2, terms outside the image = 0
  w_s(p)     = window mean of exp(-max(0, patch_s)), terms outside the image = 0
  out(p)     = sum_s w_s(p) I(q_s(p)) / sum_s w_s(p)
in float64; window means come from summed-area tables of zero-padded arrays.

Parity status: unpinned by fixtures (the script needs OpenCV, absent here,
and the reference holds no denoiser outputs).
"""
import numpy as np


def window_mean(a, h):
    """Mean over the (2h+1)^2 window centred on each pixel, zero outside."""
    rows, cols = a.shape
    n = 2 * h + 1
    pad = np.zeros((rows + n, cols + n))
    pad[h + 1:h + 1 + rows, h + 1:h + 1 + cols] = a
    sat = pad.cumsum(axis=0).cumsum(axis=1)
    return (sat[n:, n:] - sat[:-n, n:] - sat[n:, :-n] + sat[:-n, :-n]) / (n * n)


def nlmeans(img, var, r=3, f=3, k=0.02, mode=0):
    I = np.asarray(img, np.float64)
    V = np.asarray(var, np.float64)
    rows, cols = V.shape
    ii = np.arange(rows)[:, None]
    jj = np.arange(cols)[None, :]
    num = np.zeros_like(I)
    den = np.zeros((rows, cols))
    for a in range(-r, r + 1):
        for b in range(-r, r + 1):
            qi, qj = (ii - a) % rows, (jj - b) % cols
            Iq, Vq = I[qi, qj], V[qi, qj]
            if mode == 0:
                v1 = v2 = 2.0 * Vq
            else:
                v1, v2 = V + np.minimum(V, Vq), V + Vq
            dist = (((Iq - I) ** 2).sum(axis=2) - v1) / (1e-3 + k * k * v2)
            w = window_mean(np.exp(-np.maximum(0.0, window_mean(dist, f - 1))), f - 1)
            num += w[..., None] * Iq
            den += w
    return num / den[..., None]
