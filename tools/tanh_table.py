"""Coefficients of the float32 policy's tanh (lz_policy.hip tanh_tab, lz_oracle.c
orc_tanh_tab): 72 segments of width 1/8 over [0, 9), a degree-5 polynomial in
t = |x| - k/8 per segment (segment 0: t * q(t), so tanh(x) = x + O(x^3) keeps full
relative accuracy near 0), fitted in float64 by least squares on Chebyshev nodes
(relative error weighting), rounded to float32; evaluated by Horner in fmaf: max error
vs float64 tanh 1.01 ulp (was 1.11 ulp with 36 segments of degree 6).  (Round 2
before this: 36 segments of width 1/4, degree 6 -- one fma more per tanh.)  Prints the C
table (8 floats per segment: c0..c5, 0, 0) that both files embed; the kernel's packer
scales c_j by 8^-j (exact) so the kernel can run Horner in u = 8 t = fract(8 |x|)."""
import math

import numpy as np

W, DEG, XMAX = 0.125, 5, 9.0


def fit():
    nseg = int(math.ceil(XMAX / W))
    out = []
    for k in range(nseg):
        a, b = k * W, (k + 1) * W
        j = np.arange(4 * DEG + 40)
        xs = (a + b) / 2 + (b - a) / 2 * np.cos(np.pi * (j + 0.5) / len(j))
        t = xs - a
        if k == 0:
            V = np.vander(t, DEG, increasing=True)
            c = np.linalg.lstsq(V, np.tanh(xs) / xs, rcond=None)[0]
            c = np.concatenate([[0.0], c])
        else:
            y = np.tanh(xs)
            V = np.vander(t, DEG + 1, increasing=True)
            c = np.linalg.lstsq(V / y[:, None], np.ones_like(y), rcond=None)[0]
        out.append(np.concatenate([np.float32(c), np.zeros(7 - DEG, np.float32)]))
    return np.array(out, np.float32)


def main():
    tab = fit()
    print("/* tools/tanh_table.py: %d segments x 8 floats (c0..c5, 0, 0) */" % len(tab))
    for row in tab:
        print("    " + ", ".join(float(v).hex() + "f" if v != 0 else "0.0f" for v in row) + ",")


if __name__ == "__main__":
    main()
