"""Model of the d = 4096 quarter transform's stage 1 on the i8 matrix cores
(DESIGN.md section 14, item 5), checked against the VALU form kernels_n4k.hip
runs today. For quarter m0 and a = j1 + 32 j2, with s = psi^(2 m0 - 3),
c_b = 2^(120 b (2 m0 + 1)) and x_b[a] the ternary digit of coefficient a + 1024 b:
  old:  y[a] = s^a sum_b c_b x_b[a];  Y[j1][m1] = sum_j2 zeta^((2 m1 + 1) j2) y[j1 + 32 j2]
        Te[m1][j1] = Y[j1][m1] p1^((2 m1 + 1) j1)
  new:  Z''[m1][32 b + j2] = zeta^((2 m1 + 1) j2) s^(32 j2) c_b   (8 signed D8 byte planes)
        D[m1][j1] = sum_K Z''[m1][K] B[K][j1],  B[32 b + j2][j1] = x_b[j1 + 32 j2]
        Te[m1][j1] = D[m1][j1] (p1^((2 m1 + 1) j1) s^j1)
The D8 planes recombine exactly (sum_t 256^t D_t), so both give the same Te.
usage: python tools/ntt4096_mx_model.py"""
import random

import numpy as np

P = 2**64 - 2**32 + 1
d = 4096
psi = pow(7, (P - 1) // (2 * d), P)
p1 = pow(psi, 4, P)
zeta = pow(p1, 32, P)
assert zeta == pow(2, 39, P)


def d8(x):
    """frag.hpp d8: signed base-256 digits of x mod p (as int8)"""
    t = x if x <= 0x7F7F7F7F7F7F7F7F else x + 0xFFFFFFFF
    dd = ((t + 0x8080808080808080) % 2**64) ^ 0x8080808080808080
    out = [((dd >> (8 * b)) & 0xFF) for b in range(8)]
    return [v - 256 if v >= 128 else v for v in out]


def main():
    rng = random.Random(5)
    for m0 in range(4):
        s = pow(psi, (2 * m0 - 3) % 8192, P)
        c = [pow(2, (120 * b * (2 * m0 + 1)) % 192, P) for b in range(4)]
        # one ternary plane of a 4096-coefficient element
        x = [rng.choice((-1, 0, 0, 1)) for _ in range(4096)]
        xb = lambda b, a: x[a + 1024 * b]
        # old
        y = [pow(s, a, P) * sum(c[b] * xb(b, a) for b in range(4)) % P for a in range(1024)]
        Te_old = [[sum(pow(zeta, (2 * m1 + 1) * j2, P) * y[j1 + 32 * j2] for j2 in range(32)) % P
                   * pow(p1, (2 * m1 + 1) * j1, P) % P for j1 in range(32)] for m1 in range(32)]
        # new: D8 planes of Z'' and the ternary B, int64 products per plane
        Z = [[pow(zeta, (2 * m1 + 1) * j2, P) * pow(s, 32 * j2, P) % P * c[b] % P
              for b in range(4) for j2 in range(32)] for m1 in range(32)]
        planes = np.array([[d8(Z[m1][k]) for k in range(128)] for m1 in range(32)], dtype=np.int64)  # [m1][K][t]
        B = np.array([[xb(k // 32, j1 + 32 * (k % 32)) for j1 in range(32)] for k in range(128)], dtype=np.int64)
        Dt = [planes[:, :, t] @ B for t in range(8)]  # [m1][j1] per plane, |.| <= 128 * 128
        assert max(int(np.abs(D).max()) for D in Dt) <= 128 * 128
        Te_new = [[sum(int(Dt[t][m1][j1]) * 256**t for t in range(8)) % P
                   * (pow(p1, (2 * m1 + 1) * j1, P) * pow(s, j1, P) % P) % P for j1 in range(32)] for m1 in range(32)]
        assert Te_new == Te_old, m0
        print(f"m0 = {m0}: new stage 1 == old stage 1 on all 32 x 32 outputs")


if __name__ == "__main__":
    main()
