# model of the d = 4096 negacyclic NTT as a radix-4 DIF split into four
# 1024-point negacyclic NTTs (the n32 register transform), kernels_n4k.hip:
#   X[m0 + 4 m1] = NTT1024_{psi^4}(y_m0)[m1]
#   y_m0[a]      = psi^((2 m0 - 3) a) * sum_b x[a + 1024 b] w8^(b (2 m0 + 1)),  w8 = psi^1024
# and the inverse  x[a + 1024 b] = 1/4 sum_m0 w8^(-b (2 m0 + 1)) psi^(-(2 m0 - 3) a) INTT1024(X[m0 + 4 .])[a]
import random
P = 2**64 - 2**32 + 1
d = 4096
psi = pow(7, (P - 1) // (2 * d), P)
assert pow(psi, d, P) == P - 1
w8 = pow(psi, 1024, P)
e8 = [e for e in range(192) if pow(2, e, P) == w8]
print("w8 = 2^%d" % e8[0])
psi4 = pow(psi, 4, P)
assert psi4 == pow(7, (P - 1) // 2048, P)  # the d = 1024 psi
def ntt(x, ps):
    n = len(x)
    return [sum(x[j] * pow(ps, (2 * m + 1) * j, P) for j in range(n)) % P for m in range(n)]
def intt(X, ps):
    n = len(X); ni = pow(n, P - 2, P); pi = pow(ps, P - 2, P)
    return [ni * sum(X[m] * pow(pi, (2 * m + 1) * j, P) for m in range(n)) % P for j in range(n)]
# small check with the same structure at d = 16 (4 x 4) to keep it fast, then the real exponents
for dd in (16, 64):
    ps = pow(7, (P - 1) // (2 * dd), P); q = dd // 4; w = pow(ps, q, P)
    x = [random.randrange(P) for _ in range(dd)]
    ref = ntt(x, ps)
    out = [0] * dd
    for m0 in range(4):
        y = [pow(ps, ((2 * m0 - 3) * a) % (2 * dd), P) * sum(x[a + q * b] * pow(w, b * (2 * m0 + 1), P) for b in range(4)) % P
             for a in range(q)]
        Y = ntt(y, pow(ps, 4, P))
        for m1 in range(q): out[m0 + 4 * m1] = Y[m1]
    assert out == ref, dd
    back = [0] * dd
    for m0 in range(4):
        y = intt([ref[m0 + 4 * m1] for m1 in range(q)], pow(ps, 4, P))
        for a in range(q):
            z = y[a] * pow(ps, (-(2 * m0 - 3) * a) % (2 * dd), P) % P
            for b in range(4):
                back[a + q * b] = (back[a + q * b] + z * pow(4, P - 2, P) * pow(w, (-b * (2 * m0 + 1)) % 8, P)) % P
    assert back == x, dd
print("radix-4 DIF split ok")
