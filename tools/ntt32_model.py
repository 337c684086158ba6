# model of the 32x32 negacyclic NTT for d = 1024 over Goldilocks
P = 2**64 - 2**32 + 1
d = 1024
psi = pow(7, (P - 1) // (2 * d), P)
assert pow(psi, 1024, P) == P - 1
zeta = pow(psi, 32, P); w32 = pow(psi, 64, P)
def e2(e): return pow(2, e % 192, P)
assert zeta == e2(39), (zeta, [e for e in range(192) if e2(e) == zeta])
assert w32 == e2(78)
brv5 = lambda i: int(f"{i:05b}"[::-1], 2)
import random
random.seed(1)
x = [random.randrange(P) for _ in range(d)]
ref = [sum(x[j] * pow(psi, (2 * m + 1) * j, P) for j in range(d)) % P for m in range(d)]

def neg_ct32(a, z):  # merged CT, natural in, bit-reversed out; z = 64th root (zeta)
    a = a[:]; k = 0; ln = 16
    while ln >= 1:
        for st in range(0, 32, 2 * ln):
            k += 1
            t_exp = brv5(k)
            for j in range(st, st + ln):
                t = a[j + ln] * pow(z, t_exp, P) % P
                a[j + ln] = (a[j] - t) % P
                a[j] = (a[j] + t) % P
        ln //= 2
    return a
def cyc_dif32(a, w):
    a = a[:]; ln = 16
    while ln >= 1:
        for st in range(0, 32, 2 * ln):
            for j in range(ln):
                u, v = a[st + j], a[st + j + ln]
                a[st + j] = (u + v) % P
                a[st + j + ln] = (u - v) * pow(w, j * (16 // ln), P) % P
        ln //= 2
    return a
def neg_gs32(a, z):  # transpose of neg_ct32 network: levels reversed, (a,b)->(a+b, t(a-b))
    a = a[:]
    # replay forward schedule to know twiddles
    sched = []; k = 0; ln = 16
    while ln >= 1:
        for st in range(0, 32, 2 * ln):
            k += 1; sched.append((ln, st, brv5(k)))
        ln //= 2
    for ln, st, te in reversed(sched):
        for j in range(st, st + ln):
            u, v = a[j], a[j + ln]
            a[j] = (u + v) % P
            a[j + ln] = (u - v) * pow(z, te, P) % P
    return a
# forward: lane j1 holds x[j1 + 32 j2] at register j2
Y = [neg_ct32([x[j1 + 32 * j2] for j2 in range(32)], zeta) for j1 in range(32)]  # Y[j1][i] -> m1 = brv5(i)
T = [[pow(psi, (2 * brv5(i) + 1) * j1, P) for i in range(32)] for j1 in range(32)]
Yp = [[Y[j1][i] * T[j1][i] % P for i in range(32)] for j1 in range(32)]
# transpose: lane m1 holds Yp[j1][m1] for j1 = 0..31 (register j1)
V = [[Yp[j1][brv5_inv] for j1 in range(32)] for brv5_inv in [None]*0] if False else None
out = [0] * d
for m1 in range(32):
    i_of_m1 = brv5(m1)  # register index in stage-1 output holding m1
    col = [Yp[j1][i_of_m1] for j1 in range(32)]
    Z = cyc_dif32(col, w32)  # Z[i] -> m2 = brv5(i)
    for i in range(32):
        out[m1 + 32 * brv5(i)] = Z[i]
assert out == ref, "forward mismatch"
print("forward ok")
# inverse: lane m1 holds X[m1 + 32 m2] at register m2
X = ref
dinv = pow(d, P - 2, P)
zi, wi = pow(zeta, P - 2, P), pow(w32, P - 2, P)
Zs = [cyc_dif32([X[m1 + 32 * m2] for m2 in range(32)], wi) for m1 in range(32)]  # reg i -> j1 = brv5(i)
Ti = [[dinv * pow(psi, (P - 1) - ((2 * m1 + 1) * brv5(i)) % (P - 1), P) % P for i in range(32)] for m1 in range(32)]
Zp = [[Zs[m1][i] * Ti[m1][i] % P for i in range(32)] for m1 in range(32)]
xr = [0] * d
for j1 in range(32):
    ij = brv5(j1)
    col = [Zp[brv5(i)][ij] for i in range(32)]  # register i holds m1 = brv5(i)
    r = neg_gs32(col, zi)
    for j2 in range(32):
        xr[j1 + 32 * j2] = r[j2]
assert xr == x, "inverse mismatch"
print("inverse ok")
# print twiddle exponents (base 2) for code generation
def lg(v):
    for e in range(192):
        if e2(e) == v: return e
sched = []; k = 0; ln = 16
while ln >= 1:
    for st in range(0, 32, 2 * ln):
        k += 1; sched.append((ln, st, (39 * brv5(k)) % 192))
    ln //= 2
print("ct exps", [s[2] for s in sched])
