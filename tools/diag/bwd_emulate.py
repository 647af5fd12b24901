"""Exact host emulation (fractions) of the device backward recurrence at 3x3, to see which shape deviates."""
import os, sys
from fractions import Fraction
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import maxent_oracle as O

def rnd(q):  # round an exact Fraction to nearest double (ties to even) via float()
    return float(q)

def fma(a, b, c):
    return rnd(Fraction(a) * Fraction(b) + Fraction(c))

size, n = 3, 9
P = O.icy_gridworld_table(size, 0.2)
s_ = np.arange(n); x, y = s_ % size, s_ // size
def nbr(s, k):
    X, Y = s % size, s // size
    return [s, s + 1 if X + 1 < size else s, s - 1 if X > 0 else s, s + size if Y + 1 < size else s, s - size if Y > 0 else s][k]
def valid(s, k):
    X, Y = s % size, s // size
    return [True, X + 1 < size, X > 0, Y + 1 < size, Y > 0][k]
rv = np.zeros((4, 5, n))
for s in range(n):
    for k in range(5):
        if valid(s, k):
            for a in range(4):
                rv[a, k, s] = P[s, nbr(s, k), a]
bw = np.zeros((5, n))
for s in range(n):
    for k in range(5):
        acc = 0.0
        for a in range(4):
            acc = acc + rv[a, k, s]
        bw[k, s] = acc
er = float(np.exp(1.0))
zs = [0.0] * n; zs[n - 1] = 1.0
for it in range(2 * n - 1):
    new = []
    for s in range(n):
        acc = 0.0
        for k in range(5):
            acc = fma(bw[k, s], zs[nbr(s, k)], acc)
        new.append(er * acc)
    zs = new
pi = np.zeros((n, 4))
for s in range(n):
    za = []
    for a in range(4):
        acc = 0.0
        for k in range(5):
            acc = fma(rv[a, k, s], zs[nbr(s, k)], acc)
        za.append(er * acc)
    zsum = 0.0
    for v in za: zsum += v
    pi[s] = [v / zsum for v in za]
np.save("/tmp/pi_emul.npy", pi)
print(pi[2])
