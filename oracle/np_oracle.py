"""Independent numpy restatement — TEST INFRASTRUCTURE ONLY.

Used to pin the C oracle and libdmt's host set-up without the reference (which cannot run
here; see oracle/oracle.py).  Everything here is written from the published guided-proposal
method (Schauer, van der Meulen & van Zanten 2017; Mider, Schauer & van der Meulen 2021),
not from the C code:

  * ``backward_filter_expm``: exact discrete backward filter of a linear auxiliary law with
    the transition computed by scipy's matrix exponential (Van Loan), the second
    implementation against which libdmt's series-based dmt_guiding_linear is checked;
  * ``ou1d_guiding``: closed-form H, F, c of a scalar OU auxiliary law with one Gaussian
    observation (the analytic KAT);
  * ``solve_segment_naive``: the guided Euler–Maruyama recursion and Girsanov sum in plain
    float64 numpy (no fma, left-to-right sum) — agrees with the canonical C restatement to
    rounding only;
  * ``gaussian_logpdf``: log N(v; m, S).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg as sla


def transition_expm(B, beta, at, h):
    """X_{t+h} = Phi X_t + mu + N(0, K) for dX = (BX + beta)dt + sigma dW (a = sigma sigma')."""
    d = B.shape[0]
    M = np.zeros((2 * d, 2 * d))
    M[:d, :d] = -B
    M[:d, d:] = at
    M[d:, d:] = B.T
    E = sla.expm(M * h)
    Phi = E[d:, d:].T
    K = Phi @ E[:d, d:]
    K = 0.5 * (K + K.T)
    A = np.zeros((d + 1, d + 1))
    A[:d, :d] = B
    A[:d, d] = beta
    E2 = sla.expm(A * h)
    mu = E2[:d, d]
    return Phi, mu, K


def backward_filter_expm(B, beta, at, t, HT, FT, cT):
    """(H, F, c) on grid t of rho~(t,x) = exp(-c - x'Hx/2 + F'x) for the linear law, given
    the terminal information at t[-1]."""
    B = np.atleast_2d(np.asarray(B, dtype=np.float64))
    d = B.shape[0]
    beta = np.asarray(beta, dtype=np.float64).reshape(d)
    at = np.atleast_2d(np.asarray(at, dtype=np.float64))
    n = len(t)
    Hs = np.empty((n, d, d))
    Fs = np.empty((n, d))
    cs = np.empty(n)
    H = np.atleast_2d(np.asarray(HT, dtype=np.float64))
    F = np.asarray(FT, dtype=np.float64).reshape(d)
    c = float(cT)
    Hs[-1], Fs[-1], cs[-1] = H, F, c
    for i in range(n - 2, -1, -1):
        Phi, mu, K = transition_expm(B, beta, at, t[i + 1] - t[i])
        S = np.linalg.inv(np.eye(d) + H @ K)
        Hh = S @ H
        Hh = 0.5 * (Hh + Hh.T)
        Fh = S @ F
        ch = c + 0.5 * math.log(abs(np.linalg.det(np.eye(d) + H @ K))) - 0.5 * Fh @ K @ F
        H = Phi.T @ Hh @ Phi
        H = 0.5 * (H + H.T)
        F = Phi.T @ (Fh - Hh @ mu)
        c = ch - Fh @ mu + 0.5 * mu @ Hh @ mu
        Hs[i], Fs[i], cs[i] = H, F, c
    return Hs, Fs, cs


def gaussian_logpdf(v, m, S):
    v = np.atleast_1d(v)
    m = np.atleast_1d(m)
    S = np.atleast_2d(S)
    k = v.size
    r = v - m
    return float(-0.5 * r @ np.linalg.solve(S, r) - 0.5 * k * math.log(2 * math.pi)
                 - 0.5 * math.log(np.linalg.det(S)))


def ou1d_guiding(theta, mu, sigma, T, t, v, Sig):
    """Closed form for dX = -theta(X - mu)dt + sigma dW observed as v ~ N(X_T, Sig):
    X_T | X_t = x ~ N(mu + e^{-theta s}(x - mu), sigma^2 (1 - e^{-2 theta s})/(2 theta))."""
    s = T - np.asarray(t, dtype=np.float64)
    ph = np.exp(-theta * s)
    var = sigma ** 2 * (1 - np.exp(-2 * theta * s)) / (2 * theta) + Sig
    # log N(v; mu + ph (x - mu), var) = -(v - mu(1-ph) - ph x)^2/(2 var) - ...
    H = ph ** 2 / var
    m0 = mu * (1 - ph)
    F = ph * (v - m0) / var
    c = (v - m0) ** 2 / (2 * var) + 0.5 * np.log(2 * math.pi * var)
    return H, F, c


def drift(model, theta, x):
    if model == 0:
        d = len(x)
        Th = np.asarray(theta[: d * d]).reshape(d, d)
        mu = np.asarray(theta[9: 9 + d])
        return -Th @ (x - mu)
    if model == 1:
        ie, s, g, b = theta[:4]
        y, v = x
        return np.array([(y - y ** 3 - v + s) * ie, g * y - v + b])
    s, r, b = theta[:3]
    return np.array([s * (x[1] - x[0]), x[0] * (r - x[2]) - x[1], x[0] * x[1] - b * x[2]])


def _unpack(p, d):
    M = np.zeros((d, d))
    k = 0
    for a in range(d):
        for b in range(a, d):
            M[a, b] = M[b, a] = p[k]
            k += 1
    return M


def solve_segment_naive(model, d, m, law, t, H, F, W, y1):
    """Guided Euler–Maruyama + Girsanov sum, plain numpy, left-to-right summation."""
    th = law[0:16]
    sg = np.asarray(law[16:16 + d * m]).reshape(d, m)
    a = sg @ sg.T
    Bt = np.asarray(law[31:31 + d * d]).reshape(d, d)
    beta = np.asarray(law[40:40 + d])
    hp = d * (d + 1) // 2
    da = _unpack(law[43:43 + hp], d)
    trace = law[50] != 0
    X = np.empty((len(t), d))
    x = np.array(y1, dtype=np.float64)
    X[0] = x
    ll = 0.0
    for i in range(len(t) - 1):
        dt = t[i + 1] - t[i]
        Hm = _unpack(H[i], d)
        r = F[i] - Hm @ x
        b = drift(model, th, x)
        bt = Bt @ x + beta
        G = (b - bt) @ r
        if trace:
            G -= 0.5 * np.sum(da * (Hm - np.outer(r, r)))
        ll += G * dt
        x = x + (b + a @ r) * dt + sg @ (W[i + 1] - W[i])
        X[i + 1] = x
    return X, ll
