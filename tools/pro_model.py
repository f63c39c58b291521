#!/usr/bin/env python3
"""CPU model of the product's implicitly restarted Lanczos (ctx.cpp
ek_lanczos_fiedler: deflated u0, ncv 100, nev 1, restart floor ncv/5,
convergence checked every chunk) with FULL classical Gram-Schmidt per step
against PARTIAL reorthogonalisation (Simon's omega recurrence, as in
PROPACK's update_mu / compute_int): a step projects f' onto the basis only
when the estimated loss of orthogonality of the next vector exceeds a
threshold, and the step after it too.  Reports matvecs, projected steps,
max|V^T V - I| at every restart, lambda and the median split against a
tight reference vector.  Used to choose the device design.

usage: python tools/pro_model.py [hgr|lcc:MULT:SEED] [thresh ...]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
EPS = np.finfo(float).eps


def lanczos(A, n, thresh=None, m=100, tol=1e-10, keep_min=20, check=9, seed=1, est_beta=True, trace=False,
            restart_proj=False, eta=None):
    """thresh None: full CGS every step; else partial reorthogonalisation.
    eta: PROPACK's selective form (compute_int): a triggered step and its
    pair partner project only against the columns in the intervals around
    every |omega_j| > thresh where |omega| > eta (u0 when its omega > eta);
    the rule-forced steps (a run's first, the cycle's last, a lost estimate)
    against all.  Counts the column passes (cols_projected / cols_full)."""
    u0 = np.full(n, 1.0 / np.sqrt(n))
    rng = np.random.default_rng(seed)
    f = rng.random(n) - 0.5
    f -= f.mean()
    V = np.zeros((n, m + 1))
    alpha = np.zeros(m + 1)
    beta = np.zeros(m + 2)  # beta[i] = ||f_i||, f_i forms v_i
    beta[0] = np.linalg.norm(f)
    anorm_est = 0.0
    # omega[k]: estimated v_i^T v_k (k < i), last entry: v_i^T u0
    om_cur = np.zeros(m + 1)   # omega of v_i
    om_prev = np.zeros(m + 1)  # omega of v_{i-1}
    force = True
    forced = False
    k = 0
    matvecs = projected = restarts = 0
    ortho = []
    eps1 = EPS * np.sqrt(n)
    cols_projected = cols_full = 0
    sel_prev = None  # the interval set of a triggered step, for its pair partner
    while True:
        from_ = k
        conv_j = None
        for i in range(k, m):
            V[:, i] = f / beta[i]
            w = A @ V[:, i]
            matvecs += 1
            a = V[:, i] @ w
            alpha[i] = a
            fp = w - a * V[:, i] - (beta[i] * V[:, i - 1] if i > 0 else 0.0)
            anorm_est = max(anorm_est, abs(a) + beta[i] + (beta[i + 1] if i + 1 <= m else 0))
            do = True
            if thresh is not None:
                # estimate of beta_{i+1} (device: ||w||^2 - alpha^2 - beta_i^2)
                if est_beta:
                    b2 = w @ w - a * a - beta[i] ** 2
                    bn = np.sqrt(b2) if b2 > 1e-20 * (w @ w) else 0.0
                else:
                    bn = np.linalg.norm(fp)
                new = np.zeros(m + 1)
                if bn > 0 and i > 0:
                    # omega recurrence (Simon 1984; PROPACK dupdate_mu) for v_{i+1} vs v_j, j < i
                    for j in range(i):  # (omega of a vector with itself: 1)
                        t = beta[j + 1] * (om_cur[j + 1] if j + 1 < i else 1.0)
                        t += (alpha[j] - a) * om_cur[j]
                        if j > 0:
                            t += beta[j] * om_cur[j - 1]
                        t -= beta[i] * (om_prev[j] if j < i - 1 else 1.0)
                        new[j] = (t + np.copysign(eps1 * anorm_est, t)) / bn
                    # against u0 (L u0 = 0): (0 - alpha_i) om_cur[u] - beta_i om_prev[u]
                    t = -a * om_cur[m] - beta[i] * om_prev[m]
                    new[m] = (t + np.copysign(eps1 * anorm_est, t)) / bn
                    new[i] = eps1  # v_{i+1} vs v_i: local rounding
                forced = force
                rule = bn == 0.0 or i == m - 1 or i == from_
                trig = np.max(np.abs(new)) > thresh
                do = force or rule or trig
                force = False
            sel = None  # None: every column
            if do and thresh is not None and eta is not None and not rule:
                if trig:
                    om = np.abs(new[: i + 1])
                    sel = np.zeros(i + 1, bool)
                    for j in np.nonzero(om > thresh)[0]:
                        lo = j
                        while lo > 0 and om[lo - 1] > eta:
                            lo -= 1
                        hi = j
                        while hi < i and om[hi + 1] > eta:
                            hi += 1
                        sel[lo: hi + 1] = True
                    sel_u0 = abs(new[m]) > eta
                    if forced and sel_prev is not None:  # a pair partner also triggered: the union
                        ps, pu = sel_prev
                        sel[: len(ps)] |= ps
                        sel_u0 = sel_u0 or pu
                    sel = (sel, sel_u0)
                elif sel_prev is not None:  # the pair partner: the same intervals
                    ps, pu = sel_prev
                    s2 = np.zeros(i + 1, bool)
                    s2[: len(ps)] = ps
                    sel = (s2, pu)
            if do:
                if sel is None:
                    B = np.column_stack([V[:, : i + 1], u0])
                    h = B.T @ fp
                    fp = fp - B @ h
                    alpha[i] += h[i]
                    cols_projected += i + 2
                else:
                    cs, cu = sel
                    idx = np.nonzero(cs)[0]
                    B = np.column_stack([V[:, idx]] + ([u0] if cu else []))
                    h = B.T @ fp
                    fp = fp - B @ h
                    hi_ = dict(zip(idx.tolist(), h[: len(idx)].tolist()))
                    alpha[i] += hi_.get(i, 0.0)
                    cols_projected += len(idx) + (1 if cu else 0)
                projected += 1
                if thresh is not None:
                    force = not forced  # the next step too (a triggered step starts a pair)
                    if sel is None:
                        new = np.full(m + 1, eps1)
                        sel_prev = None
                    else:
                        cs, cu = sel
                        new[: i + 1][cs] = eps1
                        if cu:
                            new[m] = eps1
                        new[i] = eps1
                        sel_prev = sel if not forced else None
            cols_full += i + 2
            f = fp
            beta[i + 1] = np.linalg.norm(f)
            if thresh is not None:
                om_prev, om_cur = om_cur, new
            # mid-cycle convergence check
            j = i + 1
            if restarts > 0 and (j - from_) % check == 0 and j < m:
                th, Z = eig_tri(alpha[:j], beta[1:j])
                if abs(Z[-1, 0]) * beta[j] < tol * max(EPS ** (2 / 3), abs(th[0])):
                    conv_j = j
                    break
        mm = conv_j or m
        th, Z = eig_tri(alpha[:mm], beta[1:mm])
        if conv_j or abs(Z[-1, 0]) * beta[m] < tol * max(EPS ** (2 / 3), abs(th[0])):
            x = V[:, :mm] @ Z[:, 0]
            break
        restarts += 1
        W = np.column_stack([V[:, :m], u0])
        G = W.T @ W - np.eye(m + 1)
        ortho.append(float(np.max(np.abs(G))))
        if trace:
            kk = from_ if restarts > 1 else 0
            blk = (np.max(np.abs(G[:kk, :kk])) if kk else 0.0, np.max(np.abs(G[kk:m, :kk])) if kk else 0.0,
                   np.max(np.abs(G[kk:m, kk:m])), np.max(np.abs(G[m, :m])))
            print(f"  restart {restarts}: matvecs {matvecs}, projected {projected}, max|V^TV-I| {ortho[-1]:.2e} "
                  f"(kept/kept {blk[0]:.1e}, new/kept {blk[1]:.1e}, new/new {blk[2]:.1e}, u0 {blk[3]:.1e}), "
                  f"theta0 {th[0]:.15g}", flush=True)
        # implicit restart with the m - knew unwanted Ritz values as shifts (explicit QR on T)
        nconv = 0
        zl = Z[-1, :]
        knew = 1 + sum(1 for i in range(1, m) if abs(zl[i]) < EPS)
        if knew == 1:
            knew = m // 2
        knew = max(knew, keep_min)
        T = np.diag(alpha[:m]) + np.diag(beta[1:m], 1) + np.diag(beta[1:m], -1)
        Q = np.eye(m)
        for mu in th[knew:]:
            q, r = np.linalg.qr(T - mu * np.eye(m))
            T = r @ q + mu * np.eye(m)
            Q = Q @ q
        sigma = Q[m - 1, knew - 1]
        hk = T[knew, knew - 1]
        Vn = V[:, :m] @ Q[:, : knew + 1]
        f = Vn[:, knew] * hk + f * sigma
        V[:, :knew] = Vn[:, :knew]
        alpha[:knew] = np.diag(T)[:knew]
        beta[1:knew] = np.diag(T, -1)[: knew - 1]
        if thresh is not None and restart_proj:
            # the restart residual against the kept basis (and u0): its first
            # vector inherits the old basis's loss of orthogonality otherwise
            B = np.column_stack([V[:, :knew], u0])
            h = B.T @ f
            f = f - B @ h
            alpha[knew - 1] += h[knew - 1]
            if knew > 1:
                beta[knew - 1] += h[knew - 2]
        beta[knew] = np.linalg.norm(f)
        k = knew
        force = True
        om_cur = np.full(m + 1, eps1)
        om_prev = np.full(m + 1, eps1)
    x /= np.linalg.norm(x)
    lam = th[0]
    return dict(lam=lam, x=x, matvecs=matvecs, projected=projected, restarts=restarts,
                cols_projected=cols_projected, cols_full=cols_full,
                ortho_max=max(ortho) if ortho else 0.0, resid=float(np.linalg.norm(A @ x - lam * x)))


def eig_tri(a, b):
    from scipy.linalg import eigh_tridiagonal
    return eigh_tridiagonal(a, b)


def main():
    from conftest import load_package
    ek = load_package()
    src = sys.argv[1] if len(sys.argv) > 1 else "lcc:1.15:1"
    if src.startswith("lcc:"):
        _, mult, seed = src.split(":")
        h, _ = ek.Hypergraph.generate(float(mult), int(seed)).largest_component()
    else:
        h = ek.Hypergraph.read(src)
    L = h.laplacian()
    n = h.nodes
    A = sp.csr_matrix((L.val, L.col, L.rowptr), shape=(n, n))
    # thresholds, or thresh:eta for the selective form
    specs = [None] + sys.argv[2:] if len(sys.argv) > 2 else [None, "1e-10", "1e-10:1.8e-12"]
    ref = None
    for spec in specs:
        th = eta = None
        if spec is not None:
            th, *e = spec.split(":")
            th = float(th)
            eta = float(e[0]) if e else None
        r = lanczos(A, n, th, trace=True, eta=eta)
        x = r["x"] * np.sign(r["x"][np.argmax(np.abs(r["x"]))])
        med, bits = ek.median_split(x)
        if ref is None:
            ref = (r["lam"], x, bits)
        print(f"thresh {spec}: column passes {r['cols_projected']} of {r['cols_full']} "
              f"({r['cols_projected'] / r['cols_full']:.3f})")
        print(f"thresh {th}: lambda {r['lam']!r} (d {r['lam'] - ref[0]:.2e}), matvecs {r['matvecs']}, projected "
              f"{r['projected']} ({r['projected'] / r['matvecs']:.2f}), restarts {r['restarts']}, max|V^TV-I| "
              f"{r['ortho_max']:.2e}, resid {r['resid']:.2e}, max|dx| {np.abs(x - ref[1]).max():.2e}, split diff "
              f"{int((bits != ref[2]).sum())}", flush=True)


if __name__ == "__main__":
    main()
