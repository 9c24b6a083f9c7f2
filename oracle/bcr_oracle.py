"""CPU restatement of the block-cyclic-reduction evaluation (portfoliooptgp_amd/csrc/gpx_bcr.hip),
TEST INFRASTRUCTURE ONLY (never imported by the package): the same levels, nodes, pending updates,
couplings and selected-inverse recurrences as the device kernels, in numpy fp64 block algebra,
so that the algorithm (not the kernels' arithmetic) can be checked on the CPU against the dense
oracle (oracle/gp_oracle.py: GPflow 2.9.1's GPR logML / gradient / predict restated; SURVEY §8c,
parity against GPflow itself unpinned as for every row of this repo).

bcr_eval(Kfull, y, bs) takes the dense K + σn²I (block tridiagonal in blocks of bs rows: entries
beyond one block off the diagonal are ignored, exactly as the device path never reads them) and
returns logML, α = K⁻¹y, the band of Z = K⁻¹ as {(J, J): Z_JJ, (J+1, J): Z_{J+1,J}} and the band
check max_j |Σ_i K_ji Z_ij − 1|."""
from __future__ import annotations

import math

import numpy as np


def _levels(n0):
    m, l, out = n0, 0, []
    while True:
        out.append(m)
        if m == 1:
            return out
        m = (m + 1) // 2
        l += 1


def bcr_eval(K: np.ndarray, y: np.ndarray, bs: int, n: int | None = None):
    N = K.shape[0] if n is None else n
    n0 = (N + bs - 1) // bs
    Np = n0 * bs
    Kp = np.eye(Np)
    Kp[:N, :N] = K[:N, :N]
    yp = np.zeros(Np)
    yp[:N] = np.asarray(y, dtype=np.float64).reshape(-1)[:N]

    def blk(i, j):
        return Kp[i * bs:(i + 1) * bs, j * bs:(j + 1) * bs].copy()

    A = {}            # A[X]: the diagonal block (updates applied)
    C = {}            # C[X]: coupling of X with its left neighbour (rows X, cols left)
    dL, dR, dyL, dyR = {}, {}, {}, {}
    Wm, PI, PK, z = {}, {}, {}, {}
    yv = {}
    logdet = 0.0
    ms = _levels(n0)
    top = len(ms) - 1
    for l, m in enumerate(ms):
        h = 1 << (l - 1) if l > 0 else 0
        for j in range(m):
            X = j << l
            is_top = l == top
            elim = is_top or (j & 1)
            pl = l > 0 and X > 0
            pr = l > 0 and X + h < n0
            if l == 0:
                Ax, yx = blk(X, X), yp[X * bs:(X + 1) * bs].copy()
            else:
                Ax = A[X] - ((dR[X - h] if pl else 0.0) + (dL[X + h] if pr else 0.0))
                yx = yv[X] - ((dyR[X - h] if pl else 0.0) + (dyL[X + h] if pr else 0.0))
            if not elim:
                A[X], yv[X] = Ax, yx
                continue
            I, Kn = X - (1 << l), X + (1 << l)
            hasI, hasK = not is_top, (not is_top) and Kn < n0
            L = np.linalg.cholesky(Ax)
            W = np.linalg.inv(L)
            logdet += 2.0 * np.log(np.diag(L)).sum()
            Wm[X] = W
            z[X] = W @ yx
            if hasI:
                EXI = blk(X, I) if l == 0 else C[X]
                PI[X] = W @ EXI                      # P_Iᵀ
            if hasK:
                EKX = blk(Kn, X) if l == 0 else C[Kn]
                PK[X] = W @ EKX.T                    # P_Kᵀ
            if hasI:
                dL[X] = PI[X].T @ PI[X]
                dyL[X] = PI[X].T @ z[X]
            if hasK:
                dR[X] = PK[X].T @ PK[X]
                dyR[X] = PK[X].T @ z[X]
                C[Kn] = -PK[X].T @ PI[X]             # E_KI
    zz = sum(float(v @ v) for v in z.values())
    lml = -0.5 * zz - 0.5 * logdet - 0.5 * N * math.log(2.0 * math.pi)
    # backward: α and the selected inverse
    al, ZD, ZC = {}, {}, {}
    for l in range(top, -1, -1):
        m = ms[l]
        if l == top:
            xs = [0]
        else:
            xs = [j << l for j in range(1, m, 2)]
        for X in xs:
            is_top = l == top
            I, Kn = X - (1 << l), X + (1 << l)
            hasI, hasK = not is_top, (not is_top) and Kn < n0
            W = Wm[X]
            t = z[X].copy()
            if hasI:
                t -= PI[X] @ al[I]
            if hasK:
                t -= PK[X] @ al[Kn]
            al[X] = W.T @ t
            Zxx = W.T @ W
            if hasI:
                GI = PI[X].T @ W
                GK = PK[X].T @ W if hasK else np.zeros_like(W)
                ZKI = ZC[Kn] if hasK else np.zeros_like(W)
                ZII, ZKK = ZD[I], (ZD[Kn] if hasK else np.zeros_like(W))
                ZIX = -(ZII @ GI + ZKI.T @ GK)
                ZKX = -(ZKI @ GI + ZKK @ GK)
                Zxx = Zxx - GI.T @ ZIX - GK.T @ ZKX
                ZC[X] = ZIX.T
                if hasK:
                    ZC[Kn] = ZKX
            ZD[X] = Zxx
    alpha = np.concatenate([al[J] for J in range(n0)])[:N]
    band = {}
    chk = 0.0
    for J in range(n0):
        band[(J, J)] = ZD[J]
        if J + 1 < n0:
            band[(J + 1, J)] = ZC[J + 1]
        r = (blk(J, J) * ZD[J]).sum(axis=0)
        if J + 1 < n0:
            r += (blk(J + 1, J) * ZC[J + 1]).sum(axis=0)
        if J >= 1:
            r += (blk(J, J - 1) * ZC[J]).sum(axis=1)
        rows = np.arange(J * bs, (J + 1) * bs) < N
        if rows.any():
            chk = max(chk, float(np.abs(r[rows] - 1.0).max()))
    return lml, alpha, band, chk
