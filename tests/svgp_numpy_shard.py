"""CPU stand-in for SVGPEngine (test infrastructure): the same eval_local / partials /
eval_finish protocol and the same shard decomposition as gpx_svgp.hip, in numpy, so the
distributed orchestration (one all_reduce of the packed partial buffer) is testable with gloo
on the CPU. Partial layout: G [M*M] | w [M] | θ [16] | Z [M*D] | Σ(y−μ)², Σk_nn, n_local, 0."""
import math

import numpy as np
import torch

JITTER = 1e-6


class NumpySVGPShard:
    def __init__(self, kernel, X, Y, M, num_data, n_total):
        self.k = kernel                       # oracle kernel (K, K_diag, dK, dK_dX1)
        self.X = np.asarray(X, np.float64).reshape(len(X), -1)
        self.Y = np.asarray(Y, np.float64).reshape(-1)
        self.M, self.D = M, self.X.shape[1]
        self.num_data, self.n_total = float(num_data), int(n_total)
        self.partials = torch.zeros(M * M + M + 16 + M * self.D + 4, dtype=torch.float64)

    def _set_theta(self, theta):
        ps = self.k.params()
        for p, v in zip(ps, theta):
            p.value = float(v)
        self.s2 = float(theta[len(ps)])

    def eval_local(self, theta, Z, q, R):
        self._set_theta(theta)
        M, D = self.M, self.D
        self.Z, self.q, self.R = np.asarray(Z).reshape(M, D), np.asarray(q).reshape(M), np.tril(np.asarray(R))
        W = np.linalg.inv(np.linalg.cholesky(self.k.K(self.Z) + JITTER * np.eye(M)))
        S = self.R @ self.R.T
        P = W.T @ (S - np.eye(M)) @ W
        u = W.T @ self.q
        scale = self.num_data / self.n_total
        c = -0.5 * scale / self.s2
        Kmn = self.k.K(self.Z, self.X)
        mu = Kmn.T @ u
        g = scale * (self.Y - mu) / self.s2
        Kbar = np.outer(u, g) + 2 * c * P @ Kmn
        XA = np.concatenate([self.Z, self.X])
        dth = np.zeros(16)
        for i, d in enumerate(self.k.dK(XA)):
            dth[i] = np.sum(Kbar * d[:M, M:]) + c * np.sum(np.diag(d)[M:])
        dZ = np.einsum("mn,mnd->md", Kbar, self.k.dK_dX1(self.Z, self.X))
        sc = [np.sum((self.Y - mu) ** 2), np.sum(self.k.K_diag(self.X)), len(self.X), 0.0]
        self.partials.copy_(torch.as_tensor(np.concatenate(
            [(Kmn @ Kmn.T).ravel(), Kmn @ g, dth, dZ.ravel(), sc])))
        self.W, self.S, self.scale, self.c = W, S, scale, c

    def eval_finish(self):
        M, D = self.M, self.D
        p = self.partials.numpy()
        G = p[: M * M].reshape(M, M)
        w = p[M * M: M * M + M]
        dth = p[M * M + M: M * M + M + 16].copy()
        dZ = p[M * M + M + 16: M * M + M + 16 + M * D].reshape(M, D).copy()
        sq, kd, nl = p[-4], p[-3], p[-2]
        assert round(nl) == self.n_total
        W, S, c, q, R = self.W, self.S, self.c, self.q, self.R
        Gh = W @ G @ W.T
        ah = W @ w
        F = -(np.outer(q, ah) + 2 * c * (S - np.eye(M)) @ Gh)
        Phi = np.tril(F)
        Phi[np.diag_indices(M)] *= 0.5
        Sb = W.T @ Phi @ W
        Sb = 0.5 * (Sb + Sb.T)
        for i, d in enumerate(self.k.dK(self.Z)):
            dth[i] += np.sum(Sb * d)
        dZ += 2 * np.einsum("mj,mjd->md", Sb, self.k.dK_dX1(self.Z, self.Z))
        tr = np.sum((S - np.eye(M)) * Gh)
        kl = 0.5 * (q @ q + np.sum(R * R) - M - np.sum(np.log(np.diag(R) ** 2)))
        s, s2 = self.scale, self.s2
        elbo = s * (-0.5 * self.n_total * math.log(2 * math.pi * s2) - (sq + kd + tr) / (2 * s2)) - kl
        np_ = len(self.k.params())
        dth[np_] = s * (-0.5 * self.n_total / s2 + 0.5 * (sq + kd + tr) / s2 ** 2)
        dR = np.tril(2 * c * Gh @ R - R + np.diag(1 / np.diag(R)))
        return elbo, dth, dZ, ah - q, dR
