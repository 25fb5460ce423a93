"""The sparse (leaves-first) factorisation variants of the env kernel assume each robot's
DOFs form equal chains hanging from the base, in DFS order (leggedsim.hip l_nz /
dof_chain_length).  Pins that structure for the shipped models, so a model change that
breaks it is caught here (the kernel itself then falls back to the dense variant)."""
import os

import numpy as np
import pytest

from leggedsim.model import Model

MODELS = os.path.join(os.path.dirname(__file__), "..", "unitree-rl-gym_amd", "leggedsim", "models")


def dof_parents(m):
    par = {}
    for b in range(m.num_bodies):
        j = int(m.dof[b])
        if j < 0:
            continue
        a = int(m.parent[b])
        while a > 0 and m.dof[a] < 0:
            a = int(m.parent[a])
        par[j] = int(m.dof[a]) if a > 0 else -1
    return [par[j] for j in range(m.num_dofs)]


def chain_length(par):
    D = len(par)
    for ch in range(1, D + 1):
        if D % ch == 0 and all(par[j] == (-1 if j % ch == 0 else j - 1) for j in range(D)):
            return ch
    return 0


@pytest.mark.parametrize("name,ch", [("go2", 3), ("g1_12dof", 6), ("h1", 5), ("h1_2_12dof", 6)])
def test_shipped_models_are_chains_from_the_base(name, ch):
    m = Model.load(os.path.join(MODELS, name + ".npz"))
    assert chain_length(dof_parents(m)) == ch


def test_leaves_first_order_has_no_fill_in():
    """Cholesky of a chain-structured mass-matrix pattern in the reversed (leaves-first)
    order: every entry outside the predicted pattern (chain ancestors + base rows) is an
    exact zero, the property the kernel's skipped updates rely on."""
    rng = np.random.default_rng(0)
    D, ch = 12, 3
    n = D + 6
    anc = np.zeros((D, D), bool)  # anc[i, j]: DOF i is an ancestor-or-self of DOF j
    for j in range(D):
        for i in range(j - j % ch, j + 1):
            anc[i, j] = True
    M = np.zeros((n, n))
    M[:6, :] = M[:, :6] = 1.0
    M[6:, 6:] = anc | anc.T
    S = M * rng.uniform(0.1, 1.0, size=(n, n))
    S = (S + S.T) / 2 + n * np.eye(n)  # the mass-matrix pattern, diagonally dominant
    P = S[::-1, ::-1]  # leaves-first
    L = np.linalg.cholesky(P)
    for i in range(n):
        for k in range(i):
            predicted = k >= D or i >= D or i <= k + (D - 1 - k) % ch
            if not predicted:
                assert L[i, k] == 0.0, (i, k)
