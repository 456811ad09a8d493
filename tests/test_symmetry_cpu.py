"""Symmetry-adapted sectors on the CPU (include/grape.h grape_symmetry_basis, host code only;
robustgrape_amd/csrc/grape_symmetry.hpp).

The plan may run its sector path in a rotated basis V that block-diagonalises the algebra of the
operators H0 and the error sources use, when that splits the permutation sectors further.  Checked
here without a GPU:
* the C2 operators (rydberg_hamiltonian_full, Omega1 = Omega2, RydbergTools.jl:118-130): the
  atom-swap symmetry splits {11, 1r, r1, rr} into {11, (1r + r1)/sqrt2, rr} and the dark state
  (1r - r1)/sqrt2; V is the identity on every other level;
* the C3 operators (single-atom Rabi errors break the symmetry): no rotation;
* hidden block structure behind a random unitary (irreducible blocks, and an irreducible block
  with multiplicity two): V^dag H V block-diagonal with the right block sizes;
* the claim the engine relies on, with the oracle (FidelityCalculations.jl:19-119 restated):
  F and F_dx of the C2 problem rotated by V (H0, target, projector) equal the original's."""
import ctypes

import numpy as np
import pytest

from robustgrape_amd import rydberg as R
from robustgrape_amd.operators import (FN_LINEAR, VAR_X, DescriptorBuffers, OperatorBasisHamiltonian,
                                       OperatorBasisTarget, Term)
from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
from tests import problems as P


def _basis(fp, nparam=1):
    from robustgrape_amd import _capi
    buf = DescriptorBuffers(fp, nparam=nparam, max_batch=1)
    d = fp.unitary_problem.ndim
    V = np.zeros(2 * d * d)
    blk = (ctypes.c_int * d)()
    rc = _capi.lib().grape_symmetry_basis(ctypes.byref(buf.desc), _capi.dptr(V), blk)
    assert rc in (0, 1), rc
    Vc = (V[0::2] + 1j * V[1::2]).reshape(d, d, order="F")
    return rc, Vc, np.array(list(blk)), buf


def _used_ops(fp):
    up = fp.unitary_problem
    ops = [t.op for t in up.H0.terms]
    for es in up.error_sources:
        ops += [t.op for t in es.Herror.terms]
    return [np.asarray(o, np.complex128) for o in ops]


def _check_block_diagonal(V, blk, ops):
    d = V.shape[0]
    np.testing.assert_allclose(V.conj().T @ V, np.eye(d), atol=1e-14)
    off = blk[:, None] != blk[None, :]
    for H in ops:
        Hr = V.conj().T @ H @ V
        assert np.max(np.abs(Hr[off])) <= 1e-13 * max(1.0, np.max(np.abs(H)))


def test_c2_swap_symmetry_splits_the_four_level_component():
    fp = P.full9_problem(8)
    rc, V, blk, _ = _basis(fp)
    assert rc == 1
    _check_block_diagonal(V, blk, _used_ops(fp))
    s = 1 / np.sqrt(2)
    E = np.eye(9, dtype=complex)
    E[6:8, 6:8] = [[s, s], [-s, s]]  # columns 6, 7: (1r - r1)/sqrt2 (dark), (1r + r1)/sqrt2
    np.testing.assert_allclose(V, E, atol=1e-15)
    # invariant subspaces: {11, sym, rr} one block, the dark state its own
    assert blk[3] == blk[7] == blk[8] and blk[6] not in (blk[3],)
    Hs = [V.conj().T @ H @ V for H in _used_ops(fp)]
    for H in Hs:  # the dark state decouples completely (no operator touches it)
        assert np.all(H[6, :] == 0) and np.all(H[:, 6] == 0)


def test_c3_errors_break_the_symmetry():
    rc, V, blk, _ = _basis(P.full9_problem(8, nerr=4))
    assert rc == 0
    np.testing.assert_array_equal(V, np.eye(9))


def _hidden(blocks, mult_block=None, seed=3, nops=3):
    """Operators W (+) B_i W^dag with random Hermitian blocks B_i (mult_block: one block repeated
    twice, identical in every operator: an irreducible representation of multiplicity two)."""
    rng = np.random.default_rng(seed)
    d = sum(blocks) + (2 * mult_block if mult_block else 0)
    G = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    W, _ = np.linalg.qr(G)
    ops = []
    for _ in range(nops):
        B = np.zeros((d, d), complex)
        o = 0
        for n in blocks:
            h = rng.normal(size=(n, n)) + 1j * rng.normal(size=(n, n))
            B[o:o + n, o:o + n] = (h + h.conj().T) / 2
            o += n
        if mult_block:
            n = mult_block
            h = rng.normal(size=(n, n)) + 1j * rng.normal(size=(n, n))
            h = (h + h.conj().T) / 2
            B[o:o + n, o:o + n] = h
            B[o + n:o + 2 * n, o + n:o + 2 * n] = h
        ops.append(W @ B @ W.conj().T)
    return d, ops


def _fp_of(d, ops):
    terms = [Term(ops[0])] + [Term(o, var=VAR_X, index=i, func=FN_LINEAR) for i, o in enumerate(ops[1:])]
    up = UnitaryRobustGRAPEProblem(t0=1.0, ntimes=4, ndim=d, H0=OperatorBasisHamiltonian(terms),
                                   nb_additional_param=0)
    return FidelityRobustGRAPEProblem(up, np.eye(d), OperatorBasisTarget([Term(np.eye(d, dtype=complex))]))


@pytest.mark.parametrize("blocks,mult", [((3, 2), None), ((2, 2, 1), None), ((3,), 2), ((4, 3), None)])
def test_hidden_blocks_are_found(blocks, mult):
    d, ops = _hidden(blocks, mult)
    fp = _fp_of(d, ops)
    rc, V, blk, _ = _basis(fp, nparam=len(ops) - 1)
    assert rc == 1
    _check_block_diagonal(V, blk, ops)
    sizes = sorted(np.bincount(blk)[np.bincount(blk) > 0].tolist())
    want = sorted(list(blocks) + ([mult, mult] if mult else []))
    assert sizes == want, (sizes, want)


def test_irreducible_operators_keep_the_identity():
    d, ops = _hidden((5,))
    rc, V, blk, _ = _basis(_fp_of(d, ops), nparam=2)
    assert rc == 0 and len(set(blk.tolist())) == 1
    np.testing.assert_array_equal(V, np.eye(5))


def test_rotated_problem_has_the_same_fidelity_and_gradient():
    """F and F_dx are trace expressions invariant under X -> V^dag X V for U, U0, P0 and the
    pattern P (FidelityCalculations.jl:47-117): the C2 problem in the symmetry basis, evaluated by
    the oracle, equals the original (T1 for F, the T2s tier for F_dx)."""
    from oracle import grape_oracle as O
    fp = P.full9_problem(24, device=False)
    rc, V, blk, _ = _basis(P.full9_problem(24))
    assert rc == 1
    up = fp.unitary_problem
    H0, tgt = up.H0, fp.target_unitary
    rot = lambda M: V.conj().T @ np.asarray(M, np.complex128) @ V  # noqa: E731
    P0r = rot(fp.projector).real
    assert np.max(np.abs(rot(fp.projector).imag)) < 1e-15
    # C2: the rotation mixes only levels of weight 0, so P0' stays diagonal with its pattern P'
    np.testing.assert_allclose(P0r, np.diag(np.diag(P0r)), atol=1e-15)
    fr = FidelityRobustGRAPEProblem(up.replace(H0=lambda t, p, xa: rot(H0(t, p, xa))), np.round(P0r, 14),
                                    lambda xa: rot(tgt(xa)))
    x = P.random_x(24, 5)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    F1, g1 = O.calculate_fidelity_and_derivatives(fr, x)[:2]
    assert abs(F0 - F1) <= 1e-12
    g0, g1 = np.asarray(g0), np.asarray(g1)
    assert np.max(np.abs(g0 - g1)) <= 1e-7 * np.max(np.abs(g0)) + 1e-9
