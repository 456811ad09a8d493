"""CPU-side checks of the boundary: the library builds, loads, exports every
symbol include/grape.h declares, and the host-side descriptor packing is right.
No compute call is made (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests import problems as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "grape.h")).read()
    return sorted(set(re.findall(r"\b(grape_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from robustgrape_amd import _capi
    from robustgrape_amd.build import build_library
    build_library(verbose=False)
    L = _capi.lib()
    declared = _header_symbols()
    assert set(declared) == set(_capi.EXPORTED)
    for name in declared:
        assert hasattr(L, name), name
    assert L.grape_abi_version() == _capi.ABI_VERSION
    src = open(os.path.join(ROOT, "include", "grape.h")).read()
    assert len(_capi.KERNEL_NAMES) == int(re.search(r"GRAPE_NUM_KERNELS = (\d+)", src).group(1))


def test_library_build_id_is_the_source_hash(tmp_path):
    """Provenance: the loaded library embeds the content hash of the sources it
    was built from, equal to the hash of csrc/ + include/ as they are now; a changed source gives
    a different hash (so _capi.lib() would refuse the stale library)."""
    from robustgrape_amd import _capi, build
    build.build_library(verbose=False)
    assert _capi.build_id() == build.source_id()
    with open(build.ID_FILE) as fh:
        assert fh.read().strip() == build.source_id()
    src = build.DEPS[-1]
    orig = open(src, "rb").read()
    try:
        with open(src, "ab") as fh:
            fh.write(b"\n")
        assert build.source_id() != _capi.build_id() and build.needs_build()
    finally:
        with open(src, "wb") as fh:
            fh.write(orig)
    assert build.source_id() == _capi.build_id() and not build.needs_build()


def test_descriptor_packing_roundtrip():
    """The ctypes descriptor reproduces the operator basis (column-major, interleaved)."""
    from robustgrape_amd.operators import DescriptorBuffers
    fp = P.full9_problem(16)
    buf = DescriptorBuffers(fp, nparam=1, max_batch=8)
    d = buf.desc
    assert (d.ndim, d.ntimes, d.nparam, d.nadd, d.nerr) == (9, 16, 1, 1, 0)
    ops = buf.ops.reshape(d.n_ops, 9 * 9 * 2)
    x = np.array([0.37])
    H = np.zeros((9, 9), complex)
    for k in range(d.n_h0_terms):
        t = d.h0_terms[k]
        op = (ops[t.op, 0::2] + 1j * ops[t.op, 1::2]).reshape(9, 9, order="F")
        coef = {2: np.cos, 3: np.sin}.get(t.func, lambda v: 1.0)(t.a * x[0] + t.b)
        H += complex(t.scale_re, t.scale_im) * coef * op
    np.testing.assert_allclose(H, fp.unitary_problem.H0(1, x, [0.0]), atol=1e-15)
    np.testing.assert_array_equal(buf.pdiag, np.diag(P.W_FULL9))


def test_closure_problems_are_rejected_by_the_device_path():
    from robustgrape_amd.operators import DescriptorBuffers
    with pytest.raises(TypeError):
        DescriptorBuffers(P.sym_problem(8, device=False), nparam=1)


def test_closure_problems_take_the_table_descriptor():
    """Closure H0 / target (no error sources): GRAPE_DESC_HOST_TABLES descriptor and host tables
    laid out as grape_fidelity_grad_tables expects (column-major, variant order 0 | dx | dxa)."""
    from robustgrape_amd.operators import (GRAPE_DESC_HOST_TABLES, TableDescriptor, has_operator_basis,
                                           host_tables)
    fp = P.sym_problem(4, device=False)
    assert not has_operator_basis(fp) and has_operator_basis(P.sym_problem(4))
    t = TableDescriptor(fp, nparam=1, max_batch=2)
    assert t.desc.reserved[0] == GRAPE_DESC_HOST_TABLES and t.desc.n_ops == 0 and t.desc.nerr == 0
    x = P.random_x(4, 3)
    H, U0 = host_tables(fp, np.stack([x, x]), 1)
    assert H.shape == (2, 4, 3, 5, 5) and U0.shape == (2, 2, 5, 5)
    up = fp.unitary_problem
    eps = up.eps
    k = 2
    Hk = np.asarray(up.H0(k + 1, np.array([x[k]]), x[-1:]))
    np.testing.assert_array_equal(H[1, k, 0], Hk.T)  # column-major storage
    np.testing.assert_array_equal(H[1, k, 1], np.asarray(up.H0(k + 1, np.array([x[k] + eps]), x[-1:])).T)
    np.testing.assert_array_equal(H[1, k, 2], Hk.T)  # H0 ignores x_add: the dxa variant equals the nominal
    np.testing.assert_array_equal(U0[0, 1], np.asarray(fp.target_unitary(x[-1:] + eps)).T)
    # with error sources: n = np + na gradient parameters, 1 + 2 n + ne (2 + n) variants in the
    # UnitaryCalculations.jl:45-95 order (x_add sites included: closures may read x_add)
    fe = P.sym_problem(4, errors=("amp", "freq"), device=False)
    assert TableDescriptor(fe, nparam=1).desc.nerr == 2
    He, _ = host_tables(fe, x[None, :], 1)
    assert He.shape == (1, 4, 1 + 2 * 2 + 2 * 4, 5, 5)
    upe = fe.unitary_problem
    xk, xa = np.array([x[k]]), x[-1:]
    H0k = np.asarray(upe.H0(k + 1, xk, xa), complex)
    np.testing.assert_array_equal(He[0, k, 3], np.asarray(upe.H0(k + 1, xk + upe.eps2, xa)).T)  # dx2
    np.testing.assert_array_equal(He[0, k, 4], np.asarray(upe.H0(k + 1, xk, xa + upe.eps2)).T)  # dxa2
    herr = upe.error_sources[1].Herror
    np.testing.assert_array_equal(He[0, k, 9], (np.asarray(herr(k + 1, xk, xa, upe.eps)) + H0k).T)  # freq, eps
    mix = np.asarray(herr(k + 1, xk + upe.eps2, xa, upe.eps2)) + np.asarray(upe.H0(k + 1, xk + upe.eps2, xa))
    np.testing.assert_array_equal(He[0, k, 11], mix.T)  # freq, mixed stencil (control)
    mixa = np.asarray(herr(k + 1, xk, xa + upe.eps2, upe.eps2)) + np.asarray(upe.H0(k + 1, xk, xa + upe.eps2))
    np.testing.assert_array_equal(He[0, k, 12], mixa.T)  # freq, mixed stencil (x_add)


def test_projector_in_descriptor():
    """A diagonal projector travels as projector_diag only; any other real matrix (the reference
    accepts one, FidelityCalculations.jl:47-51) also as the full column-major complex matrix."""
    from robustgrape_amd.operators import DescriptorBuffers
    fp = P.sym_problem(8)
    buf = DescriptorBuffers(fp, nparam=1)
    assert not buf.desc.projector and buf.pfull is None
    W = np.array(P.W_SYM, dtype=float)
    W[0, 1] = 0.5
    W[3, 2] = -0.25
    buf = DescriptorBuffers(fp.replace(projector=W), nparam=1)
    d = W.shape[0]
    full = np.ctypeslib.as_array(buf.desc.projector, shape=(2 * d * d,))
    np.testing.assert_array_equal(full[0::2].reshape(d, d, order="F"), W)
    assert not full[1::2].any()
    np.testing.assert_array_equal(np.ctypeslib.as_array(buf.desc.projector_diag, shape=(d,)), np.diag(W))


def _create(fp, nparam=1):
    """grape_plan_create on this host: descriptor validation runs before the device lookup, so
    a refusal of the descriptor is observable without a GPU."""
    from robustgrape_amd import _capi
    from robustgrape_amd.operators import DescriptorBuffers
    buf = DescriptorBuffers(fp, nparam=nparam, max_batch=1)
    h = ctypes.c_void_p()
    rc = _capi.lib().grape_plan_create(ctypes.byref(buf.desc), 0, ctypes.byref(h))
    return rc, _capi.lib().grape_last_error().decode()


def test_non_hermitian_h0_selects_the_general_path():
    """A non-Hermitian H0 (a -i Gamma/2 decay term, a non-Hermitian scale * operator) passes
    validation on the small engine (the general-H0 path: LU-inverted chain, include/grape.h
    GRAPE_OPT_GENERAL_H0) -- here the device lookup then reports -6 -- and is refused by the
    dense engine (d > 12), whose solve relies on a Hermitian H."""
    from robustgrape_amd.operators import OperatorBasisHamiltonian, Term
    fp = P.sym_problem(8)
    up = fp.unitary_problem
    decay = np.diag([0, 0, 0, 0, 1.0]).astype(complex)
    terms = list(up.H0.terms)
    for f in [fp.replace(unitary_problem=up.replace(H0=OperatorBasisHamiltonian(terms + [Term(decay, scale=-0.5j)]))),
              fp.replace(unitary_problem=up.replace(H0=OperatorBasisHamiltonian(
                  terms + [Term(np.triu(np.ones((5, 5))).astype(complex))])))]:
        rc, msg = _create(f)
        assert rc in (0, -6), (rc, msg)
    # a non-Hermitian ERROR generator (decay-rate error) is accepted: only H0 chains
    from robustgrape_amd.operators import OperatorBasisError
    from robustgrape_amd.types import ErrorSource
    derr = fp.replace(unitary_problem=up.replace(error_sources=[ErrorSource(OperatorBasisError([Term(decay, scale=-0.5j)]))]))
    rc, msg = _create(derr)
    assert rc in (0, -6), (rc, msg)
    # dense engine: refused with the reason
    from robustgrape_amd import synthetic as S
    dfp = S.dense_problem(d=16, ntimes=4)
    dup = dfp.unitary_problem
    dterms = list(dup.H0.terms)
    ddecay = np.zeros((16, 16), complex)
    ddecay[3, 3] = 1.0
    bad = dfp.replace(unitary_problem=dup.replace(H0=OperatorBasisHamiltonian(dterms + [Term(ddecay, scale=-0.5j)])))
    rc, msg = _create(bad, nparam=2)  # the C5 family's two controls
    assert rc == -2 and "Hermitian" in msg, (rc, msg)


def test_plan_cache_is_bounded_and_keyed_by_problem(monkeypatch):
    """get_plan keeps one plan per (problem, nparam, device), grows it up to PLAN_BATCH_CAP and
    evicts the least recently used beyond MAX_CACHED_PLANS."""
    from robustgrape_amd import engine

    made = []

    class FakePlan:
        def __init__(self, fp, nparam, device, max_batch):
            import threading
            self.fp, self.max_batch, self.closed, self.lock = fp, max_batch, False, threading.Lock()
            self.requested_batch, self.handle = max_batch, object()
            made.append(self)

        def close(self):
            self.closed, self.handle = True, None

    monkeypatch.setattr(engine, "GrapePlan", FakePlan)
    engine.clear_plans()
    fp = P.sym_problem(4)
    a = engine.get_plan(fp, 1, 0, max_batch=1)
    assert engine.get_plan(fp, 1, 0, max_batch=1) is a and a.max_batch == 1
    b = engine.get_plan(fp, 1, 0, max_batch=10 ** 6)  # grows once, capped
    assert a.closed and b.max_batch == engine.PLAN_BATCH_CAP
    assert engine.get_plan(fp, 1, 0, max_batch=3) is b  # a big plan serves small batches
    others = [P.sym_problem(4) for _ in range(engine.MAX_CACHED_PLANS + 3)]
    for o in others:
        engine.get_plan(o, 1, 0)
    assert engine.cached_plan_count() == engine.MAX_CACHED_PLANS
    assert b.closed  # least recently used, evicted
    engine.clear_plans()
    assert engine.cached_plan_count() == 0 and all(p.closed for p in made)


def test_closure_tables_detect_non_hermitian_h0():
    """Closure fallback: a non-Hermitian nominal H0 is tabulated and detected on the host
    (tables.is_hermitian_h0 -> GrapePlan.general_h0_for moves the plan to the general-H0 path);
    a non-Hermitian error generator is tabulated as is."""
    from robustgrape_amd.tables import host_tables, is_hermitian_h0
    from robustgrape_amd.types import ErrorSource
    fp = P.sym_problem(6, device=False)
    up = fp.unitary_problem
    decay = np.diag([0, 0, 0, 0, 1.0]).astype(complex)
    x = P.random_x(6, 2)
    bad = fp.replace(unitary_problem=up.replace(H0=lambda t, p, xa: up.H0(t, p, xa) - 0.5j * decay))
    H, _ = host_tables(bad, x[None, :], 1)
    assert np.isfinite(H).all() and not is_hermitian_h0(H[:, :, 0])
    H, _ = host_tables(fp, x[None, :], 1)
    assert is_hermitian_h0(H[:, :, 0])
    ok = fp.replace(unitary_problem=up.replace(error_sources=[ErrorSource(lambda t, p, xa, e: -0.5j * e * decay)]))
    H, _ = host_tables(ok, x[None, :], 1)
    assert np.isfinite(H).all() and is_hermitian_h0(H[:, :, 0])


def test_plan_option_constants_match_the_header():
    """Every GRAPE_OPT_* of include/grape.h has its operators.OPT_* twin with the same value."""
    import os
    import re

    from robustgrape_amd import operators as OPS
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "grape.h")).read()
    defs = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define GRAPE_OPT_(\w+) (\d+)", hdr))
    assert len(defs) >= 12
    for name, val in defs.items():
        assert getattr(OPS, "OPT_" + name) == val, name


def test_build_id_names_the_variant():
    """an A/B variant (scripts/build_variants.py, -D defines) has its own build id, and the
    id recorded next to a library carries the defines it was built with."""
    from robustgrape_amd import build
    base = build.source_id()
    assert build.source_id(("GRAPE_WALK_TWIN_SUM=0",)) != base
    assert build.source_id(("A=1", "B=2")) == build.source_id(("B=2", "A=1"))
    sid, defines = build.read_id_file(build.LIB)
    assert sid == base and defines == ()
