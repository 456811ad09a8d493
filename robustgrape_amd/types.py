"""Problem descriptors, mirroring src/Types.jl of RobustGRAPE.jl.

Field names follow the reference (``t0``, ``ntimes``, ``ndim``, ``H0``,
``nb_additional_param``, ``error_sources``, ``unitary_problem``,
``projector``, ``target_unitary``); the Greek ``ϵ``/``ϵ2`` fields are exposed
as ``eps``/``eps2`` with the reference defaults 1e-8 / 1e-4 (Types.jl:38-39).

``H0``, ``Herror`` and ``target_unitary`` may be plain Python callables with
the reference signatures (Types.jl:10,25,50) -- host-evaluated -- or the
operator-basis descriptors from :mod:`robustgrape_amd.operators`, which the
device path builds on the GPU.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Sequence

import numpy as np


@dataclass(frozen=True)
class ErrorSource:
    """Types.jl:12-14. ``Herror(time_step, x, x_add, err) -> matrix``."""
    Herror: Callable


@dataclass(frozen=True)
class UnitaryRobustGRAPEProblem:
    """Types.jl:31-40."""
    t0: float
    ntimes: int
    ndim: int
    H0: Callable
    nb_additional_param: int
    error_sources: Sequence[ErrorSource] = ()
    eps: float = 1e-8
    eps2: float = 1e-4

    def __post_init__(self):
        if self.ntimes <= 0 or self.ndim <= 0 or self.nb_additional_param < 0:
            raise AssertionError("ntimes, ndim must be positive and nb_additional_param >= 0")
        object.__setattr__(self, "error_sources", tuple(self.error_sources))

    def replace(self, **kw) -> "UnitaryRobustGRAPEProblem":
        """Setfield.@set equivalent (examples/ar_cz.jl:33-36)."""
        return dataclasses.replace(self, **kw)


@dataclass(frozen=True)
class FidelityRobustGRAPEProblem:
    """Types.jl:52-56."""
    unitary_problem: UnitaryRobustGRAPEProblem
    projector: Any
    target_unitary: Callable

    def __post_init__(self):
        P = np.asarray(self.projector, dtype=np.float64)
        n = self.unitary_problem.ndim
        if P.shape != (n, n):
            raise AssertionError(f"projector must be {n}x{n}")
        object.__setattr__(self, "projector", P)

    def replace(self, **kw) -> "FidelityRobustGRAPEProblem":
        return dataclasses.replace(self, **kw)


@dataclass
class FidelityRobustGRAPEParameters:
    """Types.jl:74-84 (optimiser configuration; consumed by the driver)."""
    x_initial: Any
    regularization_functions: List[Callable]
    regularization_coeff1: Sequence[float]
    regularization_coeff2: Sequence[float]
    error_source_coeff: Sequence[float]
    time_limit: float = float("nan")
    iterations: int = 1000
    solver_algorithm: Any = "LBFGS"  # optimize.LBFGS(m) / optimize.GradientDescent() or their names
    additional_parameters: Dict[str, Any] = field(default_factory=dict)


def split_x(problem: UnitaryRobustGRAPEProblem, x):
    """UnitaryCalculations.jl:21-26: returns (x_main (nparam, ntimes), x_add, nparam)."""
    x = np.asarray(x, dtype=np.float64)
    na = problem.nb_additional_param
    nmain = x.shape[-1] - na
    if nmain < 0 or nmain % problem.ntimes != 0:
        raise AssertionError("Control parameter size must be a multiple of time steps")
    nparam = nmain // problem.ntimes
    x_main = x[..., :nmain].reshape(x.shape[:-1] + (problem.ntimes, nparam))
    x_main = np.swapaxes(x_main, -1, -2)
    return x_main, x[..., nmain:], nparam
