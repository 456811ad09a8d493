"""robustgrape_amd -- MI355X-native GRAPE propagator-and-gradient engine.

Drop-in for the hot path of RobustGRAPE.jl (src/RobustGRAPE.jl:6-13 exports):
the problem types and ``calculate_fidelity_and_derivatives`` keep the
reference's names, arguments and return tuples; the computation runs in
hand-written HIP kernels for gfx950 behind the C ABI in include/grape.h.
The north-star names (FidelityOptimProblem, compute_fidelity_and_gradient,
compute_unitary_and_derivatives) are aliases.
"""
from .types import (ErrorSource, FidelityRobustGRAPEParameters, FidelityRobustGRAPEProblem,
                    UnitaryRobustGRAPEProblem)
from .operators import (OperatorBasisError, OperatorBasisHamiltonian, OperatorBasisTarget, Term,
                        FN_CIS, FN_COS, FN_LINEAR, FN_ONE, FN_SIN, VAR_ONE, VAR_TSTEP, VAR_X, VAR_XADD)
from .engine import (GrapePlan, calculate_fidelity_and_derivatives, calculate_unitary_and_derivatives,
                     clear_plans, get_plan)
from . import rydberg as RydbergTools
from .analysis import (calculate_expectation_values, calculate_fidelity_response, calculate_fidelity_response_fft,
                       calculate_interaction_error_operators)
from .regularization import regularization_cost, regularization_cost_phase
from .optimize import (LBFGS, GradientDescent, OptimizationResult, minimizer, minimum,
                       optimize_fidelity_and_error_sources, optimize_restarts)

# north-star aliases (BASELINE.json)
FidelityOptimProblem = FidelityRobustGRAPEProblem
compute_fidelity_and_gradient = calculate_fidelity_and_derivatives
compute_unitary_and_derivatives = calculate_unitary_and_derivatives

__all__ = [
    "LBFGS", "GradientDescent",
    "ErrorSource", "UnitaryRobustGRAPEProblem", "FidelityRobustGRAPEProblem", "FidelityRobustGRAPEParameters",
    "calculate_fidelity_and_derivatives", "calculate_unitary_and_derivatives", "GrapePlan", "get_plan",
    "clear_plans", "OperatorBasisHamiltonian", "OperatorBasisError", "OperatorBasisTarget", "Term",
    "RydbergTools", "regularization_cost", "regularization_cost_phase", "optimize_fidelity_and_error_sources",
    "optimize_restarts", "calculate_interaction_error_operators", "calculate_expectation_values",
    "calculate_fidelity_response", "calculate_fidelity_response_fft", "OptimizationResult", "minimizer", "minimum", "FidelityOptimProblem", "compute_fidelity_and_gradient", "compute_unitary_and_derivatives",
]
