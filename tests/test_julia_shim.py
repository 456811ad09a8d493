"""Static checks of the Julia shim (julia/RobustGRAPEMI355X.jl) against the reference's Julia
interface.  Julia is not in the image, so the shim cannot run here; these checks pin what a
reference caller relies on:

* the exported entry points take the reference's argument types, first argument included:
    calculate_unitary_and_derivatives(problem::UnitaryRobustGRAPEProblem, x::Vector{<:Real})
        -- src/UnitaryCalculations.jl:20
    calculate_interaction_error_operators(problem::UnitaryRobustGRAPEProblem, x::Vector{<:Real})
        -- src/UnitaryCalculations.jl:180
    calculate_fidelity_and_derivatives(fidelity_problem::FidelityRobustGRAPEProblem, x::Vector{<:Real})
        -- src/FidelityCalculations.jl:19
    calculate_expectation_values(fidelity_problem::FidelityRobustGRAPEProblem, x::Vector{<:Real})
        -- src/FidelityCalculations.jl:368
* those types are the reference's own (imported from RobustGRAPE, not redefined);
* OperatorBasis is a Function, so it fits H0::Function / Herror::Function /
  target_unitary::Function (src/Types.jl:13,35,55);
* plans are cached per (problem, nparam, kind), so the fidelity plan (max_batch 256) and the
  single-x analysis plan (max_batch 1) and the closure-table plan never collide.
The reference signatures are restated here (with their file:line) rather than read from the
reference tree."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "julia", "RobustGRAPEMI355X.jl")

REFERENCE_SIGNATURES = {
    "calculate_unitary_and_derivatives": ("UnitaryRobustGRAPEProblem", "Vector{<:Real}"),      # UnitaryCalculations.jl:20
    "calculate_interaction_error_operators": ("UnitaryRobustGRAPEProblem", "Vector{<:Real}"),  # UnitaryCalculations.jl:180
    "calculate_fidelity_and_derivatives": ("FidelityRobustGRAPEProblem", "Vector{<:Real}"),    # FidelityCalculations.jl:19
    "calculate_expectation_values": ("FidelityRobustGRAPEProblem", "Vector{<:Real}"),          # FidelityCalculations.jl:368
}


def _src():
    with open(SHIM) as fh:
        return fh.read()


def _signatures(src):
    sigs = {}
    for name, args in re.findall(r"^function (\w+)\((.*?)\)\s*$", src, re.M):
        types = [a.split("::", 1)[1].strip() if "::" in a else None
                 for a in re.split(r",\s*(?![^{]*\})", args.split(";")[0]) if a.strip()]
        sigs.setdefault(name, []).append(types)
    return sigs


def test_exported_entry_points_take_the_reference_types():
    src = _src()
    exported = re.search(r"export (.*?)\n\n", src, re.S).group(1)
    sigs = _signatures(src)
    for name, (t0, t1) in REFERENCE_SIGNATURES.items():
        assert name in exported, name
        assert name in sigs, name
        assert [t0, t1] in sigs[name], (name, sigs[name])


def test_reference_types_are_imported_not_redefined():
    src = _src()
    assert re.search(r"^using RobustGRAPE: .*\bUnitaryRobustGRAPEProblem\b.*\bFidelityRobustGRAPEProblem\b", src, re.M)
    for t in ("UnitaryRobustGRAPEProblem", "FidelityRobustGRAPEProblem", "ErrorSource"):
        assert not re.search(r"^\s*(mutable\s+)?struct %s\b" % t, src, re.M), t


def test_operator_basis_is_a_function():
    src = _src()
    assert re.search(r"^struct OperatorBasis <: Function$", src, re.M)
    # callable in the three closure shapes of src/Types.jl:10,25,50
    assert "(B::OperatorBasis)(nt, x, x_add) =" in src
    assert "(B::OperatorBasis)(nt, x, x_add, err) =" in src
    assert "(B::OperatorBasis)(x_add) =" in src


def test_plan_cache_is_keyed_by_problem_nparam_and_kind():
    src = _src()
    assert re.search(r"const _plans = Dict\{Tuple\{UInt,Int,Symbol\},DevicePlan\}\(\)", src)
    assert "key = (objectid(problem), nparam, kind)" in src
    kinds = set(re.findall(r"kind=:(\w+)", src)) | set(re.findall(r"_cached\(fp, nparam, :(\w+)\)", src))
    assert {"unitary", "table"} <= kinds, kinds
    # the unitary-level entry points wrap a UnitaryRobustGRAPEProblem (identity projector / target)
    assert "function fidelity_wrapper(problem::UnitaryRobustGRAPEProblem)" in src


def test_shim_checks_the_abi_version():
    from robustgrape_amd import _capi
    src = _src()
    m = re.search(r"const GRAPE_ABI_VERSION = (\d+)", src)
    assert m and int(m.group(1)) == _capi.ABI_VERSION
