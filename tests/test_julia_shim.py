"""Static checks of the Julia shim (julia/RobustGRAPEMI355X.jl) against the reference's Julia
interface.  Julia is not in the image, so the shim cannot run here; these checks pin what a
reference caller relies on:

* the entry points are METHODS OF THE REFERENCE'S OWN GENERICS (imported with
  `import RobustGRAPE: ...`), with a signature strictly more specific than the reference's, so
  the reference's own callers (optimize_fidelity_and_error_sources, FidelityCalculations.jl:177;
  the fidelity response, :246-343) dispatch to the device:
    reference: calculate_unitary_and_derivatives(problem::UnitaryRobustGRAPEProblem, x::Vector{<:Real})
        -- src/UnitaryCalculations.jl:20
    reference: calculate_interaction_error_operators(problem::UnitaryRobustGRAPEProblem, x::Vector{<:Real})
        -- src/UnitaryCalculations.jl:180
    reference: calculate_fidelity_and_derivatives(fidelity_problem::FidelityRobustGRAPEProblem, x::Vector{<:Real})
        -- src/FidelityCalculations.jl:19
    reference: calculate_expectation_values(fidelity_problem::FidelityRobustGRAPEProblem, x::Vector{<:Real})
        -- src/FidelityCalculations.jl:368
    shim: the same first argument, x::Vector{Float64} (never Vector{<:Real}: that would overwrite
    the reference's method instead of adding one);
* the shim defines no optimiser of its own: the reference's driver is re-exported and reaches the
  device through dispatch;
* closure tables with a non-Hermitian nominal H0 select the general-H0 plan (GRAPE_OPT_GENERAL_H0),
  above 12 levels non-Hermitian tables are refused (robustgrape_amd/engine.py general_h0_for);
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

# reference generic -> first-argument type of its method (x::Vector{<:Real} in every case)
REFERENCE_SIGNATURES = {
    "calculate_unitary_and_derivatives": "UnitaryRobustGRAPEProblem",      # UnitaryCalculations.jl:20
    "calculate_interaction_error_operators": "UnitaryRobustGRAPEProblem",  # UnitaryCalculations.jl:180
    "calculate_fidelity_and_derivatives": "FidelityRobustGRAPEProblem",    # FidelityCalculations.jl:19
    "calculate_expectation_values": "FidelityRobustGRAPEProblem",          # FidelityCalculations.jl:368
}


def _src():
    with open(SHIM) as fh:
        return fh.read()


def _signatures(src):
    sigs = {}
    found = re.findall(r"^function (\w+)\((.*?)\)\s*$", src, re.M)
    found += re.findall(r"^(\w+)\((.*?)\) =\s*$", src, re.M)  # one-expression methods
    for name, args in found:
        types = [a.split("::", 1)[1].strip() if "::" in a else None
                 for a in re.split(r",\s*(?![^{]*\})", args.split(";")[0]) if a.strip()]
        sigs.setdefault(name, []).append(types)
    return sigs


def _imported_generics(src):
    m = re.search(r"^import RobustGRAPE: (.*?)\n(?!\s)", src, re.M | re.S)
    assert m, "the shim must import the reference's generics to extend them"
    return {n.strip() for n in m.group(1).replace("\n", " ").split(",") if n.strip()}


def test_entry_points_extend_the_reference_generics():
    src = _src()
    imported = _imported_generics(src)
    sigs = _signatures(src)
    exported = re.search(r"export (.*?)\n\n", src, re.S).group(1)
    for name, t0 in REFERENCE_SIGNATURES.items():
        assert name in imported, name          # a method of RobustGRAPE.<name>, not a new function
        assert name in exported, name          # re-exported: the same binding as RobustGRAPE's
        assert [t0, "Vector{Float64}"] in sigs[name], (name, sigs[name])
        # Vector{<:Real} would REPLACE the reference's method (same signature), not add one
        assert [t0, "Vector{<:Real}"] not in sigs[name], (name, sigs[name])


def test_reference_driver_reaches_the_device_by_dispatch():
    src = _src()
    # no optimiser of the shim's own: RobustGRAPE.optimize_fidelity_and_error_sources calls
    # calculate_fidelity_and_derivatives(fidelity_problem, x) with x::Vector{Float64}
    # (FidelityCalculations.jl:177,209-211), which is the method above
    assert not re.search(r"^function optimize_fidelity_and_error_sources", src, re.M)
    assert re.search(r"^using RobustGRAPE: .*\boptimize_fidelity_and_error_sources\b", src, re.M | re.S)
    assert "optimize_fidelity_and_error_sources" in re.search(r"export (.*?)\n\n", src, re.S).group(1)


def test_closure_tables_check_hermiticity():
    from robustgrape_amd.operators import OPT_GENERAL_H0
    src = _src()
    m = re.search(r"const GRAPE_OPT_GENERAL_H0 = Int32\((\d+)\)", src)
    assert m and int(m.group(1)) == OPT_GENERAL_H0
    # every closure entry point picks its table plan from the tables it built
    assert src.count("table_plan(fp, np; general=_closure_general(") == 4
    assert "table_plan(fp, np)" not in src
    assert re.search(r"up\.ndim > 12", src) and "_is_hermitian(Hall)" in src


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
    kinds |= set(re.findall(r":(table\w*)", src))
    assert {"unitary", "table", "table_general"} <= kinds, kinds
    # the unitary-level entry points wrap a UnitaryRobustGRAPEProblem (identity projector / target)
    assert "function fidelity_wrapper(problem::UnitaryRobustGRAPEProblem)" in src


def test_shim_checks_the_abi_version():
    from robustgrape_amd import _capi
    src = _src()
    m = re.search(r"const GRAPE_ABI_VERSION = (\d+)", src)
    assert m and int(m.group(1)) == _capi.ABI_VERSION


def test_every_entry_point_falls_back_to_the_reference_method():
    """a problem libgrape refuses (GRAPE_ERR_UNSUPPORTED: d > 64, non-Hermitian
    closure tables above 12 levels, the dense engine's limits) is evaluated by the reference's own
    CPU method through `invoke` with the reference's signature -- never an error where the
    reference worked.  Other libgrape errors still raise."""
    src = _src()
    assert re.search(r"const GRAPE_ERR_UNSUPPORTED = Cint\(-2\)", src)
    from robustgrape_amd import _capi
    assert _capi.STATUS_NAMES[-2] == "GRAPE_ERR_UNSUPPORTED"
    # _check turns exactly that code into GrapeUnsupported, everything else into error(...)
    chk = re.search(r"^function _check\(rc\)\n(.*?)^end", src, re.M | re.S).group(1)
    assert "rc == GRAPE_ERR_UNSUPPORTED && throw(GrapeUnsupported(msg))" in chk and 'error("libgrape: "' in chk
    fb = re.search(r"^function _or_reference\(device_call, f, sig, args\.\.\.\)\n(.*?)^end", src, re.M | re.S).group(1)
    assert "e isa GrapeUnsupported || rethrow()" in fb and "return invoke(f, sig, args...)" in fb
    for name, t0 in REFERENCE_SIGNATURES.items():
        m = re.search(r"^%s\((\w+)::%s, x::Vector\{Float64\}\) =\n\s*_or_reference\(\(\) -> _device_\w+\(\1, x\), "
                      r"%s,\n\s*Tuple\{%s,Vector\{<:Real\}\}, \1, x\)" % (name, t0, name, t0), src, re.M)
        assert m, name
    # refusals found on the host side take the same path instead of error(...)
    assert "error(\"closure problems above 12 levels" not in src
    assert src.count('throw(GrapeUnsupported("ndim > GRAPE_MAX_DENSE_DIM (64)"))') == 4
