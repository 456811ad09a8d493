"""Throughput benchmark: GRAPE gradient-evals/sec, Rydberg CZ d=9, N_t=512 (BASELINE.json).

One step = one fidelity+gradient evaluation of every restart this rank owns
(SURVEY.md 8d C2 problem; restarts r with x_main = 2pi*0.001*U, theta = 2pi*U,
seed 1000+r as config C4), inputs resident in HBM, evaluated in device passes of
--chunk restarts.  After the K timed steps, still inside the timed region, the
sweep's exchange (robustgrape_amd/sweep.py): one all_gather of (best F, restart id)
over RCCL and a broadcast of the winning x, when N > 1.  Weak scaling: every rank
owns --batch restarts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--chunk C]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line on rank 0 (contract in the task statement), with
``roofline`` for the dominant kernel (per-launch HIP-event time on the plan's
stream), ``host_path`` (the drop-in grape_fidelity_grad with host arrays, PCIe
included) and ``single_eval`` (nbatch = 1, as Optim's loop calls the reference),
``cpu_baseline`` (the C++ port, 1 thread) and ``cpu_baseline_allcores`` (the port
over restarts on the job's CPU share), all on rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X dense FP64 (vector == matrix rate on gfx950)
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E (MI355X_MICROARCH.md)
D, NT, T0 = 9, 512, 7.613


def problem():
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    up = UnitaryRobustGRAPEProblem(t0=T0, ntimes=NT, ndim=D, H0=R.rydberg_full_operator_basis(1.0, 1.0, 0.0, 0.0, 10.0),
                                   nb_additional_param=1)
    return FidelityRobustGRAPEProblem(up, np.diag([1.0] * 4 + [0.0] * 5), R.cz_full_target())


def problem_c3():
    """C2 + 4 error sources (Omega1, Omega2 amplitude, delta1, delta2 detuning;
    the reference idiom Herror = H(perturbed) - H0, runtests.jl:475-476, as operator bases)."""
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    errs = [ErrorSource(R.full_rabi_error(1)), ErrorSource(R.full_rabi_error(2)),
            ErrorSource(R.full_detuning_error(1)), ErrorSource(R.full_detuning_error(2))]
    up = UnitaryRobustGRAPEProblem(t0=T0, ntimes=NT, ndim=D, H0=R.rydberg_full_operator_basis(1.0, 1.0, 0.0, 0.0, 10.0),
                                   nb_additional_param=1, error_sources=errs)
    return FidelityRobustGRAPEProblem(up, np.diag([1.0] * 4 + [0.0] * 5), R.cz_full_target())


T0_AR, NT_AR = 14.32, 200  # examples/ar_cz.jl:14-15


def problem_arcz():
    """examples/ar_cz.jl:17-36: the d = 5 symmetric blockaded CZ (RydbergTools.jl:31-39) with one
    amplitude error source, N_t = 200, t0 = 14.32 -- the reference's robust-optimisation call pattern
    (optimize_fidelity_and_error_sources evaluates one x per call, FidelityCalculations.jl:174-207)."""
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    up = UnitaryRobustGRAPEProblem(t0=T0_AR, ntimes=NT_AR, ndim=5, H0=R.rydberg_symmetric_blockaded_operator_basis(),
                                   nb_additional_param=1, error_sources=[ErrorSource(R.symmetric_amplitude_error())])
    return FidelityRobustGRAPEProblem(up, np.diag([1.0, 2.0, 1.0, 0.0, 0.0]), R.cz_symmetric_target())


def arcz_inputs(first, count):
    """x_initial of examples/ar_cz.jl:40: [2pi 0.001 U(N_t); 2pi U] (numpy seeds 43 + r)."""
    xs = []
    for r in range(first, first + count):
        rng = np.random.default_rng(43 + r)
        xs.append(np.concatenate([2 * math.pi * 0.001 * rng.uniform(size=NT_AR), [2 * math.pi * rng.uniform()]]))
    return np.stack(xs)


def restart_inputs(first, count):
    xs = []
    for r in range(first, first + count):
        rng = np.random.default_rng(1000 + r)
        xs.append(np.concatenate([2 * math.pi * 0.001 * rng.uniform(size=NT), [2 * math.pi * rng.uniform()]]))
    return np.stack(xs)


def c5_inputs(first, count):
    """C5 restarts: x ~ U[-1, 1) with seed 67 + r (r = 0 is the golden fixture's x)."""
    from robustgrape_amd import synthetic as S
    return np.stack([S.dense_x(seed=67 + r) for r in range(first, first + count)])


def flops_expm(d, m=5, s=0):
    """Algorithmic FP64 flops of one d x d complex Pade-m exp ((pi_m + s + 5/3) * 8 d^3)."""
    pi = {3: 2, 5: 3, 7: 4, 9: 5, 13: 6}[m]
    return (pi + s + 5.0 / 3.0) * 8 * d ** 3


PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")
WALK_STORE_LEVELS = 4  # csrc/grape_walk_api.hpp kWalkStoreMinD: walk classes of >= this many levels store E
PMC_SUMMARY_C5 = os.path.join(ROOT, "profiles", "pmc_c5_latest.json")
PMC_SUMMARY_C3 = os.path.join(ROOT, "profiles", "pmc_c3_latest.json")


def pmc_traffic(kernel, batch, path=PMC_SUMMARY, dims=None):
    """HBM bytes per launch of `kernel` from the committed PMC summary (scripts/gpu_profile.sh:
    separate FETCH_SIZE / WRITE_SIZE passes, FETCH doubled per the gfx950 correction), if it was
    recorded at this launch size (evaluations per device pass); else None."""
    if path is None:
        return None
    try:
        with open(path) as fh:
            js = json.load(fh)
    except (OSError, ValueError):
        return None
    if js.get("batch") != batch:
        return None
    # every instantiation of the kernel (the sector classes launch one each per device pass),
    # restricted to the template dimensions `dims` when given (the summary may also hold the
    # whole-matrix leg's instantiation)
    def dim(name):
        try:
            return int(name.split("<")[1].split(",")[0].split(">")[0])
        except (IndexError, ValueError):
            return None
    rows = [row["hbm_bytes_per_launch"] for name, row in js.get("kernels", {}).items()
            if name.split("<")[0].split("::")[-1] in (kernel, kernel + "_lane", kernel + "_chain_lane",  # lane variants
                                                       kernel + "_m")  # merged walks (both sector classes)
            and "hbm_bytes_per_launch" in row
            and (dims is None or dim(name) in dims)]
    return sum(rows) if rows else None


PMC_MIX = os.path.join(ROOT, "profiles", "pmc_mix_latest.json")


def pmc_executed_flop(kernel, batch, dims, path=PMC_MIX):
    """Executed FP64 FLOP per device pass of `kernel` (all its instantiations of the sector
    dimensions `dims`) from the committed instruction-mix summary recorded at this pass size, or None."""
    try:
        with open(path) as fh:
            js = json.load(fh)
        ks = js["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    if js.get("batch") != batch:
        return None
    tot = 0.0
    for name, row in ks.items():
        base = name.split("<")[0].split("::")[-1]
        try:
            dim = int(name.split("<")[1].split(",")[0].split(">")[0])
        except (IndexError, ValueError):
            dim = None
        if base in (kernel, kernel + "_m") and dim in dims and "fp64_flop_per_dispatch" in row:
            tot += row["fp64_flop_per_dispatch"]
    return tot or None


def pmc_mix(batch, path=PMC_MIX):
    """The committed instruction-mix summary (scripts/pmc_mix.py) if it was recorded at this pass size."""
    try:
        with open(path) as fh:
            js = json.load(fh)
    except (OSError, ValueError):
        return None
    return js if js.get("batch") == batch else None


def pmc_pass_flop(mix, per_pass_kernel, batch):
    """Executed FP64 FLOP per evaluation over every kernel of one device pass: sum over kernels of
    FLOP per dispatch x dispatches per pass (dispatch count over that of `per_pass_kernel`, which runs
    once per pass), divided by the pass's evaluations; None without dispatch counts."""
    if not mix:
        return None
    ks = mix.get("kernels", {})
    ref = [r.get("dispatches") for n, r in ks.items() if n.split("<")[0].split("::")[-1] in (per_pass_kernel, per_pass_kernel + "_m")]
    if not ref or not ref[0]:
        return None
    tot = 0.0
    for n, r in ks.items():
        if "fp64_flop_per_dispatch" in r and r.get("dispatches"):
            tot += r["fp64_flop_per_dispatch"] * r["dispatches"] / ref[0]
    return tot / batch


def pmc_pipeline(batch, per_pass_kernel, dims, path=PMC_SUMMARY):
    """PMC HBM bytes of one whole device pass: every kernel's mean bytes per dispatch times its
    dispatches per pass (dispatch count over that of `per_pass_kernel`, which runs once per pass
    per sector class), over kernels of the sector dimensions `dims` and the dimension-free ones."""
    try:
        with open(path) as fh:
            js = json.load(fh)
    except (OSError, ValueError):
        return None
    if js.get("batch") != batch:
        return None
    ks = js.get("kernels", {})
    def dim(name):
        try:
            return int(name.split("<")[1].split(",")[0].split(">")[0])
        except (IndexError, ValueError):
            return None
    ref = [r.get("dispatches") for n, r in ks.items()
           if n.split("<")[0].split("::")[-1] in (per_pass_kernel, per_pass_kernel + "_m") and dim(n) in dims]
    if not ref or not ref[0]:
        return None
    total = 0.0
    for n, r in ks.items():
        if "hbm_bytes_per_launch" not in r or not r.get("dispatches"):
            continue
        dn = dim(n)
        if dn is not None and dn not in dims:
            continue
        total += r["hbm_bytes_per_launch"] * r["dispatches"] / ref[0]
    return total


def _host_cpu():
    """CPU model and logical CPU count of the host (SURVEY.md 8d asks for both)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "logical_cpus": os.cpu_count()}


def cpu_baseline(seconds=15.0, fp=None, label="C2"):
    """Time the CPU restatement on a bounded sample of the same workload (rank 0, N = 1)."""
    try:
        from oracle.cref import cref
        have_c = cref.available()
    except Exception:
        have_c = False
    x = restart_inputs(0, 1)[0]
    if have_c:
        fp = fp or problem()
        t = time.perf_counter()
        n = 0
        while True:
            cref.fidelity_grad(fp, x)
            n += 1
            if time.perf_counter() - t > seconds:
                break
        dt = time.perf_counter() - t
        return {"value": n / dt, "unit": "gradient-evals/s", "cores": 1, "kind": "port",
                "sample": f"{n} sequential {label} evaluations (d=9, N_t=512) by the reference-faithful C++ "
                          f"restatement oracle/cref (same exp/inv/product counts as the Julia code), 1 thread",
                "host_cpu": _host_cpu()}
    from oracle import grape_oracle as O
    from tests import problems as P
    fp = P.full9_problem(NT, device=False)
    t = time.perf_counter()
    n = 0
    while True:
        O.calculate_fidelity_and_derivatives(fp, x)
        n += 1
        if time.perf_counter() - t > seconds:
            break
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "gradient-evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} sequential C2 evaluations by the numpy restatement oracle/grape_oracle.py, 1 thread"}


def cpu_baseline_c5(seconds, fp, x, label="C5"):
    """SURVEY.md 8d C5 CPU baseline: the reference-faithful C++ port (oracle/cref, 1 thread) on
    whole C5 evaluations (d = 64, N_t = 1 024: 5 120 Pade exponentials of 64 x 64 plus the LU
    inverses and trace products per evaluation, UnitaryCalculations.jl:44-100).  Warm-up: one
    evaluation of the same problem cut to 16 steps; then whole evaluations until `seconds` have
    passed (at least one; about 18-30 s each)."""
    from oracle.cref import cref
    from robustgrape_amd import synthetic as S
    if not cref.available():
        return None
    up = fp.unitary_problem
    ne = len(up.error_sources)
    nparam = (len(x) - up.nb_additional_param) // up.ntimes
    warm = (S.dense_error_problem(ntimes=16, nerr=ne) if ne else S.dense_problem(ntimes=16))
    cref.fidelity_grad(warm, S.dense_x(ntimes=16, nparam=nparam))
    t = time.perf_counter()
    n = 0
    while True:
        cref.fidelity_grad(fp, x)
        n += 1
        if time.perf_counter() - t > seconds:
            break
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "gradient-evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} whole {label} evaluation(s) (d=64, N_t=1024) by the reference-faithful C++ restatement "
                      f"oracle/cref after a 16-step warm-up, 1 thread", "seconds_per_eval": dt / n,
            "host_cpu": _host_cpu()}


def cpu_baseline_allcores(seconds=10.0, fp=None, label="C4"):
    """SURVEY.md 8d C4 CPU baseline: the C++ port over restarts on every host core this job may
    use (OpenMP; OMP_NUM_THREADS, the GPU box grants 16 CPUs per GPU), timed on a bounded sample."""
    try:
        from oracle.cref import cref
        if not cref.available():
            return None
    except Exception:
        return None
    fp = fp or problem()
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
    batch = 4 * threads
    X = restart_inputs(0, batch)
    t = time.perf_counter()
    n = 0
    while True:
        cref.fidelity_grad_batch(fp, X, threads)
        n += batch
        if time.perf_counter() - t > seconds:
            break
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "gradient-evals/s", "cores": threads, "kind": "port",
            "sample": f"{n} {label} restart evaluations (d=9, N_t=512) by oracle/cref, OpenMP over restarts "
                      f"on {threads} threads (the job's CPU share)", "host_cpu": _host_cpu()}


def host_path(fp, nparam, X, reps, label):
    """The drop-in entry the Julia shim calls: grape_fidelity_grad with HOST arrays in and out
    (PCIe included), as GrapePlan.fidelity_grad.  Returns evals/s over `reps` calls."""
    from robustgrape_amd.engine import GrapePlan
    plan = GrapePlan(fp, nparam=nparam, device=0, max_batch=min(len(X), 4096))
    plan.fidelity_grad(X)  # warm-up
    t = time.perf_counter()
    for _ in range(reps):
        plan.fidelity_grad(X)
    dt = time.perf_counter() - t
    plan.close()
    return {"value": reps * len(X) / dt, "unit": "gradient-evals/s", "batch": len(X), "calls": reps,
            "ms_per_call": dt / reps * 1e3,
            "note": f"{label}: grape_fidelity_grad, host x in / host F, F_dx out (pageable numpy buffers, "
                    "PCIe-inclusive), synchronous per call"}


def single_eval(fp, nparam, x, seconds=3.0):
    """nbatch = 1 through the host-array path: how Optim's loop calls the reference
    (FidelityCalculations.jl:177) -- one x per call, latency-bound."""
    from robustgrape_amd.engine import GrapePlan
    plan = GrapePlan(fp, nparam=nparam, device=0, max_batch=1)
    X = x[None, :]
    for _ in range(5):
        plan.fidelity_grad(X)
    lat = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        t = time.perf_counter()
        plan.fidelity_grad(X)
        lat.append(time.perf_counter() - t)
    # the same C entry called as a Julia ccall would: preallocated buffers, no Python wrapper
    from robustgrape_amd import _capi
    L, h = _capi.lib(), plan.handle
    X = np.ascontiguousarray(X, dtype=np.float64)
    F, Fdx = np.empty(1), np.empty((1, plan.nx))
    Fd2 = np.empty((1, plan.nerr)) if plan.nerr else None
    Fd2dx = np.empty((1, plan.nerr, plan.nx)) if plan.nerr else None
    args = (h, 1, _capi.dptr(X), _capi.dptr(F), _capi.dptr(Fdx), _capi.dptr(Fd2), _capi.dptr(Fd2dx))
    raw = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < min(1.0, seconds):
        t = time.perf_counter()
        L.grape_fidelity_grad(*args)
        raw.append(time.perf_counter() - t)
    plan.close()
    lat, raw = np.array(lat), np.array(raw)
    return {"value": len(lat) / lat.sum(), "unit": "gradient-evals/s", "calls": len(lat),
            "latency_ms_median": float(np.median(lat) * 1e3), "latency_ms_p90": float(np.percentile(lat, 90) * 1e3),
            "c_entry_latency_ms_median": float(np.median(raw) * 1e3),
            "note": "nbatch = 1, host arrays in and out (grape_fidelity_grad), one synchronous call per evaluation; "
                    "c_entry_*: the same entry through a bare ctypes call with preallocated buffers (a ccall's view)"}


def _roofline(kname, flop_launch, ktimes, batch, pmc_path=PMC_SUMMARY):
    ms_k, n_k = ktimes[kname]
    per_launch_ms = ms_k / max(1, n_k)
    achieved = flop_launch / (per_launch_ms * 1e-3) / 1e12
    return {"bound": "mfma", "kernel": kname, "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
            "traffic": pmc_traffic(kname, batch, pmc_path), "traffic_unit": "HBM bytes per launch (PMC)",
            "per_launch_ms": per_launch_ms, "flop_per_launch": flop_launch}


def _kernel_fracs(flop_model, ktimes):
    """Fraction of the FP64 peak per modelled kernel (algorithmic FLOP per launch / mean launch time)."""
    out = {}
    for k, f in flop_model.items():
        ms, n = ktimes.get(k, (0.0, 0))
        if n and ms > 0:
            out[k] = f / (ms / n * 1e-3) / 1e12 / FP64_PEAK_TFLOPS
    return out


def c2_report(args, B, L, world, value, elapsed, ktimes, sectors=None, passes=None, info=None):
    """C2 bench line.  `sectors`: GrapePlan.sectors() -- ((S, nsec), ...) per sector class, or
    ((D, 1),) for whole matrices; `passes`: device passes in the timed region (per-pass kernel
    times = total / passes: the sector classes launch each kernel once per class)."""
    nvg = 1  # np = 1 control; H0 does not read x_add, so no x_add variants
    classes = tuple(sectors) if sectors else ((D, 1),)
    sec = classes[0][0] < D
    twins = tuple((info or {}).get("twin", ())) + (False,) * len(classes)
    gauges = tuple((info or {}).get("gauge", ())) + (False,) * len(classes)
    per_step = lambda f: sum(ns * f(S) for S, ns in classes)  # noqa: E731
    ladders = tuple((info or {}).get("ladder", ())) + (False,) * len(classes)
    walk = ktimes.get("k_walk_grad", (0.0, 0))[1] > 0
    # both classes walked by one lane (grape_walk.hpp k_walk_fwd_m / k_walk_grad_m): one walk launch per
    # stage and pass instead of one per class
    merged = bool(walk and passes and ktimes.get("k_walk_grad", (0.0, 0))[1] == passes)
    from robustgrape_amd import _capi
    defines = set(_capi.build_defines())
    # merged gradient walk, twin class: ONE summed state for both sectors (GRAPE_WALK_TWIN_SUM, on by
    # default): its products and contraction run once per step, not once per sector
    twin_sum = merged and "GRAPE_WALK_TWIN_SUM=0" not in defines
    ladder_contr = merged and "GRAPE_WALK_LADDER_CONTR=0" not in defines
    nX = lambda c, ns: 1 if (twins[c] and twin_sum) else ns  # noqa: E731  (gradient states of a class)
    # Executed FP64 FLOP (FMA = 2, MUL / ADD = 1) per step of the phase-covariant walks
    # (grape_walk.hpp), term by term:
    #  E_k = D_k E~ D_k^dag: one complex product (6) per off-diagonal entry, plus the pair phases' powers
    #    p^2 .. p^{S-1} (one product each);
    #  a product of two S x S complex matrices: 8 S^3 (Y = X E^dag and X <- E Y in the gradient walk,
    #    Q <- E Q in the forward walk);
    #  the eps-difference contraction: ladder charges grouped by charge difference (merged walks,
    #    GRAPE_WALK_LADDER_CONTR): 4 FMA per off-diagonal entry, 2 FMA per charge difference, the
    #    weights rho(m) (10 each beyond m = 1) and 1/eps; otherwise per entry E_rj f_rj / eps (8) and a
    #    real MAC pair (4), the weights per level pair;
    #  per step and lane (shared by the classes of a merged lane): e^{i a x_k} (grape_cis.hpp: ~37) and,
    #    in the gradient walk, e^{i phi} - 1 of the FD phase (~27).
    # A non-phase-covariant class is credited SURVEY 8d's Pade-5 exponential instead of E_k's formation.
    gform = lambda S: 6 * (S * S - S) + 6 * max(0, S - 2)  # noqa: E731
    prop = lambda c, S: gform(S) if gauges[c] else flops_expm(S)  # noqa: E731
    contr = lambda c, S: ((8 * (S * S - S) + 4 * (S - 1) + 1 + 10 * max(0, S - 2))  # noqa: E731
                          if (gauges[c] and ladders[c] and ladder_contr) else
                          (12 * (S * S - S) + 10 * max(0, S - 2)) if gauges[c] else 8 * S ** 2)
    trig_f, trig_g = (37, 64) if any(gauges[:len(classes)]) else (0, 0)
    lanes_per_step = 1 if merged else len(classes)  # the trig runs once per lane and step
    xbytes = L * 8 * (NT + 1)  # the x rows every per-step kernel streams
    if walk:
        # chunk walks (grape_walk.hpp), executed work per device pass: the forward walk
        # forms every state's E_k and its chain product; the gradient walk forms E_k again, Y = X E^dag,
        # the contraction and X <- E Y per gradient state.  The 4-level class of a non-phase-covariant
        # plan stores E once (walk_store_e) and the gradient walk reads it back -- the only per-step HBM
        # intermediate left.
        store = lambda S: S >= WALK_STORE_LEVELS and not any(gauges)  # noqa: E731
        nE = lambda c, ns: 1 if twins[c] else ns  # noqa: E731
        flop_model = {"k_walk_fwd": L * NT * (sum(nE(c, ns) * (prop(c, S) + 8 * S ** 3)
                                                  for c, (S, ns) in enumerate(classes)) + lanes_per_step * trig_f),
                      "k_walk_grad": L * NT * (nvg * sum(nE(c, ns) * prop(c, S) + nX(c, ns) * (2 * 8 * S ** 3 + contr(c, S))
                                                         for c, (S, ns) in enumerate(classes)) + lanes_per_step * trig_g)}
        byte_model = {"k_walk_fwd": xbytes + L * NT * per_step(lambda S: 16 * S * S if store(S) else 0),
                      "k_walk_grad": xbytes + L * NT * per_step(lambda S: 16 * S * S if store(S) else 0)}
    else:
        # stored-intermediate pipeline (GRAPE_OPT_NO_WALK / whole matrices): k_expm writes E;
        # k_scan reads E, writes Q; k_expm_grad reads E_k and Q_k
        flop_model = {"k_expm": L * NT * per_step(flops_expm),
                      "k_expm_grad": L * NT * nvg * per_step(lambda S: flops_expm(S) + 2 * 8 * S ** 3 + 8 * S ** 2)}
        byte_model = {"k_expm": L * NT * per_step(lambda S: 16 * S * S),
                      "k_scan": L * NT * per_step(lambda S: 2 * 16 * S * S),
                      "k_expm_grad": L * NT * nvg * per_step(lambda S: 2 * 16 * S * S)}
    eval1 = ktimes.get("k_eval1", (0.0, 0))[1] > 0
    if eval1:
        # one workgroup per evaluation (grape_eval1.hip): the walks' per-step work of both classes (the
        # merged walks' model with one lane per chunk of 256) in one kernel
        walk = True
        merged = True
        nE = lambda c, ns: 1 if twins[c] else ns  # noqa: E731
        store = lambda S: False  # noqa: E731
        step = sum(nE(c, ns) * (2 * prop(c, S) + 8 * S ** 3) + nX(c, ns) * (2 * 8 * S ** 3 + contr(c, S))
                   for c, (S, ns) in enumerate(classes)) + trig_f + trig_g
        flop_model = {"k_eval1": L * NT * step}
        byte_model = {"k_eval1": xbytes + L * 8 * (NT + 2)}
    grad_name = "k_eval1" if eval1 else ("k_walk_grad" if walk else "k_expm_grad")
    npass = passes or max(1, ktimes.get(grad_name, (0.0, 1))[1])
    per_pass = {k: v[0] / npass for k, v in ktimes.items() if v[1]}
    kname = max(flop_model, key=lambda k: per_pass.get(k, 0.0))
    ms = per_pass[kname]
    dims = {S for S, _ in classes}
    # FLOP per launch: the FP64 the VALU issued, from the instruction-mix PMC pass recorded on THIS build
    # at this pass size (profiles/pmc_mix_latest.json, scripts/gpu_pmc_mix.sh: 64 x (2 FMA + MUL + ADD)
    # F64 instructions per dispatch) when there is one; else the term-by-term model above.  Both are in
    # the line with their ratio, so the credited work can be checked against the counters.
    mix = pmc_mix(L)
    mix_build = (mix or {}).get("build_id")
    this_build = _capi.build_id()
    ex = pmc_executed_flop(kname, L, dims) if mix_build == this_build else None
    flop = ex if ex is not None else flop_model[kname]
    fp = flop / (ms * 1e-3) / 1e12
    hb = byte_model[kname] / (ms * 1e-3) / 1e9
    traffic = pmc_traffic(kname, L, dims=dims)
    fp_frac, hb_frac = fp / FP64_PEAK_TFLOPS, hb / HBM_PEAK_GBS
    if hb_frac > fp_frac:
        roof = {"bound": "hbm", "kernel": kname, "achieved": hb, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": hb_frac, "traffic": traffic}
    else:
        roof = {"bound": "fp64-valu", "kernel": kname, "achieved": fp, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": fp_frac, "traffic": traffic,
                "pipe": "fp64 (VALU; gfx950 FP64 vector peak == matrix peak)"}
    roof.update({"traffic_unit": "HBM bytes per device pass (PMC)", "per_launch_ms": ms,
                 "per_launch_note": "per device pass of evals_per_device_pass evaluations (all sector classes)",
                 "flop_per_launch": flop,
                 "flop_source": ("pmc: FP64 VALU instructions of this build (profiles/pmc_mix_latest.json)"
                                 if ex is not None else "model (no instruction-mix PMC of this build)"),
                 "flop_per_launch_model": flop_model[kname],
                 "model_over_pmc": (flop_model[kname] / ex) if ex else None,
                 "pmc_mix_build_id": mix_build, "build_id": this_build,
                 "algorithmic_bytes_per_launch": byte_model[kname],
                 "fp64": {"achieved_TFLOPs": fp, "frac": fp_frac},
                 "hbm": {"achieved_GBs": hb, "frac": hb_frac,
                         "traffic_GBs": (traffic / (ms * 1e-3) / 1e9) if traffic else None}})
    pipe = pmc_pipeline(L, grad_name, dims)
    if pipe is not None:
        total_ms = sum(per_pass.values())
        roof["pipeline_traffic"] = {"bytes_per_pass": pipe, "bytes_per_eval": pipe / L,
                                    "GBs_over_pass": pipe / (total_ms * 1e-3) / 1e9,
                                    "note": "PMC HBM bytes of every kernel of one device pass (sector classes, "
                                            "scans, head, reductions), over the summed kernel time"}
    out = {
        "metric": "GRAPE gradient-evals/sec (fidelity+∇), Rydberg CZ d=9 N_t=512, 1→8 GPU",
        "value": value, "unit": "gradient-evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C2/C4: Rydberg CZ d=9 (rydberg_hamiltonian_full, B=10), N_t=512, "
                               "np=1, na=1, ne=0; restart sweep",
                   "restarts_per_gpu": B, "global_batch": B * world, "parallelism": f"restarts x{world}",
                   "pipeline": "chunk walks" if walk else ("sector kernels" if sec else "whole matrices"),
                   "sectors": [{"levels": S, "sectors": ns, "stored_propagators": bool(walk and store(S)),
                                "twin": bool(twins[c])}
                               for c, (S, ns) in enumerate(classes)] if sec else None,
                   "symmetry_adapted": bool((info or {}).get("symmetric", False)),
                   "phase_covariant": [bool(g) for g in gauges[:len(classes)]],
                   # both classes in one lane (grape_walk.hpp k_walk_fwd_m / k_walk_grad_m): one walk
                   # launch per stage and pass instead of one per class
                   "merged_walks": merged, "twin_sum": twin_sum,
                   "ladder_charges": [bool(x) for x in ladders[:len(classes)]]},
        "roofline": roof,
        "kernels_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in ktimes.items() if v[1]},
        "kernels_ms_per_pass": per_pass,
    }
    # whole-evaluation view: FLOP executed per evaluation -- the PMC FP64 count of every
    # kernel of one device pass of this build (dispatches per pass from the same profile) over the pass's
    # evaluations when recorded, else the walks' model (the head and scan not modelled) -- and the
    # survey's canonical whole-matrix C2 figure (not executed, not credited with sectors)
    exe_model = NT * (sum((1 if twins[c] else ns) * ((1 + nvg) * prop(c, S) + 8 * S ** 3)
                          + nX(c, ns) * (2 * 8 * S ** 3 + nvg * contr(c, S)) for c, (S, ns) in enumerate(classes))
                      + lanes_per_step * (trig_f + trig_g)) if walk else None
    exe_pmc = pmc_pass_flop(mix, kname, L) if mix_build == this_build else None
    exe = exe_pmc if exe_pmc is not None else exe_model
    canon = NT * (3 * flops_expm(D) + 3 * 8 * D ** 3 + 2 * 8 * D ** 2)
    out["roofline"]["whole_eval"] = {
        "flop_per_eval_executed": exe, "achieved_executed": (exe * value / 1e12) if exe else None,
        "frac_executed": (exe * value / 1e12 / FP64_PEAK_TFLOPS) if exe else None,
        "source": "pmc (every kernel of a pass, this build)" if exe_pmc is not None else "model (walks only)",
        "flop_per_eval_model_walks": exe_model, "flop_per_eval_survey": canon}
    if sec:
        out["roofline"]["whole_eval"]["note"] = (
            "sectors: the executed work is the block-diagonal work; SURVEY 8d's whole-matrix "
            "figure (flop_per_eval_survey) is not executed and is not credited")
    else:
        out["roofline"]["whole_eval"].update({"achieved_survey": canon * value / 1e12,
                                              "frac_survey": canon * value / 1e12 / FP64_PEAK_TFLOPS})
    out["kernels_frac"] = {k: f / (per_pass[k] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS
                           for k, f in flop_model.items() if per_pass.get(k)}
    out["kernels_hbm_frac"] = {k: f / (per_pass[k] * 1e-3) / 1e9 / HBM_PEAK_GBS
                               for k, f in byte_model.items() if per_pass.get(k)}
    return out


def whole_matrix_leg(fp, nparam, X, F, Fdx, L, stream, args):
    """The same C2 step on whole 9 x 9 matrices (plan option GRAPE_OPT_NO_SECTORS): the row-group kernels'
    own efficiency, and the speed-up the sector decomposition adds on top of it."""
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_NO_SECTORS
    import torch
    plan = GrapePlan(fp, nparam=nparam, device=X.device.index or 0, max_batch=L, options=OPT_NO_SECTORS)
    plan.set_stream(stream.cuda_stream)
    n = X.shape[0]
    steps = max(3, args.steps // 5)
    step = lambda: plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), Fdx.data_ptr(), n, 0, 0)  # noqa: E731
    step()
    plan.synchronize()
    plan.kernel_times(reset=True)
    plan.set_profiling(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    plan.synchronize()
    kt = plan.kernel_times()
    plan.close()
    passes = steps * ((n + L - 1) // L)
    ms = kt["k_expm_grad"][0] / passes
    fl = L * NT * (flops_expm(D) + 2 * 8 * D ** 3 + 8 * D ** 2)
    tr = pmc_traffic("k_expm_grad", L, dims={D})
    return {"value": steps * n / dt, "unit": "gradient-evals/s", "steps": steps,
            "k_expm_grad": {"per_launch_ms": ms, "achieved_TFLOPs": fl / (ms * 1e-3) / 1e12,
                            "frac": fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, "traffic": tr,
                            "traffic_GBs": (tr / (ms * 1e-3) / 1e9) if tr else None},
            "kernels_ms_per_step": {k: v[0] / steps for k, v in kt.items() if v[1]},
            "note": "same workload with sectors disabled (GRAPE_OPT_NO_SECTORS): whole 9 x 9 matrices"}


def c4_points(fp, nparam, inputs, dev, batches=(256, 32), seconds=1.5):
    """BASELINE C4 as specified: 256 restarts over 8 GPUs = 32 per GPU (and the whole 256 on one
    GPU), device-resident x, one plan sized to the batch, back-to-back steps on one stream."""
    import torch
    from robustgrape_amd.engine import GrapePlan
    out = {}
    for b in batches:
        plan = GrapePlan(fp, nparam=nparam, device=dev.index or 0, max_batch=b)
        st = torch.cuda.Stream(device=dev)
        plan.set_stream(st.cuda_stream)
        X = torch.from_numpy(inputs(0, b)).to(dev)
        F = torch.empty(b, dtype=torch.float64, device=dev)
        G = torch.empty(b, X.shape[1], dtype=torch.float64, device=dev)
        step = lambda: plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), G.data_ptr(), b, 0, 0)  # noqa: E731
        tw = time.perf_counter()  # warm-up by the clock (the GPU leaves its idle state: see c4_strong)
        while time.perf_counter() - tw < 0.3:
            for _ in range(10):
                step()
            plan.synchronize()
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(10):
                step()
            n += 10
            plan.synchronize()
        dt = time.perf_counter() - t0
        plan.close()
        out[f"batch_{b}"] = {"value": n * b / dt, "unit": "gradient-evals/s", "ms_per_step": dt / n * 1e3,
                             "steps": n}
    if "batch_256" in out and "batch_32" in out:
        # 1 -> 8 GPU strong scaling of the 256-restart sweep implied by the two single-GPU points,
        # before the (microsecond-scale) all_gather: 8 GPUs at 32 each against one GPU at 256
        out["projected_8gpu_strong_ratio"] = 8 * out["batch_32"]["value"] / out["batch_256"]["value"]
    out["note"] = ("C4 as BASELINE names it: 256 restarts / 8 GPUs = 32 per GPU; per-GPU rate at that batch "
                   "(x resident in HBM, steps queued back to back on the plan's stream)")
    return out


def c3_report(args, B, L, world, value, elapsed, ktimes, ne, sectors=None, passes=None, info=None):
    # k_expm exponentiates every stored variant of every step: nominal, x + eps, x + eps2,
    # and per error source err(eps), err(eps2), (x + eps2, err eps2) -> 3 + 3 ne (Pade 5);
    # the x_add variants are skipped (H0 does not read x_add: their differences are exactly 0)
    nv = 3 + 3 * ne
    # k_err_local: per step nz = np (1 + ne) + ne local-frame images, 2 complex S x S products
    # each; k_err_grad: per (step, error) 2 products (the B_k recurrence, grape_errpath.hpp).
    # With sectors every item is one S x S sector, summed over the classes.
    nz = 1 * (1 + ne) + ne
    classes = tuple(sectors) if sectors else ((D, 1),)
    sec = classes[0][0] < D
    per_step = lambda f: sum(ns * f(S) for S, ns in classes)  # noqa: E731
    prod = lambda S: 8 * S ** 3  # noqa: E731
    tile = lambda S: 16 * S * S  # noqa: E731
    walk = ktimes.get("k_walk_fwd", (0.0, 0))[1] > 0
    gauges = tuple((info or {}).get("gauge", ())) + (False,) * len(classes)
    # the phase-covariant image walk (grape_walk.hpp k_walk_img_gauge) per (step, sector): no
    # exponential; E_k from E0 and the level phases, one product each for Z1 and Z2_e (E0^dag (M o f)),
    # two per image (Q^dag Z Q), the chain product, and the phase sandwiches / stencil weights
    img_gauge = lambda S: 8 * S ** 3 * (1 + 3 * (1 + ne) + 2 * ne) + (S * S - S) * (12 + 34 * (1 + ne) + 12 * ne)  # noqa: E731
    img_step = lambda c, S: img_gauge(S) if gauges[c] else nv * flops_expm(S) + prod(S) * (1 + 3 * nz)  # noqa: E731
    # the lab-frame error walks (grape_walk.hpp GRAPE_WALK_ERR_LAB, round 6: every class phase-covariant, no
    # images).  Per (step, sector, error): k_walk_wsum_lab 3 products (E~ R~ + N_e, . E~^dag, E~ Q^), the
    # pair-phase rotation of R~ and the row phases of Q^; k_walk_err_lab 6 products (Y~, Lambda, G~, E~ G~,
    # N_e Y~, E~ Y~), two weighted traces (a complex product and 2 FMAs per off-diagonal entry) and two
    # rotations, plus per (step, sector) its F_dx lanes: 2 products, a trace, a rotation.  HBM: the x rows
    # (one 8-B read per lane and step), the per-(step, error) terms written, the chunk states.
    from robustgrape_amd import _capi
    lab = walk and all(gauges[:len(classes)]) and "GRAPE_WALK_ERR_LAB=0" not in set(_capi.build_defines())
    off = lambda S: S * S - S  # noqa: E731
    lab_fwd = lambda S: ne * (3 * prod(S) + 6 * off(S) + 6 * S * S + 2 * S * S)  # noqa: E731
    lab_err = lambda S: ne * (6 * prod(S) + 2 * 10 * off(S) + 2 * 6 * off(S)) + (2 * prod(S) + 16 * off(S))  # noqa: E731
    if lab:
        flop_model = {"k_walk_fwd": L * NT * per_step(lab_fwd), "k_err_grad": L * NT * per_step(lab_err)}
        nsub = sum(ns for _, ns in classes)
        byte_model = {"k_walk_fwd": L * 8 * NT * ne * len(classes) + L * (ne + 1) * 16 * per_step(lambda S: S * S) * 8,
                      "k_grad/k_err_local": 0,
                      "k_err_grad": L * 8 * NT * (ne + 1) * len(classes) + L * NT * 8 * nsub * (ne + 1)}
    elif walk:
        # image walk (grape_walk.hpp k_walk_img) per (step, sector): the nv variant
        # exponentials, the chain product Q <- E Q and per image Z = E^dag dX, Y = Q^dag Z Q (3
        # products); HBM: the x row and the nz images written.  k_img_fdx (reported under
        # "k_grad/k_err_local") reads Z1 and M'_c; k_err_grad reads W, Z1, Z2 per (step, error).
        flop_model = {"k_walk_fwd": L * NT * sum(ns * img_step(c, S) for c, (S, ns) in enumerate(classes)),
                      "k_err_grad": L * NT * ne * 2 * per_step(prod)}
        byte_model = {"k_walk_fwd": L * 8 * (NT + 1) + L * NT * nz * per_step(tile),
                      "k_grad/k_err_local": L * NT * per_step(tile),
                      "k_err_grad": L * NT * ne * 3 * per_step(tile)}
    else:
        flop_model = {"k_expm": L * NT * nv * per_step(flops_expm),
                      "k_grad/k_err_local": L * NT * nz * 2 * per_step(prod),
                      "k_err_grad": L * NT * ne * 2 * per_step(prod)}
        # algorithmic HBM bytes per pass: k_expm writes the nv variants; k_err_local reads them and
        # Q_k, writes the nz images; k_err_grad reads W, Z1, Z2 per (step, error)
        byte_model = {"k_expm": L * NT * nv * per_step(tile),
                      "k_grad/k_err_local": L * NT * (nv + 1 + nz) * per_step(tile),
                      "k_err_grad": L * NT * ne * 3 * per_step(tile)}
    npass = passes or max(1, ktimes.get("k_walk_fwd" if walk else "k_expm", (0.0, 1))[1])
    per_pass = {k: v[0] / npass for k, v in ktimes.items() if v[1]}
    kname = max(flop_model, key=lambda k: per_pass.get(k, 0.0))
    ms = per_pass[kname]
    fp = flop_model[kname] / (ms * 1e-3) / 1e12
    hb = byte_model[kname] / (ms * 1e-3) / 1e9
    img_kernel = "k_walk_wsum_lab" if lab else "k_walk_img_gauge" if any(gauges[:len(classes)]) else "k_walk_img"
    short = {"k_grad/k_err_local": "k_err_local", "k_walk_fwd": img_kernel,
             "k_err_grad": "k_walk_err_lab" if lab else "k_walk_err_grad" if walk else "k_err_grad"}.get(kname, kname)
    traffic = pmc_traffic(short, L, PMC_SUMMARY_C3, dims={S for S, _ in classes})
    if hb / HBM_PEAK_GBS > fp / FP64_PEAK_TFLOPS:
        roof = {"bound": "hbm", "kernel": kname, "achieved": hb, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": hb / HBM_PEAK_GBS}
    else:
        roof = {"bound": "fp64-valu", "kernel": kname, "achieved": fp, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": fp / FP64_PEAK_TFLOPS, "pipe": "fp64 (VALU; gfx950 FP64 vector peak == matrix peak)"}
    roof.update({"traffic": traffic, "traffic_unit": "HBM bytes per device pass (PMC)", "per_launch_ms": ms,
                 "per_launch_note": "per device pass of evals_per_device_pass evaluations (all sector classes)",
                 "flop_per_launch": flop_model[kname], "algorithmic_bytes_per_launch": byte_model[kname],
                 "fp64": {"achieved_TFLOPs": fp, "frac": fp / FP64_PEAK_TFLOPS},
                 "hbm": {"achieved_GBs": hb, "frac": hb / HBM_PEAK_GBS}})
    out = {
        "metric": "GRAPE gradient-evals/sec (fidelity+sensitivity+gradients), Rydberg CZ d=9 N_t=512, 4 error sources",
        "value": value, "unit": "gradient-evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C3: Rydberg CZ d=9 + 4 error operators (Omega1, Omega2, delta1, delta2), N_t=512, "
                               "np=1, na=1; F, F_dx, F_d2err, F_d2err_dx",
                   "restarts_per_gpu": B, "global_batch": B * world, "parallelism": f"restarts x{world}",
                   "sectors": [{"levels": S, "sectors": ns} for S, ns in classes] if sec else None,
                   "phase_covariant": [bool(g) for g in gauges[:len(classes)]],
                   "error_walks": "lab-frame (no images)" if lab else "image walk" if walk else "stored variants"},
        "roofline": roof,
        "kernels_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in ktimes.items() if v[1]},
    }
    # SURVEY.md 8d canonical (whole-matrix) C3 figure: 352.7 MFLOP per evaluation
    canon = NT * (1 + 2 + 2 + ne * (2 + 1 + 1)) * flops_expm(D) + 3 * NT * 8 * D ** 3 \
        + 4 * NT * ne * 8 * D ** 3 + 8 * D ** 2 * NT * 2 * (1 + ne)
    # FLOP of the work executed per evaluation: the stored variant exps, the nominal chain,
    # the local-frame images (3 products each in the image walk: E^dag dX, Q^dag . Q), the B_k
    # recurrence and the contractions (+ the sector heads)
    nimg = 3 if walk else 2
    exe = NT * sum(ns * ((img_step(c, S) if walk else nv * flops_expm(S) + prod(S) + nz * nimg * prod(S))
                         + ne * 2 * prod(S) + 8 * S ** 2 * (1 + ne)) for c, (S, ns) in enumerate(classes))
    if lab:
        exe = NT * per_step(lambda S: lab_fwd(S) + lab_err(S))
    if sec:
        exe += (16 + 24 * ne) * 8 * D ** 3
    out["roofline"]["whole_eval"] = {"flop_per_eval_executed": exe, "achieved_executed": exe * value / 1e12,
                                     "frac_executed": exe * value / 1e12 / FP64_PEAK_TFLOPS,
                                     "flop_per_eval_survey": canon}
    if walk:  # PMC HBM bytes of one whole device pass (every kernel), against the pass time
        pipe = pmc_pipeline(L, img_kernel, {S for S, _ in classes}, PMC_SUMMARY_C3)
        if pipe:
            pass_ms = sum(per_pass.values())
            out["roofline"]["pipeline_traffic"] = {
                "bytes_per_pass": pipe, "bytes_per_eval": pipe / L, "GBs_over_pass": pipe / (pass_ms * 1e-3) / 1e9,
                "frac_hbm": pipe / (pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "note": ("PMC HBM bytes of every kernel of one device pass (lab-frame walks: x rows, chunk states, "
                         "per-step terms; no images), over the summed kernel time" if lab else
                         "PMC HBM bytes of every kernel of one device pass (images written by the image walk and "
                         "re-read by k_walk_img_sum and k_walk_err_grad dominate), over the summed kernel time")}
    if not sec:
        out["roofline"]["whole_eval"].update({"achieved_survey": canon * value / 1e12,
                                              "frac_survey": canon * value / 1e12 / FP64_PEAK_TFLOPS})
    out["kernels_frac"] = {k: f / (per_pass[k] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS
                           for k, f in flop_model.items() if per_pass.get(k)}
    out["kernels_hbm_frac"] = {k: f / (per_pass[k] * 1e-3) / 1e9 / HBM_PEAK_GBS
                               for k, f in byte_model.items() if per_pass.get(k)}
    # PMC bytes of the error-path kernels (committed C3 summary) over their per-pass time
    hbm = {}
    for k, sh in (("k_grad/k_err_local", "k_err_local"), ("k_err_grad", "k_err_grad"),
                  ("k_err_scan", "k_err_scan"), ("k_scan", "k_scan")):
        t = pmc_traffic(sh, L, PMC_SUMMARY_C3, dims={S for S, _ in classes})
        if per_pass.get(k) and t:
            gbs = t / (per_pass[k] * 1e-3) / 1e9
            hbm[sh] = {"traffic_bytes": t, "achieved_GBs": gbs, "frac_hbm": gbs / HBM_PEAK_GBS}
    out["kernels_hbm"] = hbm
    return out


def c5err_report(args, B, L, world, value, elapsed, ktimes, d, nt, nparam, ne):
    # C5 + error sources (dense error path): per step nv = 1 + 2 np + ne (2 + np) stored variant
    # exponentials (Pade 7 at this scale), nz = np (1 + ne) + ne local-frame images (2 products
    # each), 2 products per (step, error) in k_derr_grad
    fe = flops_expm(d, 7)
    nv, nz = 1 + 2 * nparam + ne * (2 + nparam), nparam * (1 + ne) + ne
    prod = 8 * d ** 3
    flop_model = {"k_dexp": L * nt * nv * fe, "k_grad/k_err_local": L * nt * nz * 2 * prod,
                  "k_err_grad": L * nt * ne * 2 * prod}
    kname = max(flop_model, key=lambda k: ktimes.get(k, (0.0, 0))[0])
    out = {
        "metric": "GRAPE gradient-evals/sec (fidelity+sensitivity+gradients), synthetic d=64 N_t=1024, 2 error sources",
        "value": value, "unit": "gradient-evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C5 + 2 error sources (control-1 amplitude, static Ginibre), d=64, N_t=1024, np=2",
                   "restarts_per_gpu": B, "global_batch": B * world, "parallelism": f"restarts x{world}"},
        "roofline": dict(_roofline(kname, flop_model[kname], ktimes, L, None),
                         pipe="fp64 MFMA v_mfma_f64_16x16x4_f64"),
        "kernels_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in ktimes.items() if v[1]},
    }
    # SURVEY.md 8d canonical FLOP per evaluation (ne > 0 form, na = 0)
    canon = nt * nv * fe + 3 * nt * prod + 4 * nt * ne * prod + 8 * d ** 2 * nt * nparam * (1 + ne)
    out["roofline"]["whole_eval"] = {"flop_per_eval_survey": canon, "achieved_survey": canon * value / 1e12,
                                     "frac_survey": canon * value / 1e12 / FP64_PEAK_TFLOPS}
    out["kernels_frac"] = _kernel_fracs(flop_model, ktimes)
    return out


def c5_report(args, B, L, world, value, elapsed, ktimes, d, nt, nparam):
    # C5 draws Pade m = 7 for every exponential (tests/golden/c5.npz pade_hist); per launch:
    # k_dexp: B*nt nominal exps; k_dgrad: per step 2 products (Q_{k-1} M'_c, Z_k) and, per
    # control, one eps-variant exp + the contraction; k_dscan: one product per step.
    fe = flops_expm(d, 7)
    flop_model = {"k_dexp": L * nt * fe,
                  "k_dgrad": L * nt * (2 * 8 * d ** 3 + nparam * (fe + 8 * d ** 2)),
                  "k_dscan": L * nt * 8 * d ** 3}
    kname = max(flop_model, key=lambda k: ktimes.get(k, (0.0, 0))[0])
    out = {
        "metric": "GRAPE gradient-evals/sec (fidelity+∇), synthetic d=64 N_t=1024 (SURVEY C5)",
        "value": value, "unit": "gradient-evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C5: d=64 Hermitian Ginibre basis, N_t=1024, dt=0.5, np=2, na=0, ne=0",
                   "restarts_per_gpu": B, "global_batch": B * world, "parallelism": f"restarts x{world}"},
        "roofline": dict(_roofline(kname, flop_model[kname], ktimes, L, PMC_SUMMARY_C5),
                         pipe="fp64 MFMA v_mfma_f64_16x16x4_f64"),
        "kernels_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in ktimes.items() if v[1]},
    }
    # SURVEY.md 8d canonical FLOP per C5 evaluation (na = 0, ne = 0: the survey's exp count
    # N_t (1 + np) is exactly what this engine executes)
    canon = nt * ((1 + nparam) * fe + 3 * 8 * d ** 3 + nparam * 8 * d ** 2)
    out["roofline"]["whole_eval"] = {"flop_per_eval": canon, "achieved": canon * value / 1e12,
                                     "frac": canon * value / 1e12 / FP64_PEAK_TFLOPS}
    out["kernels_frac"] = _kernel_fracs(flop_model, ktimes)
    return out


def c4opt(args):
    """SURVEY.md 8d C4 run as the optimiser the reference wraps (FidelityCalculations.jl:161-218):
    B restarts (x_main = 2pi*0.001*U, theta = 2pi*U, seed 1000 + r) advance together in a
    batched strong-Wolfe L-BFGS whose every line-search round is one device pass
    (robustgrape_amd/optimize.py).  Warm-up: W iterations; timed: K more iterations from
    there.  Reports gradient-evaluations/s including the optimiser's own host/device work,
    and the best fidelity reached.  One GPU; the multi-GPU form is sweep.optimize_sweep."""
    import torch
    from robustgrape_amd import optimize as OPT
    from robustgrape_amd import regularization as REG
    from robustgrape_amd.types import FidelityRobustGRAPEParameters
    B = args.batch or 1024
    fp = problem()
    X0 = restart_inputs(0, B)
    params = FidelityRobustGRAPEParameters(
        x_initial=X0[0], regularization_functions=[REG.regularization_cost_phase], regularization_coeff1=[1e-7],
        regularization_coeff2=[1e-7], error_source_coeff=[], iterations=10 ** 9)
    cost = OPT.RobustCost(fp, params, nparam=1, max_batch=B, device=0, scan_waves=args.scan_waves,
                          options=args.plan_options)
    dev = torch.device("cuda", 0)
    opts = OPT._solver_options(params)
    opts.update(g_tol=0.0)  # no early stop: every restart iterates through the timed region
    opts["asynchronous"] = not args.sync_rows
    res = OPT.lbfgs_batched(cost, torch.as_tensor(X0, device=dev), **dict(opts, iterations=args.warmup))
    torch.cuda.synchronize()
    calls0 = int(res.f_calls.sum())
    t0 = time.perf_counter()
    res2 = OPT.lbfgs_batched(cost, res.minimizer, **dict(opts, iterations=args.steps))
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    calls = int(res2.f_calls.sum())
    F = 1.0 - cost.fidelity_terms(res2.minimizer)[0]
    cost.close()
    out = {"metric": "GRAPE gradient-evals/sec inside batched L-BFGS (C4 sweep), Rydberg CZ d=9 N_t=512",
           "value": calls / elapsed, "unit": "gradient-evals/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C4 as an optimisation: B restarts, strong-Wolfe L-BFGS (m=10), "
                                  "regularization_cost_phase 1e-7/1e-7", "restarts_per_gpu": B,
                      "parallelism": "restarts x1"},
           "optimizer": {"evals_per_iteration": calls / (B * args.steps), "warmup_evals": calls0,
                         "best_infidelity": float(torch.min(F)), "median_infidelity": float(torch.median(F))}}
    print(json.dumps(out), flush=True)


def arcz(args):
    """The ar_cz-shaped latency leg (examples/ar_cz.jl): one x per call through the host-array entry,
    as optimize_fidelity_and_error_sources calls the reference (FidelityCalculations.jl:174-207):
    F, F_dx, F_d2err, F_d2err_dx of the d = 5 problem with one amplitude error, N_t = 200.  Beside
    it the 1-core C++ port on the same input."""
    fp = problem_arcz()
    x = arcz_inputs(0, 1)[0]
    out = {"metric": "GRAPE single-evaluation latency (fidelity+sensitivity+gradients), ar_cz d=5 N_t=200, 1 error source",
           "unit": "gradient-evals/s", "n_gpus": 1, "higher_is_better": True, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "examples/ar_cz.jl: symmetric blockaded d=5, t0=14.32, N_t=200, np=1, na=1, "
                                  "ne=1 (amplitude error); nbatch=1 per call"}}
    se = single_eval(fp, 1, x, seconds=3.0)
    out.update({"value": se["value"], "single_eval": se})
    if not args.no_cpu_baseline:
        try:
            from oracle.cref import cref
            if cref.available():
                t, n = time.perf_counter(), 0
                while time.perf_counter() - t < min(args.cpu_seconds, 5.0):
                    cref.fidelity_grad(fp, x)
                    n += 1
                dt = time.perf_counter() - t
                out["cpu_baseline"] = {"value": n / dt, "unit": "gradient-evals/s", "cores": 1, "kind": "port",
                                       "sample": f"{n} sequential ar_cz evaluations by oracle/cref, 1 thread",
                                       "host_cpu": _host_cpu()}
                out["vs_cpu"] = se["value"] / (n / dt)
        except Exception as exc:  # the baseline is a report, not the measurement
            out["cpu_baseline_error"] = repr(exc)
    print(json.dumps(out), flush=True)


def c2_closure(args):
    """SURVEY.md 8b closure fallback on C2: the same physics as plain Python closures (the
    reference's idiom, src/Types.jl:10,50 -- tests/problems.full9_problem(device=False)), so
    every evaluation pays the reference's closure calls on the host (robustgrape_amd/tables.py:
    a worker pool fills shared-memory tables chunk by chunk while the device evaluates the
    previous chunk) and grape_fidelity_grad_tables does the rest.  Host arrays in and out."""
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd import tables as TB
    from tests import problems as P
    B = args.batch or 1024
    chunk = args.chunk or 128
    fp = P.full9_problem(NT, device=False)
    X = restart_inputs(0, B)
    plan = GrapePlan(fp, nparam=1, device=0, max_batch=min(B, chunk))
    for _ in range(max(1, args.warmup)):
        plan.fidelity_grad(X[:chunk])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.fidelity_grad(X)
    elapsed = time.perf_counter() - t0
    value = args.steps * B / elapsed
    # the two halves on their own: serial closure tables (one core) and the device part
    t = time.perf_counter()
    H, U0 = TB.host_tables(fp, X[:8], 1)
    serial_ms = (time.perf_counter() - t) / 8 * 1e3
    from robustgrape_amd import _capi
    nx = X.shape[1]
    F, G = np.empty(8), np.empty((8, nx))
    Xs = np.ascontiguousarray(X[:8])
    t = time.perf_counter()
    for _ in range(5):
        _capi.check(_capi.lib().grape_fidelity_grad_tables(plan.handle, 8, _capi.dptr(Xs), _capi.dptr(H),
                                                           _capi.dptr(U0), _capi.dptr(F), _capi.dptr(G), None, None))
    device_ms = (time.perf_counter() - t) / 40 * 1e3
    workers = TB.default_workers()
    plan.close()
    out = {"metric": "GRAPE gradient-evals/sec, closure fallback (host-evaluated Python closures), Rydberg CZ d=9 N_t=512",
           "value": value, "unit": "gradient-evals/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C2 with H0 / target as plain Python closures (grape_fidelity_grad_tables)",
                      "restarts_per_gpu": B, "evals_per_chunk": min(B, chunk), "table_workers": workers},
           "closure_tables_serial_ms_per_eval": serial_ms,
           "device_ms_per_eval_tables_prebuilt": device_ms}
    if not args.no_cpu_baseline:
        cb = cpu_baseline(args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["vs_cpu"] = value / cb["value"]
    print(json.dumps(out), flush=True)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without a launcher (WORLD_SIZE unset): start N rank processes of this script,
    one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would,
    and wait for them.  The parent makes no GPU call (it never initialises HIP), so the children
    own the devices; rank 0 prints the JSON line.  If one rank fails the others are stopped (their
    exact PIDs) and the failing status is returned."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = set(range(n))
    while pending:
        for i in sorted(pending):
            c = procs[i].poll()
            if c is None:
                continue
            pending.discard(i)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {i} exited with status {c}; stopping the other ranks", file=sys.stderr)
                for j in pending:
                    procs[j].terminate()
        time.sleep(0.05)
    return rc


def c4_strong(make_step, world, rank, use_dist, sync, total=256, evals_per_restart=100):
    """BASELINE C4 as a strong-scaling sweep: `total` restarts sharded over the ranks (contiguous
    blocks, robustgrape_amd/sweep.py), `evals_per_restart` fidelity+gradient evaluations of every
    restart (examples/time_optimal_cz.jl:32 initialises them; the optimiser's evaluations are the
    unit), then the sweep's exchange -- one all_gather of (best F, id) and the winner's broadcast --
    INSIDE the timed region, bracketed by barrier + synchronize and maxed over ranks.
    make_step(first, count) -> (step, F, X, ids, close)."""
    import torch
    import torch.distributed as dist
    from robustgrape_amd.sweep import gather_best, gather_best_local, shard
    first, count = shard(total, world, rank)
    step, F, X, ids, close = make_step(first, count)
    # warm-up by the clock, not by a step count: a whole sweep lasts 2-10 ms, less than the GPU
    # needs to leave an idle state (scripts/probes/c4_strong_probe.py); 0.3 s of back-to-back sweeps
    tw = time.perf_counter()
    while True:
        for _ in range(max(3, evals_per_restart)):
            step()
        sync()
        if time.perf_counter() - tw >= 0.3:
            break
    # ... and the exchange once: the first use of its torch ops (and collectives) loads their code,
    # ~0.4 s that a cold first sweep would count (measured 4.06 -> 0.025 ms per round)
    if use_dist:
        gather_best(F, ids, X)
        dist.barrier()
    else:
        gather_best_local(F, ids, X)
    sync()
    t0 = time.perf_counter()
    for _ in range(evals_per_restart):
        step()
    sync()  # the steps run on the plan's stream; the exchange below reads F on torch's
    if use_dist:
        fb, rid, owner, _ = gather_best(F, ids, X)
        dist.barrier()
    else:
        fb, rid, owner, _ = gather_best_local(F, ids, X)
    sync()
    elapsed = time.perf_counter() - t0
    close()
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=F.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return {"value": total * evals_per_restart / elapsed, "unit": "gradient-evals/s", "n_gpus": world,
            "restarts_total": total, "restarts_per_rank": count, "evals_per_restart": evals_per_restart,
            "ms_per_eval_round": elapsed / evals_per_restart * 1e3, "scaling": "strong",
            "sweep": {"best_F": fb, "restart": rid, "owner_rank": owner},
            "note": "256 restarts sharded over the ranks, 100 evaluations each, all_gather + broadcast of the "
                    "best inside the timed region (max over ranks)"}


def dry_run(args, world, rank, use_dist):
    """Plumbing check of the multi-rank bench (no GPU, gloo): the launcher, the world-size check,
    the barrier / max-over-ranks timing and the sweep exchange, with a placeholder score in place
    of the evaluation.  Its line says "dry_run" and carries no throughput claim."""
    import torch
    from robustgrape_amd.sweep import gather_best, gather_best_local, shard
    B = args.batch or 16
    first, count = shard(B * world, world, rank)
    X = torch.from_numpy(restart_inputs(first, count))
    ids = torch.arange(first, first + count)
    F = torch.empty(count, dtype=torch.float64)

    def make_step(f, c):
        Xs = torch.from_numpy(restart_inputs(f, c))
        Fs = torch.empty(c, dtype=torch.float64)
        return (lambda: torch.sum(torch.cos(Xs), dim=1, out=Fs)), Fs, Xs, torch.arange(f, f + c), (lambda: None)

    torch.sum(torch.cos(X), dim=1, out=F)
    best = gather_best(F, ids, X) if use_dist else gather_best_local(F, ids, X)
    strong = c4_strong(make_step, world, rank, use_dist, lambda: None, total=args.c4_total,
                       evals_per_restart=2)
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher and exchange only)", "value": None, "dry_run": True,
                          "n_gpus": world, "restarts_per_gpu": B,
                          "sweep": {"best_F": best[0], "restart": best[1], "owner_rank": best[2]},
                          "c4_strong": strong}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="restarts per GPU per step; default 262144 (c2), 16384 (c3), 16 (c5)")
    ap.add_argument("--chunk", type=int, default=None,
                    help="evaluations per device pass (the plan's workspace; larger steps are chunked "
                         "by the C side); default 32768 (c2), 8192 (c3), 16 (c5)")
    ap.add_argument("--workload", choices=("c2", "c3", "c5", "c5err", "c4opt", "c2-closure", "arcz"), default="c2",
                    help="c2: the BASELINE metric (d=9 Rydberg CZ); c3: C2 + 4 error sources "
                         "(sensitivities and their gradients); c5: synthetic d=64, N_t=1024 "
                         "(dense MFMA engine, SURVEY.md 8d C5); c4opt: the C4 restart sweep as "
                         "batched L-BFGS (one step = one iteration of every restart); c2-closure: C2 as "
                         "plain Python closures through the host-table fallback; arcz: examples/ar_cz.jl's d=5 "
                         "problem with one amplitude error, single-evaluation latency")
    ap.add_argument("--scan-waves", type=int, default=None, choices=(0, 1, 4, 8, 16),
                    help="c4opt: the plan's scan width (chunking); 0 = by batch size, default: RobustCost's choice")
    ap.add_argument("--plan-options", type=int, default=0,
                    help="GRAPE_OPT_* flags of the timed plan (A/B runs; c2/c3/c5 device legs and c4opt)")
    ap.add_argument("--sync-rows", action="store_true",
                    help="c4opt: the synchronous optimiser loop (rows wait for each other every iteration)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-paths", action="store_true",
                    help="skip the host-array (PCIe-inclusive) and nbatch = 1 legs")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-whole-matrix", action="store_true",
                    help="skip the C2 whole-matrix comparison leg (PMC passes: one pipeline per run)")
    ap.add_argument("--no-c4-strong", action="store_true",
                    help="skip the C4 strong-scaling leg (256 restarts over the ranks)")
    ap.add_argument("--c4-total", type=int, default=256, help="restarts of the C4 strong-scaling leg")
    ap.add_argument("--dist", action="store_true",
                    help="run the multi-rank path (RCCL process group, the sweep's all_gather + "
                         "broadcast, max-over-ranks timing) even with one rank")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU plumbing check: gloo ranks, no GPU, placeholder scores (tests/test_bench_launch.py)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks (WORLD_SIZE); refusing "
              "to print a mislabelled line", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.workload in ("c4opt", "c2-closure", "arcz"):
        print(f"bench.py: --workload {args.workload} is a single-GPU leg", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    use_dist = world > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("NCCL_DEBUG", "WARN")  # keep RCCL's banner off stdout (one JSON line)
    if args.dry_run:
        if use_dist:
            dist.init_process_group("gloo")
        dry_run(args, world, rank, use_dist)
        if use_dist:
            dist.destroy_process_group()
        return
    if args.workload == "c4opt":
        return c4opt(args)
    if args.workload == "c2-closure":
        return c2_closure(args)
    if args.workload == "arcz":
        return arcz(args)
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.sweep import gather_best, shard
    c5err = args.workload == "c5err"
    c5, c3 = args.workload == "c5" or c5err, args.workload == "c3"
    if c5:
        from robustgrape_amd import synthetic as S
        fp, nparam, d, nt, inputs = S.dense_problem(), 2, S.C5_DIM, S.C5_NTIMES, c5_inputs
        if c5err:
            fp = S.dense_error_problem()
    elif c3:
        fp, nparam, d, nt, inputs = problem_c3(), 1, D, NT, restart_inputs
    else:
        fp, nparam, d, nt, inputs = problem(), 1, D, NT, restart_inputs
    ne = len(fp.unitary_problem.error_sources)
    # One step = B restarts per GPU, evaluated in device passes of `chunk` (C2 passes of 16 384 /
    # 32 768 / 65 536 / 131 072 measured 8.12 / 8.11 / 7.76 / 7.98 M evals/s in round 3, DESIGN.md
    # 10).  B is sized so that the default steps last long enough for the driver's GPU-busy
    # sampler to see them.
    B = args.batch or (16 if c5 else 16384 if c3 else 262144)
    chunk = args.chunk or (16 if c5 else 8192 if c3 else 32768)
    first, count = shard(B * world, world, rank)  # weak scaling: B restarts per GPU
    plan = GrapePlan(fp, nparam=nparam, device=local, max_batch=min(count, chunk), options=args.plan_options)
    X = torch.from_numpy(inputs(first, count)).to(dev)
    F = torch.empty(count, dtype=torch.float64, device=dev)
    Fdx = torch.empty(count, X.shape[1], dtype=torch.float64, device=dev)
    Fd2 = torch.empty(count, max(ne, 1), dtype=torch.float64, device=dev)
    Fd2dx = torch.empty(count, max(ne, 1), X.shape[1], dtype=torch.float64, device=dev)
    ids = torch.arange(first, first + count, device=dev)

    # The evaluation is enqueued on one torch stream, so steps queue back to back without
    # a host round trip; the timed region still ends with a full synchronize.
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    plan.set_stream(stream.cuda_stream)

    def step():
        plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), Fdx.data_ptr(), count,
                                        Fd2.data_ptr() if ne else 0, Fd2dx.data_ptr() if ne else 0)

    for _ in range(args.warmup):
        step()
    plan.synchronize()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    plan.kernel_times(reset=True)
    plan.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    best = None
    if use_dist:  # the sweep's exchange: all_gather of (best F, id), winner broadcasts its x
        best = gather_best(F, ids, X)
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    plan.synchronize()  # resolves the per-kernel events, raises on a singular Pade denominator
    plan.set_profiling(False)
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    evals = args.steps * B * world
    value = evals / elapsed
    ktimes = plan.kernel_times()
    sectors = plan.sectors()
    info = plan.sector_info()
    if rank == 0:
        L = min(count, chunk)
        if c5err:
            out = c5err_report(args, B, L, world, value, elapsed, ktimes, d, nt, nparam, ne)
        elif c5:
            out = c5_report(args, B, L, world, value, elapsed, ktimes, d, nt, nparam)
        elif c3:
            out = c3_report(args, B, L, world, value, elapsed, ktimes, ne, sectors,
                            args.steps * ((count + L - 1) // L), info)
        else:
            out = c2_report(args, B, L, world, value, elapsed, ktimes, sectors,
                            args.steps * ((count + L - 1) // L), info)
        if best is not None:
            out["sweep"] = {"best_F": best[0], "restart": best[1], "owner_rank": best[2]}
        out["config"]["evals_per_device_pass"] = min(count, chunk)
        from robustgrape_amd import _capi
        out["build_id"] = _capi.build_id()  # the library the timed region ran (robustgrape_amd/build.py)
        if _capi.build_defines():
            out["build_defines"] = list(_capi.build_defines())
    plan.close()

    if not (c3 or c5) and not args.no_c4_strong:
        def make_step(f, c):
            p = GrapePlan(fp, nparam=nparam, device=local, max_batch=max(1, c))
            p.set_stream(stream.cuda_stream)
            Xs = torch.from_numpy(inputs(f, c)).to(dev)
            Fs = torch.empty(c, dtype=torch.float64, device=dev)
            Gs = torch.empty(c, Xs.shape[1], dtype=torch.float64, device=dev)
            return ((lambda: p.fidelity_grad_device_async(Xs.data_ptr(), Fs.data_ptr(), Gs.data_ptr(), c, 0, 0)),
                    Fs, Xs, torch.arange(f, f + c, device=dev), p.close)
        strong = c4_strong(make_step, world, rank, use_dist, torch.cuda.synchronize, total=args.c4_total)
        if rank == 0:
            out["c4_strong"] = strong
    if rank == 0 and world == 1 and not (c3 or c5) and sectors[0][0] < d and not args.no_whole_matrix:
        out["whole_matrix_path"] = whole_matrix_leg(fp, nparam, X, F, Fdx, min(count, chunk), stream, args)
    if rank == 0:
        if world == 1 and not args.no_host_paths:
            # the drop-in path as the reference's callers use it (host arrays, SURVEY.md 8d's
            # metric definition): a 4 096-restart batch per call, and single evaluations
            Xh = inputs(0, min(4096, B))
            out["host_path"] = host_path(fp, nparam, Xh, reps=3 if c5 else 10, label=args.workload.upper())
            out["single_eval"] = single_eval(fp, nparam, Xh[0])
            if not (c3 or c5):
                out["c4_points"] = c4_points(fp, nparam, inputs, dev)
        if world == 1 and not args.no_cpu_baseline:
            if c5:
                out["cpu_baseline"] = cpu_baseline_c5(args.cpu_seconds, fp, c5_inputs(0, 1)[0],
                                                      "C5 + 2 error sources" if c5err else "C5")
            else:
                out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, fp if c3 else None, "C3" if c3 else "C2")
            if not (c3 or c5):
                allc = cpu_baseline_allcores(args.cpu_seconds * 2 / 3, fp, "C4")
                if allc is not None:
                    out["cpu_baseline_allcores"] = allc
            cb = out["cpu_baseline"]["value"]
            out["vs_cpu"] = {"device_value": value / cb,
                             "host_path": out["host_path"]["value"] / cb if "host_path" in out else None,
                             "single_eval": out["single_eval"]["value"] / cb if "single_eval" in out else None,
                             "device_value_vs_allcores": (value / out["cpu_baseline_allcores"]["value"]
                                                          if "cpu_baseline_allcores" in out else None)}
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
