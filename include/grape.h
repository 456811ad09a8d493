/*
 * grape.h -- C ABI of the MI355X GRAPE propagator-and-gradient engine.
 *
 * Drop-in boundary for RobustGRAPE.jl's hot path.  Every entry point takes
 * plain pointers and sizes (no torch, no C++ types) so that a Julia `ccall`
 * shim, Python `ctypes` or C/C++ can bind it.  The reference interfaces each
 * entry point replaces are cited per function (paths are into the reference
 * tree, srtweezer/RobustGRAPE).
 *
 * Layout conventions (match the reference / Julia):
 *   - complex numbers are interleaved (re, im) float64 pairs (Julia ComplexF64);
 *   - matrices are COLUMN-MAJOR d x d (element (i,j) at [i + j*d]);
 *   - a control vector x has n_x = nparam*ntimes + nadd entries with
 *     x[p + k*nparam] = control p at time step k (0-based) and x_add in the
 *     last nadd slots (src/UnitaryCalculations.jl:21-26);
 *   - batched inputs are n_x-major: eval b's vector starts at x + b*n_x;
 *   - F_dx has n_x entries per eval (src/FidelityCalculations.jl:116),
 *     F_d2err_dx is (n_x, nerr) column-major per eval (:117).
 *
 * Ownership: all host buffers are caller-owned; the library never keeps a
 * pointer to them after a call returns.  Calls are synchronous unless their
 * name ends in _async.  A plan is bound to one device and one HIP stream;
 * distinct plans may be used from different threads concurrently.
 *
 * Errors: every int-returning function returns GRAPE_OK (0) or a negative
 * grape_status; grape_last_error() returns a thread-local message.
 */
#ifndef GRAPE_H
#define GRAPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRAPE_ABI_VERSION 11

typedef enum grape_status {
    GRAPE_OK = 0,
    GRAPE_ERR_INVALID = -1,     /* bad descriptor / shape (reference: AssertionError, UnitaryCalculations.jl:22) */
    GRAPE_ERR_UNSUPPORTED = -2, /* valid but outside this engine (e.g. ndim > GRAPE_MAX_SMALL_DIM) */
    GRAPE_ERR_ALLOC = -3,       /* device or host allocation failed */
    GRAPE_ERR_HIP = -4,         /* a HIP runtime call failed */
    GRAPE_ERR_SINGULAR = -5,    /* singular Pade denominator (Julia: SingularException from gesv!) */
    GRAPE_ERR_NO_DEVICE = -6    /* no usable GPU */
} grape_status;

/* Largest Hilbert-space dimension served by the small-d (VALU row-group) engine. */
#define GRAPE_MAX_SMALL_DIM 12
/* Largest dimension served by the dense (MFMA) engine, used for
 * GRAPE_MAX_SMALL_DIM < ndim <= GRAPE_MAX_DENSE_DIM (zero-padded to 64).  It
 * requires a Hermitian H0 operator basis (Hermitian operators, real
 * coefficients) and H0 / error terms independent of x_add; error sources are
 * served (Hermitian error operators). */
#define GRAPE_MAX_DENSE_DIM 64

/*
 * Operator-basis description of the reference's Hamiltonian closures.
 *
 * The reference takes arbitrary Julia closures H0(nt, x, x_add) and
 * Herror(nt, x, x_add, err) (src/Types.jl:10,25) and target_unitary(x_add)
 * (src/Types.jl:50).  Closures cannot run on the GPU, so the device path
 * takes them as a sum of fixed operators with scalar coefficients:
 *
 *     H0(nt, x, x_add)        = sum_t  c_t(nt, x, x_add)        * OPS[op_t]
 *     Herror_e(nt,x,x_add,err) = err * sum_t c_t(nt, x, x_add)  * OPS[op_t]
 *     U0(x_add)               = sum_t  c_t(x_add)               * OPS[op_t]
 *
 * with c_t = scale_t * f_t(a_t * v_t + b_t), f in {one, identity, cos, sin,
 * cis = exp(i .)} and v the variable named by var/index.  This covers every
 * Hamiltonian, error source and target in the reference's tests, examples and
 * RydbergTools.jl (phase control: cos/sin terms; amplitude/detuning errors:
 * linear in err).
 */
typedef enum grape_var {
    GRAPE_VAR_ONE = 0,   /* v = 1 */
    GRAPE_VAR_X = 1,     /* v = x_main[index] at the current time step */
    GRAPE_VAR_XADD = 2,  /* v = x_add[index] */
    GRAPE_VAR_TSTEP = 3  /* v = nt, the 1-based time step (Types.jl:25) */
} grape_var;

typedef enum grape_func {
    GRAPE_FN_ONE = 0,    /* f(t) = 1 */
    GRAPE_FN_LINEAR = 1, /* f(t) = t */
    GRAPE_FN_COS = 2,    /* f(t) = cos t */
    GRAPE_FN_SIN = 3,    /* f(t) = sin t */
    GRAPE_FN_CIS = 4     /* f(t) = cos t + i sin t  (target terms only) */
} grape_func;

typedef struct grape_term {
    int32_t op;        /* index into grape_desc.ops */
    int32_t var;       /* grape_var */
    int32_t index;     /* parameter index for GRAPE_VAR_X / GRAPE_VAR_XADD */
    int32_t func;      /* grape_func */
    double a, b;       /* argument t = a*v + b */
    double scale_re;   /* complex scale */
    double scale_im;
} grape_term;

typedef struct grape_desc {
    int32_t ndim;       /* UnitaryRobustGRAPEProblem.ndim   (Types.jl:34) */
    int32_t ntimes;     /* UnitaryRobustGRAPEProblem.ntimes (Types.jl:33) */
    int32_t nparam;     /* controls per step: (n_x - nadd)/ntimes (UnitaryCalculations.jl:24) */
    int32_t nadd;       /* nb_additional_param (Types.jl:36) */
    int32_t nerr;       /* length(error_sources) (Types.jl:37) */
    int32_t n_ops;
    double t0;          /* total time (Types.jl:32) */
    double eps;         /* first-order FD step, default 1e-8 (Types.jl:38) */
    double eps2;        /* second-order FD step, default 1e-4 (Types.jl:39) */
    const double *projector_diag; /* ndim reals: diagonal of FidelityRobustGRAPEProblem.projector (Types.jl:54) */
    const double *ops;            /* n_ops * ndim * ndim complex, column-major, interleaved */
    int32_t n_h0_terms;
    const grape_term *h0_terms;
    const int32_t *err_term_offsets; /* nerr+1 offsets into err_terms (NULL when nerr == 0) */
    const grape_term *err_terms;
    int32_t n_target_terms;
    const grape_term *target_terms;  /* may only use GRAPE_VAR_ONE / GRAPE_VAR_XADD */
    int32_t max_batch;  /* largest nbatch a single call will use (workspace sizing); <=0 -> 256 */
    int32_t reserved[5]; /* reserved[0]: flags (GRAPE_DESC_*); [1]: engine options (GRAPE_OPT_*, ABI 6);
                          * [2]: k_scan width override (1, 4, 8 or 16 waves -- 16 for the chunk-walk classes only; 0 = chosen by batch size, ABI 6);
                          * the rest must be 0 */
    /* ABI 4: the full projector P0 (FidelityRobustGRAPEProblem.projector, Types.jl:54), ndim x ndim
     * complex, column-major, interleaved; any matrix, as FidelityCalculations.jl:47-51 accepts.
     * NULL: projector_diag is used.  When given, projector_diag is ignored (may be NULL).  The
     * struct size and the offsets of every earlier field are those of ABI 3 (a zero-filled
     * ABI-3 descriptor reads as projector = NULL). */
    const double *projector;
} grape_desc;

/*
 * reserved[0] flag: closure fallback (SURVEY.md 8b "host-evaluated H tensors").
 * H0 and the target stay opaque host closures (the reference's own idiom,
 * src/Types.jl:10,50); the caller evaluates them at every call site of the
 * reference and passes the tables to grape_fidelity_grad_tables.  ops / terms
 * may then be NULL (n_ops = 0); ndim <= GRAPE_MAX_DENSE_DIM (above GRAPE_MAX_SMALL_DIM the
 * tables go through the general path below with the dense engine's exponential, which needs
 * Hermitian tabulated generators -- the Python host checks).  The closures may read x_add:
 * every x_add call site of the reference is tabulated.
 */
#define GRAPE_DESC_HOST_TABLES 1

/*
 * reserved[1]: engine options (ABI 6), fixed at plan creation; 0 selects the defaults.  They
 * choose between implementations of the SAME outputs (A/B measurements, the bit-identity and
 * cross-path tests); none changes a result beyond the parity tiers.  Nothing is read from the
 * environment by the library.
 */
#define GRAPE_OPT_NO_SECTORS 1  /* whole matrices even when the operators are block-diagonal */
#define GRAPE_OPT_NO_LANE 2     /* row-group exponentials for d <= 3 (no lane matrices) */
#define GRAPE_OPT_NO_CHAIN 4    /* sector chunk chains through k_expm + k_scan, not k_expm_chain_lane */
#define GRAPE_OPT_NO_WALK 8     /* sector classes of <= 4 levels through the stored-intermediate
                                   kernels instead of the chunk walks (grape_walk.hpp) */
#define GRAPE_OPT_NO_GRAPH 16   /* no HIP-graph replay of small host-array calls */
#define GRAPE_OPT_WALK_RECOMPUTE 32 /* chunk walks: the gradient walk of the 4-level class recomputes the
                                       nominal propagators instead of reading the forward walk's copy */
/*
 * General (non-Hermitian) H0, e.g. a -i Gamma/2 decay term (ABI 7): the chain C_k is inverted
 * by LU as the reference does (UnitaryCalculations.jl:47, inv(cum_evo)) instead of C_k^dagger,
 * and the fidelity path runs from the materialised unitary derivatives, one evaluation at a
 * time (FidelityCalculations.jl:19-119).  Selected automatically for an operator-basis H0
 * that is not Hermitian; host-table plans (closures) set it when the host sees a
 * non-Hermitian H0 table.  Operator bases: ndim <= GRAPE_MAX_SMALL_DIM; host-table plans above
 * GRAPE_MAX_SMALL_DIM always take this path (Hermitian tables only).
 */
#define GRAPE_OPT_GENERAL_H0 64
/* Calls of at most 4096 evaluations on a plan with two sector classes run the second class on an
 * auxiliary stream beside the first (joined before the sector heads; latency-bound calls such as
 * the optimiser's line-search rounds).  This option keeps every call on the plan's one stream. */
#define GRAPE_OPT_NO_FORK 128
/* Sector problems with a diagonal projector and a diagonal target form F and M with a
 * one-thread-per-evaluation head over the sector blocks; this option keeps the general
 * (d x d products) sector head for every problem (A/B and parity checks). */
#define GRAPE_OPT_GENERAL_HEAD 256
/* Latency-bound calls (16-wave scans: fewer sub-evaluations than CUs) of the Rydberg sector layout
 * (one 4-level sector + two 2-level sectors, no error sources) run both sector classes' walks and
 * scans in one launch per stage; this option keeps one launch per class. */
#define GRAPE_OPT_NO_PAIR 512
/* Symmetry-adapted sectors (ABI 8): when a unitary change of basis V splits the operators'
 * sparsity components further (the commutant of the operator algebra; e.g. the atom-swap symmetry
 * of rydberg_hamiltonian_full with equal Rabi frequencies and detunings: a 3-level sector and a
 * dark level instead of a 4-level sector), the sector path runs in that basis -- operators, target
 * and projector rotated (V^dag X V), the outputs (traces) unchanged.  This option keeps the
 * permutation sectors. */
#define GRAPE_OPT_NO_SYMMETRY 1024
/* Twin sectors (ABI 8): two sectors of a chunk-walk class whose blocks of every H0 operator are
 * identical (the Rydberg sectors {01, 0r} and {10, r0} at equal Rabi frequencies and detunings)
 * share one exponential per step; this option computes each sector's own. */
#define GRAPE_OPT_NO_TWIN 2048
/* Accepted and ignored since round 5: captured small calls no longer fork the second sector class
   (the experimental captured fork was removed).  Kept so that old callers still build. */
#define GRAPE_OPT_GRAPH_FORK 4096
/* Phase-covariant walk classes (ABI 9): when the one control enters every sector block as a phase,
 * H(x) = D(a x) H(0) D(a x)^dag with D(t) = diag(e^{i t N_j}) -- the laser phase of the Rydberg models
 * (RydbergTools.jl:31-130) -- the chunk walks form E_k = D_k exp(-i dt H(0)) D_k^dag and the
 * eps-variant's difference from the level phases: one exponential per walk lane instead of one per
 * step and variant.  This option keeps the per-step exponentials. */
#define GRAPE_OPT_NO_GAUGE 8192
/* One workgroup per evaluation (ABI 10): calls of at most 256 evaluations of a plan with the Rydberg
 * sector layout (one 3-level and two 2-level phase-covariant classes, one control per step, no error
 * sources) run each evaluation -- propagators, chain scan, head, gradient -- inside one workgroup,
 * every intermediate in LDS; host-array calls read x from and write F, F_dx to
 * mapped pinned memory.  This option keeps the pair-kernel pipeline. */
#define GRAPE_OPT_NO_EVAL1 16384
/* Merged walks (ABI 10): throughput passes of the Rydberg layout with phase-covariant classes walk
 * both sector classes of an (evaluation, chunk) in one lane; this option launches
 * one walk kernel per class instead (the same chunking, the same results bit for bit). */
#define GRAPE_OPT_NO_MERGE 32768

typedef struct grape_plan grape_plan;

/* Library / ABI identification. */
int grape_abi_version(void);
/* Content hash of the sources and flags the library was built from (robustgrape_amd/build.py
 * source_id; round 5).  The Python binding refuses a library whose id differs from the sources
 * next to it. */
const char *grape_build_id(void);
const char *grape_last_error(void);
/* ABI 11: opt-in SIGSEGV / SIGBUS handler that prints libgrape's native frames when the fault lies in
 * the library's own host code and then hands the signal to the handler it displaced (every other
 * fault goes there directly).  Nothing is installed at load time; the Python binding calls this
 * (unless GRAPE_NO_SIGNAL_HANDLER=1); a Julia host should not (Julia uses SIGSEGV itself).
 * Returns 1 when installed (or already installed), 0 when the library's text range is unknown. */
int grape_install_fault_handler(void);

/* Number of visible HIP devices (0 when none); does not create a context. */
int grape_device_count(void);

/*
 * Build a plan: validates the descriptor, uploads the operator basis to
 * `device`, allocates the workspace for desc->max_batch evaluations and
 * creates the plan's stream.  Replaces the problem structs
 * UnitaryRobustGRAPEProblem / FidelityRobustGRAPEProblem (src/Types.jl:31-56).
 */
int grape_plan_create(const grape_desc *desc, int device, grape_plan **out);
void grape_plan_destroy(grape_plan *plan);

/* Device stream of the plan (a hipStream_t), for callers that enqueue around it. */
void *grape_plan_stream(grape_plan *plan);

/* Enqueue the plan's work on the caller's hipStream_t from now on (NULL: the
 * plan's own stream).  Lets a caller keep the evaluation stream-ordered with
 * its own kernels and collectives instead of synchronising between them. */
int grape_plan_set_stream(grape_plan *plan, void *stream);

/*
 * Fidelity + gradient (+ error sensitivity and its gradient) for a batch of
 * control vectors.  One evaluation b equals one reference call
 *   (F, F_dx_tot, F_d2err, F_d2err_dx_tot) =
 *       calculate_fidelity_and_derivatives(fidelity_problem, x_b)
 * (src/FidelityCalculations.jl:19-119, which calls
 *  calculate_unitary_and_derivatives, src/UnitaryCalculations.jl:20-155).
 *
 *   x          [nbatch][n_x]             host, read-only
 *   F          [nbatch]                  host, written
 *   F_dx       [nbatch][n_x]             host, written
 *   F_d2err    [nbatch][nerr]            host, written (may be NULL if nerr == 0)
 *   F_d2err_dx [nbatch][nerr][n_x]       host, written (may be NULL if nerr == 0)
 *              (per eval: column-major (n_x, nerr) like the reference's matrix)
 */
int grape_fidelity_grad(grape_plan *plan, int nbatch, const double *x,
                        double *F, double *F_dx, double *F_d2err, double *F_d2err_dx);

/*
 * Same as grape_fidelity_grad with DEVICE pointers, enqueued on the plan's
 * stream without synchronising (inputs resident in HBM; used by the
 * throughput benchmark and by callers that keep x on the GPU).
 */
int grape_fidelity_grad_device_async(grape_plan *plan, int nbatch, const double *d_x,
                                     double *d_F, double *d_F_dx,
                                     double *d_F_d2err, double *d_F_d2err_dx);

/* Time sharding of ONE evaluation over devices (robustgrape_amd/timeshard.py).
 * The plan is created for a time SLICE of the problem: ntimes = the slice's steps, t0 = dt * steps,
 * the slice's controls as x (np * steps values, no x_add); dense engine (12 < ndim <= 64) without
 * error sources, general projector or step-index terms (else GRAPE_ERR_UNSUPPORTED).
 * grape_slice_forward: the slice total U_slice = E_last ... E_first (ndim x ndim complex,
 *   column-major interleaved, host); the slice's propagators and chunk prefixes stay in the plan.
 * grape_slice_gradient: given M' = B M B^dagger (same layout) -- B the product of the earlier
 *   slices' totals, M = G U for the whole evaluation's U (FidelityCalculations.jl:56-65 as
 *   F_dx = Re tr(G U_dx)) -- the slice's F_dx entries (np x steps, x's layout), from the
 *   propagators of the last grape_slice_forward on this plan.  Both synchronous. */
int grape_slice_forward(grape_plan *plan, const double *x, double *U_slice);
int grape_slice_gradient(grape_plan *plan, const double *M_prime, double *F_dx);
/* The same with DEVICE buffers (round 4), enqueued on the plan's stream without a synchronize
 * (grape_plan_synchronize reports a singular Pade denominator): the time-sharded evaluation then
 * exchanges slice totals and F_dx slices device to device (robustgrape_amd/timeshard.py). */
int grape_slice_forward_device(grape_plan *plan, const double *x, double *U_slice);
int grape_slice_gradient_device(grape_plan *plan, const double *M_prime, double *F_dx);

/*
 * Closure fallback (plans created with GRAPE_DESC_HOST_TABLES): the outputs of
 * grape_fidelity_grad for problems whose H0 / target are host closures.  The
 * caller evaluates the closures at exactly the reference's call sites
 * (src/UnitaryCalculations.jl:45,51,59; src/FidelityCalculations.jl:32-40):
 *   H  [nbatch][ntimes][nv][ndim*ndim] complex, column-major, interleaved, variants v:
 *      with n = nparam + nadd gradient parameters u (u < nparam: control x[u,k];
 *      u >= nparam: x_add[u - nparam]):
 *      nerr == 0: nv = 1 + n
 *        0: H0(k, x[:,k], x_add) | 1 + u: parameter u + eps
 *      nerr > 0: nv = 1 + 2 n + nerr (2 + n)                (UnitaryCalculations.jl:45-95)
 *        0: H0 | 1 + u: parameter u + eps | 1 + n + u: parameter u + eps2 |
 *        per error e, base 1 + 2 n + e (2 + n):
 *          base: H0 + Herror_e(.., eps) | base + 1: H0 + Herror_e(.., eps2) |
 *          base + 2 + u: H0 + Herror_e(.., eps2), both at parameter u + eps2
 *   U0 [nbatch][1 + nadd][ndim*ndim] complex, column-major, interleaved:
 *      slot 0: target(x_add); 1 + q: target(x_add + eps e_q)
 * The device runs the exponentials, the scan and the gradient contractions.
 * F_d2err / F_d2err_dx as in grape_fidelity_grad (may be NULL when nerr == 0).
 * Synchronous; host buffers.
 */
int grape_fidelity_grad_tables(grape_plan *plan, int nbatch, const double *x, const double *H,
                               const double *U0, double *F, double *F_dx, double *F_d2err,
                               double *F_d2err_dx);

/*
 * Optimiser support (robustgrape_amd/optimize.py, the batched replacement of the
 * Optim.jl LBFGS that drives calculate_fidelity_and_derivatives,
 * src/FidelityCalculations.jl:199-217): the L-BFGS two-loop recursion for R
 * restarts at once, DEVICE pointers, enqueued on `stream` (a hipStream_t, NULL =
 * default stream), asynchronous.
 *   S, Y [m][R][n], rho [m][R]: ring-buffer history; head [R]: next slot;
 *   hist [R]: stored pairs (<= m); gamma [R]: initial scaling; g [R][n]: gradients;
 *   D [R][n] (written): the directions -H g.   m <= 64.
 */
int grape_lbfgs_direction(int R, int n, int m, const double *S, const double *Y, const double *rho,
                          const int64_t *head, const int64_t *hist, const double *gamma,
                          const double *g, double *D, void *stream);

/*
 * The rest of one L-BFGS iteration of every restart on the device (ABI 7): the strong-Wolfe
 * line search's state machine (Nocedal & Wright alg. 3.5 / 3.6, c1 = 1e-4, c2 = 0.9) and the
 * ring-buffer update with Optim's stopping rules, as optimize.py lbfgs_batched runs them.  All
 * pointers are DEVICE memory for R rows (vectors [R][n], ring [m][R][n]); flags int32, counters
 * int64.  Per iteration: grape_lbfgs_direction, grape_lbfgs_ls_init (active rows, descent check,
 * the search state at a = 1), then per round grape_lbfgs_ls_begin (the searching rows in row
 * order -> rows[0, *count), their trial points -> Xt, f_calls += 1), the caller evaluates the
 * compact batch (ft [count], gt [count][n]), grape_lbfgs_ls_end; finally grape_lbfgs_step.
 */
typedef struct grape_lbfgs_state {
    int R, n, m, reserved0;
    double *X, *f, *g, *D, *Xn, *fn, *gn, *Xt;
    double *f0, *dphi0, *a_cur, *a_prev, *f_prev, *dp_prev, *a_lo, *f_lo, *dp_lo, *a_hi, *f_hi, *dp_hi;
    double *S, *Y, *rho, *gamma, *g_thr;
    int64_t *f_calls, *iters, *hist, *head, *rows;
    int32_t *phase, *first, *accepted, *gconv, *fconv, *xconv, *lsfail, *active, *count;
    double f_abstol, f_reltol, x_abstol, x_reltol;
    int64_t iterations, f_calls_limit;
} grape_lbfgs_state;
int grape_lbfgs_ls_init(const grape_lbfgs_state *state, void *stream);
int grape_lbfgs_ls_begin(const grape_lbfgs_state *state, void *stream);
int grape_lbfgs_ls_end(const grape_lbfgs_state *state, int count, const double *ft, const double *gt, void *stream);
int grape_lbfgs_step(const grape_lbfgs_state *state, void *stream);
/* Asynchronous rows (round 4): instead of the per-iteration sequence above, call this at the start
 * of every round, then grape_lbfgs_ls_begin / evaluate / grape_lbfgs_ls_end.  Every row advances on
 * its own: a row whose line search ended (accepted, or max_rounds trial evaluations spent) takes its
 * step (grape_lbfgs_step), then its direction and line-search start (grape_lbfgs_direction,
 * grape_lbfgs_ls_init), so each round evaluates every searching row whatever its iteration; each
 * row's arithmetic and order are those of the per-iteration sequence (bitwise the same trajectory).
 * Rows start with phase = 3; rounds: int32 [R] device scratch; steepest != 0 clears the history after
 * every step (gradient descent).  Done when ls_begin's count is 0. */
int grape_lbfgs_async_advance(const grape_lbfgs_state *state, int steepest, int max_rounds, int *rounds, void *stream);

/*
 * The optimiser's cost of R restarts in one launch (calculate_common!, FidelityCalculations.jl:
 * 172-196; ABI 7): cost = 1 - F + sum_e c_e F_d2err_e^2 + sum_p (c1_p reg1_p + c2_p reg2_p),
 * grad = -F_dx + 2 sum_e c_e F_d2err_e F_d2err_dx[e] + the regulariser gradients on each control's
 * entries.  reg_kind[p]: 0 none, 1 regularization_cost(x_p), 2 regularization_cost_phase(x_p)
 * (Regularization.jl:26-48, :111-115; 4 <= ntimes <= 4096).  DEVICE pointers: X, F_dx, grad
 * [R][n_x]; F, cost [R]; F_d2err [R][nerr]; F_d2err_dx [R][nerr][n_x] (the device layout of
 * grape_fidelity_grad_device_async); err_coeff [nerr], coeff1 / coeff2 / reg_kind [nparam].
 */
int grape_robust_cost(int R, int nparam, int ntimes, int nadd, int nerr, const double *X, const double *F,
                      const double *F_dx, const double *F_d2err, const double *F_d2err_dx, const double *err_coeff,
                      const double *coeff1, const double *coeff2, const int32_t *reg_kind, double *cost,
                      double *grad, void *stream);

/* Block until all work enqueued on the plan's stream finished; reports device-side errors. */
int grape_plan_synchronize(grape_plan *plan);

/*
 * Materialised unitary derivatives for ONE control vector, replacing
 * calculate_unitary_and_derivatives (src/UnitaryCalculations.jl:20-155).
 * Output shapes are the reference's (complex, column-major):
 *   U (d,d); U_dx (d,d,nparam,ntimes); U_dx_add (d,d,nadd); U_derr (d,d,nerr);
 *   U_derr_dx (d,d,nparam,ntimes,nerr); U_derr_dx_add (d,d,nadd,nerr).
 * Any output pointer may be NULL to skip it.
 */
int grape_unitary_derivs(grape_plan *plan, const double *x,
                         double *U, double *U_dx, double *U_dx_add,
                         double *U_derr, double *U_derr_dx, double *U_derr_dx_add);

/*
 * Interaction-picture error operators for ONE control vector, replacing
 * calculate_interaction_error_operators (src/UnitaryCalculations.jl:180-204):
 *   O (d, d, ntimes, nerr) complex column-major,
 *   O[:, :, k, e] = C_{k-1}^{-1} (Herror_e(k, x, x_add, eps) / eps) C_{k-1}, C_0 = I.
 * Nothing is written when the problem has no error sources.
 */
int grape_interaction_error_operators(grape_plan *plan, const double *x, double *O);

/*
 * The same operators written into DEVICE memory d_O (same layout, d*d*ntimes*nerr
 * complex), for callers that post-process them on the GPU (the fidelity-response
 * rows, src/FidelityCalculations.jl:246-343).  x is a host vector.  Synchronous.
 */
int grape_interaction_error_operators_device(grape_plan *plan, const double *x, double *d_O);

/*
 * Time-resolved expectation values of the error generators for ONE control
 * vector, replacing calculate_expectation_values (src/FidelityCalculations.jl:368-390):
 *   ev (ntimes, nerr) real column-major, ev[k, e] = Re(dt tr(P0 sum_{j<=k} O_j,e)) / tr(P0).
 */
int grape_expectation_values(grape_plan *plan, const double *x, double *ev);

/*
 * Closure fallback of the three analysis entry points above (plans created with
 * GRAPE_DESC_HOST_TABLES; the reference's closures evaluated by the caller):
 *   grape_unitary_derivs_tables: H [ntimes][nv][ndim*ndim] complex column-major, the
 *     variant layout of grape_fidelity_grad_tables for ONE control vector (every x_add
 *     call site present); outputs as grape_unitary_derivs.
 *   grape_interaction_error_operators_tables / grape_expectation_values_tables:
 *     H0   [ntimes][ndim*ndim]        H0(k, x[:,k], x_add)                (UnitaryCalculations.jl:196)
 *     Oerr [ntimes][nerr][ndim*ndim]  (1/eps) Herror_e(k, x[:,k], x_add, eps) (:193)
 *     (complex, column-major); O as grape_interaction_error_operators, written to host
 *     memory or, with O_on_device != 0, to device memory; ev as grape_expectation_values.
 * Synchronous.
 */
int grape_unitary_derivs_tables(grape_plan *plan, const double *x, const double *H,
                                double *U, double *U_dx, double *U_dx_add,
                                double *U_derr, double *U_derr_dx, double *U_derr_dx_add);
int grape_interaction_error_operators_tables(grape_plan *plan, const double *x, const double *H0,
                                             const double *Oerr, double *O, int O_on_device);
int grape_expectation_values_tables(grape_plan *plan, const double *x, const double *H0,
                                    const double *Oerr, double *ev);

/*
 * Per-kernel timing for measurement (bench.py's roofline): when enabled, every
 * launch of the plan's pipeline is bracketed by HIP events recorded ON THE
 * PLAN'S STREAM; grape_plan_synchronize accumulates the elapsed times.
 * grape_plan_kernel_times copies GRAPE_NUM_KERNELS totals (ms) and launch
 * counts, indexed by grape_kernel, and optionally resets them.
 */
typedef enum grape_kernel {
    GRAPE_KERNEL_EXPM = 0,      /* propagators of every FD variant (Pade m <= 5) */
    GRAPE_KERNEL_EXPM_HIGH = 1, /* Pade m = 7/9/13 items parked by the above */
    GRAPE_KERNEL_SCAN = 2,      /* chunked prefix products, fidelity, gradient kernels */
    GRAPE_KERNEL_GRAD = 3,      /* per-step contractions: k_grad (closure tables, no error sources) / k_err_local (error sources) */
    GRAPE_KERNEL_REDUCE = 4,    /* x_add reductions */
    GRAPE_KERNEL_ERR_SCAN = 5,  /* error sources: U_derr, F_d2err, per-chunk kernels */
    GRAPE_KERNEL_ERR_GRAD = 6,  /* error sources: F_d2err_dx contractions */
    GRAPE_KERNEL_EXPM_GRAD = 7, /* no error sources: eps-variant propagators contracted in place */
    GRAPE_KERNEL_GRAD_HIGH = 8, /* Pade m > 5 items parked by the above */
    GRAPE_KERNEL_DEXP = 9,      /* dense engine: nominal propagators (MFMA) */
    GRAPE_KERNEL_DSCAN = 10,    /* dense engine: chunk-local prefix products */
    GRAPE_KERNEL_DCARRY = 11,   /* dense engine: carries, U, F, M = G U */
    GRAPE_KERNEL_DMC = 12,      /* dense engine: per-chunk M'_c */
    GRAPE_KERNEL_DGRAD = 13,    /* dense engine: eps-variant propagators contracted in place */
    GRAPE_KERNEL_WALK_FWD = 14, /* sector chunk walks: propagators + chunk totals (grape_walk.hpp) */
    GRAPE_KERNEL_WALK_GRAD = 15,/* sector chunk walks: eps-variants contracted along the chunk */
    GRAPE_KERNEL_EVAL1 = 16,    /* one workgroup per evaluation (latency-bound calls, ABI 10) */
    GRAPE_NUM_KERNELS = 17
} grape_kernel;

int grape_plan_set_profiling(grape_plan *plan, int enable);
int grape_plan_kernel_times(grape_plan *plan, double *total_ms, long long *launches, int reset);

/*
 * Sectors (ABI 5).  When every operator that H0 uses is block-diagonal in one common
 * permutation of the basis (a conserved quantity: for rydberg_hamiltonian_full the 9 levels
 * split into blocks of 4, 2 and 2 plus |00>, which no operator touches), exp, chain and
 * contractions never leave the blocks, so grape_fidelity_grad runs each evaluation as
 * independent sector problems -- one or two classes of `nsectors[c]` sectors of `sector_dims[c]`
 * levels (blocks packed first-fit, padded with decoupled levels) -- and assembles U only for the
 * fidelity (and error) heads.  Same outputs; no API change.  Chosen at plan creation for
 * operator-basis plans (H0 and error operators) when it cuts the work at least in half;
 * GRAPE_OPT_NO_SECTORS turns it off.  Fills up to max_classes entries and returns the
 * number of classes; a plan that runs whole matrices reports one class (ndim, 1).
 */
int grape_plan_sectors(grape_plan *plan, int *sector_dims, int *nsectors, int max_classes);
/* (ABI 8) Per sector class of grape_plan_sectors: twin[c] = 1 when its two sectors share one
 * exponential per step (GRAPE_OPT_NO_TWIN), symmetric (optional) = 1 when the sectors are the
 * symmetry-adapted ones (GRAPE_OPT_NO_SYMMETRY).  Returns the number of classes. */
int grape_plan_sector_info(grape_plan *plan, int *twin, int *symmetric, int max_classes);
/* Which sector classes run the phase-covariant walks (ABI 9; GRAPE_OPT_NO_GAUGE): gauge[c] = 1 per
 * class, 2 (ABI 11) when the class's charges are the ladder N_j = j (the merged walks then use
 * compile-time charge differences); returns the number of classes (1 for whole matrices, gauge[0] = 0). */
int grape_plan_gauge_info(grape_plan *plan, int *gauge, int max_classes);
/* 1 when every call of the plan runs one workgroup per evaluation (ABI 10; GRAPE_OPT_NO_EVAL1 above:
 * an eligible layout and max_batch <= 256), 0 otherwise, or a negative grape_status. */
int grape_plan_eval1(grape_plan *plan);

/*
 * Symmetry-adapted basis (ABI 8, host only: no device needed).  The unitary V (ndim x ndim,
 * column-major interleaved complex, caller-owned) that grape_plan_create would use for the sector
 * path of `desc` (GRAPE_OPT_NO_SYMMETRY above): per sparsity component of H0's and the error
 * sources' operators, the minimal invariant subspaces of the algebra they generate, each with the
 * basis closest to the unit vectors.  block (optional, ndim ints) receives the invariant-subspace id
 * of each column.  Returns 1 when V splits some component further than its sparsity pattern (V may
 * still be returned as the identity when the plan would not use it), 0 when V is the identity,
 * negative on errors.  Plans use V only when the rotated sectors cost less work.
 */
int grape_symmetry_basis(const grape_desc *desc, double *V, int *block);

/*
 * Batched matrix exponential exp(A) of n column-major ndim x ndim complex
 * matrices (2 <= ndim <= GRAPE_MAX_DENSE_DIM; above GRAPE_MAX_SMALL_DIM the
 * dense engine's solve needs a skew-Hermitian A, see grape_dense.hpp) on `device`, with the reference's algorithm (Julia
 * LinearAlgebra.exp!: Pade degree by 1-norm, gesv, squaring).  Host buffers.
 * stats (optional, 5 ints) receives how many matrices used Pade m=3,5,7,9,13.
 */
int grape_expm_batch(int device, int ndim, int n, const double *A, double *E, int *stats);

#ifdef __cplusplus
}
#endif
#endif /* GRAPE_H */
