/*
 * abi_check.c -- a plain-C caller of libgrape.so built by gcc against include/grape.h.
 *
 *   abi_check layout   prints sizeof / offsetof of grape_term and grape_desc (no GPU);
 *                      tests/test_c_abi.py compares them with the ctypes mirror
 *                      (robustgrape_amd/operators.py) and the Julia shim's structs
 *                      (julia/RobustGRAPEMI355X.jl)
 *   abi_check gpu      one grape_fidelity_grad call on device 0 for a 2-level problem
 *                      (H = cos(x) X + sin(x) Y + 0.3 Z, target X, N_t = 4, one x_add phase
 *                      on the target) and prints F and F_dx; the GPU test compares them with
 *                      the CPU oracle
 */
#define _POSIX_C_SOURCE 200809L
#include <signal.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "grape.h"

#define PRINT_OFF(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))

static int layout(void) {
    printf("sizeof.grape_term %zu\n", sizeof(grape_term));
    PRINT_OFF(grape_term, op);
    PRINT_OFF(grape_term, var);
    PRINT_OFF(grape_term, index);
    PRINT_OFF(grape_term, func);
    PRINT_OFF(grape_term, a);
    PRINT_OFF(grape_term, b);
    PRINT_OFF(grape_term, scale_re);
    PRINT_OFF(grape_term, scale_im);
    printf("sizeof.grape_desc %zu\n", sizeof(grape_desc));
    PRINT_OFF(grape_desc, ndim);
    PRINT_OFF(grape_desc, ntimes);
    PRINT_OFF(grape_desc, nparam);
    PRINT_OFF(grape_desc, nadd);
    PRINT_OFF(grape_desc, nerr);
    PRINT_OFF(grape_desc, n_ops);
    PRINT_OFF(grape_desc, t0);
    PRINT_OFF(grape_desc, eps);
    PRINT_OFF(grape_desc, eps2);
    PRINT_OFF(grape_desc, projector_diag);
    PRINT_OFF(grape_desc, ops);
    PRINT_OFF(grape_desc, n_h0_terms);
    PRINT_OFF(grape_desc, h0_terms);
    PRINT_OFF(grape_desc, err_term_offsets);
    PRINT_OFF(grape_desc, err_terms);
    PRINT_OFF(grape_desc, n_target_terms);
    PRINT_OFF(grape_desc, target_terms);
    PRINT_OFF(grape_desc, max_batch);
    PRINT_OFF(grape_desc, reserved);
    PRINT_OFF(grape_desc, projector);
    printf("sizeof.grape_lbfgs_state %zu\n", sizeof(grape_lbfgs_state));
    PRINT_OFF(grape_lbfgs_state, R);
    PRINT_OFF(grape_lbfgs_state, n);
    PRINT_OFF(grape_lbfgs_state, m);
    PRINT_OFF(grape_lbfgs_state, X);
    PRINT_OFF(grape_lbfgs_state, f);
    PRINT_OFF(grape_lbfgs_state, g);
    PRINT_OFF(grape_lbfgs_state, D);
    PRINT_OFF(grape_lbfgs_state, Xn);
    PRINT_OFF(grape_lbfgs_state, fn);
    PRINT_OFF(grape_lbfgs_state, gn);
    PRINT_OFF(grape_lbfgs_state, Xt);
    PRINT_OFF(grape_lbfgs_state, f0);
    PRINT_OFF(grape_lbfgs_state, dphi0);
    PRINT_OFF(grape_lbfgs_state, a_cur);
    PRINT_OFF(grape_lbfgs_state, a_prev);
    PRINT_OFF(grape_lbfgs_state, f_prev);
    PRINT_OFF(grape_lbfgs_state, dp_prev);
    PRINT_OFF(grape_lbfgs_state, a_lo);
    PRINT_OFF(grape_lbfgs_state, f_lo);
    PRINT_OFF(grape_lbfgs_state, dp_lo);
    PRINT_OFF(grape_lbfgs_state, a_hi);
    PRINT_OFF(grape_lbfgs_state, f_hi);
    PRINT_OFF(grape_lbfgs_state, dp_hi);
    PRINT_OFF(grape_lbfgs_state, S);
    PRINT_OFF(grape_lbfgs_state, Y);
    PRINT_OFF(grape_lbfgs_state, rho);
    PRINT_OFF(grape_lbfgs_state, gamma);
    PRINT_OFF(grape_lbfgs_state, g_thr);
    PRINT_OFF(grape_lbfgs_state, f_calls);
    PRINT_OFF(grape_lbfgs_state, iters);
    PRINT_OFF(grape_lbfgs_state, hist);
    PRINT_OFF(grape_lbfgs_state, head);
    PRINT_OFF(grape_lbfgs_state, rows);
    PRINT_OFF(grape_lbfgs_state, phase);
    PRINT_OFF(grape_lbfgs_state, first);
    PRINT_OFF(grape_lbfgs_state, accepted);
    PRINT_OFF(grape_lbfgs_state, gconv);
    PRINT_OFF(grape_lbfgs_state, fconv);
    PRINT_OFF(grape_lbfgs_state, xconv);
    PRINT_OFF(grape_lbfgs_state, lsfail);
    PRINT_OFF(grape_lbfgs_state, active);
    PRINT_OFF(grape_lbfgs_state, count);
    PRINT_OFF(grape_lbfgs_state, f_abstol);
    PRINT_OFF(grape_lbfgs_state, f_reltol);
    PRINT_OFF(grape_lbfgs_state, x_abstol);
    PRINT_OFF(grape_lbfgs_state, x_reltol);
    PRINT_OFF(grape_lbfgs_state, iterations);
    PRINT_OFF(grape_lbfgs_state, f_calls_limit);
    printf("abi_version %d\n", grape_abi_version());
    return 0;
}

static int gpu(void) {
    /* operators, column-major interleaved: X, Y, Z, I */
    double ops[4][8];
    memset(ops, 0, sizeof ops);
    ops[0][2] = 1.0; ops[0][4] = 1.0;                 /* X: (1,0) = (0,1) = 1 */
    ops[1][3] = 1.0; ops[1][5] = -1.0;                /* Y: (1,0) = i, (0,1) = -i */
    ops[2][0] = 1.0; ops[2][6] = -1.0;                /* Z */
    ops[3][0] = 1.0; ops[3][6] = 1.0;                 /* I */
    grape_term h0[3] = {
        {0, GRAPE_VAR_X, 0, GRAPE_FN_COS, 1.0, 0.0, 1.0, 0.0},
        {1, GRAPE_VAR_X, 0, GRAPE_FN_SIN, 1.0, 0.0, 1.0, 0.0},
        {2, GRAPE_VAR_ONE, 0, GRAPE_FN_ONE, 1.0, 0.0, 0.3, 0.0},
    };
    /* target = X * exp(i theta) */
    grape_term tgt[1] = {{0, GRAPE_VAR_XADD, 0, GRAPE_FN_CIS, 1.0, 0.0, 1.0, 0.0}};
    double pdiag[2] = {1.0, 1.0};
    grape_desc d;
    memset(&d, 0, sizeof d);
    d.ndim = 2; d.ntimes = 4; d.nparam = 1; d.nadd = 1; d.nerr = 0; d.n_ops = 4;
    d.t0 = 1.7; d.eps = 1e-8; d.eps2 = 1e-4;
    d.projector_diag = pdiag; d.ops = &ops[0][0];
    d.n_h0_terms = 3; d.h0_terms = h0;
    d.n_target_terms = 1; d.target_terms = tgt;
    d.max_batch = 1;
    grape_plan *plan = NULL;
    int rc = grape_plan_create(&d, 0, &plan);
    if (rc) { fprintf(stderr, "plan_create %d: %s\n", rc, grape_last_error()); return 1; }
    const double x[5] = {0.1, 0.7, -0.4, 1.3, 0.25};
    double F = 0.0, Fdx[5];
    rc = grape_fidelity_grad(plan, 1, x, &F, Fdx, NULL, NULL);
    if (rc) { fprintf(stderr, "fidelity_grad %d: %s\n", rc, grape_last_error()); grape_plan_destroy(plan); return 1; }
    printf("F %.17g\n", F);
    for (int i = 0; i < 5; ++i) printf("F_dx %d %.17g\n", i, Fdx[i]);
    grape_plan_destroy(plan);
    return 0;
}

/* the fault handler is opt-in (ABI 11): loading the library leaves SIGSEGV / SIGBUS alone */
static int signals(void) {
    struct sigaction sa;
    sigaction(SIGSEGV, NULL, &sa);
    printf("segv_default_at_load %d\n", sa.sa_handler == SIG_DFL);
    sigaction(SIGBUS, NULL, &sa);
    printf("bus_default_at_load %d\n", sa.sa_handler == SIG_DFL);
    printf("installed %d\n", grape_install_fault_handler());
    sigaction(SIGSEGV, NULL, &sa);
    printf("segv_default_after %d\n", sa.sa_handler == SIG_DFL);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) return gpu();
    if (argc > 1 && strcmp(argv[1], "signals") == 0) return signals();
    return layout();
}
