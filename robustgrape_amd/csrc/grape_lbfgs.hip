// grape_lbfgs.hip -- the L-BFGS two-loop recursion of the batched restart optimiser
// (robustgrape_amd/optimize.py, lbfgs_batched) as one launch per iteration.
//
// The optimiser replaces Optim.jl's LBFGS driving calculate_fidelity_and_derivatives
// (src/FidelityCalculations.jl:199-217).  All restarts advance together; their
// histories are ring buffers S, Y [m][R][n] and rho [m][R].  In torch the recursion
// is ~160 small launches per iteration (2 m gathers, dots and axpys); here one
// workgroup per restart walks its own history: the q vector lives in the output
// row D[r] (each thread owns the same elements in every pass, so only the dot
// products need the workgroup barrier).  HBM-bound: reads 2 m n doubles of
// history twice per restart.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "grape.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxHistory = 64;

// Sum over the workgroup; every thread gets the result.
__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();  // red[] free (previous reduction consumed)
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    return s;
}

// D[r] = -H_r g[r]: H_r the L-BFGS inverse-Hessian estimate of restart r from its
// newest hist[r] pairs (ring buffer, newest at head[r] - 1), scaled by gamma[r].  One workgroup.
__device__ void dir_row(int r, int R, int n, int m, const double *__restrict__ S, const double *__restrict__ Y,
                        const double *__restrict__ rho, const int64_t *__restrict__ head,
                        const int64_t *__restrict__ hist, const double *__restrict__ gamma,
                        const double *__restrict__ g, double *__restrict__ D) {
    __shared__ double red[kThreads / 64];
    __shared__ double alpha[kMaxHistory];
    const size_t row = (size_t)r * n;
    double *q = D + row;
    for (int i = threadIdx.x; i < n; i += kThreads) q[i] = -g[row + i];
    const int h = (int)hist[r], hd = (int)head[r];
    for (int j = 0; j < h; ++j) {  // newest first
        const int slot = ((hd - 1 - j) % m + m) % m;
        const double *s = S + ((size_t)slot * R) * n + row, *y = Y + ((size_t)slot * R) * n + row;
        double part = 0.0;
        for (int i = threadIdx.x; i < n; i += kThreads) part += s[i] * q[i];
        const double a = rho[(size_t)slot * R + r] * block_sum(part, red);
        if (threadIdx.x == 0) alpha[j] = a;
        for (int i = threadIdx.x; i < n; i += kThreads) q[i] -= a * y[i];
    }
    const double gm = gamma[r];
    for (int i = threadIdx.x; i < n; i += kThreads) q[i] *= gm;
    __syncthreads();  // alpha[] visible
    for (int j = h - 1; j >= 0; --j) {  // oldest first
        const int slot = ((hd - 1 - j) % m + m) % m;
        const double *s = S + ((size_t)slot * R) * n + row, *y = Y + ((size_t)slot * R) * n + row;
        double part = 0.0;
        for (int i = threadIdx.x; i < n; i += kThreads) part += y[i] * q[i];
        const double c = alpha[j] - rho[(size_t)slot * R + r] * block_sum(part, red);
        for (int i = threadIdx.x; i < n; i += kThreads) q[i] += c * s[i];
    }
}
__global__ __launch_bounds__(kThreads) void k_lbfgs_dir(int R, int n, int m, const double *__restrict__ S,
                                                        const double *__restrict__ Y,
                                                        const double *__restrict__ rho,
                                                        const int64_t *__restrict__ head,
                                                        const int64_t *__restrict__ hist,
                                                        const double *__restrict__ gamma,
                                                        const double *__restrict__ g, double *__restrict__ D) {
    dir_row(blockIdx.x, R, n, m, S, Y, rho, head, hist, gamma, g, D);  // grid == R
}

// ---------------------------------------------------------------------------
// The strong-Wolfe line search and the L-BFGS update of every restart, on the device
// (optimize.py lbfgs_batched, Nocedal & Wright alg. 3.5 / 3.6, c1 = 1e-4, c2 = 0.9): the
// per-row state machine that was ~60 masked torch ops per line-search round is one workgroup
// per row here, so a round is: compaction of the searching rows (k_ls_compact, one workgroup)
// and their trial points (k_ls_trial) -> the host reads the count (the round's only sync) ->
// the cost of the compact batch -> k_ls_end.  Row-local arithmetic only (a row's trajectory
// does not depend on the others: the batched-equals-single property of the torch version).
// ---------------------------------------------------------------------------
constexpr double kC1 = 1e-4, kC2 = 0.9;
constexpr int kCompactThreads = 1024;

__device__ __forceinline__ double row_dot(const double *a, const double *b, int n, double *red) {
    double part = 0.0;
    for (int i = threadIdx.x; i < n; i += kThreads) part += a[i] * b[i];
    return block_sum(part, red);
}
__device__ __forceinline__ double row_amax(const double *a, int n, double *red) {
    double part = 0.0;
    for (int i = threadIdx.x; i < n; i += kThreads) part = fmax(part, fabs(a[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part = fmax(part, __shfl_down(part, o, 64));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = part;
    __syncthreads();
    double m = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) m = fmax(m, red[w]);
    return m;
}

// optimize.py _cubic_min: minimiser of the cubic through (a0, f0, g0), (a1, f1, g1), kept in the
// middle 80 % of the interval; bisection where the cubic is unusable
__device__ double cubic_min(double a0, double f0, double g0, double a1, double f1, double g1) {
    const double d1 = g0 + g1 - 3.0 * (f0 - f1) / (a0 - a1);
    const double disc = d1 * d1 - g0 * g1;
    const double sg = (a1 - a0 > 0.0) ? 1.0 : (a1 - a0 < 0.0 ? -1.0 : 0.0);
    const double d2 = sg * sqrt(fmax(disc, 0.0));
    const double den = g1 - g0 + 2.0 * d2;
    double a = a1 - (a1 - a0) * (g1 + d2 - d1) / den;
    const double lo = fmin(a0, a1), hi = fmax(a0, a1), w = hi - lo;
    const bool ok = disc >= 0.0 && isfinite(a) && den != 0.0;
    if (!ok) a = 0.5 * (a0 + a1);
    return fmin(fmax(a, lo + 0.1 * w), hi - 0.1 * w);
}

// per row: which rows still search, the descent check (-g where D is not a descent direction)
// and the line-search state at a = 1
__device__ void ls_init_row(const grape_lbfgs_state &s, int r) {
    __shared__ double red[kThreads / 64];
    const size_t row = (size_t)r * s.n;
    const bool active = !(s.gconv[r] | s.fconv[r] | s.xconv[r] | s.lsfail[r]) && s.iters[r] < s.iterations &&
                        (s.f_calls_limit <= 0 || s.f_calls[r] < s.f_calls_limit);
    double d0 = row_dot(s.g + row, s.D + row, s.n, red);
    if (active && !(d0 < 0.0)) {  // not a descent direction: restart from -g
        for (int i = threadIdx.x; i < s.n; i += kThreads) s.D[row + i] = -s.g[row + i];
        d0 = row_dot(s.g + row, s.D + row, s.n, red);
        if (threadIdx.x == 0) {
            s.hist[r] = 0;
            s.gamma[r] = 1.0;
        }
    }
    for (int i = threadIdx.x; i < s.n; i += kThreads) {
        s.Xn[row + i] = s.X[row + i];
        s.gn[row + i] = s.g[row + i];
    }
    if (threadIdx.x == 0) {
        const double f = s.f[r];
        s.active[r] = active;
        s.phase[r] = active ? 0 : 2;
        s.dphi0[r] = d0;
        s.f0[r] = f;
        s.fn[r] = f;
        s.a_cur[r] = 1.0;
        s.a_prev[r] = 0.0;
        s.f_prev[r] = f;
        s.dp_prev[r] = d0;
        s.a_lo[r] = s.a_hi[r] = 0.0;
        s.f_lo[r] = s.f_hi[r] = f;
        s.dp_lo[r] = s.dp_hi[r] = d0;
        s.accepted[r] = 0;
        s.first[r] = 1;
    }
}
__global__ __launch_bounds__(kThreads) void k_ls_init(grape_lbfgs_state s) { ls_init_row(s, blockIdx.x); }

// the rows still searching, in row order (one workgroup: an exclusive scan of per-thread counts)
__global__ __launch_bounds__(kCompactThreads) void k_ls_compact(grape_lbfgs_state s) {
    __shared__ int sums[kCompactThreads];
    const int per = (s.R + kCompactThreads - 1) / kCompactThreads, t = threadIdx.x;
    const int lo = min(s.R, t * per), hi = min(s.R, lo + per);
    int c = 0;
    for (int r = lo; r < hi; ++r) c += s.phase[r] < 2;
    sums[t] = c;
    __syncthreads();
    for (int o = 1; o < kCompactThreads; o <<= 1) {
        const int v = t >= o ? sums[t - o] : 0;
        __syncthreads();
        sums[t] += v;
        __syncthreads();
    }
    int at = sums[t] - c;
    for (int r = lo; r < hi; ++r)
        if (s.phase[r] < 2) {
            s.rows[at++] = r;
            s.f_calls[r] += 1;
        }
    if (t == kCompactThreads - 1) s.count[0] = sums[t];
}

// trial points of the compact batch: Xt[i] = X[row] + a_row D[row]
__global__ __launch_bounds__(kThreads) void k_ls_trial(grape_lbfgs_state s) {
    const int i = blockIdx.x;
    if (i >= s.count[0]) return;
    const int64_t r = s.rows[i];
    const double a = s.a_cur[r];
    const size_t row = (size_t)r * s.n, out = (size_t)i * s.n;
    for (int j = threadIdx.x; j < s.n; j += kThreads) s.Xt[out + j] = s.X[row + j] + a * s.D[row + j];
}

// one row's strong-Wolfe step after its trial evaluation (ft, gt: compact row i)
__global__ __launch_bounds__(kThreads) void k_ls_end(grape_lbfgs_state s, const double *ft_, const double *gt_) {
    __shared__ double red[kThreads / 64];
    __shared__ int keep_s;
    const int i = blockIdx.x;
    const int64_t r = s.rows[i];
    const size_t row = (size_t)r * s.n, ti = (size_t)i * s.n;
    const double dpt = row_dot(gt_ + ti, s.D + row, s.n, red);
    if (threadIdx.x == 0) {
        const double a = s.a_cur[r], ft = ft_[i], f0r = s.f0[r], d0r = s.dphi0[r];
        const bool armijo = ft <= f0r + kC1 * a * d0r;
        const bool curv = fabs(dpt) <= -kC2 * d0r;
        const int ph = s.phase[r];
        const bool br = ph == 0;
        const bool to_zoom_a = br && (!armijo || (!s.first[r] && ft >= s.f_prev[r]));
        const bool acc_b = br && !to_zoom_a && curv;
        const bool to_zoom_b = br && !to_zoom_a && !acc_b && dpt >= 0.0;
        const bool expand = br && !to_zoom_a && !acc_b && !to_zoom_b;
        const bool zm = ph == 1;
        const bool z_hi = zm && (!armijo || ft >= s.f_lo[r]);
        const bool z_acc = zm && !z_hi && curv;
        const bool z_flip = zm && !z_hi && !z_acc && dpt * (s.a_hi[r] - s.a_lo[r]) >= 0.0;
        const bool z_lo = zm && !z_hi && !z_acc;
        const bool acc = acc_b || z_acc;
        double A_lo = s.a_lo[r], F_lo = s.f_lo[r], P_lo = s.dp_lo[r];
        double A_hi = s.a_hi[r], F_hi = s.f_hi[r], P_hi = s.dp_hi[r];
        const double Ap = s.a_prev[r], Fp = s.f_prev[r], Pp = s.dp_prev[r];
        if (to_zoom_a) {  // zoom(a_prev, a)
            A_lo = Ap; F_lo = Fp; P_lo = Pp;
            A_hi = a; F_hi = ft; P_hi = dpt;
        }
        if (to_zoom_b) {  // zoom(a, a_prev)
            A_lo = a; F_lo = ft; P_lo = dpt;
            A_hi = Ap; F_hi = Fp; P_hi = Pp;
        }
        if (z_hi) {
            A_hi = a; F_hi = ft; P_hi = dpt;
        }
        if (z_flip) {  // hi <- lo, then lo <- a
            A_hi = s.a_lo[r]; F_hi = s.f_lo[r]; P_hi = s.dp_lo[r];
        }
        if (z_lo) {
            A_lo = a; F_lo = ft; P_lo = dpt;
        }
        int newph = ph;
        if (to_zoom_a || to_zoom_b) newph = 1;
        if (acc) newph = 2;
        const bool better = armijo && ft < s.fn[r];  // the best Armijo point so far: the fallback
        const bool keep = acc || better;
        if (keep) s.fn[r] = ft;
        if (acc) s.accepted[r] = 1;
        const bool zoom_now = newph == 1;
        double a_next = expand ? 4.0 * a : a;
        if (zoom_now) a_next = cubic_min(A_lo, F_lo, P_lo, A_hi, F_hi, P_hi);
        if (zoom_now && fabs(A_hi - A_lo) <= 1e-12 * fmax(fabs(A_lo), 1.0)) newph = 2;  // collapsed bracket
        s.a_prev[r] = expand ? a : Ap;
        s.f_prev[r] = expand ? ft : Fp;
        s.dp_prev[r] = expand ? dpt : Pp;
        s.a_lo[r] = A_lo; s.f_lo[r] = F_lo; s.dp_lo[r] = P_lo;
        s.a_hi[r] = A_hi; s.f_hi[r] = F_hi; s.dp_hi[r] = P_hi;
        s.a_cur[r] = a_next;
        s.phase[r] = newph;
        s.first[r] = 0;
        keep_s = keep;
    }
    __syncthreads();
    if (keep_s)
        for (int j = threadIdx.x; j < s.n; j += kThreads) {
            s.Xn[row + j] = s.Xt[ti + j];
            s.gn[row + j] = gt_[ti + j];
        }
}

// per row after the line search: the accepted point, the ring-buffer update and Optim's
// stopping rules (optimize.py lbfgs_batched)
__device__ void step_row(const grape_lbfgs_state &s, int r) {
    __shared__ double red[kThreads / 64];
    const size_t row = (size_t)r * s.n;
    const bool active = s.active[r] != 0;
    const bool moved = active && s.fn[r] < s.f0[r];
    const bool step = active && (s.accepted[r] || moved);
    // s = Xn - X, y = gn - g (kept in Xt / D's row: D is recomputed next iteration)
    double *sv = s.Xt + row, *yv = s.D + row;  // Xt has R rows of room; the compact batch is consumed
    for (int i = threadIdx.x; i < s.n; i += kThreads) {
        sv[i] = s.Xn[row + i] - s.X[row + i];
        yv[i] = s.gn[row + i] - s.g[row + i];
    }
    __syncthreads();
    const double sy = row_dot(sv, yv, s.n, red), yy = row_dot(yv, yv, s.n, red);
    const double dx = row_amax(sv, s.n, red);
    const bool upd = step && sy > 0.0;
    const int64_t slot = s.head[r];
    if (upd) {
        double *Sd = s.S + ((size_t)slot * s.R) * s.n + row, *Yd = s.Y + ((size_t)slot * s.R) * s.n + row;
        for (int i = threadIdx.x; i < s.n; i += kThreads) {
            Sd[i] = sv[i];
            Yd[i] = yv[i];
        }
    }
    if (step)
        for (int i = threadIdx.x; i < s.n; i += kThreads) {
            s.X[row + i] = s.Xn[row + i];
            s.g[row + i] = s.gn[row + i];
        }
    __syncthreads();
    const double gmax = row_amax(s.g + row, s.n, red), xmax = row_amax(s.X + row, s.n, red);
    if (threadIdx.x == 0) {
        if (active && !moved && !s.accepted[r]) s.lsfail[r] = 1;
        if (upd) {
            s.rho[(size_t)slot * s.R + r] = 1.0 / sy;
            s.head[r] = (slot + 1) % s.m;
            s.hist[r] = s.hist[r] + 1 < s.m ? s.hist[r] + 1 : s.m;
            s.gamma[r] = sy / yy;
        }
        if (step) {
            const double fold = s.f[r], f = s.fn[r];
            s.f[r] = f;
            s.iters[r] += 1;
            if (gmax <= s.g_thr[r]) s.gconv[r] = 1;
            const double df = fabs(f - fold);
            if (df <= s.f_abstol || df <= s.f_reltol * fabs(f)) s.fconv[r] = 1;
            if (dx <= s.x_abstol || dx <= s.x_reltol * xmax) s.xconv[r] = 1;
        }
    }
}
__global__ __launch_bounds__(kThreads) void k_lbfgs_step(grape_lbfgs_state s) { step_row(s, blockIdx.x); }

// Asynchronous rows (optimize.py _lbfgs_device, asynchronous=True): at the start of every round each
// row advances on its own -- a row whose line search ended (accepted, or its round budget spent)
// takes its step, its next direction and its line-search start at a = 1, so the round evaluates
// every searching row whatever its iteration.  Rows are independent, so every row runs exactly the
// per-row arithmetic of the synchronous loop (direction -> ls_init -> rounds -> step) in the same
// order: bitwise the same trajectory.  phase 3 = a row that has not started its first iteration;
// rounds[r] = trial evaluations of the current line search (the synchronous loop's round cap).
__global__ __launch_bounds__(kThreads) void k_async_advance(grape_lbfgs_state s, int steepest, int max_rounds,
                                                            int *rounds) {
    __shared__ int ph_s;
    const int r = blockIdx.x;
    if (threadIdx.x == 0) {
        int ph = s.phase[r];
        if (ph < 2 && rounds[r] >= max_rounds) ph = 2;  // the synchronous loop's MAX_LS_ROUNDS: the search ends
        ph_s = ph;
    }
    __syncthreads();
    const int ph = ph_s;
    if (ph < 2) {  // still searching: one more trial this round
        if (threadIdx.x == 0) rounds[r] += 1;
        return;
    }
    if (ph == 2) {
        if (!s.active[r]) return;  // finished for good
        step_row(s, r);
        __syncthreads();
        if (steepest && threadIdx.x == 0) {  // GradientDescent: drop the pair just stored
            s.hist[r] = 0;
            s.gamma[r] = 1.0;
        }
        __syncthreads();
    }
    // phase 3 (first iteration) or after the step: direction, line-search start
    dir_row(r, s.R, s.n, s.m, s.S, s.Y, s.rho, s.head, s.hist, s.gamma, s.g, s.D);
    __syncthreads();
    ls_init_row(s, r);
    __syncthreads();
    if (threadIdx.x == 0) rounds[r] = s.phase[r] < 2 ? 1 : 0;  // (an inactive row ends in phase 2)
}

// ---------------------------------------------------------------------------
// The optimiser's cost (calculate_common!, FidelityCalculations.jl:172-196) for one batch of
// restarts in one launch: the fidelity terms from the engine, the error-sensitivity penalty and
// the reference's pulse regularisers (Regularization.jl:26-48, :111-115) per control.  One
// workgroup per restart; each control's transformed series staged in LDS.
// ---------------------------------------------------------------------------
constexpr int kCostMaxSteps = 4096;  // LDS staging: 2 series of ntimes doubles

// reg1 = sum d^2, reg2 = sum dd^2 and their gradients jac1 / jac2 of the series y (Regularization.jl:26-48)
__device__ __forceinline__ double reg_jac1(const double *y, int n, int k) {
    if (k == 0) return -2.0 * (y[1] - y[0]);
    if (k == n - 1) return 2.0 * (y[n - 1] - y[n - 2]);
    return -2.0 * ((y[k + 1] - y[k]) - (y[k] - y[k - 1]));
}
__device__ __forceinline__ double reg_jac2(const double *y, int n, int k) {
    if (k == 0) return 2.0 * (y[2] - 2.0 * y[1] + y[0]);
    if (k == 1) return 2.0 * (y[3] - 4.0 * y[2] + 5.0 * y[1] - 2.0 * y[0]);
    if (k == n - 2) return 2.0 * (y[n - 4] - 4.0 * y[n - 3] + 5.0 * y[n - 2] - 2.0 * y[n - 1]);
    if (k == n - 1) return 2.0 * (y[n - 3] - 2.0 * y[n - 2] + y[n - 1]);
    return 2.0 * (y[k + 2] - 4.0 * y[k + 1] + 6.0 * y[k] - 4.0 * y[k - 1] + y[k - 2]);
}

__global__ __launch_bounds__(kThreads) void k_robust_cost(int R, int np, int nt, int na, int ne, const double *X,
                                                          const double *F, const double *Fdx, const double *Fd2,
                                                          const double *Fd2dx, const double *ce, const double *c1,
                                                          const double *c2, const int32_t *kind, double *cost,
                                                          double *grad) {
    __shared__ double red[kThreads / 64];
    __shared__ double ya[kCostMaxSteps], yb[kCostMaxSteps];
    const int r = blockIdx.x, nx = np * nt + na;
    const double *x = X + (size_t)r * nx;
    double *gr = grad + (size_t)r * nx;
    // -F_dx + 2 sum_e c_e F_d2err_e F_d2err_dx[e]
    for (int i = threadIdx.x; i < nx; i += kThreads) {
        double v = -Fdx[(size_t)r * nx + i];
        for (int e = 0; e < ne; ++e) v += 2.0 * (ce[e] * Fd2[(size_t)r * ne + e]) * Fd2dx[((size_t)r * ne + e) * nx + i];
        gr[i] = v;
    }
    double c = 1.0 - F[r];
    for (int e = 0; e < ne; ++e) {
        const double d2 = Fd2[(size_t)r * ne + e];
        c += ce[e] * d2 * d2;
    }
    for (int p = 0; p < np; ++p) {
        const int kd = kind[p];
        if (kd == 0) continue;
        __syncthreads();  // ya / yb of the previous control consumed, grad rows written
        for (int k = threadIdx.x; k < nt; k += kThreads) {
            const double v = x[p + (size_t)k * np];
            ya[k] = kd == 2 ? cos(v) : v;
            yb[k] = kd == 2 ? sin(v) : 0.0;
        }
        __syncthreads();
        double s1 = 0.0, s2 = 0.0;
        for (int k = threadIdx.x; k < nt; k += kThreads) {
            if (k + 1 < nt) {
                const double da = ya[k + 1] - ya[k], db = yb[k + 1] - yb[k];
                s1 += da * da + db * db;
            }
            if (k + 2 < nt) {
                const double dda = (ya[k + 2] - ya[k + 1]) - (ya[k + 1] - ya[k]);
                const double ddb = (yb[k + 2] - yb[k + 1]) - (yb[k + 1] - yb[k]);
                s2 += dda * dda + ddb * ddb;
            }
            double j1 = reg_jac1(ya, nt, k), j2 = reg_jac2(ya, nt, k);
            if (kd == 2) {  // regularization_cost_phase: d/dx of reg(cos x) + reg(sin x)
                const double sn = yb[k], cs = ya[k];
                j1 = -sn * j1 + cs * reg_jac1(yb, nt, k);
                j2 = -sn * j2 + cs * reg_jac2(yb, nt, k);
            }
            gr[p + (size_t)k * np] += c1[p] * j1 + c2[p] * j2;
        }
        const double r1 = block_sum(s1, red), r2 = block_sum(s2, red);
        c += c1[p] * r1 + c2[p] * r2;
    }
    if (threadIdx.x == 0) cost[r] = c;
}

}  // namespace

extern "C" int grape_robust_cost(int R, int nparam, int ntimes, int nadd, int nerr, const double *X, const double *F,
                                 const double *F_dx, const double *F_d2err, const double *F_d2err_dx,
                                 const double *err_coeff, const double *coeff1, const double *coeff2,
                                 const int32_t *reg_kind, double *cost, double *grad, void *stream) {
    if (R < 0 || nparam < 1 || ntimes < 4 || ntimes > kCostMaxSteps || nadd < 0 || nerr < 0) return GRAPE_ERR_INVALID;
    if (R == 0) return GRAPE_OK;
    if (!X || !F || !F_dx || !coeff1 || !coeff2 || !reg_kind || !cost || !grad ||
        (nerr > 0 && (!F_d2err || !F_d2err_dx || !err_coeff)))
        return GRAPE_ERR_INVALID;
    hipLaunchKernelGGL(k_robust_cost, dim3(R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), R, nparam, ntimes,
                       nadd, nerr, X, F, F_dx, F_d2err, F_d2err_dx, err_coeff, coeff1, coeff2, reg_kind, cost, grad);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_ls_init(const grape_lbfgs_state *st, void *stream) {
    if (!st || st->R < 0 || st->n < 1) return GRAPE_ERR_INVALID;
    if (st->R == 0) return GRAPE_OK;
    hipLaunchKernelGGL(k_ls_init, dim3(st->R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), *st);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_ls_begin(const grape_lbfgs_state *st, void *stream) {
    if (!st || st->R < 0 || st->n < 1) return GRAPE_ERR_INVALID;
    if (st->R == 0) return GRAPE_OK;
    hipStream_t hs = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_ls_compact, dim3(1), dim3(kCompactThreads), 0, hs, *st);
    hipLaunchKernelGGL(k_ls_trial, dim3(st->R), dim3(kThreads), 0, hs, *st);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_ls_end(const grape_lbfgs_state *st, int count, const double *ft, const double *gt,
                                  void *stream) {
    if (!st || count < 0 || count > st->R || (count > 0 && (!ft || !gt))) return GRAPE_ERR_INVALID;
    if (count == 0) return GRAPE_OK;
    hipLaunchKernelGGL(k_ls_end, dim3(count), dim3(kThreads), 0, static_cast<hipStream_t>(stream), *st, ft, gt);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_step(const grape_lbfgs_state *st, void *stream) {
    if (!st || st->R < 0 || st->n < 1 || st->m < 1) return GRAPE_ERR_INVALID;
    if (st->R == 0) return GRAPE_OK;
    hipLaunchKernelGGL(k_lbfgs_step, dim3(st->R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), *st);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_async_advance(const grape_lbfgs_state *st, int steepest, int max_rounds, int *rounds,
                                         void *stream) {
    if (!st || st->R < 0 || st->n < 1 || st->m < 1 || st->m > kMaxHistory || !rounds || max_rounds < 1)
        return GRAPE_ERR_INVALID;
    if (st->R == 0) return GRAPE_OK;
    hipLaunchKernelGGL(k_async_advance, dim3(st->R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), *st,
                       steepest, max_rounds, rounds);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}

extern "C" int grape_lbfgs_direction(int R, int n, int m, const double *S, const double *Y, const double *rho,
                                     const int64_t *head, const int64_t *hist, const double *gamma,
                                     const double *g, double *D, void *stream) {
    if (R < 0 || n < 1 || m < 1 || m > kMaxHistory) return GRAPE_ERR_INVALID;
    if (R == 0) return GRAPE_OK;
    if (!S || !Y || !rho || !head || !hist || !gamma || !g || !D) return GRAPE_ERR_INVALID;
    hipLaunchKernelGGL(k_lbfgs_dir, dim3(R), dim3(kThreads), 0, static_cast<hipStream_t>(stream), R, n, m, S, Y,
                       rho, head, hist, gamma, g, D);
    return hipGetLastError() == hipSuccess ? GRAPE_OK : GRAPE_ERR_HIP;
}
