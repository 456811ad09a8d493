// grape_dense.hpp -- CDNA4 (gfx950) building blocks of the DENSE engine
// (13 <= d <= 64; SURVEY.md 8d config C5, the dense-GEMM regime).
//
// One workgroup of 8 waves (two per SIMD) owns one 64 x 64 complex FP64 matrix problem at a
// time (smaller d is zero-padded to 64: exp, products and the fidelity are
// unchanged by a zero block with zero weight).  Every d x d complex product is
// four real GEMMs on v_mfma_f64_16x16x4_f64 (16 x 16 output, K = 4, one f64 per
// lane for A and B, 4 f64 accumulators per lane):
//
//   A fragment (16 x 4):  lane l holds A[l & 15][l >> 4]
//   B fragment (4 x 16):  lane l holds B[l >> 4][l & 15]
//   C tile (16 x 16):     lane l, element r holds C[(l >> 4) + 4r][l & 15]
//
// (checked on the hardware with exact integer data, scripts/probes/mfma_probe.hip).
// The four real GEMMs run as Gauss's three (Lr Rr, Li Ri, (Lr + Li)(Rr + Ri); see mm).
// Element r of a C tile is therefore the B fragment of k-rows 4r..4r+3: a
// matrix kept in registers in C-tile layout IS the right operand of the next
// product, with no data movement.  Register matrices (HM) are distributed by
// tile: wave (w, h) holds columns 16w..16w+15 of row tiles 2h and 2h+1 (2 C
// tiles, re and im: 32 VGPRs per complex matrix, so an exponential keeps its
// five live matrices in registers at two waves per SIMD).  A product
// P = L . R reads both operands from LDS (A and B fragments); each wave
// computes its own two tiles of P.
//
// LDS matrices (SM) are two row-major 64 x 64 double planes with the column
// swizzle  col ^ swz64(row) (below):  C-tile stores (16 contiguous columns of
// one row per 16 lanes), A-fragment reads of L and of L^T, and B-fragment reads
// of R and R^T are all bank-conflict free, as ds_read_b64 (two 32-lane groups
// over 64 banks) and as ds_read2st64_b64 / ds_write_b64 (four 16-lane groups
// over 32 banks).
//
// HBM images: a complex matrix is stored as its register file, plane by plane
// (re then im), index ((w*4 + t)*4 + r)*64 + lane: a wave loads or stores its
// 16 KB as 32 fully coalesced 512-B rows.
//
// The matrix exponential follows Julia's LinearAlgebra.exp! (Pade degree by
// 1-norm thresholds 0.015/0.25/0.95/2.1, else Pade 13 with squarings; U and
// V as in exp!; X = (V-U) \ (V+U)).  The solve is a blocked Gauss-Jordan
// elimination WITHOUT row interchanges, all on MFMA (4 block steps of 16
// columns; the 16 x 16 diagonal block is inverted by one wave).  That is safe
// here: for a Hermitian H (checked at plan creation) A = -i dt H is
// skew-Hermitian, the Pade denominator q(A) = V - U has Hermitian part V with
// eigenvalues Re q(i theta) = |q(i theta)| cos(theta/2) > 0 for
// |theta| <= |A|_2 <= |A|_1 < pi, so every leading block and Schur complement
// is nonsingular with bounded growth (no pivoting needed).  For Pade 13 the
// scaling is raised, if necessary, until |A/2^s|_1 <= 1.6 (Julia: 5.4) to keep
// that margin; the result differs from exp! by rounding only.
#pragma once
#include <hip/hip_runtime.h>

#include "grape_kernels.hpp"

namespace grape_dense {

using grape::cd;
using grape::Term;
typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int N = 64;          // padded dimension
constexpr int NT = 4;          // 16-row tiles per dimension
constexpr int NW = 8;          // waves per workgroup: (column block w, row half h)
constexpr int NTHREADS = 64 * NW;
constexpr int PLANE = N * N;   // doubles per plane
constexpr int IMG = 2 * PLANE; // doubles per complex matrix image (64 KB)
constexpr int SMALL = 16 * 16; // doubles per plane of a 16 x 16 block

// LDS (doubles): matrix region 0 | matrix region 1 | reduction scratch
constexpr int LDS_R0 = 0;
constexpr int LDS_R1 = 2 * PLANE;
constexpr int LDS_RED = 4 * PLANE;
constexpr int LDS_TOTAL = LDS_RED + 2 * N + 16;
// Gauss-Jordan buffers overlay region 0 (even block steps) and region 1 (odd)
constexpr int GJ_DINV = 0;                        // D^-1: 2 planes x 16 x 16
constexpr int GJ_PCOL = GJ_DINV + 2 * SMALL;      // -Q[:, block kb]: 2 planes x 64 x 16
constexpr int GJ_NR = GJ_PCOL + 2 * 4 * SMALL;    // new row block: [w][q|p][plane][16 x 16]
constexpr int GJ_SET = GJ_NR + 4 * 2 * 2 * SMALL; // 6 656 doubles <= 2 * PLANE
static_assert(GJ_SET <= 2 * PLANE, "GJ buffers must fit one matrix region");

struct HM {
    v4d re[2];  // tiles 2h, 2h+1 of column block w
    v4d im[2];
};

struct SM {
    double *re, *im;
    int boff;  // byte offset of re from the LDS start (mm's fragment addresses)
};

__device__ __forceinline__ SM sm_at(double *lds, int off) {
    SM s;
    s.re = lds + off;
    s.im = lds + off + PLANE;
    s.boff = 8 * off;
    return s;
}

// The swizzle f(row) = (row & 15) | (row & 1) << 4: its low four bits and its bits 4..1 are both
// permutations of row & 15, and bit 4 alternates with the row parity.  So the fragment reads are
// conflict free both as ds_read_b64 (two 32-lane groups over 64 banks: needs bits 4..1 distinct over 16 rows
// and bit 4 split between rows 2k, 2k + 1) and as the ds_read2st64_b64 the compiler forms from the re / im
// plane pair (four 16-lane groups over 32 banks: needs the low four bits distinct over 16 rows).  Round 6:
// the round-2 swizzle ((row & 15) << 1) ^ ((row & 1) << 4) met only the first -- the A-fragment reads of L
// and the B-fragment reads of R^T were 2-way conflicted as ds_read2st64_b64 (C5's LDS conflict
// cycles above its LDS-active cycles).  Checked exhaustively for every access pattern below by
// scripts/probes/lds_banks.py.
#ifndef GRAPE_DENSE_SWZ_R2  // 1: the round-2 swizzles (A/B)
#define GRAPE_DENSE_SWZ_R2 0
#endif
__device__ __forceinline__ int swz64(int row) {
    if (GRAPE_DENSE_SWZ_R2) return ((row & 15) << 1) ^ ((row & 1) << 4);
    return (row & 15) | ((row & 1) << 4);
}
__device__ __forceinline__ int sidx(int row, int col) { return row * N + (col ^ swz64(row)); }
// 64 x 16 / 16 x 16 buffers read as A fragments: conflict-free in both models with this swizzle (round 2:
// row & 14, 2-way in the 16-lane one)
__device__ __forceinline__ int sidx16(int row, int col) { return row * 16 + (col ^ (row & (GRAPE_DENSE_SWZ_R2 ? 14 : 15))); }

__device__ __forceinline__ v4d mfma(double a, double b, v4d c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

struct Lane {
    int l;    // lane in the wave
    int w;    // column block (wave-uniform)
    int h;    // row half: tiles 2h, 2h+1 (wave-uniform)
    int wid;  // wave in the workgroup
    __device__ __forceinline__ int tile(int i) const { return 2 * h + i; }
    __device__ __forceinline__ int row(int i, int r) const { return 16 * (2 * h + i) + (l >> 4) + 4 * r; }
    __device__ __forceinline__ int col() const { return 16 * w + (l & 15); }
    __device__ __forceinline__ int img(int i, int r) const { return ((w * NT + 2 * h + i) * 4 + r) * 64 + l; }
};

__device__ __forceinline__ Lane make_lane() {
    Lane L;
    L.l = threadIdx.x & 63;
    L.wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    L.w = L.wid & 3;
    L.h = L.wid >> 2;
    return L;
}

__device__ __forceinline__ void hm_zero(HM &M) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        M.re[i] = v4d{0.0, 0.0, 0.0, 0.0};
        M.im[i] = v4d{0.0, 0.0, 0.0, 0.0};
    }
}

__device__ __forceinline__ void hm_identity(HM &M, const Lane &ln, double s) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            M.re[i][r] = ln.row(i, r) == ln.col() ? s : 0.0;
            M.im[i][r] = 0.0;
        }
}

// M += c X
__device__ __forceinline__ void hm_axpy(HM &M, double c, const HM &X) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            M.re[i][r] = fma(c, X.re[i][r], M.re[i][r]);
            M.im[i][r] = fma(c, X.im[i][r], M.im[i][r]);
        }
}

__device__ __forceinline__ void hm_scale(HM &M, double c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        M.re[i] *= c;
        M.im[i] *= c;
    }
}

// ---------------------------------------------------------------------------
// HBM images and LDS stores
// ---------------------------------------------------------------------------
// (pinned lane: a load of a loop-invariant image must not be hoisted out of a
// loop around an exponential, where it would hold 32 VGPRs through the Pade)
__device__ __forceinline__ void img_load(const double *img, HM &M, const Lane &ln_in) {
    Lane ln = ln_in;
    asm volatile("" : "+v"(ln.l));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            M.re[i][r] = img[ln.img(i, r)];
            M.im[i][r] = img[PLANE + ln.img(i, r)];
        }
}

__device__ __forceinline__ void img_store(double *img, const HM &M, const Lane &ln) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            img[ln.img(i, r)] = M.re[i][r];
            img[PLANE + ln.img(i, r)] = M.im[i][r];
        }
}

// a copy of the lane descriptor whose lane id the compiler cannot see through:
// index math derived from it is recomputed where used instead of being hoisted
// out of every enclosing loop and kept live
__device__ __forceinline__ Lane pinned(const Lane &ln) {
    Lane p = ln;
    asm volatile("" : "+v"(p.l));
    return p;
}

__device__ __forceinline__ void sm_store(SM S, const HM &M, const Lane &ln_in) {
    const Lane ln = pinned(ln_in);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = sidx(ln.row(i, r), ln.col());
            S.re[o] = M.re[i][r];
            S.im[o] = M.im[i][r];
        }
}

__device__ __forceinline__ void sm_load(SM S, HM &M, const Lane &ln_in) {
    const Lane ln = pinned(ln_in);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = sidx(ln.row(i, r), ln.col());
            M.re[i][r] = S.re[o];
            M.im[i][r] = S.im[o];
        }
}

// ---------------------------------------------------------------------------
// P += op(L) . op(R), both operands in LDS (LT/RT: transpose, LC/RC: conjugate).
// Wave (w, h) computes tiles (2h, w), (2h+1, w): 16 k-steps x 6 MFMAs (Gauss 3M).
// ---------------------------------------------------------------------------

struct Frag {
    double aR[2], aI[2], bR, bI;
};

// Round 6 (GRAPE_DENSE_FRAG_ADDR): the fragment addresses in closed form.  With the round-6 swizzle,
// for k-step s (a compile-time constant in the unrolled loop) and byte offsets
//   A of L:    a + ((32 s) ^ ac) (+ 8 192 for the second tile),   A of L^T: (a ^ (32 (s & 3) [+ 128])) + 2 048 s
//   B of R^T:  b + ((32 s) ^ bc),                                  B of R:   (b ^ (32 (s & 3))) + 2 048 s
// from four per-lane values formed once per product (frag_addr) -- one or two VALU instructions per address
// and step, the rest the loads' immediate offsets, where recomputing sidx from the lane id cost ~15 per
// step (checked for every lane, tile and step against sidx by scripts/probes/lds_banks.py).
#ifndef GRAPE_DENSE_FRAG_ADDR
#define GRAPE_DENSE_FRAG_ADDR 1
#endif
struct FragAddr {
    int a, ac, b, bc;
};
template <bool LT, bool RT>
__device__ __forceinline__ FragAddr frag_addr(const Lane &ln) {
    const int l = ln.l, g = l >> 4, c = l & 15, gp = g | ((g & 1) << 4);
    FragAddr f;
    const int ir = 16 * ln.tile(0) + c, jc = 16 * ln.w + c;
    if (LT) {
        f.a = 8 * (64 * g + (ir ^ gp));
        f.ac = 0;
    } else {
        const int sw = swz64(ir);
        f.a = 8 * (ir * 64 + (g ^ (sw & 3)));
        f.ac = 32 * (sw >> 2);
    }
    if (RT) {
        const int sw = swz64(jc);
        f.b = 8 * (jc * 64 + (g ^ (sw & 3)));
        f.bc = 32 * (sw >> 2);
    } else {
        f.b = 8 * (64 * g + (jc ^ gp));
        f.bc = 0;
    }
    return f;
}
__device__ __forceinline__ double lds_at(const double *base, int byte_off) {
    return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + byte_off);
}
// GRAPE_DENSE_FA_BASE: both operands addressed from the LDS start, their regions' byte offsets folded
// into fa.a / fa.b once per product.  Region 1 starts at 64 KB, beyond a ds_read_b64's 16-bit immediate:
// addressed from its own base, every B (and, for L in region 1, A) fragment load of a step took two
// v_add_u32 (base + re plane, base + im plane) and the re / im pair was not merged into one
// ds_read2st64_b64.
#ifndef GRAPE_DENSE_FA_BASE
#define GRAPE_DENSE_FA_BASE 0
#endif
template <bool LT, bool RT, bool RC>
__device__ __forceinline__ void mm_load_fa(SM L, SM R, int s, Frag &f, FragAddr &fa) {
    // made opaque in place at every step (no copies): each step's addresses are formed here instead of being
    // hoisted out of the product as 16 x 3 VGPRs; only the fields this product reads
    if constexpr (LT) asm volatile("" : "+v"(fa.a));
    else asm volatile("" : "+v"(fa.a), "+v"(fa.ac));
    if constexpr (RT) asm volatile("" : "+v"(fa.b), "+v"(fa.bc));
    else asm volatile("" : "+v"(fa.b));
    const double *lre = GRAPE_DENSE_FA_BASE ? L.re - L.boff / 8 : L.re, *lim = lre + PLANE;
    const double *rre = GRAPE_DENSE_FA_BASE ? R.re - R.boff / 8 : R.re, *rim = rre + PLANE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int o = LT ? (fa.a ^ ((i ? 128 : 0) + 32 * (s & 3))) + 2048 * s : fa.a + ((32 * s) ^ fa.ac) + 8192 * i;
        f.aR[i] = lds_at(lre, o);
        f.aI[i] = lds_at(lim, o);
    }
    const int o = RT ? fa.b + ((32 * s) ^ fa.bc) : (fa.b ^ (32 * (s & 3))) + 2048 * s;
    f.bR = lds_at(rre, o);
    f.bI = RC ? -lds_at(rim, o) : lds_at(rim, o);
}
template <bool LT, bool RT, bool RC>
__device__ __forceinline__ void mm_load(SM L, SM R, int s, Frag &f, const Lane &ln) {
    // Indices are recomputed from a freshly pinned lane id every step: otherwise
    // the compiler hoists all 16 steps' swizzled addresses of every product
    // out of the enclosing loops and keeps them live (~100 VGPRs -> spills).
    int l = ln.l;
    asm volatile("" : "+v"(l));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ir = 16 * ln.tile(i) + (l & 15), kc = 4 * s + (l >> 4);
        const int o = LT ? sidx(kc, ir) : sidx(ir, kc);
        f.aR[i] = L.re[o];
        f.aI[i] = L.im[o];
    }
    const int kr = 4 * s + (l >> 4), jc = 16 * ln.w + (l & 15);
    const int o = RT ? sidx(jc, kr) : sidx(kr, jc);
    f.bR = R.re[o];
    f.bI = RC ? -R.im[o] : R.im[o];
}

// Software-pipelined over the 16 k-steps: the fragments of step s+1 are loaded
// while step s's 8 MFMAs issue; the "memory" pin stops the compiler from hoisting
// every step's loads to the top (that costs ~100 VGPRs and forces spills).
// Gauss's 3-multiplication complex product: 3 real MFMA streams per complex product instead
// of 4; rounding-level differences only (the dense parity tests hold at T0).  Measured at C5:
// 940 -> 1 064 evals/s, k_dgrad 0.52 -> 0.58 of the FP64 peak credited with the algorithmic
// 8 d^3 per complex product (executed: 6 d^3).
#ifndef GRAPE_DENSE_4M
#define GRAPE_DENSE_4M 0
#endif
#ifndef GRAPE_DENSE_CONJ_EPI
#define GRAPE_DENSE_CONJ_EPI 0
#endif
#ifndef GRAPE_DENSE_PINGPONG  // 3M products: fragment buffers by step parity (mm, below)
#define GRAPE_DENSE_PINGPONG 1
#endif
template <bool LT, bool LC, bool RT, bool RC>
__device__ __forceinline__ void mm(SM L, SM R, HM &P, const Lane &ln) {
    if constexpr (GRAPE_DENSE_4M) {
        // the conventional four real products: re += Lr Rr - Li Ri, im += Lr Ri + Li Rr
        Frag fc, fn;
        v4d tr[2], ti[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) tr[i] = ti[i] = v4d{0.0, 0.0, 0.0, 0.0};
        mm_load<LT, RT, RC>(L, R, 0, fc, ln);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if (s < 15) mm_load<LT, RT, RC>(L, R, s + 1, fn, ln);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double ai = LC ? -fc.aI[i] : fc.aI[i];
                tr[i] = mfma(fc.aR[i], fc.bR, tr[i]);
                tr[i] = mfma(-ai, fc.bI, tr[i]);
                ti[i] = mfma(fc.aR[i], fc.bI, ti[i]);
                ti[i] = mfma(ai, fc.bR, ti[i]);
            }
            if (s < 15) {
                fc = fn;
                asm volatile("" : "+v"(fc.aR[0]), "+v"(fc.aR[1]), "+v"(fc.aI[0]), "+v"(fc.aI[1]), "+v"(fc.bR),
                             "+v"(fc.bI)::"memory");
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            P.re[i] += tr[i];
            P.im[i] += ti[i];
        }
        return;
    }
    // Gauss's three-multiplication complex product: T1 = Lr Rr, T2 = Li Ri, T3 = (Lr + Li)(Rr + Ri),
    // P += (T1 - T2) + i (T3 - T1 - T2): 3 MFMAs per tile and k-step instead of 4.
    // GRAPE_DENSE_CONJ_EPI: a conjugated operand's sign goes to the sums (a - b: a free source modifier)
    // and to T2's sign in the combination below, instead of a negated copy of the fragment per step (two
    // VALU instructions each: sign flip and move)
    constexpr bool kCE = GRAPE_DENSE_CONJ_EPI;
    constexpr bool kT2Neg = kCE && (LC != RC);  // T2 accumulated as -(Li Ri)
    Frag fc, fn;
    v4d t1[2], t2[2], t3[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) t1[i] = t2[i] = t3[i] = v4d{0.0, 0.0, 0.0, 0.0};
    constexpr bool kFA = GRAPE_DENSE_FRAG_ADDR && !GRAPE_DENSE_SWZ_R2;
    FragAddr fa = kFA ? frag_addr<LT, RT>(pinned(ln)) : FragAddr{0, 0, 0, 0};
    if constexpr (kFA && GRAPE_DENSE_FA_BASE) {
        fa.a += L.boff;
        fa.b += R.boff;
    }
    auto load = [&](int s, Frag &f) {
        if constexpr (kFA) mm_load_fa<LT, RT, RC && !kCE>(L, R, s, f, fa);
        else mm_load<LT, RT, RC && !kCE>(L, R, s, f, ln);
    };
    auto step = [&](const Frag &fc) {
        const double bs = (kCE && RC) ? fc.bR - fc.bI : fc.bR + fc.bI;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (kCE) {
                t1[i] = mfma(fc.aR[i], fc.bR, t1[i]);
                t2[i] = mfma(fc.aI[i], fc.bI, t2[i]);
                t3[i] = mfma(LC ? fc.aR[i] - fc.aI[i] : fc.aR[i] + fc.aI[i], bs, t3[i]);
                continue;
            }
            const double ai = LC ? -fc.aI[i] : fc.aI[i];
            t1[i] = mfma(fc.aR[i], fc.bR, t1[i]);
            t2[i] = mfma(ai, fc.bI, t2[i]);
            t3[i] = mfma(fc.aR[i] + ai, bs, t3[i]);
        }
    };
    if constexpr (GRAPE_DENSE_PINGPONG) {
        // two fragment buffers alternating by step parity (the loop is unrolled): no copy fc = fn, and
        // the barrier between steps is a bare compiler fence (it keeps later steps' loads from being
        // hoisted) instead of a pin on the fresh fragment, which forced the wait for step s+1's loads
        // into step s after its first two MFMAs
        Frag fb[2];
        load(0, fb[0]);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if (s < 15) load(s + 1, fb[(s + 1) & 1]);
            step(fb[s & 1]);
            if (s < 15) asm volatile("" ::: "memory");
        }
    } else {
    load(0, fc);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        if (s < 15) load(s + 1, fn);
        step(fc);
        if (s < 15) {
            fc = fn;
            asm volatile("" : "+v"(fc.aR[0]), "+v"(fc.aR[1]), "+v"(fc.aI[0]), "+v"(fc.aI[1]), "+v"(fc.bR),
                         "+v"(fc.bI)::"memory");
        }
    }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if constexpr (kT2Neg) {  // T2 = -t2: the same roundings as the negated-copy form
            P.re[i] += t1[i] + t2[i];
            P.im[i] += t3[i] - t1[i] + t2[i];
        } else {
            P.re[i] += t1[i] - t2[i];
            P.im[i] += t3[i] - t1[i] - t2[i];
        }
    }
}

// ---------------------------------------------------------------------------
// Workgroup reductions (fixed order: deterministic)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wg_sum(double v, double *lds, const Lane &ln) {
    double *red = lds + LDS_RED + 2 * N;
    v = wave_sum(v);
    __syncthreads();  // slots free
    if (ln.l == 0) red[ln.wid] = v;
    __syncthreads();
    return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
}

// |A|_1 = max_j sum_i |a_ij| (Julia opnorm(A, 1)), identical in every wave
__device__ __forceinline__ double wg_norm1(const HM &A, double *lds, const Lane &ln) {
    double *red = lds + LDS_RED;
    double cs = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs += hypot(A.re[i][r], A.im[i][r]);
    cs += __shfl_xor(cs, 16, 64);
    cs += __shfl_xor(cs, 32, 64);
    __syncthreads();  // slots free
    if (ln.l < 16) red[ln.h * N + ln.col()] = cs;
    __syncthreads();
    return wave_max(red[ln.l] + red[N + ln.l]);
}

// ---------------------------------------------------------------------------
// Operator-basis builder: M += c OP (OP image in HBM)
// ---------------------------------------------------------------------------
// (pinned lane: otherwise the loads of the second build of A inside wg_expm are
// CSE'd with the first and the operator images stay live through the Pade)
__device__ __forceinline__ void hm_cmac_img(HM &M, cd c, const double *img, const Lane &ln_in) {
    Lane ln = ln_in;
    asm volatile("" : "+v"(ln.l));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double orr = img[ln.img(i, r)], oi = img[PLANE + ln.img(i, r)];
            double re = M.re[i][r], im = M.im[i][r];
            re = fma(c.re, orr, re);
            re = fma(-c.im, oi, re);
            im = fma(c.re, oi, im);
            im = fma(c.im, orr, im);
            M.re[i][r] = re;
            M.im[i][r] = im;
        }
}

// ---------------------------------------------------------------------------
// 16 x 16 complex inverse by one wave (Gauss-Jordan without interchanges; the
// block has a positive definite Hermitian part, see the header).  In and out
// in C-tile layout: lane l holds column l & 15, rows (l >> 4) + 4r.
// ---------------------------------------------------------------------------
__device__ __forceinline__ cd crecip_smith(cd z) {
    if (fabs(z.re) >= fabs(z.im)) {
        const double q = z.im / z.re, den = z.re + z.im * q;
        return grape::cmake(1.0 / den, -q / den);
    }
    const double q = z.re / z.im, den = z.im + z.re * q;
    return grape::cmake(q / den, -1.0 / den);
}

__device__ __forceinline__ void wave_inv16(v4d &Dr, v4d &Di, v4d &Xr, v4d &Xi, int l, bool &singular) {
    const int c = l & 15, g = l >> 4;
    double dr[4], di[4], xr[4], xi[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        dr[r] = Dr[r];
        di[r] = Di[r];
        xr[r] = (g + 4 * r) == c ? 1.0 : 0.0;
        xi[r] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int kr = k >> 2, kg = k & 3;
        // pivot D[k][k] (lane k + 16 kg, element kr) and the pivot-row entries of my column
        const double pr = __shfl(dr[kr], k + 16 * kg, 64), pi = __shfl(di[kr], k + 16 * kg, 64);
        const int src = c + 16 * kg;
        const double rr = __shfl(dr[kr], src, 64), ri = __shfl(di[kr], src, 64);
        const double er = __shfl(xr[kr], src, 64), ei = __shfl(xi[kr], src, 64);
        double mr[4], mi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            mr[r] = __shfl(dr[r], k + 16 * g, 64);
            mi[r] = __shfl(di[r], k + 16 * g, 64);
        }
        if (pr == 0.0 && pi == 0.0) singular = true;
        const cd inv = crecip_smith(grape::cmake(pr, pi));
        const cd rs = grape::cmulf(grape::cmake(rr, ri), inv);
        const cd es = grape::cmulf(grape::cmake(er, ei), inv);
        const bool prow = g == kg;
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // a -= m * (scaled pivot row); the pivot row becomes it
            const bool piv = prow && (r == kr);
            const double nr = fma(-mr[r], rs.re, fma(mi[r], rs.im, dr[r]));
            const double ni = fma(-mr[r], rs.im, fma(-mi[r], rs.re, di[r]));
            const double nxr = fma(-mr[r], es.re, fma(mi[r], es.im, xr[r]));
            const double nxi = fma(-mr[r], es.im, fma(-mi[r], es.re, xi[r]));
            dr[r] = piv ? rs.re : nr;
            di[r] = piv ? rs.im : ni;
            xr[r] = piv ? es.re : nxr;
            xi[r] = piv ? es.im : nxi;
        }
        // one step at a time: keeps the compiler from overlapping steps (register blow-up)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(dr[r]), "+v"(di[r]), "+v"(xr[r]), "+v"(xi[r]));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        Dr[r] = dr[r];
        Di[r] = di[r];
        Xr[r] = xr[r];
        Xi[r] = xi[r];
    }
}

// (aR + i aI)(bR + i bI) accumulated into (cr, ci)
__device__ __forceinline__ void cmfma1(v4d &cr, v4d &ci, double aR, double aI, double bR, double bI) {
    cr = mfma(aR, bR, cr);
    ci = mfma(aR, bI, ci);
    cr = mfma(aI, -bI, cr);
    ci = mfma(aI, bR, ci);
}

// ---------------------------------------------------------------------------
// Solve Q X = Pm in place (X returned in Pm): blocked Gauss-Jordan on MFMA.
// Block step kb (buffers in LDS set kb & 1):
//   1. waves (kb, *) publish -Q[:, block kb] (the multipliers); D_kb^-1 is
//      already in the set (look-ahead, below);
//   2. waves holding row block kb replace it by D^-1 (row block) and publish it;
//   3. every wave subtracts Q[t-block, kb-block] (new row block) from its tiles.
//      Look-ahead: the wave that owns the NEXT diagonal block updates its tiles
//      first and then inverts that block into the next set while the other
//      seven waves are still in their rank-16 updates, so the serial 16-step
//      inversion no longer idles the workgroup (only D_0 is inverted up front).
// Q's column blocks left of or at kb are never read again: skipped (w <= kb).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void gj_store_dinv(double *set, const v4d &xr, const v4d &xi, int l) {
    double *dvr = set + GJ_DINV, *dvi = dvr + SMALL;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int o = sidx16((l >> 4) + 4 * r, l & 15);
        dvr[o] = xr[r];
        dvi[o] = xi[r];
    }
}

__device__ __forceinline__ void gj_solve(HM &Q, HM &Pm, double *lds, const Lane &ln_in, bool &singular) {
    __syncthreads();  // the matrix regions are free
    {  // D_0^-1 into set 0
        const Lane ln = pinned(ln_in);
        if (ln.w == 0 && ln.h == 0) {
            v4d dr = Q.re[0], di = Q.im[0], xr, xi;
            wave_inv16(dr, di, xr, xi, ln.l, singular);
            gj_store_dinv(lds + LDS_R0, xr, xi, ln.l);
        }
    }
#pragma unroll
    for (int kb = 0; kb < NT; ++kb) {
        const Lane ln = pinned(ln_in);
        double *set = lds + ((kb & 1) ? LDS_R1 : LDS_R0);
        double *nset = lds + ((kb & 1) ? LDS_R0 : LDS_R1);
        double *dvr = set + GJ_DINV, *dvi = dvr + SMALL;
        double *pcr = set + GJ_PCOL, *pci = pcr + 4 * SMALL;
        double *nr = set + GJ_NR;
        const int hk = kb >> 1, ik = kb & 1;
        const bool owner_row = ln.h == hk;  // holds row block kb of column block w (tile ik)
        if (ln.w == kb) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (ln.tile(i) == kb) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int o = sidx16(ln.row(i, r), ln.l & 15);
                    pcr[o] = -Q.re[i][r];
                    pci[o] = -Q.im[i][r];
                }
            }
        }
        __syncthreads();
        const bool doq = ln.w > kb;
        double *nq = nr + (ln.w * 2 + 0) * 2 * SMALL, *np = nr + (ln.w * 2 + 1) * 2 * SMALL;
        if (owner_row) {
            v4d nqr = {0, 0, 0, 0}, nqi = {0, 0, 0, 0}, npr = {0, 0, 0, 0}, npi = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int o = sidx16(ln.l & 15, 4 * s + (ln.l >> 4));
                const double aR = dvr[o], aI = dvi[o];
                cmfma1(npr, npi, aR, aI, Pm.re[ik][s], Pm.im[ik][s]);
                if (doq) cmfma1(nqr, nqi, aR, aI, Q.re[ik][s], Q.im[ik][s]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = ((ln.l >> 4) + 4 * r) * 16 + (ln.l & 15);
                np[o] = npr[r];
                np[SMALL + o] = npi[r];
                if (doq) {
                    nq[o] = nqr[r];
                    nq[SMALL + o] = nqi[r];
                }
            }
            Pm.re[ik] = npr;
            Pm.im[ik] = npi;
            if (doq) {
                Q.re[ik] = nqr;
                Q.im[ik] = nqi;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = ln.tile(i);
            if (t == kb) continue;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int oa = sidx16(16 * t + (ln.l & 15), 4 * s + (ln.l >> 4));
                const int ob = (4 * s + (ln.l >> 4)) * 16 + (ln.l & 15);
                const double aR = pcr[oa], aI = pci[oa];
                cmfma1(Pm.re[i], Pm.im[i], aR, aI, np[ob], np[SMALL + ob]);
                if (doq) cmfma1(Q.re[i], Q.im[i], aR, aI, nq[ob], nq[SMALL + ob]);
            }
        }
        // look-ahead: the owner of diagonal block kb+1 (updated just above) inverts it
        if (kb + 1 < NT && ln.w == kb + 1 && ln.h == ((kb + 1) >> 1)) {
            const int in = (kb + 1) & 1;
            v4d dr = Q.re[in], di = Q.im[in], xr, xi;
            wave_inv16(dr, di, xr, xi, ln.l, singular);
            gj_store_dinv(nset, xr, xi, ln.l);
        }
        __syncthreads();  // next set's D^-1 visible; this set's buffers free
    }
}

// ---------------------------------------------------------------------------
// Pade tables (Julia LinearAlgebra.exp!) and the degree choice
// ---------------------------------------------------------------------------
__constant__ const double kDPade[5][14] = {
    {120.0, 60.0, 12.0, 1.0},
    {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0},
    {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0},
    {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0, 2162160.0, 110880.0, 3960.0, 90.0, 1.0},
    {64764752532480000.0, 32382376266240000.0, 7771770303897600.0, 1187353796428800.0, 129060195264000.0,
     10559470521600.0, 670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0, 16380.0, 182.0, 1.0}};

// Julia's (m, s) for |A|_1, with the Pade-13 scaling raised until |A/2^s|_1 <= 1.6
// (keeps Re q(i theta) > 0 with margin: no-interchange solve, see the header)
__device__ __forceinline__ int dense_pade_degree(double nA, int &s) {
    s = 0;
    if (nA <= 2.1) {
        if (nA > 0.95) return 9;
        if (nA > 0.25) return 7;
        if (nA > 0.015) return 5;
        return 3;
    }
    const double l = log2(nA / 5.4);
    if (l > 0.0) s = (int)ceil(l);
    const double l2 = log2(nA / 1.6);
    const int s2 = l2 > 0.0 ? (int)ceil(l2) : 0;
    if (s2 > s) s = s2;
    return 13;
}

__device__ __forceinline__ int m_index(int m) { return m == 3 ? 0 : m == 5 ? 1 : m == 7 ? 2 : m == 9 ? 3 : 4; }

// keeps the compiler from hoisting work across a phase boundary (register pressure)
__device__ __forceinline__ void hm_pin(HM &M) {
#pragma unroll
    for (int i = 0; i < 2; ++i) asm volatile("" : "+v"(M.re[i]), "+v"(M.im[i]));
}

// ---------------------------------------------------------------------------
// X = exp(A) for the workgroup's matrix A.  `build(HM&)` (re)constructs A: it is
// called twice (at the start and for the final U = A U), so A is never live
// through the Pade polynomial (register budget: 256 VGPRs at 2 waves/SIMD).
// Uses all of LDS [0, LDS_TOTAL).  Returns the Pade degree m.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Solve-free regime (Julia's Pade 3 / 5 / 7, |A|_1 <= 0.95): the Taylor polynomial of the same
// accuracy, degree 12 (|A|_1 <= 0.25: remainder |A|^13/13! <= 2.4e-18) or 18 (|A|_1 <= 0.95:
// |A|^19/19! <= 3.1e-18), by Paterson-Stockmeyer in A^4:
//   T = B0 + A4 (B1 + A4 (B2 [+ A4 (B3 + A4 B4)])),  B_j = sum_{i<4} c_{4j+i} A^i  (top block
//   also + c_{4J} A4 for degree 12, c16 I + c17 A + c18 A^2 for degree 18).
// Products: A^2, A^3, A^4 and 2 (degree 12) or 4 (degree 18) Horner steps, all MFMA streams --
// no Gauss-Jordan solve, whose serial 16 x 16 block inversions left the MFMA pipe idle for
// about as long as the Pade products took.  Agrees with exp! to a few u (inside T0).
// ---------------------------------------------------------------------------
__constant__ const double kDInvFact[21] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720, 1.0 / 5040,
                                           1.0 / 40320, 1.0 / 362880, 1.0 / 3628800, 1.0 / 39916800,
                                           1.0 / 479001600, 1.0 / 6227020800.0, 1.0 / 87178291200.0,
                                           1.0 / 1307674368000.0, 1.0 / 20922789888000.0,
                                           1.0 / 355687428096000.0, 1.0 / 6402373705728000.0,
                                           1.0 / 121645100408832000.0, 1.0 / 2432902008176640000.0};

// x = c0 I + c1 A + c2 A2 + c3 A3 (+ c4 A4) for coefficients kDInvFact[b..]
__device__ __forceinline__ void taylor_block(HM &x, int b, int n, const HM &A, const HM &A2, const HM &A3,
                                             const HM *A4, const Lane &ln) {
    hm_identity(x, ln, kDInvFact[b]);
    if (n > 1) hm_axpy(x, kDInvFact[b + 1], A);
    if (n > 2) hm_axpy(x, kDInvFact[b + 2], A2);
    if (n > 3) hm_axpy(x, kDInvFact[b + 3], A3);
    if (n > 4 && A4) hm_axpy(x, kDInvFact[b + 4], *A4);
}

// The Taylor degree for |A|_1 <= 0.95.  Paterson-Stockmeyer in A^4 costs 4 / 5 / 6 / 7 products at
// degree 8 / 12 / 16 / 20 (degree 18 costs 7 as well).  GRAPE_DENSE_TAYLOR_U (default): the lowest of
// them whose remainder bound |A|^(m+1) / (m+1)! is at most u = 2^-53, the accuracy Julia's theta_m
// give its Pade degrees:  m = 8: |A|_1 <= 0.069,  12: <= 0.335,  16: <= 0.826,  20: <= 0.95 (bound
// 6e-5 u there).  At C5 (|A|_1 in 0.49 .. 0.88) 98 % of the steps take degree 16.
// GRAPE_DENSE_TAYLOR_U 0, GRAPE_DENSE_TAYLOR16 1: the bound of degree 18 at 0.95 (3.1e-18) for every
// degree -- 8 <= 0.047, 12 <= 0.25, 16 <= 0.668, 18 above (64 % of C5's steps at degree 16).  Both 0:
// round 2's 12 up to 0.25 and 18 above.
#ifndef GRAPE_DENSE_TAYLOR16
#define GRAPE_DENSE_TAYLOR16 1
#endif
#ifndef GRAPE_DENSE_TAYLOR_U
#define GRAPE_DENSE_TAYLOR_U 1
#endif
__device__ __forceinline__ int taylor_degree(double nA) {
    if (GRAPE_DENSE_TAYLOR_U) {
        if (nA <= 0.069) return 8;
        if (nA <= 0.335) return 12;
        if (nA <= 0.826) return 16;
        return 20;
    }
    if (GRAPE_DENSE_TAYLOR16 && nA <= 0.047) return 8;
    if (nA <= 0.25) return 12;
    if (GRAPE_DENSE_TAYLOR16 && nA <= 0.668) return 16;
    return 18;
}

// A is in S0 and in registers; returns X = T(A).  Uses both LDS regions.
__device__ __forceinline__ void wg_expm_taylor(const HM &A, int degree, HM &X, double *lds, const Lane &ln) {
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    HM A2, A3;
    hm_zero(A2);
    mm<false, false, false, false>(S0, S0, A2, ln);  // A^2
    __syncthreads();
    sm_store(S1, A2, ln);
    __syncthreads();
    hm_zero(A3);
    mm<false, false, false, false>(S0, S1, A3, ln);  // A . A^2
    {
        HM A4;
        hm_zero(A4);
        mm<false, false, false, false>(S1, S1, A4, ln);  // A^2 . A^2
        __syncthreads();
        sm_store(S0, A4, ln);  // the Horner left operand from here on
        if (degree == 18) taylor_block(X, 16, 3, A, A2, A3, nullptr, ln);  // c16..c18
        else taylor_block(X, degree - 4, 5, A, A2, A3, &A4, ln);           // c_{m-4}..c_m, m = 8 .. 20
        hm_pin(X);
    }
    const int top = degree == 18 ? 3 : degree / 4 - 2;  // blocks B_top .. B_0 below the initial one
    for (int j = top; j >= 0; --j) {
        __syncthreads();  // S1's previous contents consumed
        sm_store(S1, X, ln);
        __syncthreads();
        HM P;
        hm_zero(P);
        mm<false, false, false, false>(S0, S1, P, ln);  // A^4 . x
        taylor_block(X, 4 * j, 4, A, A2, A3, nullptr, ln);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            X.re[i] += P.re[i];
            X.im[i] += P.im[i];
        }
        hm_pin(X);
    }
    __syncthreads();  // every wave done with the LDS regions
}

template <class Build>
__device__ __forceinline__ int wg_expm(const Build &build, HM &X, double *lds, const Lane &ln, bool &singular) {
    SM S0 = sm_at(lds, LDS_R0), S1 = sm_at(lds, LDS_R1);
    int s = 0, m;
    HM U, V;
    {
        HM A;
        build(A);
        const double nA = wg_norm1(A, lds, ln);
        m = dense_pade_degree(nA, s);
        if (s > 0) hm_scale(A, ldexp(1.0, -s));
        __syncthreads();
        sm_store(S0, A, ln);
        __syncthreads();
        if (m <= 7) {  // Julia's Pade 3 / 5 / 7 regime: solve-free Taylor (above)
            wg_expm_taylor(A, taylor_degree(nA), X, lds, ln);
            return m;
        }
    }
    const double *C = kDPade[m_index(m)];
    if (m <= 9) {
        // exp!: A2 = A*A; P = I; U = c1 P; V = c0 P; repeat P *= A2; U += c_{2k+1} P;
        // V += c_{2k} P; U = A*U
        {
            HM A2;
            hm_zero(A2);
            mm<false, false, false, false>(S0, S0, A2, ln);
            hm_identity(U, ln, C[1]);
            hm_identity(V, ln, C[0]);
            hm_axpy(U, C[3], A2);
            hm_axpy(V, C[2], A2);
            __syncthreads();
            sm_store(S0, A2, ln);  // L = A2 for every further power
            __syncthreads();
        }
        const int nk = (m + 1) / 2;
        if (nk > 2) {
            HM P;
            hm_zero(P);
            mm<false, false, false, false>(S0, S0, P, ln);  // A4
            hm_axpy(U, C[5], P);
            hm_axpy(V, C[4], P);
            for (int kk = 3; kk < nk; ++kk) {
                __syncthreads();
                sm_store(S1, P, ln);
                __syncthreads();
                hm_zero(P);
                mm<false, false, false, false>(S0, S1, P, ln);  // A2 . P
                hm_axpy(U, C[2 * kk + 1], P);
                hm_axpy(V, C[2 * kk], P);
                hm_pin(U);
                hm_pin(V);
            }
        }
    } else {
        // exp! Pade 13: U = A (A6 (c13 A6 + c11 A4 + c9 A2) + c7 A6 + c5 A4 + c3 A2 + c1 I),
        //               V = A6 (c12 A6 + c10 A4 + c8 A2) + c6 A6 + c4 A4 + c2 A2 + c0 I
        // A2 and A4 live in LDS once consumed; W1 and Z1 are formed only after A6
        // exists (A2, A4 read back from LDS), so no product ever runs with more
        // than U, V and its accumulator live.
        {
            HM A2;
            hm_zero(A2);
            mm<false, false, false, false>(S0, S0, A2, ln);
            hm_identity(U, ln, C[1]);
            hm_identity(V, ln, C[0]);
            hm_axpy(U, C[3], A2);
            hm_axpy(V, C[2], A2);
            __syncthreads();
            sm_store(S0, A2, ln);
            __syncthreads();
        }
        {
            HM A4;
            hm_zero(A4);
            mm<false, false, false, false>(S0, S0, A4, ln);
            hm_axpy(U, C[5], A4);
            hm_axpy(V, C[4], A4);
            sm_store(S1, A4, ln);  // region 1 unused so far
            __syncthreads();
        }
        hm_pin(U);
        hm_pin(V);
        HM A6, W1, Z1;
        hm_zero(A6);
        mm<false, false, false, false>(S0, S1, A6, ln);  // A2 . A4
        hm_axpy(U, C[7], A6);
        hm_axpy(V, C[6], A6);
        {
            HM A2, A4;
            sm_load(S0, A2, ln);
            sm_load(S1, A4, ln);
            hm_zero(W1);
            hm_zero(Z1);
            hm_axpy(W1, C[13], A6);  // exp!'s order: c13 A6 + c11 A4 + c9 A2
            hm_axpy(W1, C[11], A4);
            hm_axpy(W1, C[9], A2);
            hm_axpy(Z1, C[12], A6);
            hm_axpy(Z1, C[10], A4);
            hm_axpy(Z1, C[8], A2);
        }
        __syncthreads();
        sm_store(S0, A6, ln);
        sm_store(S1, W1, ln);
        __syncthreads();
        hm_pin(Z1);
        mm<false, false, false, false>(S0, S1, U, ln);  // U += A6 W1
        __syncthreads();
        sm_store(S1, Z1, ln);
        __syncthreads();
        mm<false, false, false, false>(S0, S1, V, ln);  // V += A6 Z1
    }
    hm_pin(U);
    hm_pin(V);
    __syncthreads();
    sm_store(S1, U, ln);
    {
        HM A;
        build(A);
        if (s > 0) hm_scale(A, ldexp(1.0, -s));
        sm_store(S0, A, ln);
    }
    __syncthreads();
    hm_zero(U);
    mm<false, false, false, false>(S0, S1, U, ln);  // U = A U
    // Q = V - U, X = V + U: solve Q X' = X
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const v4d ur = U.re[i], ui = U.im[i], vr = V.re[i], vi = V.im[i];
        U.re[i] = vr - ur;
        U.im[i] = vi - ui;
        V.re[i] = vr + ur;
        V.im[i] = vi + ui;
    }
    gj_solve(U, V, lds, ln, singular);
    for (int q = 0; q < s; ++q) {
        sm_store(S0, V, ln);
        __syncthreads();
        hm_zero(V);
        mm<false, false, false, false>(S0, S0, V, ln);
        __syncthreads();
    }
    X = V;
    return m;
}

}  // namespace grape_dense
