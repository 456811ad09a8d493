// grape_symmetry.hpp -- symmetry-adapted sectors: the finest block decomposition of the operator
// algebra (host code, plan creation only).
//
// The sector engine (grape_engine.hip find_sectors) splits the levels into the connected components
// of the operators' union sparsity pattern: a PERMUTATION of the basis.  A symmetry can split a
// component further in a rotated basis.  In rydberg_hamiltonian_full with equal Rabi frequencies and
// detunings (the BASELINE C2 configuration, RydbergTools.jl:118-130) the atom-swap symmetry splits
// the 4-level component {11, 1r, r1, rr} into {11, (1r + r1)/sqrt2, rr} and the dark state
// (1r - r1)/sqrt2, which no operator touches: one 3-level sector instead of a 4-level one (27 instead
// of 64 complex MACs per product).
//
// General algorithm, for any set of Hermitian operators {H_j} (every operator H0 and the error
// sources use; the propagators exp(-i dt sum g_j H_j) lie in the algebra they generate):
//   1. per connected component C of the sparsity pattern, the commutant
//        A' = { X : H_j X = X H_j for all j }
//      as the null space of the stacked linear maps X -> H_j X - X H_j (complex Gauss-Jordan with
//      complete pivoting); dim A' = 1 means C is irreducible: no split;
//   2. a generic Hermitian element Z = R + R^dag of A' (R a fixed pseudo-random combination of the
//      null vectors): its eigenspaces are invariant under every H_j (H_j Z v = Z H_j v), and for a
//      generic Z they are the minimal invariant subspaces (complex Jacobi eigen-decomposition,
//      eigenvalues clustered);
//   3. in each invariant subspace, the basis closest to the standard one: pivoted Gram-Schmidt of
//      the projections of the unit vectors e_i (largest remaining norm first), so a level that lies
//      in the subspace keeps its unit vector exactly (11 and rr above) and the rotated target and
//      projector stay diagonal wherever the symmetry does not mix levels of different weight.
// The result V (unitary, d x d) is checked: V^dag V = I and V^dag H_j V block-diagonal to 1e-12 of
// |H_j|; otherwise that component keeps its levels.  Every output of the fidelity path
// (F, F_dx, F_d2err, F_d2err_dx) is a trace expression invariant under the simultaneous similarity
// U -> V^dag U V, U0 -> V^dag U0 V, P0 -> V^dag P0 V, P -> V^dag P V (FidelityCalculations.jl:47-117),
// and the finite differences are linear in the propagators, so the engine may run the sector path
// in the rotated basis (grape_plan_create) with the same outputs to rounding.
#pragma once
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <vector>

namespace grape_sym {

using cplx = std::complex<double>;

struct Split {
    bool rotated = false;   // some component splits further than its sparsity pattern
    int d = 0;
    std::vector<cplx> V;    // d x d column-major, unitary: column j = basis vector j
    std::vector<int> block; // invariant-subspace id of each column
};

// column-major complex d x d from grape_desc's interleaved column-major doubles
inline std::vector<cplx> load_op(const double *src, int d) {
    std::vector<cplx> m((size_t)d * d);
    for (size_t t = 0; t < m.size(); ++t) m[t] = cplx(src[2 * t], src[2 * t + 1]);
    return m;
}

// null space of the m x n complex matrix M (row-major), complete pivoting; columns of the
// returned n x k matrix (column-major) span it
inline std::vector<cplx> null_space(std::vector<cplx> M, int m, int n, int &k) {
    std::vector<int> colp(n);
    for (int j = 0; j < n; ++j) colp[j] = j;
    double amax = 0.0;
    for (const cplx &v : M) amax = std::max(amax, std::abs(v));
    const double tol = 1e-11 * std::max(amax, 1e-300);
    int r = 0;
    for (; r < std::min(m, n); ++r) {
        int pi = -1, pj = -1;
        double best = tol;
        for (int i = r; i < m; ++i)
            for (int j = r; j < n; ++j) {
                const double a = std::abs(M[(size_t)i * n + j]);
                if (a > best) best = a, pi = i, pj = j;
            }
        if (pi < 0) break;
        if (pi != r)
            for (int j = 0; j < n; ++j) std::swap(M[(size_t)pi * n + j], M[(size_t)r * n + j]);
        if (pj != r) {
            for (int i = 0; i < m; ++i) std::swap(M[(size_t)i * n + pj], M[(size_t)i * n + r]);
            std::swap(colp[pj], colp[r]);
        }
        const cplx inv = 1.0 / M[(size_t)r * n + r];
        for (int j = r; j < n; ++j) M[(size_t)r * n + j] *= inv;
        for (int i = 0; i < m; ++i) {  // Gauss-Jordan: clear the column above and below
            if (i == r) continue;
            const cplx f = M[(size_t)i * n + r];
            if (f == cplx(0.0, 0.0)) continue;
            for (int j = r; j < n; ++j) M[(size_t)i * n + j] -= f * M[(size_t)r * n + j];
        }
    }
    k = n - r;
    std::vector<cplx> N((size_t)n * k, cplx(0.0, 0.0));
    for (int f = 0; f < k; ++f) {  // free variable colp[r + f] = 1, pivots from the reduced rows
        N[(size_t)f * n + colp[r + f]] = 1.0;
        for (int i = 0; i < r; ++i) N[(size_t)f * n + colp[i]] = -M[(size_t)i * n + r + f];
    }
    return N;
}

// eigen-decomposition of a Hermitian n x n matrix (column-major, overwritten): cyclic complex
// Jacobi; eigenvalues in w, eigenvectors in the columns of U
inline void jacobi_herm(std::vector<cplx> A, int n, std::vector<double> &w, std::vector<cplx> &U) {
    U.assign((size_t)n * n, cplx(0.0, 0.0));
    for (int i = 0; i < n; ++i) U[(size_t)i * n + i] = 1.0;
    auto at = [&](int i, int j) -> cplx & { return A[(size_t)j * n + i]; };
    double fro = 0.0;
    for (const cplx &v : A) fro += std::norm(v);
    fro = std::sqrt(fro);
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += std::norm(at(p, q));
        if (std::sqrt(off) <= 1e-16 * std::max(fro, 1e-300)) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const cplx apq = at(p, q);
                const double g = std::abs(apq);
                if (g <= 1e-300) continue;
                const cplx e = apq / g;  // e^{i phi}
                const double app = at(p, p).real(), aqq = at(q, q).real();
                const double tau = (aqq - app) / (2.0 * g);
                const double t = (tau >= 0 ? 1.0 : -1.0) / (std::abs(tau) + std::sqrt(1.0 + tau * tau));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = t * c;
                // J = diag(1, e^{-i phi}) [[c, s], [-s, c]] on (p, q): J_pp = c, J_pq = s,
                // J_qp = -s e*, J_qq = c e*
                const cplx jpp = c, jpq = s, jqp = -s * std::conj(e), jqq = c * std::conj(e);
                for (int r = 0; r < n; ++r) {  // A <- A J, U <- U J
                    const cplx arp = at(r, p), arq = at(r, q);
                    at(r, p) = arp * jpp + arq * jqp;
                    at(r, q) = arp * jpq + arq * jqq;
                    const cplx urp = U[(size_t)p * n + r], urq = U[(size_t)q * n + r];
                    U[(size_t)p * n + r] = urp * jpp + urq * jqp;
                    U[(size_t)q * n + r] = urp * jpq + urq * jqq;
                }
                for (int r = 0; r < n; ++r) {  // A <- J^dag A
                    const cplx apr = at(p, r), aqr = at(q, r);
                    at(p, r) = std::conj(jpp) * apr + std::conj(jqp) * aqr;
                    at(q, r) = std::conj(jpq) * apr + std::conj(jqq) * aqr;
                }
                at(p, q) = at(q, p) = 0.0;
                at(p, p) = at(p, p).real();
                at(q, q) = at(q, q).real();
            }
    }
    w.resize(n);
    for (int i = 0; i < n; ++i) w[i] = at(i, i).real();
}

// The split of one component: levels `lv` (ascending), restricted operators ops (each c x c
// column-major).  Returns false (keep the levels) when the component is irreducible or the
// checks fail; else the component's new basis vectors (c x c, column-major, in component
// coordinates) and their subspace ids.
inline bool split_component(const std::vector<std::vector<cplx>> &ops, int c, std::vector<cplx> &B,
                            std::vector<int> &blk) {
    const int n = c * c, m = (int)ops.size() * n;
    std::vector<cplx> M((size_t)m * n, cplx(0.0, 0.0));
    // row (o, i, j) of H_o X - X H_o; unknown X_ab at column a + b c
    for (size_t o = 0; o < ops.size(); ++o) {
        const std::vector<cplx> &H = ops[o];
        for (int j = 0; j < c; ++j)
            for (int i = 0; i < c; ++i) {
                const size_t row = (o * n + (size_t)i + (size_t)j * c) * n;
                for (int q = 0; q < c; ++q) {
                    M[row + q + (size_t)j * c] += H[(size_t)q * c + i];  // H_iq X_qj
                    M[row + i + (size_t)q * c] -= H[(size_t)j * c + q];  // X_iq H_qj
                }
            }
    }
    int k = 0;
    const std::vector<cplx> N = null_space(M, m, n, k);
    if (k <= 1) return false;
    // generic Hermitian element of the commutant (fixed pseudo-random coefficients: deterministic plans)
    std::vector<cplx> R((size_t)n, cplx(0.0, 0.0));
    uint64_t st = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(st >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    };
    for (int f = 0; f < k; ++f) {
        const cplx a(rnd(), rnd());
        for (int t = 0; t < n; ++t) R[t] += a * N[(size_t)f * n + t];
    }
    std::vector<cplx> Z((size_t)n);
    double zmax = 0.0;
    for (int j = 0; j < c; ++j)
        for (int i = 0; i < c; ++i) {
            Z[(size_t)j * c + i] = R[(size_t)j * c + i] + std::conj(R[(size_t)i * c + j]);
            zmax = std::max(zmax, std::abs(Z[(size_t)j * c + i]));
        }
    if (zmax <= 0.0) return false;
    for (cplx &v : Z) v /= zmax;
    std::vector<double> w;
    std::vector<cplx> U;
    jacobi_herm(Z, c, w, U);
    std::vector<int> ord(c);
    for (int i = 0; i < c; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] < w[b]; });
    std::vector<std::vector<int>> clusters;
    for (int t = 0; t < c; ++t) {
        if (t == 0 || w[ord[t]] - w[ord[t - 1]] > 1e-7) clusters.emplace_back();
        clusters.back().push_back(ord[t]);
    }
    if (clusters.size() < 2) return false;
    // per invariant subspace: pivoted Gram-Schmidt of the projected unit vectors
    B.assign((size_t)c * c, cplx(0.0, 0.0));
    blk.assign(c, -1);
    int col = 0;
    for (size_t id = 0; id < clusters.size(); ++id) {
        const std::vector<int> &cl = clusters[id];
        std::vector<cplx> Pj((size_t)c * c, cplx(0.0, 0.0));  // projector onto the subspace
        for (int e : cl)
            for (int j = 0; j < c; ++j)
                for (int i = 0; i < c; ++i) Pj[(size_t)j * c + i] += U[(size_t)e * c + i] * std::conj(U[(size_t)e * c + j]);
        std::vector<std::vector<cplx>> cand(c);  // P e_i, deflated by the chosen vectors
        for (int i = 0; i < c; ++i) cand[i].assign(Pj.begin() + (size_t)i * c, Pj.begin() + (size_t)(i + 1) * c);
        std::vector<char> used(c, 0);
        for (size_t t = 0; t < cl.size(); ++t) {
            int bi = -1;
            double bn = 0.0;
            for (int i = 0; i < c; ++i) {
                if (used[i]) continue;
                double nn = 0.0;
                for (const cplx &v : cand[i]) nn += std::norm(v);
                if (nn > bn + 1e-12) bn = nn, bi = i;
            }
            if (bi < 0 || bn < 1e-6) return false;
            used[bi] = 1;
            std::vector<cplx> v = cand[bi];
            const double inv = 1.0 / std::sqrt(bn);
            int big = 0;
            for (int i = 0; i < c; ++i) {
                v[i] *= inv;
                if (std::abs(v[i]) > std::abs(v[big]) + 1e-14) big = i;
            }
            const cplx ph = std::abs(v[big]) > 0 ? std::conj(v[big]) / std::abs(v[big]) : cplx(1.0, 0.0);
            for (int i = 0; i < c; ++i) {  // largest entry real positive; rounding residue snapped to 0
                v[i] *= ph;
                if (std::abs(v[i].real()) < 1e-15) v[i].real(0.0);
                if (std::abs(v[i].imag()) < 1e-15) v[i].imag(0.0);
            }
            for (int i = 0; i < c; ++i) {  // deflate the remaining candidates
                if (used[i]) continue;
                cplx dot = 0.0;
                for (int r = 0; r < c; ++r) dot += std::conj(v[r]) * cand[i][r];
                for (int r = 0; r < c; ++r) cand[i][r] -= dot * v[r];
            }
            for (int r = 0; r < c; ++r) B[(size_t)col * c + r] = v[r];
            blk[col++] = (int)id;
        }
    }
    // checks: orthonormal, and every operator block-diagonal in the new basis
    for (int a = 0; a < c; ++a)
        for (int b = 0; b < c; ++b) {
            cplx s = 0.0;
            for (int r = 0; r < c; ++r) s += std::conj(B[(size_t)a * c + r]) * B[(size_t)b * c + r];
            if (std::abs(s - (a == b ? 1.0 : 0.0)) > 1e-12) return false;
        }
    for (const std::vector<cplx> &H : ops) {
        double hmax = 0.0;
        for (const cplx &v : H) hmax = std::max(hmax, std::abs(v));
        for (int a = 0; a < c; ++a)
            for (int b = 0; b < c; ++b) {
                if (blk[a] == blk[b]) continue;
                cplx s = 0.0;
                for (int r = 0; r < c; ++r)
                    for (int q = 0; q < c; ++q)
                        s += std::conj(B[(size_t)a * c + r]) * H[(size_t)q * c + r] * B[(size_t)b * c + q];
                if (std::abs(s) > 1e-12 * std::max(hmax, 1e-300)) return false;
            }
    }
    return true;
}

// The symmetry-adapted basis of d x d operators `ops` (grape_desc layout).  Components of the
// sparsity pattern that do not split keep their unit vectors (V is the identity there).
inline Split symmetry_split(int d, const std::vector<const double *> &ops) {
    Split s;
    s.d = d;
    s.V.assign((size_t)d * d, cplx(0.0, 0.0));
    s.block.assign(d, -1);
    for (int i = 0; i < d; ++i) s.V[(size_t)i * d + i] = 1.0;
    std::vector<int> parent(d);
    for (int i = 0; i < d; ++i) parent[i] = i;
    auto root = [&](int i) {
        while (parent[i] != i) i = parent[i] = parent[parent[i]];
        return i;
    };
    std::vector<std::vector<cplx>> full;
    for (const double *o : ops) full.push_back(load_op(o, d));
    for (const auto &H : full)
        for (int c = 0; c < d; ++c)
            for (int r = 0; r < d; ++r)
                if (H[(size_t)c * d + r] != cplx(0.0, 0.0)) parent[root(r)] = root(c);
    std::vector<std::vector<int>> comps;
    std::vector<int> slot(d, -1);
    for (int i = 0; i < d; ++i) {
        const int r = root(i);
        if (slot[r] < 0) {
            slot[r] = (int)comps.size();
            comps.emplace_back();
        }
        comps[slot[r]].push_back(i);
    }
    int next_block = 0;
    for (const std::vector<int> &lv : comps) {
        const int c = (int)lv.size();
        std::vector<cplx> B;
        std::vector<int> blk;
        bool split = false;
        if (c >= 2) {
            std::vector<std::vector<cplx>> sub;
            for (const auto &H : full) {
                std::vector<cplx> h((size_t)c * c);
                for (int b = 0; b < c; ++b)
                    for (int a = 0; a < c; ++a) h[(size_t)b * c + a] = H[(size_t)lv[b] * d + lv[a]];
                sub.push_back(std::move(h));
            }
            split = split_component(sub, c, B, blk);
        }
        if (!split) {
            for (int i : lv) s.block[i] = next_block;
            ++next_block;
            continue;
        }
        s.rotated = true;
        int nb = 0;
        for (int b : blk) nb = std::max(nb, b + 1);
        // the component's columns are its level indices: a new vector that IS a unit vector e_lv[r]
        // keeps column lv[r] (V stays the identity there), the others fill the remaining columns
        std::vector<int> colof(c, -1);
        std::vector<char> taken(c, 0);
        for (int t = 0; t < c; ++t) {
            int nz = 0, at = -1;
            for (int r = 0; r < c; ++r)
                if (B[(size_t)t * c + r] != cplx(0.0, 0.0)) ++nz, at = r;
            if (nz == 1 && B[(size_t)t * c + at] == cplx(1.0, 0.0) && !taken[at]) colof[t] = at, taken[at] = 1;
        }
        for (int t = 0, f = 0; t < c; ++t) {
            if (colof[t] >= 0) continue;
            while (taken[f]) ++f;
            colof[t] = f;
            taken[f] = 1;
        }
        for (int t = 0; t < c; ++t) {
            const int col = lv[colof[t]];
            for (int i = 0; i < d; ++i) s.V[(size_t)col * d + i] = 0.0;
            for (int r = 0; r < c; ++r) s.V[(size_t)col * d + lv[r]] = B[(size_t)t * c + r];
            s.block[col] = next_block + blk[t];
        }
        next_block += nb;
    }
    return s;
}

// out = V^dag A V (grape_desc layout: column-major interleaved doubles, in and out)
inline void rotate(const Split &s, const double *A, double *out) {
    const int d = s.d;
    const std::vector<cplx> a = load_op(A, d);
    std::vector<cplx> t((size_t)d * d, cplx(0.0, 0.0));  // A V
    for (int j = 0; j < d; ++j)
        for (int q = 0; q < d; ++q) {
            const cplx v = s.V[(size_t)j * d + q];
            if (v == cplx(0.0, 0.0)) continue;
            for (int i = 0; i < d; ++i) t[(size_t)j * d + i] += a[(size_t)q * d + i] * v;
        }
    for (int j = 0; j < d; ++j)
        for (int i = 0; i < d; ++i) {
            cplx acc = 0.0;
            for (int q = 0; q < d; ++q) {
                const cplx v = s.V[(size_t)i * d + q];
                if (v != cplx(0.0, 0.0)) acc += std::conj(v) * t[(size_t)j * d + q];
            }
            out[2 * ((size_t)j * d + i)] = acc.real();
            out[2 * ((size_t)j * d + i) + 1] = acc.imag();
        }
}

}  // namespace grape_sym
