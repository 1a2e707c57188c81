// Dominant right singular vector of a k x 3 matrix, following the path LAPACK's
// dgesdd takes for it. The reference calls np.linalg.svd(full_matrices=False) on
// the fp32 centred neighbourhoods (models/model_partseg.py:36-37); numpy's linalg
// upcasts fp32 to fp64, runs dgesdd (jobz 'S') and rounds the results back to
// fp32, so this restatement computes in double:
//   k >= 5 (dgesdd "path 3", M >> N):  A = Q R          (dgeqr2: Householder)
//   R (3 x 3) = Q_B B P_B^T                              (dgebd2: upper bidiagonal)
//   B = U_B S V_B^T                                      (dbdsdc -> dlasdq -> dbdsqr)
//   V^T = V_B^T P_B^T                                    (dormbr 'P','R','T')
// The singular vectors' signs depend on every Householder and Givens choice, so
// each step restates the LAPACK routine's arithmetic: dlarfg's beta = -sign(alpha)
// |(alpha, x)|, the Givens of LAPACK 3.10+'s la_xlartg (c >= 0, r = sign(f) d),
// dlasv2's 2 x 2 SVD, dlas2's shift and dbdsqr's sweep/convergence logic. Stage
// outputs were checked one by one against the same routines of numpy's bundled
// OpenBLAS 0.3.29 (tools/svd3_check.py). Only k >= 5 is restated (k < 5 takes
// dgesdd's path 5, not used: the reference's k is 20..40).
// Plain C++ (host and device): the HOG kernel (hog.hip) calls it per point and
// tools/svd3_check.py runs the same code on the host against numpy.
#pragma once
#include <math.h>

#ifndef DGX_HD
#if defined(__HIPCC__)
#define DGX_HD __host__ __device__
#else
#define DGX_HD
#endif
#endif

namespace svd3 {

typedef double real;
constexpr real EPS = 1.1102230246251565e-16;     // dlamch('E') = 2^-53
constexpr real SAFMIN = 2.2250738585072014e-308;  // dlamch('S')

DGX_HD inline real sgn(real a, real b) { return b >= 0. ? fabs(a) : -fabs(a); }  // Fortran SIGN(a, b)

// dlapy2: sqrt(x^2 + y^2) without unnecessary overflow
DGX_HD inline real lapy2(real x, real y) {
    const real xa = fabs(x), ya = fabs(y);
    const real w = fmax(xa, ya), z = fmin(xa, ya);
    if (z == 0. || w > 1.7976931348623157e308) return w;
    const real q = z / w;
    return w * sqrt(1. + q * q);
}

// dlarfg on (alpha, x[0..n-2]) with stride: returns tau, overwrites alpha with
// beta and x with v(2:n)
DGX_HD inline real larfg(int n, real& alpha, real* x, int incx) {
    if (n <= 1) return 0.;
    real xnorm = 0.;
    {  // dnrm2 (scaled sum of squares)
        real scale = 0., ssq = 1.;
        for (int i = 0; i < n - 1; ++i) {
            const real v = x[i * incx];
            if (v != 0.) {
                const real a = fabs(v);
                if (scale < a) {
                    ssq = 1. + ssq * (scale / a) * (scale / a);
                    scale = a;
                } else {
                    ssq += (a / scale) * (a / scale);
                }
            }
        }
        xnorm = scale * sqrt(ssq);
    }
    if (xnorm == 0.) return 0.;
    real beta = -sgn(lapy2(alpha, xnorm), alpha);
    const real tau = (beta - alpha) / beta;
    const real s = 1. / (alpha - beta);
    for (int i = 0; i < n - 1; ++i) x[i * incx] *= s;
    alpha = beta;
    (void)SAFMIN;
    return tau;
}

// la_xlartg (LAPACK 3.10+): c = |f| / d, r = sign(f) d, s = g / r
DGX_HD inline void lartg(real f, real g, real& c, real& s, real& r) {
    if (g == 0.) {
        c = 1.;
        s = 0.;
        r = f;
    } else if (f == 0.) {
        c = 0.;
        s = sgn(1., g);
        r = fabs(g);
    } else {
        const real d = sqrt(f * f + g * g);
        c = fabs(f) / d;
        r = sgn(d, f);
        s = g / r;
    }
}

// dlas2: singular values of [f g; 0 h] (smaller in ssmin, larger in ssmax)
DGX_HD inline void las2(real f, real g, real h, real& ssmin, real& ssmax) {
    const real fa = fabs(f), ga = fabs(g), ha = fabs(h);
    const real fhmn = fmin(fa, ha), fhmx = fmax(fa, ha);
    if (fhmn == 0.) {
        ssmin = 0.;
        if (fhmx == 0.) {
            ssmax = ga;
        } else {
            const real mx = fmax(fhmx, ga), mn = fmin(fhmx, ga);
            ssmax = mx * sqrt(1. + (mn / mx) * (mn / mx));
        }
    } else if (ga < fhmx) {
        const real as = 1. + fhmn / fhmx;
        const real at = (fhmx - fhmn) / fhmx;
        const real au = (ga / fhmx) * (ga / fhmx);
        const real c = 2. / (sqrt(as * as + au) + sqrt(at * at + au));
        ssmin = fhmn * c;
        ssmax = fhmx / c;
    } else {
        const real au = fhmx / ga;
        if (au == 0.) {
            ssmin = (fhmn * fhmx) / ga;
            ssmax = ga;
        } else {
            const real as = 1. + fhmn / fhmx;
            const real at = (fhmx - fhmn) / fhmx;
            const real c = 1. / (sqrt(1. + (as * au) * (as * au)) + sqrt(1. + (at * au) * (at * au)));
            ssmin = (fhmn * c) * au;
            ssmin = ssmin + ssmin;
            ssmax = ga / (c + c);
        }
    }
}

// dlasv2: SVD of [f g; 0 h]: |ssmax| >= |ssmin|, with the rotations
// [csl snl; -snl csl] [f g; 0 h] [csr -snr; snr csr] = [ssmax 0; 0 ssmin]
DGX_HD inline void lasv2(real f, real g, real h, real& ssmin, real& ssmax, real& snr, real& csr,
                         real& snl, real& csl) {
    real ft = f, fa = fabs(ft), ht = h, ha = fabs(h);
    int pmax = 1;
    const bool swap = ha > fa;
    if (swap) {
        pmax = 3;
        real tmp = ft; ft = ht; ht = tmp;
        tmp = fa; fa = ha; ha = tmp;
    }
    const real gt = g, ga = fabs(gt);
    real clt, crt, slt, srt;
    if (ga == 0.) {
        ssmin = ha;
        ssmax = fa;
        clt = 1.; crt = 1.; slt = 0.; srt = 0.;
    } else {
        bool gasmal = true;
        if (ga > fa) {
            pmax = 2;
            if (fa / ga < EPS) {
                gasmal = false;
                ssmax = ga;
                if (ha > 1.) ssmin = fa / (ga / ha);
                else ssmin = (fa / ga) * ha;
                clt = 1.;
                slt = ht / gt;
                srt = 1.;
                crt = ft / gt;
            }
        }
        if (gasmal) {
            const real d = fa - ha;
            real l = (d == fa) ? 1. : d / fa;
            const real m = gt / ft;
            real t = 2. - l;
            const real mm = m * m, tt = t * t;
            const real s = sqrt(tt + mm);
            const real r = (l == 0.) ? fabs(m) : sqrt(l * l + mm);
            const real a = 0.5 * (s + r);
            ssmin = ha / a;
            ssmax = fa * a;
            if (mm == 0.) {
                if (l == 0.) t = sgn(2., ft) * sgn(1., gt);
                else t = gt / sgn(d, ft) + m / t;
            } else {
                t = (m / (s + t) + m / (r + l)) * (1. + a);
            }
            l = sqrt(t * t + 4.);
            crt = 2. / l;
            srt = t / l;
            clt = (crt + srt * m) / a;
            slt = (ht / ft) * srt / a;
        }
    }
    if (swap) {
        csl = srt; snl = crt; csr = slt; snr = clt;
    } else {
        csl = clt; snl = slt; csr = crt; snr = srt;
    }
    real tsign = 1.;
    if (pmax == 1) tsign = sgn(1., csr) * sgn(1., csl) * sgn(1., f);
    if (pmax == 2) tsign = sgn(1., snr) * sgn(1., csl) * sgn(1., g);
    if (pmax == 3) tsign = sgn(1., snr) * sgn(1., snl) * sgn(1., h);
    ssmax = sgn(ssmax, tsign);
    ssmin = sgn(ssmin, tsign * sgn(1., f) * sgn(1., h));
}

// Apply a plane rotation to rows p, q of the 3 x 3 VT: (x, y) <- (c x + s y, c y - s x)
DGX_HD inline void rot_rows(real (&vt)[3][3], int p, int q, real c, real s) {
    for (int j = 0; j < 3; ++j) {
        const real x = vt[p][j], y = vt[q][j];
        vt[p][j] = c * x + s * y;
        vt[q][j] = c * y - s * x;
    }
}

// dbdsqr('U', n = 3, ncvt = 3, nru = 0): singular values of the upper bidiagonal
// (d, e) and VT <- VT_B^T VT, sorted decreasing, made non-negative.
DGX_HD inline void bdsqr3(real (&d)[3], real (&e)[2], real (&vt)[3][3]) {
    constexpr int n = 3;
    const real tolmul = fmax(10., fmin(100., pow(EPS, -0.125)));
    const real tol = tolmul * EPS;
    real smax = 0.;
    for (int i = 0; i < n; ++i) smax = fmax(smax, fabs(d[i]));
    for (int i = 0; i < n - 1; ++i) smax = fmax(smax, fabs(e[i]));
    real sminoa = fabs(d[0]);
    if (sminoa != 0.) {
        real mu = sminoa;
        for (int i = 1; i < n; ++i) {
            mu = fabs(d[i]) * (mu / (mu + fabs(e[i - 1])));
            sminoa = fmin(sminoa, mu);
            if (sminoa == 0.) break;
        }
    }
    sminoa = sminoa / sqrt((real)n);
    const real thresh = fmax(tol * sminoa, 6. * n * (n * SAFMIN));
    const int maxitdivn = 6 * n;
    int iterdivn = 0, iter = -1, oldll = -1, oldm = -1, idir = 0;
    int m = n;  // 1-based index of the last element of the unconverged part
    // 1-based accessors (the routine's own indexing)
#define D_(i) d[(i) - 1]
#define E_(i) e[(i) - 1]
    for (int guard = 0; guard < 200; ++guard) {
        if (m <= 1) break;
        if (iter >= n) {
            iter -= n;
            ++iterdivn;
            if (iterdivn >= maxitdivn) break;
        }
        // find diagonal block of matrix to work on
        real smx = fabs(D_(m));
        int ll = 0;
        bool split = false;
        for (int lll = 1; lll <= m - 1; ++lll) {
            ll = m - lll;
            const real abss = fabs(D_(ll)), abse = fabs(E_(ll));
            if (abse <= thresh) { split = true; break; }
            smx = fmax(smx, fmax(abss, abse));
        }
        if (split) {
            E_(ll) = 0.;
            if (ll == m - 1) { m -= 1; continue; }
        } else {
            ll = 0;
        }
        ll += 1;
        if (ll == m - 1) {  // 2 x 2 block
            real sigmn, sigmx, sinr, cosr, sinl, cosl;
            lasv2(D_(m - 1), E_(m - 1), D_(m), sigmn, sigmx, sinr, cosr, sinl, cosl);
            D_(m - 1) = sigmx;
            E_(m - 1) = 0.;
            D_(m) = sigmn;
            rot_rows(vt, m - 2, m - 1, cosr, sinr);
            m -= 2;
            continue;
        }
        if (ll > oldm || m < oldll) idir = fabs(D_(ll)) >= fabs(D_(m)) ? 1 : 2;
        real smin;
        bool conv = false;
        if (idir == 1) {
            if (fabs(E_(m - 1)) <= fabs(tol) * fabs(D_(m))) { E_(m - 1) = 0.; continue; }
            real mu = fabs(D_(ll));
            smin = mu;
            for (int lll = ll; lll <= m - 1; ++lll) {
                if (fabs(E_(lll)) <= tol * mu) { E_(lll) = 0.; conv = true; break; }
                mu = fabs(D_(lll + 1)) * (mu / (mu + fabs(E_(lll))));
                smin = fmin(smin, mu);
            }
        } else {
            if (fabs(E_(ll)) <= fabs(tol) * fabs(D_(ll))) { E_(ll) = 0.; continue; }
            real mu = fabs(D_(m));
            smin = mu;
            for (int lll = m - 1; lll >= ll; --lll) {
                if (fabs(E_(lll)) <= tol * mu) { E_(lll) = 0.; conv = true; break; }
                mu = fabs(D_(lll)) * (mu / (mu + fabs(E_(lll))));
                smin = fmin(smin, mu);
            }
        }
        if (conv) continue;
        oldll = ll;
        oldm = m;
        // shift
        real shift, r;
        if (n * tol * (smin / smx) <= fmax(EPS, 0.01 * tol)) {
            shift = 0.;
        } else {
            real sll;
            if (idir == 1) {
                sll = fabs(D_(ll));
                las2(D_(m - 1), E_(m - 1), D_(m), shift, r);
            } else {
                sll = fabs(D_(m));
                las2(D_(ll), E_(ll), D_(ll + 1), shift, r);
            }
            if (sll > 0. && (shift / sll) * (shift / sll) < EPS) shift = 0.;
        }
        iter += m - ll;
        real wc[2], ws[2];  // rotations applied to VT rows (at most 2 for n = 3)
        const int nrot = m - ll;
        if (shift == 0.) {
            if (idir == 1) {
                real cs = 1., oldcs = 1., sn = 0., oldsn = 0.;
                for (int i = ll; i <= m - 1; ++i) {
                    lartg(D_(i) * cs, E_(i), cs, sn, r);
                    if (i > ll) E_(i - 1) = oldsn * r;
                    lartg(oldcs * r, D_(i + 1) * sn, oldcs, oldsn, D_(i));
                    wc[i - ll] = cs;
                    ws[i - ll] = sn;
                }
                const real h = D_(m) * cs;
                D_(m) = h * oldcs;
                E_(m - 1) = h * oldsn;
                for (int q = 0; q < nrot; ++q) rot_rows(vt, ll - 1 + q, ll + q, wc[q], ws[q]);  // dlasr L V F
                if (fabs(E_(m - 1)) <= thresh) E_(m - 1) = 0.;
            } else {
                real cs = 1., oldcs = 1., sn = 0., oldsn = 0.;
                for (int i = m; i >= ll + 1; --i) {
                    lartg(D_(i) * cs, E_(i - 1), cs, sn, r);
                    if (i < m) E_(i) = oldsn * r;
                    lartg(oldcs * r, D_(i - 1) * sn, oldcs, oldsn, D_(i));
                    wc[i - ll - 1] = oldcs;
                    ws[i - ll - 1] = -oldsn;
                }
                const real h = D_(ll) * cs;
                D_(ll) = h * oldcs;
                E_(ll) = h * oldsn;
                for (int q = nrot - 1; q >= 0; --q) rot_rows(vt, ll - 1 + q, ll + q, wc[q], ws[q]);  // dlasr L V B
                if (fabs(E_(ll)) <= thresh) E_(ll) = 0.;
            }
        } else {
            if (idir == 1) {
                real f = (fabs(D_(ll)) - shift) * (sgn(1., D_(ll)) + shift / D_(ll));
                real g = E_(ll);
                for (int i = ll; i <= m - 1; ++i) {
                    real cosr, sinr, cosl, sinl;
                    lartg(f, g, cosr, sinr, r);
                    if (i > ll) E_(i - 1) = r;
                    f = cosr * D_(i) + sinr * E_(i);
                    E_(i) = cosr * E_(i) - sinr * D_(i);
                    g = sinr * D_(i + 1);
                    D_(i + 1) = cosr * D_(i + 1);
                    lartg(f, g, cosl, sinl, r);
                    D_(i) = r;
                    f = cosl * E_(i) + sinl * D_(i + 1);
                    D_(i + 1) = cosl * D_(i + 1) - sinl * E_(i);
                    if (i < m - 1) {
                        g = sinl * E_(i + 1);
                        E_(i + 1) = cosl * E_(i + 1);
                    }
                    wc[i - ll] = cosr;
                    ws[i - ll] = sinr;
                }
                E_(m - 1) = f;
                for (int q = 0; q < nrot; ++q) rot_rows(vt, ll - 1 + q, ll + q, wc[q], ws[q]);
                if (fabs(E_(m - 1)) <= thresh) E_(m - 1) = 0.;
            } else {
                real f = (fabs(D_(m)) - shift) * (sgn(1., D_(m)) + shift / D_(m));
                real g = E_(m - 1);
                for (int i = m; i >= ll + 1; --i) {
                    real cosr, sinr, cosl, sinl;
                    lartg(f, g, cosr, sinr, r);
                    if (i < m) E_(i) = r;
                    f = cosr * D_(i) + sinr * E_(i - 1);
                    E_(i - 1) = cosr * E_(i - 1) - sinr * D_(i);
                    g = sinr * D_(i - 1);
                    D_(i - 1) = cosr * D_(i - 1);
                    lartg(f, g, cosl, sinl, r);
                    D_(i) = r;
                    f = cosl * E_(i - 1) + sinl * D_(i - 1);
                    D_(i - 1) = cosl * D_(i - 1) - sinl * E_(i - 1);
                    if (i > ll + 1) {
                        g = sinl * E_(i - 2);
                        E_(i - 2) = cosl * E_(i - 2);
                    }
                    wc[i - ll - 1] = cosl;
                    ws[i - ll - 1] = -sinl;
                }
                E_(ll) = f;
                if (fabs(E_(ll)) <= thresh) E_(ll) = 0.;
                for (int q = nrot - 1; q >= 0; --q) rot_rows(vt, ll - 1 + q, ll + q, wc[q], ws[q]);
            }
        }
    }
#undef D_
#undef E_
    // make singular values positive (flipping the VT rows), then sort decreasing
    for (int i = 0; i < n; ++i) {
        if (d[i] < 0.) {
            d[i] = -d[i];
            for (int j = 0; j < 3; ++j) vt[i][j] = -vt[i][j];
        }
    }
    for (int i = 1; i <= n - 1; ++i) {
        int isub = 1;
        real smn = d[0];
        for (int j = 2; j <= n + 1 - i; ++j) {
            if (d[j - 1] <= smn) { isub = j; smn = d[j - 1]; }
        }
        if (isub != n + 1 - i) {
            d[isub - 1] = d[n - i];
            d[n - i] = smn;
            for (int j = 0; j < 3; ++j) {
                const real t = vt[isub - 1][j];
                vt[isub - 1][j] = vt[n - i][j];
                vt[n - i][j] = t;
            }
        }
    }
}

// dgeqr2 on A (k x 3 row-major, k >= 3, modified): R of A = Q R
DGX_HD inline void qr_r(real* A, int k, real (&R)[3][3]) {
    for (int i = 0; i < 3; ++i) {
        real alpha = A[i * 3 + i];
        const real tau = larfg(k - i, alpha, A + (i + 1) * 3 + i, 3);
        A[i * 3 + i] = alpha;
        if (i < 2 && tau != 0.) {
            // apply H = I - tau v v^T (v = [1; A(i+1:k, i)]) to columns i+1..2, rows i..k-1
            for (int j = i + 1; j < 3; ++j) {
                real w = A[i * 3 + j];
                for (int r = i + 1; r < k; ++r) w += A[r * 3 + i] * A[r * 3 + j];
                A[i * 3 + j] -= tau * w;
                for (int r = i + 1; r < k; ++r) A[r * 3 + j] -= tau * w * A[r * 3 + i];
            }
        }
    }
    R[0][0] = A[0]; R[0][1] = A[1]; R[0][2] = A[2];
    R[1][0] = 0.;  R[1][1] = A[4]; R[1][2] = A[5];
    R[2][0] = 0.;  R[2][1] = 0.;  R[2][2] = A[8];
}

// dgebd2 (m = n = 3, upper bidiagonal) on R (modified): diagonal d, superdiagonal
// e, and the one non-trivial right reflector G(1) = I - taup0 [0 1 vp]^T [0 1 vp]
DGX_HD inline void bidiag(real (&R)[3][3], real (&d)[3], real (&e)[2], real& taup0, real& vp) {
    taup0 = 0.;
    for (int i = 0; i < 3; ++i) {
        // left: annihilate R(i+1:2, i)
        real alpha = R[i][i];
        real col[2] = {i + 1 < 3 ? R[i + 1][i] : 0., i + 2 < 3 ? R[i + 2][i] : 0.};
        const real tauq = larfg(3 - i, alpha, col, 1);
        d[i] = alpha;
        if (i + 1 < 3) R[i + 1][i] = col[0];
        if (i + 2 < 3) R[i + 2][i] = col[1];
        if (i < 2 && tauq != 0.) {
            for (int j = i + 1; j < 3; ++j) {
                real w = R[i][j];
                for (int r = i + 1; r < 3; ++r) w += R[r][i] * R[r][j];
                R[i][j] -= tauq * w;
                for (int r = i + 1; r < 3; ++r) R[r][j] -= tauq * w * R[r][i];
            }
        }
        if (i < 2) {
            // right: annihilate R(i, i+2:2)
            real beta = R[i][i + 1];
            real row[1] = {i + 2 < 3 ? R[i][i + 2] : 0.};
            const real taup = larfg(2 - i, beta, row, 1);
            e[i] = beta;
            if (i + 2 < 3) R[i][i + 2] = row[0];
            if (i == 0) taup0 = taup;
            if (taup != 0.) {  // only i = 0 has a non-trivial right reflector (columns 1..2)
                for (int r = i + 1; r < 3; ++r) {
                    const real w = R[r][i + 1] + R[r][i + 2] * R[i][i + 2];
                    R[r][i + 1] -= taup * w;
                    R[r][i + 2] -= taup * w * R[i][i + 2];
                }
            }
        }
    }
    vp = R[0][2];  // right reflector G(1): v = [1, vp] on columns 1..2
}

// A: k x 3 row-major (k >= 3), modified. Returns the largest singular value in
// *s0 and the first row of LAPACK's VT (its first right singular vector) in v.
DGX_HD inline void dominant_right_vector(real* A, int k, real* s0, real (&v)[3]) {
    real R[3][3], d[3], e[2], taup0, vp;
    qr_r(A, k, R);
    bidiag(R, d, e, taup0, vp);
    real vt[3][3] = {{1., 0., 0.}, {0., 1., 0.}, {0., 0., 1.}};
    bdsqr3(d, e, vt);
    // dormbr('P','R','T'): VT <- VT P^T, P = G(1) = I - taup0 [0,1,vp]^T [0,1,vp] (symmetric)
    for (int r = 0; r < 3; ++r) {
        const real w = vt[r][1] + vt[r][2] * vp;
        vt[r][1] -= taup0 * w;
        vt[r][2] -= taup0 * w * vp;
    }
    *s0 = d[0];
    v[0] = vt[0][0];
    v[1] = vt[0][1];
    v[2] = vt[0][2];
}

}  // namespace svd3
