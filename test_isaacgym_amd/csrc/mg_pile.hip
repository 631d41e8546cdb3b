// mg_pile.hip — the free-body pile step: a coupled env of
// more than MG_ENV_MAXF free bodies and no articulation — the pyramid of 30
// balls per env of examples/1080_balls_of_solitude.py:96-136 (group i,
// filter 0), or boxes, capsules and hulls heaped on the ground and on up to
// MG_ENV_MAXS static bodies.
//
// One wavefront (one workgroup) per env; lane k owns free body k (<= 64).
// Per substep:
//   1. body lanes: free flight (gravity, external wrench, damping, speed
//      clamps), the pose, COM and world inverse inertia into LDS;
//   2. narrow phase: 64 candidate shape pairs per round, one per lane (the
//      coupled step's screen and contacts, mg_pairs.h / mg_collide.h); the pairs
//      with contacts ("active pairs") are compacted in pair order by one
//      wave-wide prefix sum, up to MG_PILE_MAXAP pairs / MG_PILE_MAXPT points
//      (the first pair that would overflow either ends the list);
//   3. pair lanes: their points' row constants;
//   4. greedy colouring in pair order, the used-colour masks held in the body
//      lanes' registers (v_readlane per pair, no LDS on the chain), then a
//      counting sort by colour (ballots) — PhysX's GPU constraint
//      partitioning: no two pairs of one colour share a free body;
//   5. TGS sweeps colour by colour: each lane solves one pair's rows (friction
//      then normal rows, solve_pair) against the body velocities in LDS. The
//      pairs of a colour touch disjoint bodies, so the parallel visit equals
//      the sequential one of oracle/migym_oracle_pile.c bit for bit;
//   6. body lanes: motion deltas, pose integration, the contact impulses summed
//      in pair order (net contact force).
// Numerics: -ffp-contract=off, explicit fmaf where the oracle has fmaf.
#include "mg_internal.h"
#include "mg_collide.h"
#include "mg_pairs.h"

namespace {

constexpr int MAXB = MG_PILE_MAXB;
constexpr int ST0 = MG_PILE_ST0;
constexpr int MAXAP = MG_PILE_MAXAP;
constexpr int MAXPT = MG_PILE_MAXPT;
static_assert(MAXB == 64 && MAXAP == 128, "one body per lane; two active pairs per lane");

struct PileLds {
    // free bodies (lane k = body k)
    V3 x[MAXB], xc[MAXB], v[MAXB], w[MAXB], dx[MAXB], dth[MAXB];
    Q4 q[MAXB];
    S3 Iw[MAXB];
    float invm[MAXB];
    // static bodies
    V3 sx[MG_ENV_MAXS];
    Q4 sq[MG_ENV_MAXS];
    // active pairs (pair order), then the visit order
    int pa[MAXAP], pb[MAXAP], pt0[MAXAP], pn[MAXAP], ord[MAXAP];
    float pmu[MAXAP], pe[MAXAP];
    int cstart[MAXB + 1];
    // points
    V3 n[MAXPT], ra[MAXPT], rb[MAXPT], t1[MAXPT], t2[MAXPT];
    float s0[MAXPT], kn[MAXPT], kt1[MAXPT], kt2[MAXPT], vn0[MAXPT], ln[MAXPT], lt1[MAXPT], lt2[MAXPT];
};

__device__ __forceinline__ V3 vfma(V3 v, V3 d, float s) {   // oracle fmad3_
    return v3(fmaf(d.x, s, v.x), fmaf(d.y, s, v.y), fmaf(d.z, s, v.z));
}
__device__ __forceinline__ Q4 inertia_frame(Q4 q, Q4 iq) {
    if (iq.x == 0.0f && iq.y == 0.0f && iq.z == 0.0f && iq.w == 1.0f) return q;
    return qmul(q, iq);
}
__device__ __forceinline__ V3 com_world(V3 x, Q4 q, V3 com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return x;
    return vadd(x, qrot(q, com));
}
__device__ __forceinline__ V3 origin_from_com(V3 xc, Q4 q, V3 com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return xc;
    return vsub(xc, qrot(q, com));
}
// 1 / effective mass of a row along d (oracle op_k_)
__device__ __forceinline__ float row_k(V3 d, V3 ra, V3 rb, float ima, float imb, const S3& Ia, const S3& Ib) {
    const V3 ca = vcross(ra, d), cb = vcross(rb, d);
    return 1.0f / (((ima + imb) + vdot(ca, symmul(Ia, ca))) + vdot(cb, symmul(Ib, cb)));
}
// TGS row targets (mg_rigid.hip pos_target / vel_target, oracle pos_target_ / vel_target_)
__device__ __forceinline__ float pos_tgt(const MgStep& P, float s) { return fminf(-s * P.inv_sub, P.max_depen); }
__device__ __forceinline__ float vel_tgt(const MgStep& P, float s, float e, float vn0) {
    float tgt = fminf(-s * P.inv_h, 0.0f);
    if (e > 0.0f && vn0 < -P.bounce_thresh) tgt = fmaxf(tgt, -e * vn0);
    return tgt;
}
__device__ __forceinline__ float clamp_sym(float x, float lim) { return fminf(fmaxf(x, -lim), lim); }

// inclusive prefix sum over the wavefront
__device__ __forceinline__ int wave_incl_scan(int x, int ln) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (ln >= d) x += y;
    }
    return x;
}
__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int k) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, k);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), k);
    return ((unsigned long long)hi << 32) | lo;
}

// the velocities a pair's rows act on: A's, and B's (zero, never stored back,
// for a static body or the ground) — oracle prow_t
struct PairRows {
    float ima, imb;
    S3 Ia, Ib;
    V3 dxa, dta, dxb, dtb, va, wa, vb, wb;
};

// the pair's normal rows, point order (oracle op_normal_rows_)
__device__ __forceinline__ void normal_rows(const MgStep& P, PileLds& S, int p0, int np, float e, PairRows& R,
                                            bool pos) {
    for (int j = 0; j < np; ++j) {
        const int c = p0 + j;
        const V3 n = S.n[c], ra = S.ra[c], rb = S.rb[c];
        const V3 ca = vcross(ra, n), cb = vcross(rb, n);
        const float s = S.s0[c] + ((vdot(n, R.dxa) + vdot(ca, R.dta)) - (vdot(n, R.dxb) + vdot(cb, R.dtb)));
        const float tgt = pos ? pos_tgt(P, s) : vel_tgt(P, s, e, S.vn0[c]);
        const float vn = (vdot(n, R.va) + vdot(ca, R.wa)) - (vdot(n, R.vb) + vdot(cb, R.wb));
        const float l0 = S.ln[c];
        const float nl = fmaxf(fmaf(S.kn[c], tgt - vn, l0), 0.0f);
        const float dl = nl - l0;
        S.ln[c] = nl;
        R.va = vfma(R.va, n, dl * R.ima);
        R.wa = vfma(R.wa, symmul(R.Ia, ca), dl);
        R.vb = vfma(R.vb, n, -(dl * R.imb));
        R.wb = vfma(R.wb, symmul(R.Ib, cb), -dl);
    }
}

// the pair's friction rows, point order, t1 then t2 (oracle op_friction_rows_):
// the pyramid clamp at mu times the point's normal impulse; a position sweep
// also closes the tangential drift of the point's two copies over the substep
__device__ __forceinline__ void friction_rows(const MgStep& P, PileLds& S, int p0, int np, float mu, PairRows& R,
                                              bool pos) {
    for (int j = 0; j < np; ++j) {
        const int c = p0 + j;
        const V3 ra = S.ra[c], rb = S.rb[c];
        const float lim = mu * S.ln[c];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const V3 t = r == 0 ? S.t1[c] : S.t2[c];
            const float kt = r == 0 ? S.kt1[c] : S.kt2[c];
            const float lt = r == 0 ? S.lt1[c] : S.lt2[c];
            const V3 ca = vcross(ra, t), cb = vcross(rb, t);
            const float vt = (vdot(t, R.va) + vdot(ca, R.wa)) - (vdot(t, R.vb) + vdot(cb, R.wb));
            const float dr = (vdot(t, R.dxa) + vdot(ca, R.dta)) - (vdot(t, R.dxb) + vdot(cb, R.dtb));
            const float ft = pos ? -dr * P.inv_sub : 0.0f;
            const float nl = clamp_sym(fmaf(kt, ft - vt, lt), lim);
            const float d = nl - lt;
            if (r == 0) S.lt1[c] = nl; else S.lt2[c] = nl;
            R.va = vfma(R.va, t, d * R.ima);
            R.wa = vfma(R.wa, symmul(R.Ia, ca), d);
            R.vb = vfma(R.vb, t, -(d * R.imb));
            R.wb = vfma(R.wb, symmul(R.Ib, cb), -d);
        }
    }
}

// one active pair in one sweep (oracle op_solve_pair_): a position sweep is
// friction, then normal rows (the first opens with the normal rows too); a
// velocity sweep is normal, friction, normal rows (DESIGN.md §3.2.1's order)
__device__ __forceinline__ void solve_pair(const MgStep& P, PileLds& S, int i, bool pos, bool first) {
    const int a = S.pa[i], b = S.pb[i], p0 = S.pt0[i], np = S.pn[i];
    const bool dynb = b >= 0 && b < ST0;
    const float mu = S.pmu[i], e = S.pe[i];
    const V3 z = v3(0.0f, 0.0f, 0.0f);
    PairRows R;
    R.ima = S.invm[a]; R.Ia = S.Iw[a];
    R.dxa = S.dx[a]; R.dta = S.dth[a]; R.va = S.v[a]; R.wa = S.w[a];
    R.imb = 0.0f;
    R.Ib.xx = 0.0f; R.Ib.yy = 0.0f; R.Ib.zz = 0.0f; R.Ib.xy = 0.0f; R.Ib.xz = 0.0f; R.Ib.yz = 0.0f;
    R.dxb = z; R.dtb = z; R.vb = z; R.wb = z;
    if (dynb) {
        R.imb = S.invm[b]; R.Ib = S.Iw[b];
        R.dxb = S.dx[b]; R.dtb = S.dth[b]; R.vb = S.v[b]; R.wb = S.w[b];
    }
    if (!pos || first) normal_rows(P, S, p0, np, e, R, pos);
    friction_rows(P, S, p0, np, mu, R, pos);
    normal_rows(P, S, p0, np, e, R, pos);
    S.v[a] = R.va;
    S.w[a] = R.wa;
    if (dynb) { S.v[b] = R.vb; S.w[b] = R.wb; }
}

__global__ void __launch_bounds__(64) k_pile_step(MgStep P, MgPileArgs A) {
    __shared__ PileLds S;
    const int ln = threadIdx.x;
    const int* ei = A.pile_i + (size_t)blockIdx.x * MG_PILE_I_N;
    const int boff = ei[0], nb = ei[1], pr0 = ei[2], npair = ei[3], ns = ei[4];
    const int N = A.nb;   // SoA stride
    const bool act = ln < nb;
    const int slot = act ? A.pile_body[boff + ln] : 0;
    const float h = P.h;

    // the lane's free body
    V3 x = v3(0.0f, 0.0f, 0.0f), v = x, w = x, invI = x, com = x, fext = x, text = x;
    Q4 q = q4(0.0f, 0.0f, 0.0f, 1.0f), iq = q;
    float invm = 0.0f, lkeep = 1.0f, akeep = 1.0f, mlv2 = 0.0f, mav2 = 0.0f, gon = 0.0f;
    if (act) {
        const float* st = A.state;
        x = v3(st[0 * N + slot], st[1 * N + slot], st[2 * N + slot]);
        q = qnormalize(q4(st[3 * N + slot], st[4 * N + slot], st[5 * N + slot], st[6 * N + slot]));
        v = v3(st[7 * N + slot], st[8 * N + slot], st[9 * N + slot]);
        w = v3(st[10 * N + slot], st[11 * N + slot], st[12 * N + slot]);
        const float* M = A.mass;
        invm = M[0 * N + slot];
        invI = v3(M[1 * N + slot], M[2 * N + slot], M[3 * N + slot]);
        iq = q4(M[4 * N + slot], M[5 * N + slot], M[6 * N + slot], M[7 * N + slot]);
        com = v3(M[8 * N + slot], M[9 * N + slot], M[10 * N + slot]);
        const float* tf = A.tbf + (size_t)A.body_tmpl[slot] * MG_TBODY_F_N;
        lkeep = 1.0f - fminf(tf[0] * h, 1.0f);
        akeep = 1.0f - fminf(tf[1] * h, 1.0f);
        mlv2 = tf[2] * tf[2];
        mav2 = tf[3] * tf[3];
        gon = tf[4];
        if (A.ext) {
            fext = v3(A.ext[0 * N + slot], A.ext[1 * N + slot], A.ext[2 * N + slot]);
            text = v3(A.ext[3 * N + slot], A.ext[4 * N + slot], A.ext[5 * N + slot]);
        }
    }
    if (ln < ns) {
        const int ss = ei[5 + ln];
        S.sx[ln] = v3(A.state[0 * N + ss], A.state[1 * N + ss], A.state[2 * N + ss]);
        S.sq[ln] = qnormalize(q4(A.state[3 * N + ss], A.state[4 * N + ss], A.state[5 * N + ss], A.state[6 * N + ss]));
    }
    const V3 gvec = v3(P.g[0], P.g[1], P.g[2]);
    V3 fsum = v3(0.0f, 0.0f, 0.0f);

    for (int sub = 0; sub < P.substeps; ++sub) {
        // ---- 1. free flight (oracle: rigid_body_step's order)
        if (act) {
            const S3 Iw = sym_rdrt(qmat(inertia_frame(q, iq)), invI);
            const V3 xc = com_world(x, q, com);
            if (gon != 0.0f) v = vmad(v, gvec, h);
            if (A.ext) {
                v = vmad(v, fext, invm * h);
                w = vmad(w, symmul(Iw, text), h);
            }
            v = vscale(v, lkeep);
            w = vscale(w, akeep);
            const float v2 = vdot(v, v);
            if (v2 > mlv2) v = vscale(v, sqrtf(mlv2 / v2));
            const float w2 = vdot(w, w);
            if (w2 > mav2) w = vscale(w, sqrtf(mav2 / w2));
            S.x[ln] = x; S.q[ln] = q; S.xc[ln] = xc;
            S.v[ln] = v; S.w[ln] = w;
            S.dx[ln] = v3(0.0f, 0.0f, 0.0f);
            S.dth[ln] = v3(0.0f, 0.0f, 0.0f);
            S.Iw[ln] = Iw;
            S.invm[ln] = invm;
        }
        __syncthreads();

        // ---- 2. narrow phase, 64 pairs per round, compacted in pair order
        int nap = 0, npt = 0;
        for (int base = 0; base < npair; base += 64) {
            const int i = base + ln;
            PairOut o;
            o.n = 0;
            int a = 0, b = -1;
            float mu = 0.0f, e = 0.0f;
            if (i < npair) {
                const int* pp = A.pairs + (size_t)(pr0 + i) * 4;
                a = pp[0];
                const int sa = pp[1];
                b = pp[2];
                const int sb = pp[3];
                const float* sha = A.shapes + (size_t)sa * MG_SHAPE_STRIDE;
                const V3 xa = S.x[a];
                const Q4 qa = S.q[a];
                if (b < 0) {
                    if (pair_near(P, sha, xa, qa, sha, xa, qa, true, nullptr, nullptr)) {
                        const CShape sA = place_shape(sha, xa, qa, A.hulls);
                        ground_pair(P, sA, o);
                    }
                    mu = 0.5f * (sha[11] + P.mu_ground);
                    e = 0.5f * (sha[12] + P.e_ground);
                } else {
                    const float* shb = A.shapes + (size_t)sb * MG_SHAPE_STRIDE;
                    const bool dynb = b < ST0;
                    const V3 xb = dynb ? S.x[b] : S.sx[b - ST0];
                    const Q4 qb = dynb ? S.q[b] : S.sq[b - ST0];
                    if (pair_near(P, sha, xa, qa, shb, xb, qb, false, A.shape_obb + (size_t)sa * MG_OBB_N,
                                  A.shape_obb + (size_t)sb * MG_OBB_N)) {
                        const CShape sA = place_shape(sha, xa, qa, A.hulls);
                        const CShape sB = place_shape(shb, xb, qb, A.hulls);
                        collide(sA, sB, P.contact_offset, o);
                    }
                    mu = 0.5f * (sha[11] + shb[11]);
                    e = 0.5f * (sha[12] + shb[12]);
                }
            }
            // packed (pairs << 16 | points) prefix: a pair is kept while both
            // running totals fit; the first that does not ends the list
            const int has = o.n > 0 ? 1 : 0;
            const int incl = wave_incl_scan((has << 16) | o.n, ln);
            const int ip = nap + (incl >> 16), it = npt + (incl & 0xFFFF);
            const bool kept = has && ip <= MAXAP && it <= MAXPT;
            const bool over = has && !kept;
            if (kept) {
                const int j = ip - 1, c0 = it - o.n;
                S.pa[j] = a; S.pb[j] = b; S.pt0[j] = c0; S.pn[j] = o.n;
                S.pmu[j] = mu; S.pe[j] = e;
                const bool dynb = b >= 0 && b < ST0;
                const V3 xca = S.xc[a];
                const V3 xcb = dynb ? S.xc[b] : v3(0.0f, 0.0f, 0.0f);
#pragma unroll
                for (int k = 0; k < MG_PAIR_MAXC; ++k) {
                    if (k < o.n) {
                        S.n[c0 + k] = o.nrm[k];
                        S.s0[c0 + k] = o.sep[k] - P.rest_offset;
                        S.ra[c0 + k] = vsub(o.p[k], xca);
                        S.rb[c0 + k] = dynb ? vsub(o.p[k], xcb) : v3(0.0f, 0.0f, 0.0f);
                    }
                }
            }
            const unsigned long long kb = __ballot(kept);
            if (kb) {   // the last kept lane's running totals
                const int lk = __builtin_amdgcn_readlane(incl, 63 - __clzll(kb));
                nap += lk >> 16;
                npt += lk & 0xFFFF;
            }
            if (__any(over)) break;
        }
        __syncthreads();

        // ---- 3. row constants, one active pair per lane
        for (int i = ln; i < nap; i += 64) {
            const int a = S.pa[i], b = S.pb[i], p0 = S.pt0[i], np = S.pn[i];
            const bool dynb = b >= 0 && b < ST0;
            const float ima = S.invm[a];
            const S3 Ia = S.Iw[a];
            const V3 va = S.v[a], wa = S.w[a];
            S3 Ib;
            Ib.xx = 0.0f; Ib.yy = 0.0f; Ib.zz = 0.0f; Ib.xy = 0.0f; Ib.xz = 0.0f; Ib.yz = 0.0f;
            float imb = 0.0f;
            V3 vb = v3(0.0f, 0.0f, 0.0f), wb = vb;
            if (dynb) { imb = S.invm[b]; Ib = S.Iw[b]; vb = S.v[b]; wb = S.w[b]; }
            for (int j = 0; j < np; ++j) {
                const int c = p0 + j;
                const V3 n = S.n[c], ra = S.ra[c], rb = S.rb[c];
                V3 t1, t2;
                env_tangents(n, &t1, &t2);
                S.t1[c] = t1;
                S.t2[c] = t2;
                S.kn[c] = row_k(n, ra, rb, ima, imb, Ia, Ib);
                S.kt1[c] = row_k(t1, ra, rb, ima, imb, Ia, Ib);
                S.kt2[c] = row_k(t2, ra, rb, ima, imb, Ia, Ib);
                S.vn0[c] = (vdot(n, va) + vdot(vcross(ra, n), wa)) - (vdot(n, vb) + vdot(vcross(rb, n), wb));
                S.ln[c] = 0.0f;
                S.lt1[c] = 0.0f;
                S.lt2[c] = 0.0f;
            }
        }

        // ---- 4. greedy colouring in pair order: pair j's bodies' masks read
        // from their lanes; the pair's (a, b) from lane j % 64's registers
        const int paA = ln < nap ? S.pa[ln] : 0, pbA = ln < nap ? S.pb[ln] : -1;
        const int paB = ln + 64 < nap ? S.pa[ln + 64] : 0, pbB = ln + 64 < nap ? S.pb[ln + 64] : -1;
        unsigned long long used = 0ull;
        int colA = -1, colB = -1, ncol = 0;
        for (int j = 0; j < nap; ++j) {
            const int jl = j & 63;
            const int a = __builtin_amdgcn_readlane(j < 64 ? paA : paB, jl);
            const int b = __builtin_amdgcn_readlane(j < 64 ? pbA : pbB, jl);
            const bool dynb = b >= 0 && b < ST0;
            const unsigned long long taken = readlane64(used, a) | (dynb ? readlane64(used, b) : 0ull);
            int c = -1;
            if (taken != ~0ull) {
                c = __builtin_ctzll(~taken);
                if (ln == a || (dynb && ln == b)) used |= 1ull << c;
                ncol = c + 1 > ncol ? c + 1 : ncol;
            }
            if (ln == jl) {
                if (j < 64) colA = c; else colB = c;
            }
        }
        // counting sort by colour (stable in pair order): lane c counts colour c
        {
            int cnt = 0;
            for (int c = 0; c < ncol; ++c) {
                const unsigned long long b0 = __ballot(colA == c), b1 = __ballot(colB == c);
                if (ln == c) cnt = __popcll(b0) + __popcll(b1);
            }
            const int incl = wave_incl_scan(cnt, ln);
            if (ln < ncol) S.cstart[ln] = incl - cnt;
            if (ln == 63) S.cstart[ncol] = incl;           // the coloured total
            for (int c = 0; c < ncol; ++c) {
                const int start = __builtin_amdgcn_readlane(incl - cnt, c);
                const unsigned long long b0 = __ballot(colA == c), b1 = __ballot(colB == c);
                const unsigned lo = (unsigned)b0, hi = (unsigned)(b0 >> 32);
                const int r0 = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0));
                if (colA == c) S.ord[start + r0] = ln;
                const unsigned lo1 = (unsigned)b1, hi1 = (unsigned)(b1 >> 32);
                const int r1 = __builtin_amdgcn_mbcnt_hi(hi1, __builtin_amdgcn_mbcnt_lo(lo1, 0));
                if (colB == c) S.ord[start + __popcll(b0) + r1] = ln + 64;
            }
        }
        __syncthreads();

        // ---- 5. TGS: position sweeps (then the motion deltas), velocity sweeps
        for (int itr = 0; itr < P.npos + P.nvel; ++itr) {
            const bool pos = itr < P.npos;
            for (int c = 0; c < ncol; ++c) {
                const int cs = S.cstart[c], ce = S.cstart[c + 1];
                for (int k = cs + ln; k < ce; k += 64) solve_pair(P, S, S.ord[k], pos, itr == 0);
                __syncthreads();
            }
            if (pos && act) {
                S.dx[ln] = vfma(S.dx[ln], S.v[ln], P.sub);
                S.dth[ln] = vfma(S.dth[ln], S.w[ln], P.sub);
            }
            __syncthreads();
        }

        // ---- 6. pose; contact impulses on the lane's body, in pair order
        if (act) {
            v = S.v[ln];
            w = S.w[ln];
            const V3 xc1 = vadd(S.xc[ln], S.dx[ln]);
            q = qintegrate(q, S.dth[ln]);
            x = origin_from_com(xc1, q, com);
            for (int i = 0; i < nap; ++i) {
                const int a = S.pa[i], b = S.pb[i];
                if (a != ln && b != ln) continue;
                const int p0 = S.pt0[i], np = S.pn[i];
                for (int j = 0; j < np; ++j) {
                    const int c = p0 + j;
                    const V3 f = vadd(vadd(vscale(S.n[c], S.ln[c]), vscale(S.t1[c], S.lt1[c])), vscale(S.t2[c], S.lt2[c]));
                    fsum = a == ln ? vadd(fsum, f) : vsub(fsum, f);
                }
            }
        }
        __syncthreads();
    }
    if (act) {
        float* st = A.state;
        st[0 * N + slot] = x.x; st[1 * N + slot] = x.y; st[2 * N + slot] = x.z;
        st[3 * N + slot] = q.x; st[4 * N + slot] = q.y; st[5 * N + slot] = q.z; st[6 * N + slot] = q.w;
        st[7 * N + slot] = v.x; st[8 * N + slot] = v.y; st[9 * N + slot] = v.z;
        st[10 * N + slot] = w.x; st[11 * N + slot] = w.y; st[12 * N + slot] = w.z;
        A.cforce[0 * N + slot] = fsum.x * P.inv_dt;
        A.cforce[1 * N + slot] = fsum.y * P.inv_dt;
        A.cforce[2 * N + slot] = fsum.z * P.inv_dt;
    }
}

}  // namespace

hipError_t mg_launch_pile_step(const MgStep& P, const MgPileArgs& A, hipStream_t s) {
    if (A.ne <= 0) return hipSuccess;
    MG_LAUNCH(k_pile_step, dim3(A.ne), dim3(64), 0, s, P, A);
    return hipGetLastError();
}
