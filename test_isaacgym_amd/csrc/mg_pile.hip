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

#ifdef MG_PILE_STAMPS
// diagnostic build only (tools/kbench_pile_stamps.py): s_memtime stamps of each
// k_pile_step wave at its phase boundaries (the last substep's), then its
// counts (candidate pairs, active pairs, points, colours), lane 0 ->
// g_pile_stamp[env]
#define MG_PILE_NSTAMP 16
__device__ unsigned long long g_pile_stamp[16384][MG_PILE_NSTAMP];
extern "C" int mg_debug_pile_stamps(unsigned long long* out, int n) {
    if (n > 16384) n = 16384;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pile_stamp), (size_t)n * MG_PILE_NSTAMP * 8) == hipSuccess ? 0 : -1;
}
__device__ __forceinline__ unsigned long long pile_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PSTAMP(k) do { const unsigned long long t_ = pile_stamp(); \
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_pile_stamp[blockIdx.x][k] = t_; } while (0)
#define PCOUNT(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 16384) g_pile_stamp[blockIdx.x][k] = (v); } while (0)
#else
#define PSTAMP(k) do { } while (0)
#define PCOUNT(k, v) do { } while (0)
#endif

namespace {

constexpr int MAXB = MG_PILE_MAXB;
constexpr int ST0 = MG_PILE_ST0;
constexpr int MAXAP = MG_PILE_MAXAP;
constexpr int MAXPT = MG_PILE_MAXPT;
constexpr int MAXSH = MG_PILE_MAXSH;
static_assert(MAXB == 64 && MAXAP == 128, "one body per lane; two active pairs per lane");

struct ShapeSphere { float x, y, z, r; };   // a local shape's bounding sphere (pair_near's first test)

struct PileLds {
    // free bodies (lane k = body k)
    V3 x[MAXB], xc[MAXB], v[MAXB], w[MAXB], dx[MAXB], dth[MAXB];
    Q4 q[MAXB];
    S3 Iw[MAXB];
    float invm[MAXB];
    // static bodies
    V3 sx[MG_ENV_MAXS];
    Q4 sq[MG_ENV_MAXS];
    // the env's local shape slots: participant, shape record, bounding sphere
    int slot_part[MAXSH], slot_shape[MAXSH];
    ShapeSphere sc[MAXSH];
    // screened candidate pairs waiting for the narrow phase (ring, pair order)
    unsigned ring[128];
    // active pairs (pair order)
    int pa[MAXAP], pb[MAXAP], pt0[MAXAP], pn[MAXAP];
    // greedy colouring: each body's used colours; the first uncoloured pair
    // of the batch touching it
    unsigned long long used[MAXB];
    unsigned first[MAXB];
    V3 facc[MAXB];   // net contact impulse per body (the force pass)
    float pmu[MAXAP], pe[MAXAP];
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
// 1 / effective mass of a row along d (oracle op_k_); B static or the ground
// (dynb false): A's terms only
__device__ __forceinline__ float row_k(bool dynb, V3 d, V3 ra, V3 rb, float ima, float imb, const S3& Ia,
                                       const S3& Ib) {
    const V3 ca = vcross(ra, d);
    const float ka = ima + vdot(ca, symmul(Ia, ca));
    if (!dynb) return 1.0f / ka;
    const V3 cb = vcross(rb, d);
    return 1.0f / ((ka + imb) + vdot(cb, symmul(Ib, cb)));
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
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) x = max(x, __shfl_xor(x, d, 64));
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
    bool dynb;
    float ima, imb;
    S3 Ia, Ib;
    V3 dxa, dta, dxb, dtb, va, wa, vb, wb;
};
// a row's relative velocity / substep motion along d, and its impulse
// (oracle op_relv_ / op_reld_ / op_apply_): B's terms only when it is a free body
__device__ __forceinline__ float rel_v(const PairRows& R, V3 d, V3 ca, V3 cb) {
    const float ua = vdot(d, R.va) + vdot(ca, R.wa);
    return R.dynb ? ua - (vdot(d, R.vb) + vdot(cb, R.wb)) : ua;
}
__device__ __forceinline__ float rel_d(const PairRows& R, V3 d, V3 ca, V3 cb) {
    const float ua = vdot(d, R.dxa) + vdot(ca, R.dta);
    return R.dynb ? ua - (vdot(d, R.dxb) + vdot(cb, R.dtb)) : ua;
}
__device__ __forceinline__ void apply_row(PairRows& R, V3 d, V3 ca, V3 cb, float dl) {
    R.va = vfma(R.va, d, dl * R.ima);
    R.wa = vfma(R.wa, symmul(R.Ia, ca), dl);
    if (R.dynb) {
        R.vb = vfma(R.vb, d, -(dl * R.imb));
        R.wb = vfma(R.wb, symmul(R.Ib, cb), -dl);
    }
}

// the pair's normal rows, point order (oracle op_normal_rows_)
__device__ __forceinline__ void normal_rows(const MgStep& P, PileLds& S, int p0, int np, float e, PairRows& R,
                                            bool pos) {
    for (int j = 0; j < np; ++j) {
        const int c = p0 + j;
        const V3 n = S.n[c], ra = S.ra[c], rb = S.rb[c];
        const V3 ca = vcross(ra, n), cb = vcross(rb, n);
        const float s = S.s0[c] + rel_d(R, n, ca, cb);
        const float tgt = pos ? pos_tgt(P, s) : vel_tgt(P, s, e, S.vn0[c]);
        const float vn = rel_v(R, n, ca, cb);
        const float l0 = S.ln[c];
        const float nl = fmaxf(fmaf(S.kn[c], tgt - vn, l0), 0.0f);
        const float dl = nl - l0;
        S.ln[c] = nl;
        apply_row(R, n, ca, cb, dl);
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
            const float vt = rel_v(R, t, ca, cb);
            const float ft = pos ? -rel_d(R, t, ca, cb) * P.inv_sub : 0.0f;
            const float nl = clamp_sym(fmaf(kt, ft - vt, lt), lim);
            const float d = nl - lt;
            if (r == 0) S.lt1[c] = nl; else S.lt2[c] = nl;
            apply_row(R, t, ca, cb, d);
        }
    }
}

// an active pair's header, held by its lane (pair j: lane j % 64)
struct PairHdr {
    int a, b, p0, np, color;
    int rnd;   // the colouring sub-round that coloured it (per body: pair order)
    float mu, e;
};

// one active pair in one sweep (oracle op_solve_pair_): a position sweep is
// friction, then normal rows (the first opens with the normal rows too); a
// velocity sweep is normal, friction, normal rows (DESIGN.md §3.2.1's order)
__device__ __forceinline__ void solve_pair(const MgStep& P, PileLds& S, const PairHdr& H, bool pos, bool first) {
    const int a = H.a, b = H.b;
    const bool dynb = b >= 0 && b < ST0;
    const V3 z = v3(0.0f, 0.0f, 0.0f);
    PairRows R;
    R.dynb = dynb;
    R.ima = S.invm[a]; R.Ia = S.Iw[a];
    R.dxa = S.dx[a]; R.dta = S.dth[a]; R.va = S.v[a]; R.wa = S.w[a];
    R.imb = 0.0f;
    R.Ib.xx = 0.0f; R.Ib.yy = 0.0f; R.Ib.zz = 0.0f; R.Ib.xy = 0.0f; R.Ib.xz = 0.0f; R.Ib.yz = 0.0f;
    R.dxb = z; R.dtb = z; R.vb = z; R.wb = z;
    if (dynb) {
        R.imb = S.invm[b]; R.Ib = S.Iw[b];
        R.dxb = S.dx[b]; R.dtb = S.dth[b]; R.vb = S.v[b]; R.wb = S.w[b];
    }
    if (!pos || first) normal_rows(P, S, H.p0, H.np, H.e, R, pos);
    friction_rows(P, S, H.p0, H.np, H.mu, R, pos);
    normal_rows(P, S, H.p0, H.np, H.e, R, pos);
    S.v[a] = R.va;
    S.w[a] = R.wa;
    if (dynb) { S.v[b] = R.vb; S.w[b] = R.wb; }
}

// the pair's row constants (oracle pile_step_ step 3)
__device__ __forceinline__ void pair_constants(PileLds& S, const PairHdr& H) {
    const int a = H.a, b = H.b;
    const bool dynb = b >= 0 && b < ST0;
    const float ima = S.invm[a];
    const S3 Ia = S.Iw[a];
    const V3 va = S.v[a], wa = S.w[a];
    S3 Ib;
    Ib.xx = 0.0f; Ib.yy = 0.0f; Ib.zz = 0.0f; Ib.xy = 0.0f; Ib.xz = 0.0f; Ib.yz = 0.0f;
    float imb = 0.0f;
    V3 vb = v3(0.0f, 0.0f, 0.0f), wb = vb;
    if (dynb) { imb = S.invm[b]; Ib = S.Iw[b]; vb = S.v[b]; wb = S.w[b]; }
    for (int j = 0; j < H.np; ++j) {
        const int c = H.p0 + j;
        const V3 n = S.n[c], ra = S.ra[c], rb = S.rb[c];
        V3 t1, t2;
        env_tangents(n, &t1, &t2);
        S.t1[c] = t1;
        S.t2[c] = t2;
        S.kn[c] = row_k(dynb, n, ra, rb, ima, imb, Ia, Ib);
        S.kt1[c] = row_k(dynb, t1, ra, rb, ima, imb, Ia, Ib);
        S.kt2[c] = row_k(dynb, t2, ra, rb, ima, imb, Ia, Ib);
        const float ua = vdot(n, va) + vdot(vcross(ra, n), wa);
        S.vn0[c] = dynb ? ua - (vdot(n, vb) + vdot(vcross(rb, n), wb)) : ua;
        S.ln[c] = 0.0f;
        S.lt1[c] = 0.0f;
        S.lt2[c] = 0.0f;
    }
}

__global__ void __launch_bounds__(64) k_pile_step(MgStep P, MgPileArgs A) {
    __shared__ PileLds S;
    const int ln = threadIdx.x;
    const int* ei = A.pile_i + (size_t)blockIdx.x * MG_PILE_I_N;
    const int boff = ei[0], nb = ei[1], pr0 = ei[2], npair = ei[3], ns = ei[4], so = ei[9], nsl = ei[10];
    const int N = A.nb;   // SoA stride
    PSTAMP(0);
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
    // local shape slots ln and ln + 64: participant, shape, its offset on the
    // body and bounding radius (pair_near: cA = x + q off, rA)
    int spt[2] = {-1, -1};
    V3 soff[2] = {v3(0.0f, 0.0f, 0.0f), v3(0.0f, 0.0f, 0.0f)};
    float srad[2] = {0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int l = ln + 64 * u;
        if (l < nsl) {
            const int part = A.slots[(size_t)(so + l) * 2 + 0], shp = A.slots[(size_t)(so + l) * 2 + 1];
            const float* sh = A.shapes + (size_t)shp * MG_SHAPE_STRIDE;
            spt[u] = part;
            soff[u] = v3(sh[4], sh[5], sh[6]);
            srad[u] = bound_radius(sh);
            S.slot_part[l] = part;
            S.slot_shape[l] = shp;
        }
    }
    const V3 gvec = v3(P.g[0], P.g[1], P.g[2]);
    const V3 gn = v3(P.n[0], P.n[1], P.n[2]);
    V3 fsum = v3(0.0f, 0.0f, 0.0f);
    PSTAMP(1);

    for (int sub = 0; sub < P.substeps; ++sub) {
        PSTAMP(2);
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
        // the local shapes' bounding spheres (pair_near's first test, op for op)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (spt[u] >= 0) {
                const int pt = spt[u];
                const V3 xp = pt < ST0 ? S.x[pt] : S.sx[pt - ST0];
                const Q4 qp = pt < ST0 ? S.q[pt] : S.sq[pt - ST0];
                const V3 c = vadd(xp, qrot(qp, soff[u]));
                ShapeSphere b;
                b.x = c.x; b.y = c.y; b.z = c.z; b.r = srad[u];
                S.sc[ln + 64 * u] = b;
            }
        }
        __syncthreads();
        PSTAMP(3);

        // ---- 2. narrow phase in pair order: each round screens 64 candidate
        // pairs by their bounding spheres (LDS only) into a ring; every 64
        // survivors (and the rest at the end) run the full pair test and the
        // contacts, compacted in pair order
        int nap = 0, npt = 0, head = 0, tail = 0;
        bool stop = false;
        for (int base = 0; base < npair && !stop; base += 64) {
            const int i = base + ln;
            bool near = false;
            unsigned pv = 0;
            if (i < npair) {
                pv = A.pairs[(size_t)pr0 + i];
                const ShapeSphere sa = S.sc[pv & 0xFF];
                const V3 cA = v3(sa.x, sa.y, sa.z);
                const int lb = (pv >> 8) & 0xFF;
                if (lb == MG_PILE_GROUND) {
                    near = vdot(gn, cA) + P.pd - sa.r < P.contact_offset;
                } else {
                    const ShapeSphere sb = S.sc[lb];
                    const V3 d = vsub(v3(sb.x, sb.y, sb.z), cA);
                    const float rr = sa.r + sb.r + P.contact_offset;
                    near = vdot(d, d) < rr * rr * 1.0001f + 1e-6f;
                }
            }
            const unsigned long long nbal = __ballot(near);
            if (near) {
                const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(nbal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)nbal, 0));
                S.ring[(tail + r) & 127] = pv;
            }
            tail += __popcll(nbal);
            const bool last = base + 64 >= npair;
            while (tail - head >= 64 || (last && tail > head)) {
                __syncthreads();
                const int cnt = tail - head < 64 ? tail - head : 64;
                PairOut o;
                o.n = 0;
                int a = 0, b = -1;
                float mu = 0.0f, e = 0.0f;
                if (ln < cnt) {
                    const unsigned rv = S.ring[(head + ln) & 127];
                    const int la = rv & 0xFF, lb = (rv >> 8) & 0xFF;
                    a = S.slot_part[la];
                    const int sa = S.slot_shape[la];
                    const float* sha = A.shapes + (size_t)sa * MG_SHAPE_STRIDE;
                    const V3 xa = S.x[a];
                    const Q4 qa = S.q[a];
                    if (lb == MG_PILE_GROUND) {   // the screen was pair_near's whole test
                        const CShape sA = place_shape(sha, xa, qa, A.hulls);
                        ground_pair(P, sA, o);
                        mu = 0.5f * (sha[11] + P.mu_ground);
                        e = 0.5f * (sha[12] + P.e_ground);
                    } else {
                        b = S.slot_part[lb];
                        const int sb = S.slot_shape[lb];
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
                head += cnt;
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
                if (__any(over)) { stop = true; break; }
            }
        }
        __syncthreads();
        PSTAMP(4);

        // ---- 3. the lane's pairs (j = ln, ln + 64): headers, row constants
        PairHdr H[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int j = ln + 64 * u;
            H[u].color = -1;
            H[u].rnd = -1;
            H[u].a = 0; H[u].b = -1; H[u].p0 = 0; H[u].np = 0; H[u].mu = 0.0f; H[u].e = 0.0f;
            if (j < nap) {
                H[u].a = S.pa[j]; H[u].b = S.pb[j]; H[u].p0 = S.pt0[j]; H[u].np = S.pn[j];
                H[u].mu = S.pmu[j]; H[u].e = S.pe[j];
                pair_constants(S, H[u]);
            }
        }
        PSTAMP(5);

        // ---- 4. greedy colouring in pair order (oracle: a sequential walk).
        // A batch of 64 pairs (lane = pair) in sub-rounds: a pair is ready once
        // it is the first uncoloured pair of the batch on each of its free
        // bodies (LDS min per body) — every earlier pair on them is then
        // coloured and no later one is — so its bodies' masks hold exactly the
        // colours the sequential walk would see; ready pairs share no body.
        if (act) S.used[ln] = 0ull;
        int ncol = 0, nrnd = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            PairHdr& Hu = H[u];
            const int j = ln + 64 * u;
            const bool dynb = Hu.b >= 0 && Hu.b < ST0;
            bool todo = j < nap;
            unsigned long long left = __ballot(todo);   // wave-uniform
            // each sub-round colours at least the batch's first uncoloured
            // pair: at most 64 sub-rounds (the bound also guards the loop)
            for (int round = 0; left != 0ull && round < 64; ++round) {
                if (todo) {
                    S.first[Hu.a] = 0xFFFFFFFFu;
                    if (dynb) S.first[Hu.b] = 0xFFFFFFFFu;
                }
                __syncthreads();
                if (todo) {
                    atomicMin(&S.first[Hu.a], (unsigned)j);
                    if (dynb) atomicMin(&S.first[Hu.b], (unsigned)j);
                }
                __syncthreads();
                bool ready = false;
                if (todo) ready = S.first[Hu.a] == (unsigned)j && (!dynb || S.first[Hu.b] == (unsigned)j);
                if (ready) {
                    const unsigned long long ua = S.used[Hu.a], ub = dynb ? S.used[Hu.b] : 0ull;
                    const unsigned long long taken = ua | ub;
                    const int c = taken == ~0ull ? -1 : __builtin_ctzll(~taken);
                    Hu.color = c;
                    Hu.rnd = nrnd + round;
                    if (c >= 0) {
                        S.used[Hu.a] = ua | (1ull << c);
                        if (dynb) S.used[Hu.b] = ub | (1ull << c);
                    }
                }
                __syncthreads();
                todo = todo && !ready;
                left = __ballot(todo);
            }
            ncol = max(ncol, wave_max(Hu.color + 1));
            nrnd = max(nrnd, wave_max(Hu.rnd + 1));
        }
        PSTAMP(6);
        PSTAMP(7);

        // ---- 5. TGS: colour by colour, each lane its pairs of that colour;
        // position sweeps (then the motion deltas), velocity sweeps
        for (int itr = 0; itr < P.npos + P.nvel; ++itr) {
            const bool pos = itr < P.npos;
            for (int c = 0; c < ncol; ++c) {
                for (int u = 0; u < 2; ++u) {   // not unrolled: one copy of the rows' code
                    const PairHdr& Hu = u == 0 ? H[0] : H[1];
                    if (Hu.color == c) solve_pair(P, S, Hu, pos, itr == 0);
                }
                __syncthreads();
            }
            if (pos && act) {
                S.dx[ln] = vfma(S.dx[ln], S.v[ln], P.sub);
                S.dth[ln] = vfma(S.dth[ln], S.w[ln], P.sub);
            }
            __syncthreads();
        }
        PSTAMP(8);

        // ---- 6. pose; contact impulses on the lane's body: its list, pair order
        if (act) {
            v = S.v[ln];
            w = S.w[ln];
            const V3 xc1 = vadd(S.xc[ln], S.dx[ln]);
            q = qintegrate(q, S.dth[ln]);
            x = origin_from_com(xc1, q, com);
        }
        // contact impulses per body in pair order: replay the colouring's
        // sub-rounds — a body's pairs were coloured in pair order, at most one
        // per sub-round — each pair lane adding its points to its bodies'
        // sums (oracle: point by point, pair by pair)
        if (act) S.facc[ln] = fsum;
        __syncthreads();
        for (int r = 0; r < nrnd; ++r) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const PairHdr& Hu = H[u];
                if (Hu.rnd == r) {
                    const bool dynb = Hu.b >= 0 && Hu.b < ST0;
                    V3 fa = S.facc[Hu.a];
                    V3 fb = dynb ? S.facc[Hu.b] : v3(0.0f, 0.0f, 0.0f);
                    for (int k = 0; k < Hu.np; ++k) {
                        const int c = Hu.p0 + k;
                        const V3 f = vadd(vadd(vscale(S.n[c], S.ln[c]), vscale(S.t1[c], S.lt1[c])),
                                          vscale(S.t2[c], S.lt2[c]));
                        fa = vadd(fa, f);
                        fb = vsub(fb, f);
                    }
                    S.facc[Hu.a] = fa;
                    if (dynb) S.facc[Hu.b] = fb;
                }
            }
            __syncthreads();
        }
        if (act) fsum = S.facc[ln];
        __syncthreads();
        PSTAMP(9);
        PCOUNT(12, npair);
        PCOUNT(13, nap);
        PCOUNT(14, npt);
        PCOUNT(15, ncol);
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
#ifdef MG_PILE_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PSTAMP(10);
#endif
}

}  // namespace

hipError_t mg_launch_pile_step(const MgStep& P, const MgPileArgs& A, hipStream_t s) {
    if (A.ne <= 0) return hipSuccess;
    MG_LAUNCH(k_pile_step, dim3(A.ne), dim3(64), 0, s, P, A);
    return hipGetLastError();
}
