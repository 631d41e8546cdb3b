// mg_env.hip — coupled per-env step: an env whose bodies touch each other
// (the Franka cube-pick scene of examples/franka_cube_ik_osc.py:111-285: a
// fixed-base arm, a table and a cube in one collision group).
//
// Layout: MG_ENV_G = 16 lanes per env, 4 envs per wavefront (one wave per
// workgroup, per-env state staged in LDS). Lane s owns generalized-velocity
// slot s: the articulation's DOFs first (0..D-1), then 6 slots (v.xyz, w.xyz)
// per free body, so every contact row is a 16-lane vector pair (J, W = M^-1 J^T)
// held in registers and every Gauss-Seidel row update is
//   vrel = sum_lanes J u  (4 DPP steps within the 16-lane row),
//   u   += W dlambda      (one multiply-add per lane).
// Per substep:
//   1. lane 0: articulated-body algorithm (as mg_artic.hip, implicit drives,
//      effort-limit re-solve) and forward kinematics into LDS; free bodies:
//      gravity, external force, damping, speed clamps;
//   2. all lanes: narrow phase, one candidate shape pair per lane per round
//      (mg_collide.h), contacts placed by a 16-lane prefix sum in pair order;
//   3. if a link is in contact: lane 0 builds M_eff = CRBA mass matrix +
//      armature + the implicit drive terms ABA added to D, Cholesky; lane j
//      solves column j of M_eff^-1; each lane forms its slot of J and W for the
//      rows n, t1, t2 of every contact;
//   4. TGS: npos position iterations (all normal rows, then all friction rows;
//      separation s0 + J_n . dpos), nvel velocity iterations; 5. integrate.
// Static bodies and the fixed base link have no slots (infinite mass).
// Restated in C by oracle/migym_oracle_env.c, with the same pair order, the
// same reduction tree (red16) and the same evaluation order.
#include <type_traits>

#include "mg_internal.h"
#include "mg_spatial.h"
#include "mg_collide.h"
#include "mg_pairs.h"
#include "mg_world.h"

#ifdef MG_ENV_PHASE_TIMING
// profiling build only: per-phase shader-clock cycles summed over waves
__device__ unsigned long long g_env_phase[24];
#define PH_T0() unsigned long long ph_t = clock64()
#define PH_MARK(k) do { const unsigned long long t_ = clock64(); \
    if (threadIdx.x == 0) atomicAdd(&g_env_phase[k], t_ - ph_t); ph_t = t_; } while (0)
#define PH_COUNT(k, v) atomicAdd(&g_env_phase[k], (unsigned long long)(v))
#define PH_SUB(k) do { const unsigned long long t_ = clock64(); \
    if (threadIdx.x == 0) atomicAdd(&g_env_phase[k], t_ - ph_sub); ph_sub = t_; } while (0)
extern "C" int mg_debug_env_phase(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_env_phase), sizeof(g_env_phase)) == hipSuccess ? 0 : -1;
}
extern "C" int mg_debug_env_phase_reset(void) {
    unsigned long long z[24] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_env_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#else
#define PH_T0() do { } while (0)
#define PH_MARK(k) do { } while (0)
#define PH_COUNT(k, v) do { } while (0)
#define PH_SUB(k) do { } while (0)
#endif
// np_collide's parts (profiling build): pair setup, one-lane pair tests, the
// cooperative convex loop, contact placement
#ifdef MG_ENV_PHASE_TIMING
#define PH_NP0() unsigned long long ph_np = clock64()
#define PH_NP(k) do { const unsigned long long t_ = clock64(); \
    if (threadIdx.x == 0) atomicAdd(&g_env_phase[k], t_ - ph_np); ph_np = t_; } while (0)
#else
#define PH_NP0() do { } while (0)
#define PH_NP(k) do { } while (0)
#endif

namespace {

// G: lanes per env, a template parameter of the kernels: 16 (4 envs per
// wavefront, DPP row reductions) or 64 (one env per wavefront: articulations of
// more than 16 links or velocity slots, the MJCF humanoid's 25 links and 27
// slots; reductions by row, then readlane across the four rows)
constexpr int G16 = MG_ENV_G;
// contacts per env per substep: 16, or 48 in a 64-lane env (a humanoid on the
// ground has ~35 capsule end caps; the rows then live partly in scratch)
template <int G>
constexpr int maxct() { return G == 64 ? MG_ENV_MAXCT_WIDE : MG_ENV_MAXCT; }
constexpr int MAXF = MG_ENV_MAXF;
constexpr int F0 = MG_ENV_FREE0;
constexpr int ST0 = MG_ENV_STATIC0;
constexpr int LIM0 = MG_ENV_LIMIT0;
constexpr int NPB = 64;               // candidate pairs per screening block
// carry record of one env between the substep launches of k_env_step
constexpr int MG_CARRY_HDR = 24;     // x0 (3), q0 (4), free body k: x (3), q (4) at 7 + 7k
constexpr int MG_CARRY_LANE = 8;     // per lane: qv, uv, lsum.xyz, fsum.xyz
constexpr int MG_CARRY_LINK = 7;     // per link (after the lanes): its pose at the next substep's start
template <int G>
constexpr int carry_n() { return MG_CARRY_HDR + MG_CARRY_LANE * G + MG_CARRY_LINK * MG_MAX_LINKS; }
template <int G>
constexpr int carry_link0() { return MG_CARRY_HDR + MG_CARRY_LANE * G; }
// MG_ENV_FK_CARRY: a substep's launch leaves the link poses at the next
// substep's start (forward kinematics of its integrated q, the same operations
// the next launches would run) in the carry record, so the next substep's
// k_env_np and k_env_step read them instead of each running the kinematic scan
// MG_ENV_SWEEP_ANF (experiment): a position sweep solves the anchors' rows then
// the normal rows (only the first opens with the normal rows), the free-body
// kernel's order since round 6 (mg_rigid.hip); 0: normal, anchor rows, the
// last position sweep and the velocity sweeps closing with the normal rows
#ifndef MG_ENV_SWEEP_ANF
#define MG_ENV_SWEEP_ANF 0
#endif
#ifndef MG_ENV_FK_CARRY
#define MG_ENV_FK_CARRY 1
#endif

template <int MAXL, int G>
struct EnvLds {
    static constexpr int NDM = G > 32 ? 32 : G;   // velocity slots of the M_eff solve
    static constexpr int MAXCT = maxct<G>();
    float q[G], u[G], qdd[G], dpos[G], mdiag[G];
    V3 xl[MAXL], zl[MAXL];
    Q4 ql[MAXL];
    unsigned amask[MAXL];            // DOF bits of the joints on the path root -> l
    int dlink[G];                    // link whose joint is DOF d
    int drev[G];                     // DOF d is revolute
    V3 fx[MAXF], fxc[MAXF];
    Q4 fq[MAXF];
    float finvm[MAXF];
    S3 fIw[MAXF];
    float Lc[NDM][NDM];              // M_eff, assembled by the DOF lanes
    int ca[MAXCT], cb[MAXCT];
    V3 cp[MAXCT], cd[MAXCT][3];      // point, (n, t1, t2)
    float cs0[MAXCT], ce[MAXCT], cvn0[MAXCT];
    float ck[MAXCT][3], clam[MAXCT][3];
    int nct, link_rows;
    // world-frame articulated-body quantities (about the base origin x0)
    float Iw[MAXL][36];              // spatial inertia -> articulated / composite inertia, row-major 6x6
    float xi[MAXL][6];               // joint motion axis (w, v at x0)
    float va[MAXL][6];               // link velocity, then acceleration
    float cc[MAXL][6];               // velocity-product acceleration
    float pa[MAXL][6];               // bias force
    float Ua[MAXL][6];               // IA xi
    float Dd[MAXL], uu[MAXL];
    Q4 qr[MAXL];                     // joint rotation / offset relative to the parent
    V3 rr[MAXL];
    float tau0[G], imp[G], arm[G];
    float ru[6];                     // floating root: (w, v_O) after the unconstrained update
    // friction anchors (patch friction): anchor k's point (its
    // A copy, world), position-sweep target velocities closing the drift of its
    // two copies along the patch tangents
    // (cd[k][1], cd[k][2]), friction coefficient, participants a | b << 16, last
    // contact of its patch | partner anchor (1: next, 2: previous) << 8 | pair << 10
    V3 apt[MAXCT];
    float ae[MAXCT][2], amu[MAXCT];
    int aab[MAXCT], alast[MAXCT];
    float psum[MAXCT];               // running normal impulse of each contact's patch
    unsigned long long pstart;       // contacts that open a patch
};
// the step kernel's LDS: a 64-lane env's rows (48 contacts x 3) do not fit in
// registers beside the rest of the step (round 4: 1,872 B of scratch per lane):
// their J and W in LDS [row][slot] (slots < 32), their impulses (the same in
// every lane) too. 16-lane envs keep them in registers.
template <int MAXL, int G>
struct EnvStepLds : EnvLds<MAXL, G> {
    static constexpr int MAXCT = maxct<G>();
    float Jl[G == 64 ? MAXCT * 3 : 1][G == 64 ? 32 : 1];
    float Wl[G == 64 ? MAXCT * 3 : 1][G == 64 ? 32 : 1];
    float laml[G == 64 ? MAXCT * 3 : 1];
};



// sum over the 16 lanes of a DPP row, the same value in every lane:
// ror 8, ror 4, quad xor 2, quad xor 1 (oracle: red16)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float red16(float v) {
    v = v + dpp<0x128>(v);   // row_ror:8
    v = v + dpp<0x124>(v);   // row_ror:4
    v = v + dpp<0x4E>(v);    // quad_perm [2,3,0,1]
    v = v + dpp<0xB1>(v);    // quad_perm [1,0,3,2]
    return v;
}
// the same over a G-lane env: G = 64 adds the four row sums read lane by lane,
// (r0 + r1) + (r2 + r3) (oracle: red_)
__device__ __forceinline__ float rdlane(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
template <int G>
__device__ __forceinline__ float redg(float v) {
    v = red16(v);
    if constexpr (G == 64) return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
    return v;
}
// lane k of the 16-lane row, to every lane of the row (DPP row_newbcast:k,
// a VALU operand modifier on gfx950: no LDS round trip). k must fold to a
// constant (fully unrolled loops).
__device__ __forceinline__ float bcast16(float v, int k) {
    switch (k) {
    case 0: return dpp<0x150>(v);  case 1: return dpp<0x151>(v);
    case 2: return dpp<0x152>(v);  case 3: return dpp<0x153>(v);
    case 4: return dpp<0x154>(v);  case 5: return dpp<0x155>(v);
    case 6: return dpp<0x156>(v);  case 7: return dpp<0x157>(v);
    case 8: return dpp<0x158>(v);  case 9: return dpp<0x159>(v);
    case 10: return dpp<0x15A>(v); case 11: return dpp<0x15B>(v);
    case 12: return dpp<0x15C>(v); case 13: return dpp<0x15D>(v);
    case 14: return dpp<0x15E>(v); default: return dpp<0x15F>(v);
    }
}
// lane k of the env to every lane of it (G = 64: readlane, k wave-uniform)
template <int G>
__device__ __forceinline__ float bcastg(float v, int k) {
    if constexpr (G == 64) return rdlane(v, k);
    return bcast16(v, k);
}

// a row's J of this lane's slot: registers (16-lane envs) or EnvLds::Jl (64)
template <int G, int N>
struct RowJ {
    float v[N];
    __device__ __forceinline__ float get(int r, int) const { return v[r]; }
    __device__ __forceinline__ void set(int r, int, float x) { v[r] = x; }
    __device__ __forceinline__ float lane(int r, int ln, int k) const { return bcastg<G>(v[r], k); }
};
template <int N>
struct RowJ<64, N> {
    float (*p)[32];
    __device__ __forceinline__ float get(int r, int ln) const { return ln < 32 ? p[r][ln] : 0.0f; }
    __device__ __forceinline__ void set(int r, int ln, float x) { if (ln < 32) p[r][ln] = x; }
    __device__ __forceinline__ float lane(int r, int, int k) const { return p[r][k]; }   // k < 32: a slot
};
// a row's accumulated impulse (the same value in every lane of the env)
template <int G, int N>
struct RowL {
    float v[N];
    __device__ __forceinline__ float get(int r) const { return v[r]; }
    __device__ __forceinline__ void set(int r, float x) { v[r] = x; }
};
template <int N>
struct RowL<64, N> {
    float* p;
    __device__ __forceinline__ float get(int r) const { return p[r]; }
    __device__ __forceinline__ void set(int r, float x) { p[r] = x; }
};

// ---- cooperative convex-convex narrow phase ---------------------------------
// A pair of convex shapes (box or hull, at least one hull) on all 16 lanes of
// an env group: the same result, in every lane, as convex_convex (mg_collide.h)
// on one lane. Vertex i of A is tested on lane i % 16 (candidate order i),
// vertex i of B likewise (order 64 + i), edges the same way (order e). Every
// per-vertex / per-edge result is computed by the sequential code's own
// functions (cvx_vertex_one, cvx_edge_one); each lane keeps its candidates in
// order, and the group merges the 4 smallest (separation, order) keys — the
// set and the order deep4_add's in-order insertion keeps (ties go to the
// earlier candidate). So no oracle change: oracle/migym_oracle_env.c's
// sequential convex_convex_ is the definition.
struct CandQ {
    int n;
    float s[MG_PAIR_MAXC];
    int id[MG_PAIR_MAXC];
    V3 p[MG_PAIR_MAXC], nrm[MG_PAIR_MAXC];
};
__device__ __forceinline__ void candq_add(CandQ& Q, float s, int id, V3 p, V3 n) {
    // ids arrive in increasing order per lane: deep4_add's rule
    if (Q.n == MG_PAIR_MAXC && !(s < Q.s[MG_PAIR_MAXC - 1])) return;
    int at = 0;
#pragma unroll
    for (int k = 0; k < MG_PAIR_MAXC; ++k)
        if (k < Q.n && Q.s[k] <= s) at = k + 1;
    // every slot through selects, top down (an indexed insert kept the queue in
    // scratch: a memory round trip per candidate)
#pragma unroll
    for (int k = MG_PAIR_MAXC - 1; k >= 0; --k) {
        const int km = k > 0 ? k - 1 : 0;
        const bool sh = k > at, put = k == at;
        Q.s[k] = sh ? Q.s[km] : (put ? s : Q.s[k]);
        Q.id[k] = sh ? Q.id[km] : (put ? id : Q.id[k]);
        Q.p[k] = vsel(sh, Q.p[km], vsel(put, p, Q.p[k]));
        Q.nrm[k] = vsel(sh, Q.nrm[km], vsel(put, n, Q.nrm[k]));
    }
    if (Q.n < MG_PAIR_MAXC) Q.n = Q.n + 1;
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ void minkey_step(float& s, int& id) {
    const float s2 = dpp<CTRL>(s);
    const int i2 = dppi<CTRL>(id);
    if (s2 < s || (s2 == s && i2 < id)) { s = s2; id = i2; }
}
// the smallest (s, id) of the env's lanes, in every lane (G = 64: the rows'
// minima read lane by lane; min with ties by id is order-free)
template <int G>
__device__ __forceinline__ void grp_minkey(float& s, int& id) {
    minkey_step<0x128>(s, id);   // row_ror:8
    minkey_step<0x124>(s, id);   // row_ror:4
    minkey_step<0x4E>(s, id);    // quad_perm [2,3,0,1]
    minkey_step<0xB1>(s, id);    // quad_perm [1,0,3,2]
    if constexpr (G == 64) {
        float bs = rdlane(s, 0);
        int bi = __builtin_amdgcn_readlane(id, 0);
#pragma unroll
        for (int r = 16; r < 64; r += 16) {
            const float s2 = rdlane(s, r);
            const int i2 = __builtin_amdgcn_readlane(id, r);
            if (s2 < bs || (s2 == bs && i2 < bi)) { bs = s2; bi = i2; }
        }
        s = bs;
        id = bi;
    }
}
template <int CTRL>
__device__ __forceinline__ void bounds_step(V3& lo, V3& hi) {
    lo = v3(fminf(lo.x, dpp<CTRL>(lo.x)), fminf(lo.y, dpp<CTRL>(lo.y)), fminf(lo.z, dpp<CTRL>(lo.z)));
    hi = v3(fmaxf(hi.x, dpp<CTRL>(hi.x)), fmaxf(hi.y, dpp<CTRL>(hi.y)), fmaxf(hi.z, dpp<CTRL>(hi.z)));
}
// vertex bounds over the env's lanes (min / max are exact: order-free)
template <int G>
__device__ __forceinline__ void grp_bounds(V3& lo, V3& hi) {
    bounds_step<0x128>(lo, hi);
    bounds_step<0x124>(lo, hi);
    bounds_step<0x4E>(lo, hi);
    bounds_step<0xB1>(lo, hi);
    if constexpr (G == 64) {
        V3 l = lo, h = hi;
#pragma unroll
        for (int r = 16; r < 64; r += 16) {
            l = v3(fminf(l.x, rdlane(lo.x, r)), fminf(l.y, rdlane(lo.y, r)), fminf(l.z, rdlane(lo.z, r)));
            h = v3(fmaxf(h.x, rdlane(hi.x, r)), fmaxf(h.y, rdlane(hi.y, r)), fmaxf(h.z, rdlane(hi.z, r)));
        }
        lo = v3(rdlane(l.x, 0), rdlane(l.y, 0), rdlane(l.z, 0));
        hi = v3(rdlane(h.x, 0), rdlane(h.y, 0), rdlane(h.z, 0));
    }
}
// ballot of the env's lanes (bit ln)
template <int G>
__device__ __forceinline__ unsigned long long grp_ballot(bool b, int gi) {
    if constexpr (G == 64) return __ballot(b);
    return (__ballot(b) >> (gi * G)) & 0xFFFFull;
}
// the cooperative hull loops' chunk: MG_NP_HULL_CHUNK vertices (3x as many
// edges) per pass of the group, the importer's default hull in one pass; a finer
// hull (up to MG_HULL_MAX_VERTS) takes more passes, in index order
#ifndef MG_NP_HULL_CHUNK
#define MG_NP_HULL_CHUNK 32
#endif
// B's vertex candidates order after every vertex of A (coop_convex_convex)
#define MG_NP_BVERT_ORDER 256
static_assert(MG_NP_BVERT_ORDER > MG_HULL_MAX_VERTS, "vertex order keys of A and B overlap");
// X's edges against Y on the group, into each lane's queue (order = edge index).
// A lane's edges (e = base + ln + G k, 6 per chunk on 16 lanes) in batches of
// 3: all the batch's edge ids, then all its endpoints are loaded before any is
// tested (two dependent round trips per batch, not two per edge)
template <int G>
__device__ __forceinline__ void coop_edges(const CShape& X, const CShape& Y, float margin, bool onY, V3 lo, V3 hi,
                                           int ln, CandQ& Q) {
    V3 t;
    M3 M;
    float ry;
    if (!cvx_edges_gate(X, Y, margin, lo, hi, t, M, ry)) return;
    const int ne = cvx_ne(X);
    constexpr int CE_PER_LANE = (3 * MG_NP_HULL_CHUNK + G - 1) / G;
    for (int base = 0; base < ne; base += G * CE_PER_LANE) {
#pragma unroll
        for (int k0 = 0; k0 < CE_PER_LANE; k0 += 3) {
            if (base + ln + G * k0 >= ne) break;
            int ia[3], ib[3];
            V3 la[3], lb[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int e = base + ln + G * (k0 + k);
                cvx_edge_ids(X, e < ne ? e : ne - 1, ia[k], ib[k]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                la[k] = cvx_vertex_l(X, ia[k]);
                lb[k] = cvx_vertex_l(X, ib[k]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int e = base + ln + G * (k0 + k);
                if (e < ne) {
                    Deep4 T;
                    T.n = 0;
                    cvx_edge_one(Y, margin, onY, t, M, ry, la[k], lb[k], T);
                    if (T.n) candq_add(Q, T.s[0], e, T.p[0], T.nrm[0]);
                }
            }
        }
    }
}
// X's vertices (i = base + ln + G k: 2 per lane per chunk on 16 lanes) against
// Y's planes, into the lane's queue (order idbase + i); all the chunk's vertices
// loaded before any is tested. (Round 6: the bound was a literal 2, so a build
// with a larger vertex cap skipped the vertices past 32 while the oracle tested
// them; now any hull up to MG_HULL_MAX_VERTS, chunk by chunk.)
template <int G>
__device__ __forceinline__ void coop_vertices(const CShape& X, const CShape& Y, float margin, bool onY, int idbase,
                                              int ln, CandQ& Q, V3& lo, V3& hi) {
    constexpr int CV_PER_LANE = (MG_NP_HULL_CHUNK + G - 1) / G;
    const int nv = cvx_nv(X);
    for (int base = 0; base < nv; base += G * CV_PER_LANE) {
        V3 vw[CV_PER_LANE];
#pragma unroll
        for (int k = 0; k < CV_PER_LANE; ++k) {
            const int i = base + ln + G * k;
            vw[k] = cvx_vertex(X, i < nv ? i : nv - 1);
        }
#pragma unroll
        for (int k = 0; k < CV_PER_LANE; ++k) {
            const int i = base + ln + G * k;
            if (i < nv) {
                const V3 v = vw[k];
                aabb_add(lo, hi, mtmul(Y.R, vsub(v, Y.c)));
                int f;
                const float sv = cvx_sd(Y, v, f, 0.0f, margin);     // cvx_vertex_one's candidate
                if (sv < margin) {
                    const V3 n = cvx_normal(Y, f);
                    if (onY) candq_add(Q, sv, idbase + i, vsub(v, vscale(n, sv)), vscale(n, -1.0f));
                    else candq_add(Q, sv, idbase + i, v, n);
                }
            }
        }
    }
}
// every lane of the group calls it with the same pair (group-uniform control)
template <int G>
__device__ __forceinline__ void coop_convex_convex(const CShape& A, const CShape& B, float margin, int ln, int gi,
                                                   PairOut& o) {
#ifdef MG_ENV_PHASE_TIMING
    unsigned long long ph_sub = clock64();
#endif
    CandQ Q;
    Q.n = 0;
    V3 loA = v3(1e30f, 1e30f, 1e30f), hiA = v3(-1e30f, -1e30f, -1e30f), loB = loA, hiB = hiA;
    coop_vertices<G>(A, B, margin, false, 0, ln, Q, loA, hiA);     // A's vertices by B's planes
    coop_vertices<G>(B, A, margin, true, MG_NP_BVERT_ORDER, ln, Q, loB, hiB);     // B's vertices by A's planes
    PH_SUB(12);
    if (grp_ballot<G>(Q.n > 0, gi) == 0ull) {
        // no vertex candidate: edge crossings (convex_convex's order of passes)
        grp_bounds<G>(loA, hiA);
        grp_bounds<G>(loB, hiB);
        if (A.type == MG_SHAPE_BOX && B.type != MG_SHAPE_BOX) {
            coop_edges<G>(B, A, margin, true, loB, hiB, ln, Q);
        } else {
            coop_edges<G>(A, B, margin, false, loA, hiA, ln, Q);
            if (B.type != MG_SHAPE_BOX && grp_ballot<G>(Q.n > 0, gi) == 0ull)
                coop_edges<G>(B, A, margin, true, loB, hiB, ln, Q);
        }
        PH_COUNT(15, 1);
    }
    PH_SUB(13);
    // merge: the group's smallest (s, order) keys, ascending
    o.n = 0;
#pragma unroll
    for (int r = 0; r < MG_PAIR_MAXC; ++r) {
        if (grp_ballot<G>(Q.n > 0, gi) == 0ull) break;     // group-uniform: nothing left
        float s = Q.n > 0 ? Q.s[0] : 3.0e38f;
        int id = Q.n > 0 ? Q.id[0] : 0x7fffffff;
        grp_minkey<G>(s, id);
        const unsigned long long m = grp_ballot<G>(Q.n > 0 && Q.id[0] == id, gi);
        const int owner = m ? __ffsll(m) - 1 : 0;
        const V3 p = v3(__shfl(Q.p[0].x, owner, G), __shfl(Q.p[0].y, owner, G), __shfl(Q.p[0].z, owner, G));
        const V3 n = v3(__shfl(Q.nrm[0].x, owner, G), __shfl(Q.nrm[0].y, owner, G), __shfl(Q.nrm[0].z, owner, G));
        if (m != 0ull && ln == owner) {         // pop the head
#pragma unroll
            for (int k = 0; k + 1 < MG_PAIR_MAXC; ++k) {
                Q.s[k] = Q.s[k + 1]; Q.id[k] = Q.id[k + 1]; Q.p[k] = Q.p[k + 1]; Q.nrm[k] = Q.nrm[k + 1];
            }
            Q.n = Q.n - 1;
        }
        if (m != 0ull) pair_push(o, p, n, s);
    }
    PH_SUB(14);
}
// lane k's placed shape, to every lane of the group (ds_bpermute: no global
// round trips for the pair record, the shape rows and the poses)
template <int G>
__device__ __forceinline__ V3 shfl3(V3 v, int k) { return v3(__shfl(v.x, k, G), __shfl(v.y, k, G), __shfl(v.z, k, G)); }
template <int G>
__device__ __forceinline__ CShape shfl_shape(const CShape& c, int k) {
    CShape r;
    r.type = __shfl(c.type, k, G);
    r.c = shfl3<G>(c.c, k);
    r.R.c0 = shfl3<G>(c.R.c0, k);
    r.R.c1 = shfl3<G>(c.R.c1, k);
    r.R.c2 = shfl3<G>(c.R.c2, k);
    r.h = shfl3<G>(c.h, k);
    const unsigned long long hp = (unsigned long long)(uintptr_t)c.hv;
    const unsigned lo = __shfl((unsigned)(hp & 0xFFFFFFFFull), k, G), hi = __shfl((unsigned)(hp >> 32), k, G);
    r.hv = (const float*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
    return r;
}

// place of DOF d in a ball joint (1, 2, 3; 0: not a ball DOF): link_f[10] of
// the link it drives (mg_spatial.h, exponential coordinates)
__device__ __forceinline__ int dof_ball(const MgEnvArgs& A, int LA, int d) {
    int r = 0;
    for (int l = 0; l < LA; ++l)
        if (A.link_i[l * MG_LINK_I_N + 2] == d) r = (int)A.link_f[l * MG_LINK_F_N + 10];
    return r;
}
// a ball DOF lane's new position: component k of log(exp(th) exp(dth)), th and
// dth the three DOFs' values in q[] and dq[] (LDS), f the ball's first DOF
__device__ __forceinline__ float ball_dof_step(const float* q, const float* dq, int f, int k) {
    const V3 tn = ball_step(v3(q[f], q[f + 1], q[f + 2]), v3(dq[f], dq[f + 1], dq[f + 2]));
    return k == 1 ? tn.x : (k == 2 ? tn.y : tn.z);
}

// substep-invariant per-lane constants: lane d < D holds DOF d's drive
// properties and targets (link constants: LinkC, mg_world.h)
struct DofC {
    int mode, haslim;
    float kp, kd, eff, maxv, lo, hi, arm, tpos, tvel, force;
};
struct FreeC {
    V3 invI, com, fext, text;
    Q4 iq;
    float lkeep, akeep, mlv2, mav2, gon;
};

// pose of a pair participant: link l (< F0), free body F0 + k, static body ST0 + s
template <class SL>
__device__ __forceinline__ void pair_pose(const SL& S, int id, V3& x, Q4& q) {
    if (id >= ST0) { x = S.sx[id - ST0]; q = S.sq[id - ST0]; }
    else if (id >= F0) { x = S.fx[id - F0]; q = S.fq[id - F0]; }
    else { x = S.xl[id]; q = S.ql[id]; }
}

// ---- friction patches -------------------------------------
// PhysX friction is patch friction: a shape pair's friction rows act at up to
// two anchors, each fixed on both bodies, kept from substep to substep and
// from step to step while the pair stays in contact (Isaac Gym exposes its two
// parameters, examples/franka_cube_ik_osc.py:124-125). Per substep, on the
// pair's lane: the patch is dropped when its normal turned (cos <
// MG_FP_NORMAL_COS); an anchor is dropped when its two copies drifted apart by
// more than the correlation distance; then anchors grow from this substep's
// contacts in emitted order — the first contact within the friction offset
// threshold, then the first one farther than the correlation distance from
// anchor 0 — fixed on both bodies at the contact point. The friction rows of
// an anchor close the drift of its two copies along the patch tangents (TGS
// position target, like a normal row's separation) and share the patch's
// Coulomb bound mu * (sum of its contacts' normal impulses) equally; a patch
// whose bound clamps a row in the last iteration is slipping and re-anchors at
// the next substep. Oracle: patch_update_ (migym_oracle_env.c).
struct Patch {
    int cnt;
    V3 nA;          // patch normal in A's body frame
    V3 aA[2], aB[2];
};
MG_HD void patch_load(Patch& R, const float* r) {
    R.cnt = (int)r[0];
    R.nA = v3(r[1], r[2], r[3]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        R.aA[k] = v3(r[4 + 6 * k], r[5 + 6 * k], r[6 + 6 * k]);
        R.aB[k] = v3(r[7 + 6 * k], r[8 + 6 * k], r[9 + 6 * k]);
    }
}
MG_HD void patch_store(const Patch& R, float* r) {
    r[0] = (float)R.cnt;
    r[1] = R.nA.x; r[2] = R.nA.y; r[3] = R.nA.z;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        r[4 + 6 * k] = R.aA[k].x; r[5 + 6 * k] = R.aA[k].y; r[6 + 6 * k] = R.aA[k].z;
        r[7 + 6 * k] = R.aB[k].x; r[8 + 6 * k] = R.aB[k].y; r[9 + 6 * k] = R.aB[k].z;
    }
}
// R: the pair's patch of the last substep (cnt 0: none) -> this substep's
MG_HD void patch_update(Patch& R, V3 xa, Q4 qa, V3 xb, Q4 qb, const PairOut& o, float fot, float corr) {
    const V3 n0 = o.nrm[0];
    const float c2 = corr * corr;
    int cnt = R.cnt;
    if (cnt > 0 && vdot(qrot(qa, R.nA), n0) < MG_FP_NORMAL_COS) cnt = 0;
    Patch N;
    N.cnt = 0;
    N.aA[0] = N.aA[1] = N.aB[0] = N.aB[1] = v3(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k < cnt) {
            const V3 d = vsub(vadd(xa, qrot(qa, R.aA[k])), vadd(xb, qrot(qb, R.aB[k])));
            if (vdot(d, d) <= c2) {
                if (N.cnt == 0) { N.aA[0] = R.aA[k]; N.aB[0] = R.aB[k]; }
                else { N.aA[1] = R.aA[k]; N.aB[1] = R.aB[k]; }
                N.cnt = N.cnt + 1;
            }
        }
    }
    // growth (PhysX growPatches; mg_rigid.hip ground_patch_update): a patch
    // still holding two anchors keeps them; otherwise the contacts within the
    // friction offset threshold, in emitted order, give anchor 0, then anchor 1
    // (the first farther than the correlation distance from anchor 0), then
    // each later one replaces the anchor it is nearer to when it lies farther
    // from the other than the two are apart (the anchors spread)
    const int kept = N.cnt;   // anchors kept from the last substep
    const bool grow = N.cnt < 2;
    V3 w0 = N.cnt > 0 ? vadd(xa, qrot(qa, N.aA[0])) : v3(0.0f, 0.0f, 0.0f), w1 = v3(0.0f, 0.0f, 0.0f);
    float dd = 0.0f;
#pragma unroll
    for (int j = 0; j < MG_PAIR_MAXC; ++j) {
        if (grow && j < o.n && o.sep[j] <= fot) {
            const V3 pj = o.p[j];
            int put = -1;
            if (N.cnt == 0) {
                put = 0;
            } else if (N.cnt == 1) {
                const V3 d = vsub(pj, w0);
                const float d2 = vdot(d, d);
                if (d2 > c2) { put = 1; dd = d2; }
            } else {
                const V3 e0 = vsub(pj, w0), e1 = vsub(pj, w1);
                const float d0 = vdot(e0, e0), d1 = vdot(e1, e1);
                if (d0 > d1) {
                    if (d0 > dd) { put = 1; dd = d0; }
                } else if (d1 > dd) {
                    put = 0;
                    dd = d1;
                }
            }
            if (put >= 0) {
                const V3 la = qrot_inv(qa, vsub(pj, xa)), lb = qrot_inv(qb, vsub(pj, xb));
                if (put == 0) { N.aA[0] = la; N.aB[0] = lb; w0 = pj; }
                else { N.aA[1] = la; N.aB[1] = lb; w1 = pj; }
                if (N.cnt <= put) N.cnt = put + 1;
            }
        }
    }
    // the patch normal is the one the patch was created with while it keeps an
    // anchor (a slowly tilting contact still drops it past MG_FP_NORMAL_COS)
    N.nA = kept > 0 ? R.nA : qrot_inv(qa, n0);
    R = N;
}

// x = M^-1 b for a symmetric positive definite 6x6 M (row-major): left-looking
// Cholesky, forward and backward substitution (oracle: spd6_solve_)
MG_HD void spd6_solve(const float* M, const float* b, float* x) {
    float Lm[36], y[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        float sj = M[j * 6 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) sj = sj - Lm[j * 6 + k] * Lm[j * 6 + k];
        const float dj = sqrtf(sj);
        const float inv = 1.0f / dj;
        Lm[j * 6 + j] = dj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            float t = M[i * 6 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) t = t - Lm[i * 6 + k] * Lm[j * 6 + k];
            Lm[i * 6 + j] = t * inv;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        float t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t = t - Lm[i * 6 + k] * y[k];
        y[i] = t / Lm[i * 6 + i];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        float t = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) t = t - Lm[k * 6 + i] * x[k];
        x[i] = t / Lm[i * 6 + i];
    }
}

// Articulated-body algorithm in the world frame about the base origin x0 (RBDA
// ch. 7 with all quantities in one frame: no spatial transforms in the inward
// pass). Every lane of the workgroup calls it (the barriers are shared); `act`
// selects the envs that do work. Lane l computes link l's joint transform,
// axis and inertia; lanes 0..5 own one spatial component in the outward scans;
// lane ln owns entries {ln, ln+16, ln+32} of every 6x6 in the inward pass.
// Implicit drives (h kd + h^2 kp added to D); a drive whose implicit force
// exceeds its effort limit is re-solved at the limit (xmask / xpos).
// Floating base (A.floating): link 0 moves with the root spatial velocity held
// by slots DA..DA+5; the inward pass also folds into link 0 and the root
// acceleration solves IA_0 a0 = -pA_0 (a0 relative to gravity, as the fixed
// base's a0 = -g). External wrenches at link COMs (A.ext) enter the bias forces.
// The articulated-body algorithm is split so that the effort-limit re-solve
// (a second pass with the flagged drives at constant force) repeats only what
// the drives change: aba_kin (joint transforms, forward kinematics, motion
// axes, world inertias, velocities, velocity-product terms) runs once per
// substep; aba_dyn (drive terms, inward and outward passes) per attempt, after
// aba_refresh restores the world inertias and bias forces the previous inward
// pass accumulated into, and the link velocities its outward pass overwrote
// (recomputed: the same values bit for bit).
template <int MAXL, int G>
__device__ __forceinline__ void aba_vp(const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA, V3 x0,
                                       const LinkC& lk, int b0) {
    // ---- velocity-product terms (lane l)
    if (act && ln < LA) {
        const int dof = A.link_i[ln * MG_LINK_I_N + 2];
        const float qd = dof >= 0 ? S.u[dof] : 0.0f;
        const SV v = sv6(S.va[ln]);
        const SV vJ = svscale(sv6(S.xi[ln]), qd);
        float Iv[6];
        for (int i = 0; i < 6; ++i) Iv[i] = dot6(&S.Iw[ln][i * 6], S.va[ln]);
        // a ball joint's later links: the velocity product with the ball's
        // parent (its three axes are fixed in the child frame: the bias of the
        // joint is v_parent x vJ, not the chain's v_{l-1} x vJ_l)
        const int ball = (int)A.link_f[ln * MG_LINK_F_N + 10];
        SV vb = v;
        if (ball >= 2) {
            int pb = A.link_i[ln * MG_LINK_I_N + 0];
            pb = A.link_i[pb * MG_LINK_I_N + 0];
            if (ball == 3) pb = A.link_i[pb * MG_LINK_I_N + 0];
            vb = sv6(S.va[pb]);
        }
        put6(S.cc[ln], crm(vb, vJ));
        SV pb = crf(v, sv6(Iv));
        const int bl = A.link_i[ln * MG_LINK_I_N + 3];      // -1: virtual link
        if (A.ext && bl >= 0) {
            // world force f and torque t at the link COM: the wrench about x0
            const int b = b0 + bl, nb = A.nb;
            const V3 f = v3(A.ext[0 * nb + b], A.ext[1 * nb + b], A.ext[2 * nb + b]);
            const V3 t = v3(A.ext[3 * nb + b], A.ext[4 * nb + b], A.ext[5 * nb + b]);
            const V3 c = vsub(vadd(S.xl[ln], qrot(S.ql[ln], lk.com)), x0);
            pb = sv(vsub(pb.w, vadd(t, vcross(c, f))), vsub(pb.v, f));
        }
        put6(S.pa[ln], pb);
    }
    __syncthreads();
}

// link velocities (lanes 0..5, one component each) from the joint speeds: the
// outward pass of aba_dyn leaves accelerations in S.va, so a re-solve
// recomputes them before its velocity-product terms
template <int MAXL, int G>
__device__ __forceinline__ void aba_vel(const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA) {
    const bool fb = A.floating != 0;
    const int DA = A.ndof;
    if (act && ln < 6) {
        S.va[0][ln] = fb ? S.u[DA + ln] : 0.0f;
        for (int l = 1; l < LA; ++l) {
            const int p = A.link_i[l * MG_LINK_I_N + 0], dof = A.link_i[l * MG_LINK_I_N + 2];
            const float qd = dof >= 0 ? S.u[dof] : 0.0f;
            S.va[l][ln] = S.va[p][ln] + S.xi[l][ln] * qd;
        }
    }
    __syncthreads();
}

// joint transforms (lane l) and forward kinematics (lane 0) of the links
// from the DOF positions S.q and the base pose (x0, q0): S.qr / S.rr, S.ql,
// S.xl, S.zl. SL: the coupled step's LDS (EnvLds) or the narrow-phase
// kernel's (NpLds) — the same operations in both, so the same bits.
template <class SL>
__device__ __forceinline__ void aba_fk(const MgEnvArgs& A, SL& S, bool act, int ln, int LA, V3 x0, Q4 q0) {
    // ---- joint transforms (lane l)
    if (act && ln < LA && ln > 0) {
        const float* lf = A.link_f + ln * MG_LINK_F_N;
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        const V3 po = v3(lf[0], lf[1], lf[2]);
        const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
        const V3 ax = v3(lf[7], lf[8], lf[9]);
        Q4 qrel;
        V3 rr;
        link_joint(jt, (int)lf[10], po, qo, ax, S.q, dof, qrel, rr);
        S.qr[ln] = qrel;
        S.rr[ln] = rr;
    }
    __syncthreads();
    // ---- forward kinematics (lane 0)
    if (act && ln == 0) {
        for (int l = 0; l < LA; ++l) {
            const int p = A.link_i[l * MG_LINK_I_N + 0];
            if (p < 0) {
                S.ql[l] = q0;
                S.xl[l] = x0;
                S.zl[l] = v3(0.0f, 0.0f, 0.0f);
            } else {
                const float* lf = A.link_f + l * MG_LINK_F_N;
                const Q4 qp = S.ql[p];
                S.ql[l] = qnormalize(qmul(qp, S.qr[l]));
                S.xl[l] = vadd(S.xl[p], qrot(qp, S.rr[l]));
                S.zl[l] = qrot(S.ql[l], v3(lf[7], lf[8], lf[9]));
            }
        }
    }
    __syncthreads();
}

template <int MAXL, int G>
__device__ __forceinline__ void aba_kin(const MgStep& P, const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA, V3 x0,
                                        Q4 q0, const LinkC& lk, int b0, const float* poses = nullptr) {
    if (poses) {
        // the link poses forward kinematics would give (MG_ENV_FK_CARRY) and the
        // joint axes from them, as aba_fk's scan forms them
        if (act && ln < LA) {
            const float* c = poses + MG_CARRY_LINK * ln;
            const Q4 ql = q4(c[3], c[4], c[5], c[6]);
            S.xl[ln] = v3(c[0], c[1], c[2]);
            S.ql[ln] = ql;
            if (A.link_i[ln * MG_LINK_I_N + 0] < 0) {
                S.zl[ln] = v3(0.0f, 0.0f, 0.0f);
            } else {
                const float* lf = A.link_f + ln * MG_LINK_F_N;
                S.zl[ln] = qrot(ql, v3(lf[7], lf[8], lf[9]));
            }
        }
        __syncthreads();
    } else {
        aba_fk(A, S, act, ln, LA, x0, q0);
    }
    // ---- axes and inertias (lane l)
    if (act && ln < LA) {
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        SV x = svzero();
        if (ln > 0 && dof >= 0) {
            const V3 z = S.zl[ln];
            if (jt == MG_JOINT_REVOLUTE) x = sv(z, vcross(vsub(S.xl[ln], x0), z));
            else x = sv(v3(0.0f, 0.0f, 0.0f), z);
        }
        put6(S.xi[ln], x);
        world_inertia(lk, S.ql[ln], S.xl[ln], x0, S.Iw[ln]);
    }
    __syncthreads();
    aba_vel<MAXL, G>(A, S, act, ln, LA);
    aba_vp<MAXL, G>(A, S, act, ln, LA, x0, lk, b0);
}

template <int MAXL, int G>
__device__ __forceinline__ void aba_refresh(const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA, V3 x0,
                                            const LinkC& lk, int b0) {
    if (act && ln < LA) world_inertia(lk, S.ql[ln], S.xl[ln], x0, S.Iw[ln]);
    aba_vel<MAXL, G>(A, S, act, ln, LA);
    aba_vp<MAXL, G>(A, S, act, ln, LA, x0, lk, b0);
}

template <int MAXL, int G>
__device__ __forceinline__ void aba_dyn(const MgStep& P, const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA, V3 x0,
                                        V3 gw, const DofC& dc, bool is_dof, bool xm, bool xp, int b0) {
    const float h = P.h;
    const bool fb = A.floating != 0;
    const int DA = A.ndof;
    // ---- drive terms (lane d): implicit PD force and its h-derivative; a DOF
    // flagged by the effort-limit test (xm) runs at constant +-effort
    if (act && is_dof) {
        const float qv = S.q[ln], uv = S.u[ln];
        float tau = 0.0f, imp = 0.0f;
        if (dc.mode == MG_DOF_MODE_POS) {
            tau = dc.kp * (dc.tpos - qv - h * uv) + dc.kd * (dc.tvel - uv);
            imp = h * dc.kd + h * h * dc.kp;
        } else if (dc.mode == MG_DOF_MODE_VEL) {
            tau = dc.kd * (dc.tvel - uv);
            imp = h * dc.kd;
        } else if (dc.mode == MG_DOF_MODE_EFFORT) {
            tau = dc.force;
        }
        if (dc.eff > 0.0f) {
            if (xm) {
                tau = xp ? dc.eff : -dc.eff;
                imp = 0.0f;
            } else if (imp == 0.0f) {
                tau = fminf(fmaxf(tau, -dc.eff), dc.eff);
            }
        }
        S.tau0[ln] = tau;
        S.imp[ln] = imp;
        S.mdiag[ln] = dc.arm + imp;
        S.arm[ln] = dc.arm;
    }
    __syncthreads();
    // ---- inward pass: articulated inertias and bias forces
    for (int l = LA - 1; l >= 1; --l) {
        const int p = A.link_i[l * MG_LINK_I_N + 0], dof = A.link_i[l * MG_LINK_I_N + 2];
        float uinvD = 0.0f;
        if (dof >= 0) {
            if (act && ln < 6) S.Ua[l][ln] = dot6(&S.Iw[l][ln * 6], S.xi[l]);
            __syncthreads();
            if (act) {
                const float Dv = dot6(S.xi[l], S.Ua[l]) + S.arm[dof] + S.imp[dof];
                const float uvv = S.tau0[dof] - dot6(S.xi[l], S.pa[l]);
                const float invD = 1.0f / Dv;
                uinvD = uvv * invD;
                for (int e = ln; e < 36; e += G) {
                    const int i = e / 6, k = e % 6;
                    S.Iw[l][e] = S.Iw[l][e] - S.Ua[l][i] * (S.Ua[l][k] * invD);
                }
                if (ln == 0) {
                    S.Dd[l] = Dv;
                    S.uu[l] = uvv;
                }
            }
            __syncthreads();
        }
        if (act && ln < 6 && (p > 0 || (fb && p == 0))) {
            float pv = S.pa[l][ln] + dot6(&S.Iw[l][ln * 6], S.cc[l]);
            if (dof >= 0) pv = pv + S.Ua[l][ln] * uinvD;
            S.pa[p][ln] = S.pa[p][ln] + pv;
        }
        if (act && (p > 0 || (fb && p == 0)))
            for (int e = ln; e < 36; e += G) S.Iw[p][e] = S.Iw[p][e] + S.Iw[l][e];
        __syncthreads();
    }
    // ---- root: a0 = -IA_0^-1 pA_0 (lane 0); the root slots' accelerations are
    // w' and the classical acceleration of the base origin, a0.v + g + w x v;
    // the root link's damping and speed limits (as a free body's) give ru
    if (fb) {
        if (act && ln == 0) {
            float nb6[6], a0[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) nb6[i] = -S.pa[0][i];
            spd6_solve(S.Iw[0], nb6, a0);
#pragma unroll
            for (int i = 0; i < 6; ++i) S.va[0][i] = a0[i];
            const V3 w = v3(S.u[DA + 0], S.u[DA + 1], S.u[DA + 2]);
            const V3 vo = v3(S.u[DA + 3], S.u[DA + 4], S.u[DA + 5]);
            const V3 av = vadd(vadd(v3(a0[3], a0[4], a0[5]), gw), vcross(w, vo));
            S.qdd[DA + 0] = a0[0]; S.qdd[DA + 1] = a0[1]; S.qdd[DA + 2] = a0[2];
            S.qdd[DA + 3] = av.x; S.qdd[DA + 4] = av.y; S.qdd[DA + 5] = av.z;
            const float* tf = A.tbf + A.body_tmpl[b0] * MG_TBODY_F_N;
            const float lkeep = 1.0f - fminf(tf[0] * h, 1.0f), akeep = 1.0f - fminf(tf[1] * h, 1.0f);
            V3 wn = vscale(vmad(w, v3(a0[0], a0[1], a0[2]), h), akeep);
            V3 vn = vscale(vmad(vo, av, h), lkeep);
            const float w2 = vdot(wn, wn), mw2 = tf[3] * tf[3];
            if (w2 > mw2) wn = vscale(wn, sqrtf(mw2 / w2));
            const float v2 = vdot(vn, vn), mv2 = tf[2] * tf[2];
            if (v2 > mv2) vn = vscale(vn, sqrtf(mv2 / v2));
            S.ru[0] = wn.x; S.ru[1] = wn.y; S.ru[2] = wn.z;
            S.ru[3] = vn.x; S.ru[4] = vn.y; S.ru[5] = vn.z;
        }
        __syncthreads();
    }
    // ---- outward pass: accelerations (lanes 0..5, one component each)
    if (act && ln < 6 && !fb) S.va[0][ln] = ln < 3 ? 0.0f : -(ln == 3 ? gw.x : (ln == 4 ? gw.y : gw.z));
    for (int l = 1; l < LA; ++l) {
        const int p = A.link_i[l * MG_LINK_I_N + 0], dof = A.link_i[l * MG_LINK_I_N + 2];
        float a = 0.0f;
        if (act && ln < 6) a = S.va[p][ln] + S.cc[l][ln];
        if (dof >= 0) {
            const float t = redg<G>(act && ln < 6 ? S.Ua[l][ln] * a : 0.0f);
            if (act) {
                const float acc = (S.uu[l] - t) / S.Dd[l];
                if (ln < 6) a = a + S.xi[l][ln] * acc;
                if (ln == 0) S.qdd[dof] = acc;
            }
        }
        if (act && ln < 6) S.va[l][ln] = a;
    }
    __syncthreads();
}


// M_eff = joint-space inertia + S.mdiag from world-frame composite inertias
// (entrywise subtree sums of the link inertias; M_ij = xi_j . IC_i xi_i for j
// on the path of i), then its Cholesky factor and M_eff^-1, both in registers:
// lane i holds row i of the factor (right-looking, column j broadcast by DPP;
// every entry sees the same subtractions in the same order as the left-looking
// loops of the oracle), lane j solves column j of M_eff^-1 into mcol[].
// Called by every lane; `act` selects the envs that work. ND: static bound on D.
// Floating base: the root slots DA..DA+5 (unit spatial axes at x0) extend the
// matrix to NA = DA + 6: M[root r][root c] = IC_0[r][c], M[d][root r] = (IC_l xi_l)[r].
template <int MAXL, int ND, int G>
__device__ __forceinline__ void meff_world(const MgEnvArgs& A, EnvLds<MAXL, G>& S, bool act, int ln, int LA, int DA, V3 x0, const LinkC& lk,
                           float (&mcol)[ND]) {
    const bool fb = A.floating != 0;
    const int NA = fb ? DA + 6 : DA;
    if (act && ln < LA) world_inertia(lk, S.ql[ln], S.xl[ln], x0, S.Iw[ln]);
    __syncthreads();
    if (act)
        for (int l = LA - 1; l >= 1; --l) {
            const int p = A.link_i[l * MG_LINK_I_N + 0];
            if (p > 0 || (fb && p == 0))
                for (int e = ln; e < 36; e += G) S.Iw[p][e] = S.Iw[p][e] + S.Iw[l][e];
        }
    if (act && ln < NA)
        for (int j = 0; j < NA; ++j) S.Lc[ln][j] = 0.0f;
    __syncthreads();
    if (act && fb && ln >= DA && ln < NA) {
        const int r = ln - DA;
        for (int c = 0; c < 6; ++c) S.Lc[ln][DA + c] = S.Iw[0][r * 6 + c];
    }
    if (act && ln < DA) {
        const int l = S.dlink[ln];
        float F[6];
        for (int r = 0; r < 6; ++r) F[r] = dot6(&S.Iw[l][r * 6], S.xi[l]);
        S.Lc[ln][ln] = dot6(S.xi[l], F) + S.mdiag[ln];
        int j = A.link_i[l * MG_LINK_I_N + 0];
        while (j > 0) {
            const int dj = A.link_i[j * MG_LINK_I_N + 2];
            if (dj >= 0) {
                const float hv = dot6(S.xi[j], F);
                S.Lc[ln][dj] = hv;
                S.Lc[dj][ln] = hv;
            }
            j = A.link_i[j * MG_LINK_I_N + 0];
        }
        if (fb)
            for (int r = 0; r < 6; ++r) {
                S.Lc[ln][DA + r] = F[r];
                S.Lc[DA + r][ln] = F[r];
            }
    }
    __syncthreads();
    // all 64 lanes run the register phases (DPP reads neighbouring lanes);
    // envs that are not `act` compute on stale data and discard it
    float a[ND], invd[ND];
    const int row = ln < NA ? ln : 0;
#pragma unroll
    for (int k = 0; k < ND; ++k) a[k] = k < NA ? S.Lc[row][k] : 0.0f;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        if (j < NA) {
            const float dj = bcastg<G>(sqrtf(a[j]), j);
            invd[j] = 1.0f / dj;
            if (ln == j) a[j] = dj;
            else if (ln > j) a[j] = a[j] * invd[j];
            const float col = a[j];                          // L[ln][j]
#pragma unroll
            for (int k = j + 1; k < ND; ++k)
                if (k < NA) {
                    const float lk = bcastg<G>(col, k);        // L[k][j]
                    if (ln >= k) a[k] = a[k] - col * lk;
                }
        }
    }
    // column ln of M_eff^-1: forward then backward substitution, L[i][k] from lane i
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        if (i < NA) {
            float t = i == ln ? 1.0f : 0.0f;
#pragma unroll
            for (int k = 0; k < i; ++k) t = t - bcastg<G>(a[k], i) * mcol[k];
            mcol[i] = t * invd[i];
        }
    }
#pragma unroll
    for (int i = ND - 1; i >= 0; --i) {
        if (i < NA) {
            float t = mcol[i];
#pragma unroll
            for (int k = i + 1; k < ND; ++k)
                if (k < NA) t = t - bcastg<G>(a[i], k) * mcol[k];
            mcol[i] = t * invd[i];
        }
    }
}

// The template's link constants (joint frames, axes, parents, DOF indices) in
// LDS for the whole kernel: the serial loops of the kinematic scan and the
// inward / outward passes read them per link, and from HBM / L2 every such read
// was a dependent round trip on the critical path (S2: ~4 us of a 24.9 us step).
template <int MAXL, int G>
__device__ __forceinline__ void stage_links(MgEnvArgs& A) {
    __shared__ float s_lf[MAXL * MG_LINK_F_N];
    __shared__ int s_li[MAXL * MG_LINK_I_N];
    const int nl = A.nl < MAXL ? A.nl : MAXL;
    for (int k = threadIdx.x; k < nl * MG_LINK_F_N; k += 64) s_lf[k] = A.link_f[k];
    for (int k = threadIdx.x; k < nl * MG_LINK_I_N; k += 64) s_li[k] = A.link_i[k];
    __syncthreads();
    A.link_f = s_lf;
    A.link_i = s_li;
}

// ---- the narrow phase as its own launch (round 5) ---------------------------
// The coupled step of one substep is two launches: k_env_np (this kernel: the
// link poses by forward kinematics, the pair screen, the narrow phase, contact
// placement and the friction patches) and k_env_step (unconstrained motion,
// limit rows, rows, TGS, integration). Round 4's single kernel held both in one
// register allocation (512 VGPRs + 276 B of scratch per lane, one wave per
// SIMD); split, the narrow phase runs with GN lanes per env (64: one env per
// wave, the cooperative convex tests on 64 lanes, four waves per SIMD at 4096
// envs) and hands its contacts to the step through a per-env table in HBM
// (ctab, MG_CT_* below); the step's state between its substep launches goes
// through a per-env carry record (qv, uv, the contact-force sums, the root and
// free-body poses) bit for bit, so the arithmetic and its order are those of
// the single kernel and of oracle/migym_oracle_env.c, unchanged.
template <int MAXL, int MAXCT>
struct NpLds {
    float q[64];                     // DOF positions (aba_fk's link_joint)
    V3 xl[MAXL], zl[MAXL], rr[MAXL];
    Q4 ql[MAXL], qr[MAXL];
    V3 fx[MAXF];
    Q4 fq[MAXF];
    V3 sx[MG_ENV_MAXS];
    Q4 sq[MG_ENV_MAXS];
    int npl[NPB];
    int ca[MAXCT], cb[MAXCT];
    V3 cp[MAXCT], cd[MAXCT][3];
    float cs0[MAXCT], ce[MAXCT];
    int ppair[MAXCT];
    V3 apt[MAXCT];
    float ae[MAXCT][2], amu[MAXCT];
    int aab[MAXCT], alast[MAXCT];
    unsigned fpv[MG_FP_W], fpn[MG_FP_W];
    unsigned long long pstart;
    int link_rows;
};

// contact table of one env (floats; ints stored by bit pattern): header, then
// MAXCT contacts, then MAXCT anchors
constexpr int MG_CT_HDR = 8;         // [0] contacts (uncapped), [1] anchors (uncapped), [2] link rows, [3..4] pstart
constexpr int MG_CT_C = 10;          // ca, cb, cp.xyz, n.xyz, cs0, ce
constexpr int MG_CT_A = 14;          // apt.xyz, t1.xyz, t2.xyz, ae0, ae1, amu, aab, alast
template <int MAXCT>
constexpr int ct_n() { return MG_CT_HDR + MAXCT * (MG_CT_C + MG_CT_A); }


__device__ __forceinline__ float ibits(int v) { return __int_as_float(v); }
__device__ __forceinline__ int fbits(float v) { return __float_as_int(v); }

// MAXL, GM: the step kernel's link bound and lanes per env (its MAXCT); GN:
// this kernel's lanes per env (16 or 64). MG_NP_WAVES: the occupancy budget
// (waves per SIMD the register allocation must allow)
#ifndef MG_NP_GN
#define MG_NP_GN 16
#endif
#ifndef MG_NP_WAVES
#define MG_NP_WAVES 1
#endif
template <int MAXL, int GM, int GN>
__global__ void __launch_bounds__(64, MG_NP_WAVES) k_env_np(MgStep P, MgEnvArgs A) {
    constexpr int G = GN;
    constexpr int EPW = 64 / G;          // envs per wavefront
    constexpr int MAXCT = maxct<GM>();
    __shared__ NpLds<MAXL, MAXCT> shm[EPW];
    stage_links<MAXL, G>(A);
    const int gi = threadIdx.x / G;
    const int ln = threadIdx.x % G;
    const int e = blockIdx.x * EPW + gi;
    const bool live = e < A.ne;
    NpLds<MAXL, MAXCT>& S = shm[gi];
    // the scene's shape records, shape boxes and hull table in LDS for the
    // launch (the dynamic allocation, mg_launch_env_step, when they fit): the
    // screen and the plane / vertex / edge scans read them over and over, and
    // from L2 each batch was a dependent round trip
    if (A.nhull >= 0) {
        extern __shared__ float s_scene[];
        float* sh_s = s_scene;
        float* sh_o = sh_s + A.nshape * MG_SHAPE_STRIDE;
        float* sh_h = sh_o + A.nshape * MG_OBB_N;
        for (int k = threadIdx.x; k < A.nshape * MG_SHAPE_STRIDE; k += 64) sh_s[k] = A.shapes[k];
        for (int k = threadIdx.x; k < A.nshape * MG_OBB_N; k += 64) sh_o[k] = A.shape_obb[k];
        for (int k = threadIdx.x; k < A.nhull; k += 64) sh_h[k] = A.hulls[k];
        __syncthreads();
        A.shapes = sh_s;
        A.shape_obb = sh_o;
        A.hulls = sh_h;
    }
    const int* ei = A.env_i + (size_t)(live ? e : 0) * MG_ENV_I_N;
    const int b0 = ei[0], d0 = ei[1];
    const int nfr = live ? ei[2] : 0;
    const int pair0 = ei[14], npair = live ? ei[15] : 0;
    const int L = (live && b0 >= 0) ? A.nl : 0;
    const int D = (live && b0 >= 0) ? A.ndof : 0;
    const int nb = A.nb;
    const float* St = A.state;
    const float* cy = A.carry + (size_t)(live ? e : 0) * carry_n<GM>();
    const int LA = A.nl;
    PH_T0();
    // poses at the substep start: the first substep's from the state (the step
    // kernel's own loads: quaternions normalised), later ones from the carry
    V3 x0 = v3(0.0f, 0.0f, 0.0f);
    Q4 q0 = q4(0.0f, 0.0f, 0.0f, 1.0f);
    if (L > 0) {
        if (A.sub == 0) {
            x0 = v3(St[0 * nb + b0], St[1 * nb + b0], St[2 * nb + b0]);
            q0 = qnormalize(q4(St[3 * nb + b0], St[4 * nb + b0], St[5 * nb + b0], St[6 * nb + b0]));
        } else {
            x0 = v3(cy[0], cy[1], cy[2]);
            q0 = q4(cy[3], cy[4], cy[5], cy[6]);
        }
    }
    if (ln < D) S.q[ln] = A.sub == 0 ? A.dof_pos[d0 + ln] : cy[MG_CARRY_HDR + MG_CARRY_LANE * ln];
    if (live && ln < ei[7]) {
        const int b = ei[8 + ln];
        S.sx[ln] = v3(St[0 * nb + b], St[1 * nb + b], St[2 * nb + b]);
        S.sq[ln] = qnormalize(q4(St[3 * nb + b], St[4 * nb + b], St[5 * nb + b], St[6 * nb + b]));
    }
    if (live && ln < nfr) {
        if (A.sub == 0) {
            const int b = ei[3 + ln];
            S.fx[ln] = v3(St[0 * nb + b], St[1 * nb + b], St[2 * nb + b]);
            S.fq[ln] = qnormalize(q4(St[3 * nb + b], St[4 * nb + b], St[5 * nb + b], St[6 * nb + b]));
        } else {
            const float* c = cy + 7 + 7 * ln;
            S.fx[ln] = v3(c[0], c[1], c[2]);
            S.fq[ln] = q4(c[3], c[4], c[5], c[6]);
        }
    }
    if (ln < MG_FP_W) {   // friction patches held at the end of the last substep
        S.fpv[ln] = live ? A.fp_mask[(size_t)e * MG_FP_W + ln] : 0u;
        S.fpn[ln] = 0u;
    }
    if (ln == 0) {
        S.pstart = 0ull;
        S.link_rows = 0;
    }
    if (MG_ENV_FK_CARRY && A.sub > 0) {   // the link poses the last substep's step kernel left
        if (live && ln < L) {
            const float* c = cy + carry_link0<GM>() + MG_CARRY_LINK * ln;
            S.xl[ln] = v3(c[0], c[1], c[2]);
            S.ql[ln] = q4(c[3], c[4], c[5], c[6]);
        }
        __syncthreads();
    } else {
        __syncthreads();
        if (LA > 0) aba_fk(A, S, live && L > 0, ln, LA, x0, q0);
    }
    PH_MARK(17);

    // ================= 2. narrow phase, per block of NPB candidate pairs:
    // (a) bounding-sphere screen, one pair per lane, survivors compacted in
    //     pair order into S.npl (the screen is conservative: a rejected pair
    //     has no contact within the margin);
    // (b) the full pair test on the survivors, one per lane per round,
    //     contacts placed by a 16-lane prefix sum in pair order.
    int base = 0, npatch = 0;   // contacts, friction patches placed so far
    for (int blk = 0; __any(blk < npair); blk += NPB) {
        int nnear = 0;
#pragma unroll
        for (int r = 0; r < NPB; r += G) {
            const int pi = blk + r + ln;
            bool near = false;
            if (pi < npair) {
                const int* pp = A.pairs + (size_t)(pair0 + pi) * 4;
                const int pa = pp[0], sa = pp[1], pb = pp[2], sb = pp[3];
                const float* sha = A.shapes + sa * MG_SHAPE_STRIDE;
                V3 xa, xb = v3(0.0f, 0.0f, 0.0f);
                Q4 qa, qb = q4(0.0f, 0.0f, 0.0f, 1.0f);
                pair_pose(S, pa, xa, qa);
                if (pb >= 0) pair_pose(S, pb, xb, qb);
                near = pair_near(P, sha, xa, qa, pb >= 0 ? A.shapes + sb * MG_SHAPE_STRIDE : sha, xb, qb, pb < 0,
                                 A.shape_obb + sa * MG_OBB_N, A.shape_obb + (pb >= 0 ? sb : sa) * MG_OBB_N);
            }
            const unsigned long long gm = grp_ballot<G>(near, gi);
            if (near) S.npl[nnear + __popcll(gm & ((1ull << ln) - 1ull))] = pi;
            nnear += __popcll(gm);
        }
        __syncthreads();
        PH_MARK(8);
        for (int rb = 0; __any(rb < nnear); rb += G) {
            PH_NP0();
            PairOut o;
            o.n = 0;
            float rest = 0.0f;
            int pa = 0, pb = -1, pidx = 0;
            bool coop = false;
            CShape cA = {}, cB = {};
            if (rb + ln < nnear) {
                PH_COUNT(10, 1);
                pidx = S.npl[rb + ln];
                const int* pp = A.pairs + (size_t)(pair0 + pidx) * 4;
                pa = pp[0];
                const int sa = pp[1];
                pb = pp[2];
                const int sb = pp[3];
                const float* sha = A.shapes + sa * MG_SHAPE_STRIDE;
                if (pb < 0) {
                    V3 xa;
                    Q4 qa;
                    pair_pose(S, pa, xa, qa);
                    ground_pair(P, place_shape(sha, xa, qa, A.hulls), o);
                    rest = 0.5f * (sha[12] + P.e_ground);
                } else {
                    const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                    coop = cvx_pair((int)sha[0], (int)shb[0]);
                    V3 xa, xb;
                    Q4 qa, qb;
                    pair_pose(S, pa, xa, qa);
                    pair_pose(S, pb, xb, qb);
                    cA = place_shape(sha, xa, qa, A.hulls);
                    cB = place_shape(shb, xb, qb, A.hulls);
                    if (!coop) collide(cA, cB, P.contact_offset, o);
                    PH_COUNT(11, ((int)sha[0] == MG_SHAPE_CONVEX || (int)shb[0] == MG_SHAPE_CONVEX) ? 1 : 0);
                    rest = 0.5f * (sha[12] + shb[12]);
                }
            }
            PH_NP(18);
            // this round's convex pairs, one at a time on the whole group (in
            // lane order; the result goes to the pair's own lane)
            unsigned long long cm = grp_ballot<G>(coop, gi);
            while (__any(cm != 0ull)) {
                if (cm != 0ull) {                     // group-uniform
                    const int k = __ffsll(cm) - 1;
                    cm &= cm - 1ull;
                    PairOut t;
                    coop_convex_convex<G>(shfl_shape<G>(cA, k), shfl_shape<G>(cB, k), P.contact_offset, ln, gi, t);
                    if (ln == k) o = t;
                    if (ln == k) PH_COUNT(16, t.n == 0 ? 1 : 0);   // convex pairs without a contact
                }
            }
            PH_NP(19);
            // exclusive prefix sum of the counts over the 16 lanes
            int incl = o.n;
#pragma unroll
            for (int off = 1; off < G; off <<= 1) {
                const int t = __shfl_up(incl, off, G);
                if (ln >= off) incl += t;
            }
            const int total = __shfl(incl, G - 1, G);
            const int slot0 = base + incl - o.n;
#pragma unroll
            for (int j = 0; j < MG_PAIR_MAXC; ++j) {
                const int c = slot0 + j;
                if (j < o.n && c < MAXCT) {
                    S.ca[c] = pa;
                    S.cb[c] = pb;
                    S.cp[c] = o.p[j];
                    S.cd[c][0] = o.nrm[j];
                    S.cs0[c] = o.sep[j] - P.rest_offset;
                    S.ce[c] = rest;
                    if (pa < F0) S.link_rows = 1;
                }
            }
            base += total;
            // the pair's friction patch (its first contact placed), in pair
            // order; updated after the narrow phase, one patch per lane
            const int pn = (o.n > 0 && slot0 < MAXCT) ? 1 : 0;
            int pin = pn;
#pragma unroll
            for (int off = 1; off < G; off <<= 1) {
                const int t = __shfl_up(pin, off, G);
                if (ln >= off) pin += t;
            }
            if (pn) S.ppair[npatch + pin - 1] = (pidx << 10) | (slot0 << 4) | (o.n < MAXCT - slot0 ? o.n : MAXCT - slot0);
            npatch += __shfl(pin, G - 1, G);
            PH_NP(20);
        }
        __syncthreads();
        PH_MARK(9);
    }
    // friction patches, one per lane: anchors kept from
    // the last substep or grown from the patch's placed contacts
    int abase = 0;
    {
        Patch R;
        R.cnt = 0;
        V3 pxa = v3(0.0f, 0.0f, 0.0f), pxb = v3(0.0f, 0.0f, 0.0f), n0 = v3(0.0f, 0.0f, 1.0f);
        Q4 pqa = q4(0.0f, 0.0f, 0.0f, 1.0f), pqb = q4(0.0f, 0.0f, 0.0f, 1.0f);
        int pidx = 0, slot0 = 0, pn = 0, pa = 0, pb = -1;
        float mu = 0.0f;
        if (live && ln < npatch) {
            const int pp = S.ppair[ln];
            pidx = pp >> 10;
            slot0 = (pp >> 4) & 63;
            pn = pp & 15;
            pa = S.ca[slot0];
            pb = S.cb[slot0];
            const int* pr = A.pairs + (size_t)(pair0 + pidx) * 4;
            const float fa = A.shapes[pr[1] * MG_SHAPE_STRIDE + 11];
            mu = pb < 0 ? 0.5f * (fa + P.mu_ground) : 0.5f * (fa + A.shapes[pr[3] * MG_SHAPE_STRIDE + 11]);
            PairOut o;
            o.n = pn;
#pragma unroll
            for (int j = 0; j < MG_PAIR_MAXC; ++j) {
                const int c = j < pn ? slot0 + j : slot0;
                o.p[j] = S.cp[c];
                o.nrm[j] = S.cd[c][0];
                o.sep[j] = S.cs0[c];   // separation beyond the rest offset
            }
            n0 = o.nrm[0];
            pair_pose(S, pa, pxa, pqa);
            if (pb >= 0) pair_pose(S, pb, pxb, pqb);
            float* rec = A.fpatch + (size_t)(pair0 + pidx) * MG_FP_N;
            const bool held = pidx < MG_FP_MAXP && ((S.fpv[pidx >> 5] >> (pidx & 31)) & 1u);
            if (held) patch_load(R, rec);
            patch_update(R, pxa, pqa, pxb, pqb, o, P.fric_offset, P.fric_corr);
            if (pidx < MG_FP_MAXP) {
                patch_store(R, rec);
                atomicOr(&S.fpn[pidx >> 5], 1u << (pidx & 31));
            }
            atomicOr(&S.pstart, 1ull << slot0);
        }
        int ain = R.cnt;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const int t = __shfl_up(ain, off, G);
            if (ln >= off) ain += t;
        }
        abase = __shfl(ain, G - 1, G);
        const int ak0 = ain - R.cnt;
        if (R.cnt > 0) {
            V3 t1, t2;
            env_tangents(n0, &t1, &t2);
            const int last = slot0 + pn - 1;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int k = ak0 + j;
                if (j < R.cnt && k < MAXCT) {
                    const V3 wA = vadd(pxa, qrot(pqa, R.aA[j])), wB = vadd(pxb, qrot(pqb, R.aB[j]));
                    const V3 dr = vsub(wA, wB);
                    S.apt[k] = wA;
                    S.cd[k][1] = t1;
                    S.cd[k][2] = t2;
                    // position sweeps' target velocity along t1, t2: close 80 %
                    // of the substep-start drift of the anchor's two copies
                    const float kd = 0.8f * P.inv_h;
                    S.ae[k][0] = fminf(fmaxf(-vdot(dr, t1) * kd, -P.max_depen), P.max_depen);
                    S.ae[k][1] = fminf(fmaxf(-vdot(dr, t2) * kd, -P.max_depen), P.max_depen);
                    // the patch's other anchor, when it has a row
                    const int pc = R.cnt == 2 ? (j == 0 ? (k + 1 < MAXCT ? 1 : 0) : 2) : 0;
                    S.amu[k] = mu;
                    S.aab[k] = (pa & 0xFFFF) | (pb << 16);
                    S.alast[k] = last | (pc << 8) | (pidx << 10);
                }
            }
        }
    }
    __syncthreads();
    // this substep's patches are the next one's; the contact table
    if (live && ln < MG_FP_W) A.fp_mask[(size_t)e * MG_FP_W + ln] = S.fpn[ln];
    if (live) {
        float* ct = A.ctab + (size_t)e * ct_n<MAXCT>();
        if (ln == 0) {
            ct[0] = ibits(base);
            ct[1] = ibits(abase);
            ct[2] = ibits(S.link_rows);
            ct[3] = ibits((int)(unsigned)(S.pstart & 0xFFFFFFFFull));
            ct[4] = ibits((int)(unsigned)(S.pstart >> 32));
        }
        const int nc = base < MAXCT ? base : MAXCT, na = abase < MAXCT ? abase : MAXCT;
        for (int c = ln; c < nc; c += G) {
            float* r = ct + MG_CT_HDR + c * MG_CT_C;
            r[0] = ibits(S.ca[c]); r[1] = ibits(S.cb[c]);
            r[2] = S.cp[c].x; r[3] = S.cp[c].y; r[4] = S.cp[c].z;
            r[5] = S.cd[c][0].x; r[6] = S.cd[c][0].y; r[7] = S.cd[c][0].z;
            r[8] = S.cs0[c]; r[9] = S.ce[c];
        }
        for (int k = ln; k < na; k += G) {
            float* r = ct + MG_CT_HDR + MAXCT * MG_CT_C + k * MG_CT_A;
            r[0] = S.apt[k].x; r[1] = S.apt[k].y; r[2] = S.apt[k].z;
            r[3] = S.cd[k][1].x; r[4] = S.cd[k][1].y; r[5] = S.cd[k][1].z;
            r[6] = S.cd[k][2].x; r[7] = S.cd[k][2].y; r[8] = S.cd[k][2].z;
            r[9] = S.ae[k][0]; r[10] = S.ae[k][1]; r[11] = S.amu[k];
            r[12] = ibits(S.aab[k]); r[13] = ibits(S.alast[k]);
        }
    }
    PH_MARK(21);
}

template <int MAXL, int G>
__global__ void __launch_bounds__(64) k_env_step(MgStep P, MgEnvArgs A) {
    constexpr int EPW = 64 / G;          // envs per wavefront
    constexpr int MAXCT = maxct<G>();
    __shared__ EnvStepLds<MAXL, G> shm[EPW];
    stage_links<MAXL, G>(A);
    const int gi = threadIdx.x / G;
    const int ln = threadIdx.x % G;
    const int e = blockIdx.x * EPW + gi;
    const bool live = e < A.ne;
    EnvStepLds<MAXL, G>& S = shm[gi];
    const int* ei = A.env_i + (size_t)(live ? e : 0) * MG_ENV_I_N;
    const int b0 = ei[0], d0 = ei[1];
    const int nfr = live ? ei[2] : 0;
    const int pair0 = ei[14];
    const int L = (live && b0 >= 0) ? A.nl : 0;
    const int D = (live && b0 >= 0) ? A.ndof : 0;
    const int nb = A.nb, nd = A.nd;
    float* St = A.state;
    const float* pr = A.dof_props;
    const float h = P.h;
    const V3 gvec = v3(P.g[0], P.g[1], P.g[2]);

    // slot of this lane: DOFs, the floating root's (w, v_O), free bodies
    const int RB = (L > 0 && A.floating) ? 6 : 0;
    const int NS = D + RB;
    const bool is_dof = ln < D;
    const int ballr = is_dof ? dof_ball(A, A.nl, ln) : 0;   // ball joints: exponential coordinates
    const bool any_ball = __any(dof_ball(A, A.nl, ln % (A.ndof > 0 ? A.ndof : 1)) > 0);   // launch-uniform
    const bool is_root = ln >= D && ln < NS;
    const int rc = ln - D;
    const int fk = ln >= NS ? (ln - NS) / 6 : MAXF;
    const int fc = ln >= NS ? (ln - NS) % 6 : 0;
    const bool is_free = fk < nfr;

    // ---- substep-invariant setup
    PH_T0();
    V3 x0 = v3(0.0f, 0.0f, 0.0f);
    Q4 q0 = q4(0.0f, 0.0f, 0.0f, 1.0f);
    // lane k < nf: free body k's constants and contact force sum; lane l < L:
    // link l's contact force sum
    FreeC fr = {};
    V3 fsum = v3(0.0f, 0.0f, 0.0f), lsum = v3(0.0f, 0.0f, 0.0f);
    V3 gw = v3(0.0f, 0.0f, 0.0f);
    const int LA = A.nl, DA = A.ndof;           // launch-uniform loop bounds (barriers inside)
    const int NA = (LA > 0 && A.floating) ? DA + 6 : DA;   // articulation velocity slots
    // one substep per launch (A.sub of P.substeps); the state of a later
    // substep comes from the carry record the previous launch wrote
    const bool first = A.sub == 0;
    float* cy = A.carry + (size_t)(live ? e : 0) * carry_n<G>();
    float* cyl = cy + MG_CARRY_HDR + MG_CARRY_LANE * ln;
    if (L > 0) {
        if (first) {
            x0 = v3(St[0 * nb + b0], St[1 * nb + b0], St[2 * nb + b0]);
            q0 = qnormalize(q4(St[3 * nb + b0], St[4 * nb + b0], St[5 * nb + b0], St[6 * nb + b0]));
        } else {
            x0 = v3(cy[0], cy[1], cy[2]);
            q0 = q4(cy[3], cy[4], cy[5], cy[6]);
        }
        const float grav_on = A.tbf[A.body_tmpl[b0] * MG_TBODY_F_N + 4];
        gw = grav_on != 0.0f ? gvec : v3(0.0f, 0.0f, 0.0f);
    }
    if (ln == 0 && live) {
        for (int l = 0; l < L; ++l) {
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], dof = li[2];
            S.amask[l] = (p >= 0 ? S.amask[p] : 0u) | (dof >= 0 ? (1u << dof) : 0u);
            if (dof >= 0) {
                S.dlink[dof] = l;
                S.drev[dof] = li[1] == MG_JOINT_REVOLUTE ? 1 : 0;
            }
        }
    }
    if (live && ln < nfr) {
        const int b = ei[3 + ln];
        if (first) {
            S.fx[ln] = v3(St[0 * nb + b], St[1 * nb + b], St[2 * nb + b]);
            S.fq[ln] = qnormalize(q4(St[3 * nb + b], St[4 * nb + b], St[5 * nb + b], St[6 * nb + b]));
        } else {
            const float* c = cy + 7 + 7 * ln;
            S.fx[ln] = v3(c[0], c[1], c[2]);
            S.fq[ln] = q4(c[3], c[4], c[5], c[6]);
        }
        const float* Ms = A.mass;
        S.finvm[ln] = Ms[0 * nb + b];
        fr.invI = v3(Ms[1 * nb + b], Ms[2 * nb + b], Ms[3 * nb + b]);
        fr.iq = q4(Ms[4 * nb + b], Ms[5 * nb + b], Ms[6 * nb + b], Ms[7 * nb + b]);
        fr.com = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
        const float* tf = A.tbf + A.body_tmpl[b] * MG_TBODY_F_N;
        fr.lkeep = 1.0f - fminf(tf[0] * h, 1.0f);
        fr.akeep = 1.0f - fminf(tf[1] * h, 1.0f);
        fr.mlv2 = tf[2] * tf[2];
        fr.mav2 = tf[3] * tf[3];
        fr.gon = tf[4];
        fr.fext = v3(0.0f, 0.0f, 0.0f);
        fr.text = v3(0.0f, 0.0f, 0.0f);
        if (A.ext) {
            fr.fext = v3(A.ext[0 * nb + b], A.ext[1 * nb + b], A.ext[2 * nb + b]);
            fr.text = v3(A.ext[3 * nb + b], A.ext[4 * nb + b], A.ext[5 * nb + b]);
        }
    }
    // slot registers
    float qv = 0.0f, uv = 0.0f, dp = 0.0f;
    DofC dc = {};
    if (is_dof) {
        const int gd = d0 + ln;
        qv = first ? A.dof_pos[gd] : cyl[0];
        uv = first ? A.dof_vel[gd] : cyl[1];
        dc.mode = (int)pr[0 * nd + gd];
        dc.kp = pr[1 * nd + gd];
        dc.kd = pr[2 * nd + gd];
        dc.eff = pr[3 * nd + gd];
        dc.maxv = pr[4 * nd + gd];
        dc.lo = pr[5 * nd + gd];
        dc.hi = pr[6 * nd + gd];
        dc.haslim = pr[7 * nd + gd] != 0.0f;
        dc.arm = pr[8 * nd + gd];
        dc.tpos = A.dof_tpos[gd];
        dc.tvel = A.dof_tvel[gd];
        dc.force = A.dof_force[gd];
        if (first && A.tpos_w) A.tpos_w[gd] = dc.tpos;
        if (first && A.tvel_w) A.tvel_w[gd] = dc.tvel;
        if (first && A.force_w) A.force_w[gd] = dc.force;
    } else if (is_root) {
        // root slots: w and the velocity of the base origin v_O = v_com - w x (R c)
        const V3 w = v3(St[10 * nb + b0], St[11 * nb + b0], St[12 * nb + b0]);
        const V3 vc = v3(St[7 * nb + b0], St[8 * nb + b0], St[9 * nb + b0]);
        const V3 c0 = v3(A.mass[8 * nb + b0], A.mass[9 * nb + b0], A.mass[10 * nb + b0]);
        const V3 vo = vsub(vc, vcross(w, qrot(q0, c0)));
        uv = first ? (rc < 3 ? v3c(w, rc) : v3c(vo, rc - 3)) : cyl[1];
    } else if (is_free) {
        const int b = ei[3 + fk];
        uv = first ? St[(7 + fc) * nb + b] : cyl[1];
    }
    if (!first) {   // the contact-force sums of the earlier substeps
        lsum = v3(cyl[2], cyl[3], cyl[4]);
        fsum = v3(cyl[5], cyl[6], cyl[7]);
    }
    // link ln's body (-1: a virtual link of a ball / multi-axis joint, no mass)
    const int blk = ln < L ? A.link_i[ln * MG_LINK_I_N + 3] : -1;
    LinkC lk = {};
    if (blk >= 0) lk = load_link(A.mass, nb, b0 + blk);
    __syncthreads();
    // the DOF lane's joint: link, revolute flag
    const int mylink = is_dof ? S.dlink[ln] : 0;
    const bool myrev = is_dof && S.drev[ln] != 0;
    constexpr int ND = MAXL <= 4 ? 4 : (G > 32 ? 32 : G);
    float mcol[ND];                  // column ln of M_eff^-1 (DOF lanes)
#pragma unroll
    for (int k = 0; k < ND; ++k) mcol[k] = 0.0f;
    RowJ<G, MAXCT * 3> Jr, Wr;
    RowL<G, MAXCT * 3> lam;
    if constexpr (G == 64) {
        Jr.p = S.Jl;
        Wr.p = S.Wl;
        lam.p = S.laml;
    }
    PH_MARK(6);

    {
        // ================= 1. unconstrained motion (lane 0)
        S.q[ln] = qv;
        S.u[ln] = uv;
        __syncthreads();
        if (LA > 0) {
            bool xm = false, xp = false;     // this DOF runs at constant +-effort
            bool redo = live && L > 0;
            aba_kin<MAXL, G>(P, A, S, redo, ln, LA, x0, q0, lk, b0,
                             (MG_ENV_FK_CARRY && !first) ? cy + carry_link0<G>() : nullptr);
            for (int att = 0; att < 2; ++att) {
                if (!__any(redo)) break;
                if (att > 0) aba_refresh<MAXL, G>(A, S, redo, ln, LA, x0, lk, b0);
                aba_dyn<MAXL, G>(P, A, S, redo, ln, LA, x0, gw, dc, is_dof, xm, xp, b0);
                // drives whose implicit force exceeds the effort limit
                bool flip = false;
                if (redo && is_dof && dc.eff > 0.0f && S.imp[ln] != 0.0f) {
                    const float actf = S.tau0[ln] - S.imp[ln] * S.qdd[ln];
                    if (actf > dc.eff) { xm = true; xp = true; flip = true; }
                    else if (actf < -dc.eff) { xm = true; flip = true; }
                }
                redo = grp_ballot<G>(flip, gi) != 0ull;
                __syncthreads();
            }
        }
        // free body k (lane k): gravity, external force, damping, speed clamps
        if (live && ln < nfr) {
            const int k = ln;
            const int s0 = NS + 6 * k;
            const S3 Iw = sym_rdrt(qmat(qmul(S.fq[k], fr.iq)), fr.invI);
            S.fIw[k] = Iw;
            S.fxc[k] = vadd(S.fx[k], qrot(S.fq[k], fr.com));
            V3 v = v3(S.u[s0 + 0], S.u[s0 + 1], S.u[s0 + 2]);
            V3 w = v3(S.u[s0 + 3], S.u[s0 + 4], S.u[s0 + 5]);
            if (fr.gon != 0.0f) v = vmad(v, gvec, h);
            v = vmad(v, fr.fext, S.finvm[k] * h);
            w = vmad(w, symmul(Iw, fr.text), h);
            v = vscale(v, fr.lkeep);
            w = vscale(w, fr.akeep);
            const float v2 = vdot(v, v);
            if (v2 > fr.mlv2) v = vscale(v, sqrtf(fr.mlv2 / v2));
            const float w2 = vdot(w, w);
            if (w2 > fr.mav2) w = vscale(w, sqrtf(fr.mav2 / w2));
            S.u[s0 + 0] = v.x; S.u[s0 + 1] = v.y; S.u[s0 + 2] = v.z;
            S.u[s0 + 3] = w.x; S.u[s0 + 4] = w.y; S.u[s0 + 5] = w.z;
        }
        __syncthreads();
        if (is_dof) {
            const float maxv = dc.maxv;
            float w = uv + h * S.qdd[ln];
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            uv = w;
        } else if (is_root) {
            uv = S.ru[rc];
        } else if (is_free) {
            uv = S.u[ln];
        }
        dp = 0.0f;
        PH_MARK(0);

        // ================= 2. the contacts and friction anchors of k_env_np
        // (this substep's narrow phase and patches, placed in pair order)
        int base = 0, abase = 0;
        {
            const float* ct = A.ctab + (size_t)(live ? e : 0) * ct_n<MAXCT>();
            base = live ? fbits(ct[0]) : 0;
            abase = live ? fbits(ct[1]) : 0;
            if (ln == 0) {
                S.link_rows = live ? fbits(ct[2]) : 0;
                S.pstart = live ? ((unsigned long long)(unsigned)fbits(ct[3]) |
                                   ((unsigned long long)(unsigned)fbits(ct[4]) << 32)) : 0ull;
            }
            const int nc = base < MAXCT ? base : MAXCT, na = abase < MAXCT ? abase : MAXCT;
            for (int c = ln; c < nc; c += G) {
                const float* r = ct + MG_CT_HDR + c * MG_CT_C;
                S.ca[c] = fbits(r[0]);
                S.cb[c] = fbits(r[1]);
                S.cp[c] = v3(r[2], r[3], r[4]);
                S.cd[c][0] = v3(r[5], r[6], r[7]);
                S.cs0[c] = r[8];
                S.ce[c] = r[9];
            }
            for (int q = ln; q < na; q += G) {
                const float* r = ct + MG_CT_HDR + MAXCT * MG_CT_C + q * MG_CT_A;
                S.apt[q] = v3(r[0], r[1], r[2]);
                S.cd[q][1] = v3(r[3], r[4], r[5]);
                S.cd[q][2] = v3(r[6], r[7], r[8]);
                S.ae[q][0] = r[9];
                S.ae[q][1] = r[10];
                S.amu[q] = r[11];
                S.aab[q] = fbits(r[12]);
                S.alast[q] = fbits(r[13]);
            }
        }
        __syncthreads();
        // joint-limit rows (PhysX solves limits as constraints): a DOF whose
        // predicted position q + h u lies within 5% of its range of a limit gets
        // one unilateral row towards the nearer limit, after the contacts
        {
            int need = 0, sgn = 0;
            float s0 = 0.0f;
            if (live && is_dof) {
                if (dc.haslim) {
                    const float lo = dc.lo, hi = dc.hi;
                    const float q1 = qv + h * uv;
                    const float mg = 0.05f * (hi - lo);
                    if (q1 - lo < mg || hi - q1 < mg) {
                        need = 1;
                        sgn = (q1 - lo) < (hi - q1) ? 1 : -1;
                        s0 = sgn > 0 ? qv - lo : hi - qv;
                    }
                }
            }
            int incl = need;
#pragma unroll
            for (int off = 1; off < G; off <<= 1) {
                const int t = __shfl_up(incl, off, G);
                if (ln >= off) incl += t;
            }
            const int total = __shfl(incl, G - 1, G);
            const int c = base + incl - need;
            if (need && c < MAXCT) {
                S.ca[c] = LIM0 + ln;
                S.cb[c] = sgn;
                S.cp[c] = v3(0.0f, 0.0f, 0.0f);
                S.cd[c][0] = v3(0.0f, 0.0f, 0.0f);
                S.cs0[c] = s0;
                S.ce[c] = 0.0f;
                S.link_rows = 1;
            }
            base += total;
        }
        const int nct = base < MAXCT ? base : MAXCT;
        const int nanc = abase < MAXCT ? abase : MAXCT;
        __syncthreads();
        PH_MARK(1);

        // ================= 3. rows
        const bool link_rows = live && S.link_rows != 0;
        if (LA > 0 && __any(link_rows)) meff_world<MAXL, ND, G>(A, S, link_rows, ln, LA, DA, x0, lk, mcol);
        PH_MARK(2);
        // this DOF lane's joint axis and origin at the substep start
        const V3 myz = S.zl[mylink], myx = S.xl[mylink];
        // a free body's slot: its inverse mass, COM and the row of its world
        // inverse inertia this slot takes (read once, not per row)
        float fb_im = 0.0f;
        V3 fb_xc = v3(0.0f, 0.0f, 0.0f), fb_iw = v3(0.0f, 0.0f, 0.0f);
        if (is_free) {
            fb_im = S.finvm[fk];
            fb_xc = S.fxc[fk];
            const S3 I = S.fIw[fk];
            fb_iw = fc == 3 ? v3(I.xx, I.xy, I.xz) : (fc == 4 ? v3(I.xy, I.yy, I.yz) : v3(I.xz, I.yz, I.zz));
        }
        // pass 1: every row's J (and a free body's W, its slots' M^-1 J)
#pragma unroll
        for (int c = 0; c < MAXCT; ++c) {
#pragma unroll
            for (int rw = 0; rw < 3; ++rw) {
                Jr.set(c * 3 + rw, ln, 0.0f);
                Wr.set(c * 3 + rw, ln, 0.0f);
                lam.set(c * 3 + rw, 0.0f);
            }
            // row 0: contact c's normal; rows 1, 2: anchor c's friction rows
            const bool cn = c < nct, cf = c < nanc;
            if (cn || cf) {
#pragma unroll
                for (int rw = 0; rw < 3; ++rw) {
                    if (rw == 0 ? !cn : !cf) continue;
                    const int ab = rw == 0 ? 0 : S.aab[c];
                    const int a = rw == 0 ? S.ca[c] : (ab & 0xFFFF), b = rw == 0 ? S.cb[c] : (ab >> 16);
                    const V3 p = vsel(rw == 0, S.cp[c], S.apt[c]);
                    const V3 dir = S.cd[c][rw];
                    float J = 0.0f, W = 0.0f;
                    if (a >= LIM0) {
                        if (rw == 0 && ln == a - LIM0) J = (float)b;
                    } else if (is_dof) {
                        if (a < F0 && ln < 32 && ((S.amask[a] >> ln) & 1u))
                            J = myrev ? vdot(vcross(myz, vsub(p, myx)), dir) : vdot(myz, dir);
                    } else if (is_root) {
                        if (a < F0) J = rc < 3 ? v3c(vcross(vsub(p, x0), dir), rc) : v3c(dir, rc - 3);
                    } else if (is_free) {
                        const float sg = a == F0 + fk ? 1.0f : (b == F0 + fk ? -1.0f : 0.0f);
                        if (sg != 0.0f) {
                            if (fc < 3) {
                                const float dc = fc == 0 ? dir.x : (fc == 1 ? dir.y : dir.z);
                                J = sg * dc;
                                W = sg * (fb_im * dc);
                            } else {
                                // row fc - 3 of symmul(fIw, rd): the same products and sums
                                const V3 rd = vcross(vsub(p, fb_xc), dir);
                                J = sg * (fc == 3 ? rd.x : (fc == 4 ? rd.y : rd.z));
                                W = sg * vdot(fb_iw, rd);
                            }
                        }
                    }
                    Jr.set(c * 3 + rw, ln, J);
                    Wr.set(c * 3 + rw, ln, W);
                }
            }
        }
        if constexpr (G == 64) __syncthreads();   // the rows' J (EnvLds::Jl) of every slot
        // pass 2: W = M_eff^-1 J over the articulation's slots (J_k broadcast
        // from lane k). Slot k outermost: M_eff^-1 entry k is read once for all
        // rows and the rows' sums are independent chains (row-outer, each row
        // was a chain of NA dependent adds behind NA AGPR reads). Every row's sum
        // still runs k = 0, 1, ... from 0.0f: the same additions in the same
        // order. Rows beyond the env's contacts hold J = 0 and are not used.
        int cmax = nct > nanc ? nct : nanc;      // rows in use, the wave's maximum
#pragma unroll
        for (int off = G; off < 64; off <<= 1) {
            const int t = __shfl_xor(cmax, off);
            cmax = t > cmax ? t : cmax;
        }
        cmax = __builtin_amdgcn_readfirstlane(cmax);
        // (two straight-line variants by the wave's row count: a guard per
        // contact inside the slot loop split it into 256 blocks, each reloading
        // its operands from AGPRs)
        auto wpass = [&](auto cm) {
            constexpr int CM = decltype(cm)::value;
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                if (k < NA) {
                    const float m = mcol[k];
#pragma unroll
                    for (int c = 0; c < CM; ++c) {
#pragma unroll
                        for (int rw = 0; rw < 3; ++rw)
                            Wr.set(c * 3 + rw, ln, Wr.get(c * 3 + rw, ln) + m * Jr.lane(c * 3 + rw, ln, k));
                    }
                }
            }
        };
        if (link_rows && (is_dof || is_root)) {
            if (cmax <= 8) wpass(std::integral_constant<int, (MAXCT < 8 ? MAXCT : 8)>{});
            else wpass(std::integral_constant<int, MAXCT>{});
        }
        // pass 3: each row's effective mass and a normal row's approach speed
#pragma unroll
        for (int c = 0; c < MAXCT; ++c) {
            const bool cn = c < nct, cf = c < nanc;
            if (cn || cf) {
#pragma unroll
                for (int rw = 0; rw < 3; ++rw) {
                    if (rw == 0 ? !cn : !cf) continue;
                    const float den = redg<G>(Jr.get(c * 3 + rw, ln) * Wr.get(c * 3 + rw, ln));
                    const float kk = den > 0.0f ? 1.0f / den : 0.0f;
                    if (ln == 0) S.ck[c][rw] = kk;
                }
                if (cn) {
                    const float vn0 = redg<G>(Jr.get(c * 3, ln) * uv);
                    if (ln == 0) S.cvn0[c] = vn0;
                }
            }
        }
        __syncthreads();
        PH_MARK(3);

        // ================= 4. TGS (the lambdas are kept by lane 0 in LDS; every
        // lane of the env computes the same value)
        // anchors whose friction bound clamped a row in the last iteration, one
        // bit per anchor, per direction (the same in every lane of the env)
        unsigned long long clamp1 = 0ull, clamp2 = 0ull;
        for (int it = 0; it < P.npos + P.nvel; ++it) {
            const bool pos = it < P.npos;
            // the normal rows (every lane of the env holds the same lambdas: red16
            // and the LDS operands are the same in all 16 lanes)
            auto normal_pass = [&]() {
#pragma unroll
                for (int c = 0; c < MAXCT; ++c) {
                    if (c < nct) {
                        const float s = S.cs0[c] + redg<G>(Jr.get(c * 3, ln) * dp);
                        float tgt;
                        if (pos) {
                            tgt = -s * P.inv_sub;
                            if (s < 0.0f) tgt = fminf(tgt, P.max_depen);
                        } else {
                            tgt = s > 0.0f ? -s * P.inv_h : 0.0f;
                            const float ev = S.ce[c], vn0 = S.cvn0[c];
                            if (ev > 0.0f && vn0 < -P.bounce_thresh) tgt = fmaxf(tgt, -ev * vn0);
                        }
                        const float lm = lam.get(c * 3);
                        float dl = S.ck[c][0] * (tgt - redg<G>(Jr.get(c * 3, ln) * uv));
                        const float nl = fmaxf(lm + dl, 0.0f);
                        dl = nl - lm;
                        uv = uv + Wr.get(c * 3, ln) * dl;
                        lam.set(c * 3, nl);
                    }
                }
            };
            if (!MG_ENV_SWEEP_ANF || it == 0 || !pos) normal_pass();
            // each patch's normal impulse: running sums in contact order,
            // restarting at the contact that opens a patch
            {
                const unsigned long long ps = S.pstart;
                float run = 0.0f;
#pragma unroll
                for (int c = 0; c < MAXCT; ++c) {
                    if (c < nct) {
                        run = ((ps >> c) & 1ull) ? lam.get(c * 3) : run + lam.get(c * 3);
                        if (ln == 0) S.psum[c] = run;
                    }
                }
            }
            __syncthreads();
            const bool last_it = it == P.npos + P.nvel - 1;
#pragma unroll
            for (int c = 0; c < MAXCT; ++c) {
                if (c < nanc) {
                    const int al = S.alast[c];
                    const int pc = (al >> 8) & 3;
                    const float mun = S.amu[c] * S.psum[al & 0xFF];
#pragma unroll
                    for (int rw = 1; rw < 3; ++rw) {
                        // the patch's Coulomb budget mu N per direction, half of it for
                        // each of two anchors (symmetric; the two saturate at mu N)
                        const float lim = (pc ? 0.5f : 1.0f) * mun;
                        const float tgt = pos ? S.ae[c][rw - 1] : 0.0f;   // drift closing (position sweeps)
                        const float lm = lam.get(c * 3 + rw);
                        const float raw = lm + S.ck[c][rw] * (tgt - redg<G>(Jr.get(c * 3 + rw, ln) * uv));
                        const float nl = fminf(fmaxf(raw, -lim), lim);
                        if (last_it && (raw > lim || raw < -lim)) {
                            if (rw == 1) clamp1 |= 1ull << c;
                            else clamp2 |= 1ull << c;
                        }
                        const float dl = nl - lm;
                        uv = uv + Wr.get(c * 3 + rw, ln) * dl;
                        lam.set(c * 3 + rw, nl);
                    }
                }
            }
            // the last position sweep and the velocity sweeps end with the normal
            // rows again: a friction bound the size of a grip cannot drag a body
            // into a unilateral contact that eight Gauss-Seidel sweeps would not
            // converge
            if (it >= P.npos - 1 || MG_ENV_SWEEP_ANF) normal_pass();
            if (pos) dp = dp + uv * P.sub;
        }
        if (ln == 0) {
#pragma unroll
            for (int c = 0; c < MAXCT; ++c) {
                if (c < nct) S.clam[c][0] = lam.get(c * 3);
                if (c < nanc) {
                    S.clam[c][1] = lam.get(c * 3 + 1);
                    S.clam[c][2] = lam.get(c * 3 + 2);
                }
            }
        }
        // a slipping patch lets go of its anchors (regrown at the next substep):
        // every anchor it holds clamped along one direction (a Gauss-Seidel sweep
        // may leave one of two anchors at its half budget while the other holds)
        bool slip = false;
        if (ln < nanc) {
            const int pc = (S.alast[ln] >> 8) & 3;
            const int o = pc == 1 ? ln + 1 : (pc == 2 ? ln - 1 : ln);
            slip = ((((clamp1 >> ln) & (clamp1 >> o)) | ((clamp2 >> ln) & (clamp2 >> o))) & 1ull) != 0ull;
        }
        if (live && slip && ln < nanc) {
            const int pidx = S.alast[ln] >> 10;
            if (pidx < MG_FP_MAXP) A.fpatch[(size_t)(pair0 + pidx) * MG_FP_N] = 0.0f;
        }
        __syncthreads();
        PH_MARK(4);

        // ================= 5. integrate (a ball joint's three lanes turn its
        // rotation vector by its dpos together: ball_dof_step)
        S.dpos[ln] = dp;
        if (any_ball) __syncthreads();
        if (is_dof) {
            const float maxv = dc.maxv;
            float w = uv;
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            float x = qv + dp;
            if (dc.haslim) {
                const float lo = dc.lo, hi = dc.hi;
                if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
            }
            if (ballr > 0) x = ball_dof_step(S.q, S.dpos, ln - (ballr - 1), ballr);
            qv = x;
            uv = w;
        }
        __syncthreads();
        // contact impulse sums in contact order: link l on lane l, free body k on lane k
        // (normal impulses in contact order, then the anchors' friction impulses)
        // (unrolled over the static bounds, so the LDS reads of all rows issue
        // together instead of one dependent round trip per row)
        if (live && (ln < L || ln < nfr)) {
#pragma unroll
            for (int c = 0; c < 2 * MAXCT; ++c) {
                const bool fr_ = c >= MAXCT;
                const int k = fr_ ? c - MAXCT : c;
                if (fr_ ? k < nanc : k < nct) {
                    const int ab = fr_ ? S.aab[k] : 0;
                    const int a = fr_ ? (ab & 0xFFFF) : S.ca[k], b = fr_ ? (ab >> 16) : S.cb[k];
                    const bool on_link = a < LIM0 && ln < L && a == ln;
                    const bool on_fa = a < LIM0 && ln < nfr && a == F0 + ln;
                    const bool on_fb = a < LIM0 && ln < nfr && b == F0 + ln;
                    if (on_link || on_fa || on_fb) {
                        V3 imp;
                        if (fr_) imp = vmad(vscale(S.cd[k][1], S.clam[k][1]), S.cd[k][2], S.clam[k][2]);
                        else imp = vscale(S.cd[k][0], S.clam[k][0]);
                        if (on_link) lsum = vadd(lsum, imp);
                        if (on_fa) fsum = vadd(fsum, imp);
                        if (on_fb) fsum = vsub(fsum, imp);
                    }
                }
            }
        }
        if (RB > 0) {
            // floating root (every lane keeps x0, q0): the origin moves by dpos_v,
            // the orientation turns by dpos_w
            x0 = vadd(x0, v3(S.dpos[D + 3], S.dpos[D + 4], S.dpos[D + 5]));
            q0 = qintegrate(q0, v3(S.dpos[D + 0], S.dpos[D + 1], S.dpos[D + 2]));
        }
        if (live && ln < nfr) {
            const int k = ln;
            const int s0 = NS + 6 * k;
            const V3 dx = v3(S.dpos[s0 + 0], S.dpos[s0 + 1], S.dpos[s0 + 2]);
            const V3 dth = v3(S.dpos[s0 + 3], S.dpos[s0 + 4], S.dpos[s0 + 5]);
            const V3 xc1 = vadd(S.fxc[k], dx);
            S.fq[k] = qintegrate(S.fq[k], dth);
            S.fx[k] = vsub(xc1, qrot(S.fq[k], fr.com));
        }
        __syncthreads();
        PH_MARK(5);
    }
    if (!A.last) {   // to the next substep's launches (k_env_np, k_env_step)
        if (MG_ENV_FK_CARRY && LA > 0) {
            // the next substep's link poses: forward kinematics of the integrated q
            // (S.q) about the moved root, the operations aba_fk would run there
            S.q[ln] = qv;
            __syncthreads();
            aba_fk(A, S, live && L > 0, ln, LA, x0, q0);
            if (live && ln < L) {
                float* c = cy + carry_link0<G>() + MG_CARRY_LINK * ln;
                const V3 xl = S.xl[ln];
                const Q4 ql = S.ql[ln];
                c[0] = xl.x; c[1] = xl.y; c[2] = xl.z;
                c[3] = ql.x; c[4] = ql.y; c[5] = ql.z; c[6] = ql.w;
            }
        }
        if (live) {
            if (ln == 0) {
                cy[0] = x0.x; cy[1] = x0.y; cy[2] = x0.z;
                cy[3] = q0.x; cy[4] = q0.y; cy[5] = q0.z; cy[6] = q0.w;
            }
            if (ln < nfr) {
                float* c = cy + 7 + 7 * ln;
                c[0] = S.fx[ln].x; c[1] = S.fx[ln].y; c[2] = S.fx[ln].z;
                c[3] = S.fq[ln].x; c[4] = S.fq[ln].y; c[5] = S.fq[ln].z; c[6] = S.fq[ln].w;
            }
            cyl[0] = qv; cyl[1] = uv;
            cyl[2] = lsum.x; cyl[3] = lsum.y; cyl[4] = lsum.z;
            cyl[5] = fsum.x; cyl[6] = fsum.y; cyl[7] = fsum.z;
        }
        return;
    }

    // ---- outputs
    S.q[ln] = qv;
    S.u[ln] = uv;
    if (is_dof) {
        A.dof_pos[d0 + ln] = qv;
        A.dof_vel[d0 + ln] = uv;
    }
    __syncthreads();
    // joint transforms (lane l)
    if (live && ln < L && ln > 0) {
        const float* lf = A.link_f + ln * MG_LINK_F_N;
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        const V3 po = v3(lf[0], lf[1], lf[2]);
        const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
        const V3 ax = v3(lf[7], lf[8], lf[9]);
        Q4 qrel;
        V3 rr;
        link_joint(jt, (int)lf[10], po, qo, ax, S.q, dof, qrel, rr);
        S.qr[ln] = qrel;
        S.rr[ln] = rr;
    }
    __syncthreads();
    // forward kinematics and link velocities (lane 0, body frames, LDS)
    if (live && ln == 0) {
        for (int l = 0; l < L; ++l) {
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], jt = li[1], dof = li[2];
            if (p < 0) {
                S.ql[l] = q0;
                S.xl[l] = x0;
                // root velocity in the base frame (zero for a fixed base)
                const V3 w = RB ? v3(S.u[D + 0], S.u[D + 1], S.u[D + 2]) : v3(0.0f, 0.0f, 0.0f);
                const V3 vo = RB ? v3(S.u[D + 3], S.u[D + 4], S.u[D + 5]) : v3(0.0f, 0.0f, 0.0f);
                put6(S.va[l], sv(qrot(qconj(q0), w), qrot(qconj(q0), vo)));
            } else {
                const V3 ax = v3(A.link_f[l * MG_LINK_F_N + 7], A.link_f[l * MG_LINK_F_N + 8],
                                 A.link_f[l * MG_LINK_F_N + 9]);
                const float qdj = dof >= 0 ? S.u[dof] : 0.0f;
                const Q4 qrel = S.qr[l];
                const V3 rr = S.rr[l];
                SV sj = svzero();
                if (jt == MG_JOINT_REVOLUTE) sj = sv(ax, v3(0.0f, 0.0f, 0.0f));
                else if (jt == MG_JOINT_PRISMATIC) sj = sv(v3(0.0f, 0.0f, 0.0f), ax);
                const Q4 qp = S.ql[p];
                S.ql[l] = qnormalize(qmul(qp, qrel));
                S.xl[l] = vadd(S.xl[p], qrot(qp, rr));
                put6(S.va[l], svadd(x_motion(m3t(qmat(qrel)), rr, sv6(S.va[p])), svscale(sj, qdj)));
            }
        }
    }
    __syncthreads();
    if (live && blk >= 0) {
        const int b = b0 + blk;
        const Q4 ql = S.ql[ln];
        const V3 xl = S.xl[ln];
        const SV vl = sv6(S.va[ln]);
        const V3 ww = qrot(ql, vl.w);
        const V3 vw = qrot(ql, vadd(vl.v, vcross(vl.w, lk.com)));
        St[0 * nb + b] = xl.x; St[1 * nb + b] = xl.y; St[2 * nb + b] = xl.z;
        St[3 * nb + b] = ql.x; St[4 * nb + b] = ql.y; St[5 * nb + b] = ql.z; St[6 * nb + b] = ql.w;
        St[7 * nb + b] = vw.x; St[8 * nb + b] = vw.y; St[9 * nb + b] = vw.z;
        St[10 * nb + b] = ww.x; St[11 * nb + b] = ww.y; St[12 * nb + b] = ww.z;
        A.cforce[0 * nb + b] = lsum.x * P.inv_dt;
        A.cforce[1 * nb + b] = lsum.y * P.inv_dt;
        A.cforce[2 * nb + b] = lsum.z * P.inv_dt;
    }
    if (live && ln < nfr) {
        const int k = ln;
        const int b = ei[3 + k];
        const int s0 = NS + 6 * k;
        const V3 x = S.fx[k];
        const Q4 q = S.fq[k];
        St[0 * nb + b] = x.x; St[1 * nb + b] = x.y; St[2 * nb + b] = x.z;
        St[3 * nb + b] = q.x; St[4 * nb + b] = q.y; St[5 * nb + b] = q.z; St[6 * nb + b] = q.w;
        for (int c = 0; c < 6; ++c) St[(7 + c) * nb + b] = S.u[s0 + c];
        A.cforce[0 * nb + b] = fsum.x * P.inv_dt;
        A.cforce[1 * nb + b] = fsum.y * P.inv_dt;
        A.cforce[2 * nb + b] = fsum.z * P.inv_dt;
    }
    PH_MARK(7);
}

// Uncoupled fixed-base articulations (the S2 gimbal, test12_add_joint.py.py:
// 69-98): the world-frame articulated-body algorithm of the coupled step
// (aba_kin / aba_dyn, 16 lanes per articulation, 4 per wavefront, the per-articulation
// quantities in LDS) followed by the joint integration of an articulation
// without contacts — q' = q + h clamp(q' + h q'', maxv), joint limits clamped
// — and the link states by forward kinematics. Restated by
// oracle/migym_oracle.c:artic_step (aba_world_ + the same integration and
// outputs).
template <int MAXL, int G>
__global__ void __launch_bounds__(64) k_artic_lanes(MgStep P, MgArticArgs AA) {
    constexpr int EPW = 64 / G;          // envs per wavefront
    __shared__ EnvLds<MAXL, G> shm[EPW];
    const int gi = threadIdx.x / G;
    const int ln = threadIdx.x % G;
    const int a = blockIdx.x * EPW + gi;
    const bool live = a < AA.na;
    EnvLds<MAXL, G>& S = shm[gi];
    MgEnvArgs A{};
    A.nb = AA.nb; A.nd = AA.nd; A.nl = AA.nl; A.ndof = AA.ndof; A.floating = 0;
    A.link_f = AA.link_f; A.link_i = AA.link_i;
    stage_links<MAXL, G>(A);
    A.state = AA.state; A.mass = AA.mass; A.body_tmpl = AA.body_tmpl; A.tbf = AA.tbf;
    A.dof_pos = AA.dof_pos; A.dof_vel = AA.dof_vel; A.dof_tpos = AA.dof_tpos; A.dof_tvel = AA.dof_tvel;
    A.dof_force = AA.dof_force; A.dof_props = AA.dof_props; A.ext = AA.ext; A.cforce = AA.cforce;
    A.tpos_w = live ? AA.tpos_w : nullptr; A.tvel_w = live ? AA.tvel_w : nullptr; A.force_w = live ? AA.force_w : nullptr;
    const int* ai = AA.artic_i + (size_t)(live ? a : 0) * MG_ARTIC_I_N;
    const int b0 = ai[0], d0 = ai[1];
    const int nb = A.nb, nd = A.nd;
    const int LA = A.nl, DA = A.ndof;           // launch-uniform (barriers inside)
    const int L = live ? LA : 0, D = live ? DA : 0;
    float* St = A.state;
    const float* pr = A.dof_props;
    const float h = P.h;
    const bool is_dof = ln < D;
    const int ballr = is_dof ? dof_ball(A, LA, ln) : 0;   // ball joints: exponential coordinates
    const bool any_ball = __any(dof_ball(A, LA, ln % (DA > 0 ? DA : 1)) > 0);   // launch-uniform

    V3 x0 = v3(0.0f, 0.0f, 0.0f), gw = v3(0.0f, 0.0f, 0.0f);
    Q4 q0 = q4(0.0f, 0.0f, 0.0f, 1.0f);
    if (live) {
        x0 = v3(St[0 * nb + b0], St[1 * nb + b0], St[2 * nb + b0]);
        q0 = qnormalize(q4(St[3 * nb + b0], St[4 * nb + b0], St[5 * nb + b0], St[6 * nb + b0]));
        if (A.tbf[A.body_tmpl[b0] * MG_TBODY_F_N + 4] != 0.0f) gw = v3(P.g[0], P.g[1], P.g[2]);
    }
    float qv = 0.0f, uv = 0.0f;
    DofC dc = {};
    if (is_dof) {
        const int gd = d0 + ln;
        qv = A.dof_pos[gd];
        uv = A.dof_vel[gd];
        dc.mode = (int)pr[0 * nd + gd];
        dc.kp = pr[1 * nd + gd];
        dc.kd = pr[2 * nd + gd];
        dc.eff = pr[3 * nd + gd];
        dc.maxv = pr[4 * nd + gd];
        dc.lo = pr[5 * nd + gd];
        dc.hi = pr[6 * nd + gd];
        dc.haslim = pr[7 * nd + gd] != 0.0f;
        dc.arm = pr[8 * nd + gd];
        dc.tpos = A.dof_tpos[gd];
        dc.tvel = A.dof_tvel[gd];
        dc.force = A.dof_force[gd];
        if (A.tpos_w) A.tpos_w[gd] = dc.tpos;
        if (A.tvel_w) A.tvel_w[gd] = dc.tvel;
        if (A.force_w) A.force_w[gd] = dc.force;
    }
    // link ln's body (-1: a virtual link of a ball joint: no mass, no state row)
    const int bl = ln < LA ? A.link_i[ln * MG_LINK_I_N + 3] : -1;
    LinkC lk = {};
    lk.iq = q4(0.0f, 0.0f, 0.0f, 1.0f);
    if (ln < L && bl >= 0) lk = load_link(A.mass, nb, b0 + bl);

    for (int st = 0; st < P.substeps; ++st) {
        S.q[ln] = qv;
        S.u[ln] = uv;
        __syncthreads();
        bool xm = false, xp = false;     // this DOF runs at constant +-effort
        bool redo = live;
        aba_kin<MAXL, G>(P, A, S, redo, ln, LA, x0, q0, lk, b0);
        for (int att = 0; att < 2; ++att) {
            if (!__any(redo)) break;
            if (att > 0) aba_refresh<MAXL, G>(A, S, redo, ln, LA, x0, lk, b0);
            aba_dyn<MAXL, G>(P, A, S, redo, ln, LA, x0, gw, dc, is_dof, xm, xp, b0);
            // drives whose implicit force exceeds the effort limit
            bool flip = false;
            if (redo && is_dof && dc.eff > 0.0f && S.imp[ln] != 0.0f) {
                const float actf = S.tau0[ln] - S.imp[ln] * S.qdd[ln];
                if (actf > dc.eff) { xm = true; xp = true; flip = true; }
                else if (actf < -dc.eff) { xm = true; flip = true; }
            }
            redo = grp_ballot<G>(flip, gi) != 0ull;
            __syncthreads();
        }
        // integrate the joint (DOF lane); a ball joint's three lanes turn its
        // rotation vector by h w together (ball_dof_step, S.dpos as scratch)
        float w = 0.0f, x = 0.0f;
        if (is_dof) {
            w = uv + h * S.qdd[ln];
            if (dc.maxv > 0.0f) w = fminf(fmaxf(w, -dc.maxv), dc.maxv);
            x = qv + h * w;
            if (dc.haslim) {
                if (x < dc.lo) { x = dc.lo; if (w < 0.0f) w = 0.0f; }
                if (x > dc.hi) { x = dc.hi; if (w > 0.0f) w = 0.0f; }
            }
            S.dpos[ln] = h * w;
        }
        if (any_ball) {
            __syncthreads();
            if (ballr > 0) x = ball_dof_step(S.q, S.dpos, ln - (ballr - 1), ballr);
        }
        if (is_dof) {
            qv = x;
            uv = w;
        }
        __syncthreads();
    }

    // outputs: DOF state; link states by forward kinematics at the new (q, qd):
    // joint transforms per link lane, the kinematic scan on lane 0, world
    // velocities and stores per link lane
    if (is_dof) {
        A.dof_pos[d0 + ln] = qv;
        A.dof_vel[d0 + ln] = uv;
    }
    S.q[ln] = qv;
    S.u[ln] = uv;
    __syncthreads();
    float* vs = &S.va[0][0];          // link velocities (body frame), 6 per link
    if (ln < L && ln > 0) {
        const float* lf = A.link_f + ln * MG_LINK_F_N;
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        const V3 po = v3(lf[0], lf[1], lf[2]);
        const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
        const V3 ax = v3(lf[7], lf[8], lf[9]);
        Q4 qrel;
        V3 rr;
        link_joint(jt, (int)lf[10], po, qo, ax, S.q, dof, qrel, rr);
        SV sj = svzero();
        if (jt == MG_JOINT_REVOLUTE) sj = sv(ax, v3(0.0f, 0.0f, 0.0f));
        else if (jt == MG_JOINT_PRISMATIC) sj = sv(v3(0.0f, 0.0f, 0.0f), ax);
        S.qr[ln] = qrel;
        S.rr[ln] = rr;
        put6(S.xi[ln], sj);
    }
    __syncthreads();
    if (live && ln == 0) {
        for (int l = 0; l < LA; ++l) {
            const int p = A.link_i[l * MG_LINK_I_N + 0], dof = A.link_i[l * MG_LINK_I_N + 2];
            if (p < 0) {
                S.ql[l] = q0;
                S.xl[l] = x0;
                put6(vs + 6 * l, svzero());
            } else {
                const Q4 qp = S.ql[p];
                const Q4 qrel = S.qr[l];
                const float qdj = dof >= 0 ? S.u[dof] : 0.0f;
                S.ql[l] = qnormalize(qmul(qp, qrel));
                S.xl[l] = vadd(S.xl[p], qrot(qp, S.rr[l]));
                put6(vs + 6 * l, svadd(x_motion(m3t(qmat(qrel)), S.rr[l], sv6(vs + 6 * p)), svscale(sv6(S.xi[l]), qdj)));
            }
        }
    }
    __syncthreads();
    if (ln < L && bl >= 0) {
        const int b = b0 + bl;
        const SV vl = sv6(vs + 6 * ln);
        const Q4 ql = S.ql[ln];
        const V3 xl = S.xl[ln];
        const V3 ww = qrot(ql, vl.w);
        const V3 vw = qrot(ql, vadd(vl.v, vcross(vl.w, lk.com)));
        St[0 * nb + b] = xl.x; St[1 * nb + b] = xl.y; St[2 * nb + b] = xl.z;
        St[3 * nb + b] = ql.x; St[4 * nb + b] = ql.y; St[5 * nb + b] = ql.z; St[6 * nb + b] = ql.w;
        St[7 * nb + b] = vw.x; St[8 * nb + b] = vw.y; St[9 * nb + b] = vw.z;
        St[10 * nb + b] = ww.x; St[11 * nb + b] = ww.y; St[12 * nb + b] = ww.z;
        A.cforce[0 * nb + b] = 0.0f; A.cforce[1 * nb + b] = 0.0f; A.cforce[2 * nb + b] = 0.0f;
    }
}

}  // namespace

// lanes per env / articulation: 16 (4 per wavefront) up to 16 links and 16
// velocity slots; 64 (one per wavefront) up to MG_MAX_LINKS links and
// MG_ENV_SLOTS_WIDE slots
static bool mg_wide(int nl, int slots) { return nl > 16 || slots > 16; }

hipError_t mg_launch_artic_lanes(const MgStep& P, const MgArticArgs& A, hipStream_t s) {
    if (A.na <= 0) return hipSuccess;
    if (!A.fixed_base || A.nl > MG_MAX_LINKS || A.ndof > MG_ENV_SLOTS_WIDE) return hipErrorNotSupported;
    if (A.chain && A.nl >= 2 && A.nl <= 4)   // serial chain, one DOF per moving link (mg_chain.hip)
        return mg_launch_artic_chain(P, A, s);
    if (mg_wide(A.nl, A.ndof)) {
        MG_LAUNCH((k_artic_lanes<MG_MAX_LINKS, 64>), dim3(A.na), dim3(64), 0, s, P, A);
        return hipGetLastError();
    }
    const int blocks = (A.na + 3) / 4;
    if (A.nl <= 4 && A.ndof <= 4)
        MG_LAUNCH((k_artic_lanes<4, G16>), dim3(blocks), dim3(64), 0, s, P, A);
    else
        MG_LAUNCH((k_artic_lanes<16, G16>), dim3(blocks), dim3(64), 0, s, P, A);
    return hipGetLastError();
}

hipError_t mg_launch_env_step(const MgStep& P, const MgEnvArgs& A, hipStream_t s) {
    if (A.ne <= 0) return hipSuccess;
    // velocity slots: DOFs, the floating root's 6, 6 per free body (at most MG_ENV_MAXF)
    const int slots = A.ndof + (A.floating ? 6 : 0) + 6 * A.max_free;
    if (A.nl > MG_MAX_LINKS || slots > MG_ENV_SLOTS_WIDE) return hipErrorNotSupported;
    // per substep: the narrow phase (one env per wavefront), then the step
    const bool wide = mg_wide(A.nl, slots);
    const bool small = A.nl <= 4 && A.ndof <= 4 && !A.floating;
    const int blocks = (A.ne + 3) / 4;
    const int np_blocks = (A.ne + 64 / MG_NP_GN - 1) / (64 / MG_NP_GN);
    MgEnvArgs B = A;
    // k_env_np's LDS copy of the scene's shapes, shape boxes and hulls (B.nhull =
    // -1: too large, read from global memory)
    size_t scene = ((size_t)A.nshape * (MG_SHAPE_STRIDE + MG_OBB_N) + (size_t)A.nhull) * sizeof(float);
#ifndef MG_NP_SCENE_LDS_MAX
#define MG_NP_SCENE_LDS_MAX (24 * 1024)
#endif
    if (scene > MG_NP_SCENE_LDS_MAX || A.nhull < 0) {
        B.nhull = -1;
        scene = 0;
    }
    for (int sub = 0; sub < P.substeps; ++sub) {
        B.sub = sub;
        B.last = sub == P.substeps - 1 ? 1 : 0;
        if (wide) {
            MG_LAUNCH((k_env_np<MG_MAX_LINKS, 64, 64>), dim3(A.ne), dim3(64), scene, s, P, B);
            MG_LAUNCH((k_env_step<MG_MAX_LINKS, 64>), dim3(A.ne), dim3(64), 0, s, P, B);
        } else if (small) {
            MG_LAUNCH((k_env_np<4, G16, MG_NP_GN>), dim3(np_blocks), dim3(64), scene, s, P, B);
            MG_LAUNCH((k_env_step<4, G16>), dim3(blocks), dim3(64), 0, s, P, B);
        } else {
            MG_LAUNCH((k_env_np<16, G16, MG_NP_GN>), dim3(np_blocks), dim3(64), scene, s, P, B);
            MG_LAUNCH((k_env_step<16, G16>), dim3(blocks), dim3(64), 0, s, P, B);
        }
    }
    return hipGetLastError();
}

// floats of the per-env carry and contact-table records the launches above
// need (migym_capi.cpp allocates them per coupled env at the widest group's size)
extern "C" int mg_env_carry_floats(void) { return carry_n<64>(); }
extern "C" int mg_env_ctab_floats(void) { return ct_n<MG_ENV_MAXCT_WIDE>(); }
int mg_env_ctab_record_floats(int wide) { return wide ? ct_n<MG_ENV_MAXCT_WIDE>() : ct_n<MG_ENV_MAXCT>(); }
