// mg_chain.hip — k_artic_chain: the S2 servo-arm step (SURVEY.md §8d S2,
// test12_add_joint.py.py:69-98's dof_test_camera.urdf gimbal): fixed-base
// serial chains of 1..3 moving links, link l driven by DOF l - 1 (revolute or
// prismatic), not touching anything. One lane per articulation, everything in
// registers; the per-template joint constants are wave-uniform (scalar loads).
//
// Per substep, all spatial quantities in the world frame
// about the base origin x0, so no spatial transform appears anywhere:
//   forward, l = 1..D: joint transform, pose (ql, xl), motion axis xi_l,
//     velocity v_l = v_{l-1} + xi_l u_l, velocity-product acceleration
//     c_l = v_l x xi_l u_l, bias acceleration a_l = a_{l-1} + c_l (a_0 = -g),
//     the link's rigid inertia I_l in compact form (10 floats: A, h = m c, m)
//     and its bias force f_l = I_l a_l + v_l x* I_l v_l - f_ext;
//     and the bias C_j += xi_j . f_l for j <= l (recursive Newton-Euler at
//     qdd = 0: C_j = xi_j . sum_{k >= j} f_k, in the order the f_k appear);
//   and the joint-space inertia M_ij = xi_i . IC_j xi_j (IC_j = sum_{k >= j} I_k)
//     accumulated in the same pass: link k adds xi_i . (I_k xi_j) for i <= j <= k;
//   (M + diag(armature + h kd + h^2 kp)) qdd = tau0 - C by LDL^T: the implicit
//     PD drive of §3.3, exact for the linearised drive; a drive whose implicit
//     torque tau0 - (h kd + h^2 kp) qdd exceeds its effort limit is re-solved as
//     a constant torque at the limit — a new diagonal and right-hand side only,
//     the kinematics, inertias and bias forces are not recomputed;
//   semi-implicit Euler with the speed and limit clamps.
// This is the joint-space form of the articulated-body recursion (same qdd up
// to rounding). For a 3-link chain with implicit drives it does ~1/2 of the
// articulated-body pass's arithmetic, and a re-solve (every step of the S2
// bench: kp 50 against a 10 N m limit) costs ~60 operations instead of a
// second inward / outward pass. Register footprint: three compact inertias,
// axes and bias forces (21 floats per link) instead of 6x6 articulated
// inertias.
//
// With the refresh fused into the step (MG_FUSE_STEP_OUT) the kernel also
// writes the bound DOF-state rows, rigid-body rows and the base's actor-root
// row (the rows refresh_*_state_tensor would gather), with 16-B stores where
// the rows of an articulation are contiguous and aligned.
// Restated op for op by oracle/migym_oracle.c chain_step_ (explicit fmaf where
// the kernel uses it, -ffp-contract=off elsewhere): bit-identical results.
#include "mg_internal.h"
#include "mg_chainlink.h"
#include "mg_spatial.h"
#include "mg_world.h"

#ifdef MG_CHAIN_STAMPS
// diagnostic build only (tools/kbench_gimbal_stamps.py): s_memtime stamps of
// each quad-kernel wave at its phase boundaries, lane 0 -> g_chain_stamp[wave]
#define MG_CHAIN_NSTAMP 8
__device__ unsigned long long g_chain_stamp[4096][MG_CHAIN_NSTAMP];
extern "C" int mg_debug_chain_stamps(unsigned long long* out, int nwaves) {
    if (nwaves > 4096) nwaves = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_stamp), (size_t)nwaves * MG_CHAIN_NSTAMP * 8) == hipSuccess ? 0
                                                                                                             : -1;
}
__device__ __forceinline__ unsigned long long chain_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define CSTAMP(k) do { const unsigned long long t_ = chain_stamp(); \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_chain_stamp[blockIdx.x][k] = t_; } while (0)
#define CUSE(v) asm volatile("" ::"v"(v))
#else
#define CSTAMP(k) do { } while (0)
#define CUSE(v) do { } while (0)
#endif

namespace {

// compact rigid spatial inertia about x0 in world axes:
// [A, [h]x; [h]x^T, m 1], A symmetric (xx, yy, zz, xy, xz, yz), h = m (c - x0)
struct RI {
    float xx, yy, zz, xy, xz, yz;
    V3 h;
    float m;
};

// element idx of field `f` of an SoA array of row stride `n`: unsigned 32-bit
// lane offsets from a wave-uniform field base, so the compiler addresses
// every field with one VGPR offset (saddr) instead of a 64-bit address per
// field (52 of them in the output pass: 248 -> 202 VGPRs)
template <class T>
__device__ __forceinline__ T& fld(T* base, int f, int n, int idx) {
    return (base + (size_t)f * (unsigned)n)[(unsigned)idx];
}

// a x b with one rounding per component
__device__ __forceinline__ V3 fcross(V3 a, V3 b) {
    return v3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
// I x = (A w + h x v, m v - h x w)
__device__ __forceinline__ SV ri_mul(const RI& I, SV x) {
    const V3 t = fcross(I.h, x.v);
    const V3 s = fcross(I.h, x.w);
    return sv(v3(fmaf(I.xx, x.w.x, fmaf(I.xy, x.w.y, fmaf(I.xz, x.w.z, t.x))),
                 fmaf(I.xy, x.w.x, fmaf(I.yy, x.w.y, fmaf(I.yz, x.w.z, t.y))),
                 fmaf(I.xz, x.w.x, fmaf(I.yz, x.w.y, fmaf(I.zz, x.w.z, t.z)))),
              v3(fmaf(I.m, x.v.x, -s.x), fmaf(I.m, x.v.y, -s.y), fmaf(I.m, x.v.z, -s.z)));
}
__device__ __forceinline__ float sdot(SV a, SV b) {
    return fmaf(a.v.z, b.v.z, fmaf(a.v.y, b.v.y, fmaf(a.v.x, b.v.x, fmaf(a.w.z, b.w.z, fmaf(a.w.y, b.w.y, a.w.x * b.w.x)))));
}
// motion x motion, motion x force
__device__ __forceinline__ SV crm_f(SV a, SV b) { return sv(fcross(a.w, b.w), vadd(fcross(a.w, b.v), fcross(a.v, b.w))); }
__device__ __forceinline__ SV crf_f(SV a, SV f) { return sv(vadd(fcross(a.w, f.w), fcross(a.v, f.v)), fcross(a.w, f.v)); }

__device__ __forceinline__ ChainLink load_chain_link(const float* Ms, int nb, int b) {
    return chain_link_make(fld(Ms, 11, nb, b), v3(fld(Ms, 8, nb, b), fld(Ms, 9, nb, b), fld(Ms, 10, nb, b)),
                           fld(Ms, 1, nb, b), fld(Ms, 2, nb, b), fld(Ms, 3, nb, b),
                           q4(fld(Ms, 4, nb, b), fld(Ms, 5, nb, b), fld(Ms, 6, nb, b), fld(Ms, 7, nb, b)));
}

// R v, one fused chain per component (the link's rotation matrix R = qmat(ql)
// is formed once per link and pass, and rotates the COM, the joint axis and the
// child's joint offset: three quaternion rotations fewer per link)
__device__ __forceinline__ V3 rmul(const M3& R, V3 v) {
    return v3(fmaf(R.c2.x, v.z, fmaf(R.c1.x, v.y, R.c0.x * v.x)), fmaf(R.c2.y, v.z, fmaf(R.c1.y, v.y, R.c0.y * v.x)),
              fmaf(R.c2.z, v.z, fmaf(R.c1.z, v.y, R.c0.z * v.x)));
}
// the link's rigid inertia about x0 (world axes); c = its COM - x0
__device__ __forceinline__ RI world_ri(const ChainLink& K, const M3& R, V3 xl, V3 x0, V3& c) {
    // T = R Ib (rows of R: (c0.i, c1.i, c2.i)), Ic = T R^T
    const float* b = K.ib;   // xx yy zz xy xz yz
    const float ib[3][3] = {{b[0], b[3], b[4]}, {b[3], b[1], b[5]}, {b[4], b[5], b[2]}};
    const float r[3][3] = {{R.c0.x, R.c1.x, R.c2.x}, {R.c0.y, R.c1.y, R.c2.y}, {R.c0.z, R.c1.z, R.c2.z}};
    float t[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) t[i][j] = fmaf(r[i][2], ib[2][j], fmaf(r[i][1], ib[1][j], r[i][0] * ib[0][j]));
#define MG_IC(i, j) fmaf(t[i][2], r[j][2], fmaf(t[i][1], r[j][1], t[i][0] * r[j][0]))
    c = vsub(vadd(xl, rmul(R, K.com)), x0);
    const V3 h = vscale(c, K.m);
    RI I;
    // R Ib R^T + m (|c|^2 1 - c c^T)
    I.xx = fmaf(h.y, c.y, fmaf(h.z, c.z, MG_IC(0, 0)));
    I.yy = fmaf(h.x, c.x, fmaf(h.z, c.z, MG_IC(1, 1)));
    I.zz = fmaf(h.x, c.x, fmaf(h.y, c.y, MG_IC(2, 2)));
    I.xy = fmaf(-h.x, c.y, MG_IC(0, 1));
    I.xz = fmaf(-h.x, c.z, MG_IC(0, 2));
    I.yz = fmaf(-h.y, c.z, MG_IC(1, 2));
#undef MG_IC
    I.h = h;
    I.m = K.m;
    return I;
}

// link l's pose from its parent's (orientation qp, rotation matrix Rp, origin
// xp): joint rotation / offset at DOF position qj. Inside the substeps the
// orientation is not renormalised (it is rebuilt from the joint angles and the
// unit base orientation every pass: no drift); the output pass (NORM) is.
// chain_rel: the joint's rotation / offset in its parent (independent of the
// parent's pose); chain_fk_rel: composed with the parent's pose
__device__ __forceinline__ void chain_rel(int jt, V3 po, Q4 qo, V3 ax, float qj, Q4& qrel, V3& rr) {
    qrel = qo;
    rr = po;
    if (jt == MG_JOINT_REVOLUTE) qrel = qmul(qo, q_axis_angle(ax, qj));
    else if (jt == MG_JOINT_PRISMATIC) rr = vadd(po, qrot(qo, vscale(ax, qj)));
}
template <bool NORM>
__device__ __forceinline__ void chain_fk_rel(Q4 qrel, V3 rr, Q4 qp, const M3& Rp, V3 xp, Q4& ql, V3& xl) {
    ql = NORM ? qnormalize(qmul(qp, qrel)) : qmul(qp, qrel);
    xl = vadd(xp, rmul(Rp, rr));
}
template <bool NORM>
__device__ __forceinline__ void chain_fk(int jt, V3 po, Q4 qo, V3 ax, float qj, Q4 qp, const M3& Rp, V3 xp, Q4& ql,
                                         V3& xl) {
    Q4 qrel;
    V3 rr;
    chain_rel(jt, po, qo, ax, qj, qrel, rr);
    chain_fk_rel<NORM>(qrel, rr, qp, Rp, xp, ql, xl);
}
// joint l's motion axis about x0 (R: the link's rotation matrix)
__device__ __forceinline__ SV chain_axis(int jt, V3 ax, const M3& R, V3 xl, V3 x0) {
    const V3 z = rmul(R, ax);
    return jt == MG_JOINT_REVOLUTE ? sv(z, fcross(vsub(xl, x0), z)) : sv(v3(0.0f, 0.0f, 0.0f), z);
}

struct ChainDof {
    int mode, haslim;
    float kp, kd, eff, maxv, lo, hi, arm, tpos, tvel, force;
};

// drive torque tau0 and implicit inertia imp of one DOF (xm:
// effort-limited on the re-solve, xp: at +effort)
__device__ __forceinline__ void chain_drive(const ChainDof& c, float q, float u, float h, bool xm, bool xp,
                                            float& tau0, float& imp) {
    float tau = 0.0f, im = 0.0f;
    if (c.mode == MG_DOF_MODE_POS) {
        tau = c.kp * (c.tpos - q - h * u) + c.kd * (c.tvel - u);
        im = h * c.kd + h * h * c.kp;
    } else if (c.mode == MG_DOF_MODE_VEL) {
        tau = c.kd * (c.tvel - u);
        im = h * c.kd;
    } else if (c.mode == MG_DOF_MODE_EFFORT) {
        tau = c.force;
    }
    if (c.eff > 0.0f) {
        if (xm) {
            tau = xp ? c.eff : -c.eff;
            im = 0.0f;
        } else if (im == 0.0f) {
            tau = fminf(fmaxf(tau, -c.eff), c.eff);
        }
    }
    tau0 = tau;
    imp = im;
}

// (M + diag(arm + imp)) x = b by LDL^T; M given by its upper triangle M[i][j], i <= j
template <int D>
__device__ __forceinline__ void chain_solve(const float (&M)[D][D], const float* arm, const float* imp,
                                            const float* b, float* x) {
    float L[D][D], Ld[D][D], r[D], y[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        float dj = M[j][j] + (arm[j] + imp[j]);
#pragma unroll
        for (int k = 0; k < j; ++k) dj = fmaf(-L[j][k], Ld[j][k], dj);
        r[j] = 1.0f / dj;
#pragma unroll
        for (int i = j + 1; i < D; ++i) {
            float s = M[j][i];
#pragma unroll
            for (int k = 0; k < j; ++k) s = fmaf(-L[i][k], Ld[j][k], s);
            Ld[i][j] = s;
            L[i][j] = s * r[j];
        }
    }
#pragma unroll
    for (int i = 0; i < D; ++i) {
        float t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t = fmaf(-L[i][k], y[k], t);
        y[i] = t;
    }
#pragma unroll
    for (int i = D - 1; i >= 0; --i) {
        float t = y[i] * r[i];
#pragma unroll
        for (int k = i + 1; k < D; ++k) t = fmaf(-L[k][i], x[k], t);
        x[i] = t;
    }
}

#ifndef MG_CHAIN_AFF
#define MG_CHAIN_AFF 1
#endif
// instance a's first body, first DOF and link stride: computed for the
// blocked layout (AA.aff: no dependent load ahead of the state loads), else
// its artic_i row
__device__ __forceinline__ void chain_row(const MgArticArgs& AA, int a, int nbody, int& b0, int& d0, int& ls) {
    if (MG_CHAIN_AFF && AA.aff) {
        const int blk = a >> 6;
        b0 = AA.ab0 + blk * 64 * nbody + (a & 63);
        ls = min(64, AA.na - blk * 64);
        d0 = AA.ad0 + a * AA.ads;
    } else {
        const int* ai = AA.artic_i + (size_t)a * MG_ARTIC_I_N;
        b0 = ai[0];
        d0 = ai[1];
        ls = ai[3];
    }
}

// contiguous stores of n floats from registers; 16-B stores when dst is aligned
template <int N>
__device__ __forceinline__ void store_row(float* dst, const float (&v)[N]) {
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
#pragma unroll
        for (int k = 0; k + 4 <= N; k += 4)
            *reinterpret_cast<float4*>(dst + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
#pragma unroll
        for (int k = N & ~3; k < N; ++k) dst[k] = v[k];
    } else {
#pragma unroll
        for (int k = 0; k < N; ++k) dst[k] = v[k];
    }
}

#ifndef MG_CHAIN_WAVES
#define MG_CHAIN_WAVES 2
#endif
// EXT: external wrenches this step (apply_rigid_body_force_tensors); UNI: every
// instance of the launch shares its link mass constants and gravity flag
// (AA.uni, migym_capi.cpp; fixed after upload); UDOF: and its DOF properties
// (wave-uniform scalar loads instead of per-lane loads and per-lane inertia
// set-up: no VGPRs for them). s_rows / s_root: the kernel's LDS row staging.
template <int NL, bool EXT, bool UNI, bool UDOF, bool AFF>
__device__ __forceinline__ void chain_body(const MgStep& P, const MgArticArgs& AA, float* s_rows, float* s_root) {
    constexpr int D = NL - 1;
    const int a = blockIdx.x * 64 + threadIdx.x;
    const bool live = a < AA.na;
    // link l: body b0 + l * ls (migym_capi.cpp); AFF (a launch-time choice, so
    // only one form is compiled into each kernel): computed from the blocked
    // layout, and the fused refresh's rows too — no dependent index load at
    // either end of the frame
    int b0, d0, ls;
    if constexpr (AFF) {
        const int ai = live ? a : 0, blk = ai >> 6;
        b0 = AA.ab0 + blk * 64 * NL + (ai & 63);
        ls = min(64, AA.na - blk * 64);
        d0 = AA.ad0 + ai * AA.ads;
    } else {
        const int* ai = AA.artic_i + (size_t)(live ? a : 0) * MG_ARTIC_I_N;
        b0 = ai[0];
        d0 = ai[1];
        ls = ai[3];
    }
    const int nb = AA.nb, nd = AA.nd;
    float* St = AA.state;
    const float* pr = AA.dof_props;
    const float h = P.h;

    // template joint constants (wave-uniform)
    V3 po[NL], ax[NL];
    Q4 qo[NL];
    int jt[NL];
#pragma unroll
    for (int l = 1; l < NL; ++l) {
        const float* lf = AA.link_f + l * MG_LINK_F_N;
        po[l] = v3(lf[0], lf[1], lf[2]);
        qo[l] = q4(lf[3], lf[4], lf[5], lf[6]);
        ax[l] = v3(lf[7], lf[8], lf[9]);
        jt[l] = AA.link_i[l * MG_LINK_I_N + 1];
    }
    const V3 x0 = v3(fld(St, 0, nb, b0), fld(St, 1, nb, b0), fld(St, 2, nb, b0));
    const Q4 q0 = qnormalize(q4(fld(St, 3, nb, b0), fld(St, 4, nb, b0), fld(St, 5, nb, b0), fld(St, 6, nb, b0)));
    const M3 R0 = qmat(q0);
    const float gflag = UNI ? AA.uni[MG_CHAIN_UNI_GRAV] : AA.tbf[fld(AA.body_tmpl, 0, 0, b0) * MG_TBODY_F_N + 4];
    const V3 gw = gflag != 0.0f ? v3(P.g[0], P.g[1], P.g[2]) : v3(0.0f, 0.0f, 0.0f);
    float qv[D], uv[D], arm[D];
    ChainDof dc[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int gd = d0 + d;
        qv[d] = fld(AA.dof_pos, 0, 0, gd);
        uv[d] = fld(AA.dof_vel, 0, 0, gd);
        if constexpr (UDOF) {
            const float* u = AA.uni + MG_CHAIN_UNI_DOF + 9 * d;
            dc[d].mode = (int)u[0];
            dc[d].kp = u[1];
            dc[d].kd = u[2];
            dc[d].eff = u[3];
            dc[d].maxv = u[4];
            dc[d].lo = u[5];
            dc[d].hi = u[6];
            dc[d].haslim = u[7] != 0.0f;
            arm[d] = u[8];
        } else {
            dc[d].mode = (int)fld(pr, 0, nd, gd);
            dc[d].kp = fld(pr, 1, nd, gd);
            dc[d].kd = fld(pr, 2, nd, gd);
            dc[d].eff = fld(pr, 3, nd, gd);
            dc[d].maxv = fld(pr, 4, nd, gd);
            dc[d].lo = fld(pr, 5, nd, gd);
            dc[d].hi = fld(pr, 6, nd, gd);
            dc[d].haslim = fld(pr, 7, nd, gd) != 0.0f;
            arm[d] = fld(pr, 8, nd, gd);
        }
        dc[d].tpos = fld(AA.dof_tpos, 0, 0, gd);
        dc[d].tvel = fld(AA.dof_tvel, 0, 0, gd);
        dc[d].force = fld(AA.dof_force, 0, 0, gd);
        if (live) {   // fused target sets: write through (the only lane of this DOF)
            if (AA.tpos_w) fld(AA.tpos_w, 0, 0, gd) = dc[d].tpos;
            if (AA.tvel_w) fld(AA.tvel_w, 0, 0, gd) = dc[d].tvel;
            if (AA.force_w) fld(AA.force_w, 0, 0, gd) = dc[d].force;
        }
    }
    ChainLink lk[NL];
#pragma unroll
    for (int l = 1; l < NL; ++l) {
        if constexpr (UNI) {
            const float* u = AA.uni + MG_CHAIN_UNI_LINK + 10 * (l - 1);
            lk[l].m = u[0];
            lk[l].com = v3(u[1], u[2], u[3]);
#pragma unroll
            for (int k = 0; k < 6; ++k) lk[l].ib[k] = u[4 + k];
        } else {
            lk[l] = load_chain_link(AA.mass, nb, b0 + l * ls);
        }
    }

    for (int st = 0; st < P.substeps; ++st) {
        // ---- forward: poses, axes, velocities, inertias, bias forces, and the
        // joint-space inertia accumulated link by link: link k's rigid inertia
        // I_k adds xi_i . (I_k xi_j) to M_ij for i <= j <= k (M_ij = xi_i . IC_j
        // xi_j with IC_j = sum_{k >= j} I_k, summed over k in link order), so no
        // inertia is kept past its own link (registers: three waves per SIMD)
        SV xi[D];
        float Cb[D];   // bias C_j = xi_j . sum_{k >= j} f_k, accumulated as f_k appears
        float M[D][D];
        {
            Q4 qp = q0;
            M3 Rp = R0;
            V3 xp = x0;
            SV vp = svzero();
            SV ap = sv(v3(0.0f, 0.0f, 0.0f), v3(-gw.x, -gw.y, -gw.z));
#pragma unroll
            for (int l = 1; l < NL; ++l) {
                Q4 ql;
                V3 xl;
                chain_fk<false>(jt[l], po[l], qo[l], ax[l], qv[l - 1], qp, Rp, xp, ql, xl);
                const M3 Rl = qmat(ql);
                const SV x = chain_axis(jt[l], ax[l], Rl, xl, x0);
                const SV vJ = svscale(x, uv[l - 1]);
                const SV v = svadd(vp, vJ);
                const SV acc = svadd(ap, crm_f(v, vJ));
                V3 c;
                const RI I = world_ri(lk[l], Rl, xl, x0, c);
                SV f = svadd(ri_mul(I, acc), crf_f(v, ri_mul(I, v)));
                if constexpr (EXT) {   // external wrench at the COM (apply_rigid_body_force_tensors)
                    const int b = b0 + l * ls;
                    const V3 fe = v3(fld(AA.ext, 0, nb, b), fld(AA.ext, 1, nb, b), fld(AA.ext, 2, nb, b));
                    const V3 te = v3(fld(AA.ext, 3, nb, b), fld(AA.ext, 4, nb, b), fld(AA.ext, 5, nb, b));
                    f = sv(vsub(f.w, vadd(te, vcross(c, fe))), vsub(f.v, fe));
                }
                xi[l - 1] = x;
#pragma unroll
                for (int j = 0; j < l; ++j) Cb[j] = j == l - 1 ? sdot(x, f) : Cb[j] + sdot(xi[j], f);
#pragma unroll
                for (int j = 0; j < l; ++j) {
                    const SV Fm = ri_mul(I, xi[j]);
#pragma unroll
                    for (int i = 0; i <= j; ++i) {
                        const float mij = sdot(xi[i], Fm);
                        M[i][j] = j == l - 1 ? mij : M[i][j] + mij;
                    }
                }
                qp = ql;
                Rp = Rl;
                xp = xl;
                vp = v;
                ap = acc;
            }
        }
        // ---- drives and the solve; one re-solve with effort-limited drives
        float qdd[D], tau0[D], imp[D], rhs[D];
        bool xm[D], xp[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            xm[d] = false;
            xp[d] = false;
            chain_drive(dc[d], qv[d], uv[d], h, false, false, tau0[d], imp[d]);
            rhs[d] = tau0[d] - Cb[d];
        }
        chain_solve<D>(M, arm, imp, rhs, qdd);
        bool flip = false;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (dc[d].eff > 0.0f && imp[d] != 0.0f) {
                const float actf = tau0[d] - imp[d] * qdd[d];
                if (actf > dc[d].eff) { xm[d] = true; xp[d] = true; flip = true; }
                else if (actf < -dc[d].eff) { xm[d] = true; flip = true; }
            }
        }
        if (__any(flip)) {   // lanes without a flip solve the same system again
#pragma unroll
            for (int d = 0; d < D; ++d) {
                chain_drive(dc[d], qv[d], uv[d], h, xm[d], xp[d], tau0[d], imp[d]);
                rhs[d] = tau0[d] - Cb[d];
            }
            chain_solve<D>(M, arm, imp, rhs, qdd);
        }
        // ---- integrate the joints
#pragma unroll
        for (int d = 0; d < D; ++d) {
            float w = uv[d] + h * qdd[d];
            if (dc[d].maxv > 0.0f) w = fminf(fmaxf(w, -dc[d].maxv), dc[d].maxv);
            float x = qv[d] + h * w;
            if (dc[d].haslim) {
                if (x < dc[d].lo) { x = dc[d].lo; if (w < 0.0f) w = 0.0f; }
                if (x > dc[d].hi) { x = dc[d].hi; if (w > 0.0f) w = 0.0f; }
            }
            qv[d] = x;
            uv[d] = w;
        }
    }
    if (!live) return;
    // ---- outputs: DOF state; link states by forward kinematics at (q, qd)
#pragma unroll
    for (int d = 0; d < D; ++d) {
        fld(AA.dof_pos, 0, 0, d0 + d) = qv[d];
        fld(AA.dof_vel, 0, 0, d0 + d) = uv[d];
    }
    if (AA.out_dof) {
        float o[2 * D];
#pragma unroll
        for (int d = 0; d < D; ++d) { o[2 * d] = qv[d]; o[2 * d + 1] = uv[d]; }
        float* R = AA.out_dof + (size_t)d0 * 2;
        if ((reinterpret_cast<uintptr_t>(R) & 7) == 0) {
#pragma unroll
            for (int d = 0; d < D; ++d) *reinterpret_cast<float2*>(R + 2 * d) = make_float2(o[2 * d], o[2 * d + 1]);
        } else {
#pragma unroll
            for (int k = 0; k < 2 * D; ++k) R[k] = o[k];
        }
    }
    // link states by forward kinematics at (q, qd), each link's row stored as
    // soon as it is formed: into the SoA state and, with the refresh fused into
    // the step, into the bound rigid-body rows (the articulation's bodies are
    // consecutive rows: 16-B stores streamed across the link boundaries, at most
    // 3 floats carried to the next link) and the base's actor-root row
    float* orb = nullptr;
    bool contiguous = false;
    // a full wave whose 64 articulations' rows form one contiguous block (consecutive
    // actors, the S2 scene): the rows go through LDS and leave as 16-B stores of
    // consecutive addresses, 1 KB per store instruction (per lane, a store would
    // touch 64 rows 208 B apart)
    constexpr int RW = NL * MG_STATE_N;            // floats of one articulation's rows
    bool wave_tr = false, root_tr = false;
    if (AA.out_rb) {
        int g0;
        if constexpr (AFF) {
            g0 = AA.og0 + a * NL;
            contiguous = true;
        } else {
            g0 = fld(AA.out_body, 0, 0, b0);
            contiguous = true;
#pragma unroll
            for (int l = 1; l < NL; ++l) contiguous = contiguous && fld(AA.out_body, 0, 0, b0 + l * ls) == g0 + l;
        }
        orb = AA.out_rb + (size_t)g0 * MG_STATE_N;
        // wave-uniform: every lane live, and a launch wider than the SIMDs can hold
        // in one round (a latency-bound launch pays the LDS round trip: 4096
        // gimbals 12.2 -> 12.8 us; 262,144: 50.4 -> 43.4 us)
        const bool full = ((int)blockIdx.x + 1) * 64 <= AA.na && gridDim.x > 1024;
        if (full) {
            const int g00 = __builtin_amdgcn_readfirstlane(g0);
            const float* wb = AA.out_rb + (size_t)g00 * MG_STATE_N;
            wave_tr = __all(contiguous && g0 == g00 + NL * (int)threadIdx.x) &&
                      (reinterpret_cast<uintptr_t>(wb) & 15) == 0;
        }
        contiguous = contiguous && (reinterpret_cast<uintptr_t>(orb) & 15) == 0;
    }
    float carry[3] = {0.0f, 0.0f, 0.0f};
    {
        Q4 qp = q0;
        M3 Rp = R0;
        V3 xp = x0;
        SV vp = svzero();
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            Q4 ql = q0;
            V3 xl = x0;
            V3 ww = v3(0.0f, 0.0f, 0.0f), vw = v3(0.0f, 0.0f, 0.0f);
            if (l > 0) {
                chain_fk<true>(jt[l], po[l], qo[l], ax[l], qv[l - 1], qp, Rp, xp, ql, xl);
                const M3 Rl = qmat(ql);
                const SV v = svadd(vp, svscale(chain_axis(jt[l], ax[l], Rl, xl, x0), uv[l - 1]));
                // COM velocity: v_O + w x (COM - x0)
                const V3 cw = vadd(vsub(xl, x0), rmul(Rl, lk[l].com));
                ww = v.w;
                vw = vadd(v.v, fcross(v.w, cw));
                qp = ql;
                Rp = Rl;
                xp = xl;
                vp = v;
            }
            const int b = b0 + l * ls;
            const float r[MG_STATE_N] = {xl.x, xl.y, xl.z, ql.x, ql.y, ql.z, ql.w, vw.x, vw.y, vw.z, ww.x, ww.y, ww.z};
#pragma unroll
            for (int k = 0; k < MG_STATE_N; ++k) fld(St, k, nb, b) = r[k];
            if (AA.out_rb) {
                if (wave_tr) {
#pragma unroll
                    for (int k = 0; k < MG_STATE_N; ++k) s_rows[threadIdx.x * RW + l * MG_STATE_N + k] = r[k];
                } else if (contiguous) {
                    // this link's floats after the carried ones: whole float4s
                    // from the row start (l * 13 floats in), the rest carried
                    const int c0 = (l * MG_STATE_N) & 3;               // floats carried in
                    const int n = c0 + MG_STATE_N;                      // floats pending
                    const int f4 = n / 4;                               // float4 stores now
                    float* dst = orb + (l * MG_STATE_N - c0);
                    auto pend = [&](int i) { return i < c0 ? carry[i] : r[i - c0]; };
#pragma unroll
                    for (int k = 0; k < f4; ++k)
                        *reinterpret_cast<float4*>(dst + 4 * k) =
                            make_float4(pend(4 * k), pend(4 * k + 1), pend(4 * k + 2), pend(4 * k + 3));
#pragma unroll
                    for (int i = 0; i < n - 4 * f4; ++i) carry[i] = pend(4 * f4 + i);
                } else {
                    float* R = AA.out_rb + (size_t)fld(AA.out_body, 0, 0, b) * MG_STATE_N;
#pragma unroll
                    for (int k = 0; k < MG_STATE_N; ++k) R[k] = r[k];
                }
            }
            if (l == 0 && AA.out_root) {
                const int rr = AFF ? AA.or0 + a : fld(AA.out_root_row, 0, 0, b0);
                // the wave's base rows one contiguous block as well: through LDS
                const int rr0 = __builtin_amdgcn_readfirstlane(rr);
                root_tr = wave_tr && __all(rr >= 0 && rr == rr0 + (int)threadIdx.x) &&
                          (reinterpret_cast<uintptr_t>(AA.out_root + (size_t)rr0 * MG_STATE_N) & 15) == 0;
                if (root_tr) {
#pragma unroll
                    for (int k = 0; k < MG_STATE_N; ++k) s_root[threadIdx.x * MG_STATE_N + k] = r[k];
                } else if (rr >= 0) {
                    float* R = AA.out_root + (size_t)rr * MG_STATE_N;
#pragma unroll
                    for (int k = 0; k < MG_STATE_N; ++k) R[k] = r[k];
                }
            }
        }
    }
    if (wave_tr) {   // wave-uniform
        __syncthreads();
        float* wb = AA.out_rb + (size_t)__builtin_amdgcn_readfirstlane(AFF ? AA.og0 + a * NL
                                                                           : fld(AA.out_body, 0, 0, b0)) * MG_STATE_N;
        constexpr int N4 = 16 * RW;                 // float4s of the wave's block (64 * RW / 4)
#pragma unroll
        for (int j = 0; j < (N4 + 63) / 64; ++j) {
            const int f4 = j * 64 + (int)threadIdx.x;
            if (f4 < N4)
                *reinterpret_cast<float4*>(wb + 4 * f4) = *reinterpret_cast<const float4*>(s_rows + 4 * f4);
        }
        if (root_tr) {   // wave-uniform
            float* wr = AA.out_root + (size_t)__builtin_amdgcn_readfirstlane(AFF ? AA.or0 + a
                                                                                 : fld(AA.out_root_row, 0, 0, b0)) *
                                          MG_STATE_N;
#pragma unroll
            for (int j = 0; j < 4; ++j) {   // 64 x 13 floats = 208 float4s
                const int f4 = j * 64 + (int)threadIdx.x;
                if (f4 < 16 * MG_STATE_N)
                    *reinterpret_cast<float4*>(wr + 4 * f4) = *reinterpret_cast<const float4*>(s_root + 4 * f4);
            }
        }
    }
    // NL * 13 floats end on a float4 boundary only for NL = 4: the last link's
    // remaining floats (NL < 4)
    if (AA.out_rb && contiguous && !wave_tr) {
        constexpr int rem = (NL * MG_STATE_N) & 3;
#pragma unroll
        for (int i = 0; i < rem; ++i) orb[NL * MG_STATE_N - rem + i] = carry[i];
    }
}

// ---- four lanes per chain (launches of at most one resident round) ----------
// At the S2 size (4096 gimbals = 64 waves of one lane per gimbal on 1024 SIMDs)
// the step is one wave's instruction stream (profiles/r05_sq_chain_4096.json:
// 3,934 VALU per wave, 65 % of its quad-cycles issuing): the chain kernel runs
// on four lanes per articulation instead, lane k of a quad owning link k.
// Lane l forms joint l's rotation in its parent (chain_rel: the sin / cos
// series) and the quad broadcasts them (DPP quad_perm); every lane then runs the
// serial scan (poses, axes, velocities, bias accelerations) itself; lane l
// forms link l's world inertia, bias force and its terms of the bias C and the
// joint-space inertia M, the quad broadcasts the terms, and every lane adds
// them in link order and solves, exactly as chain_body does. In the output pass lane l stores link l's rows (lane 0 the base's,
// the root row and the DOF rows). The same operations on the same values in
// the same order: bit-identical to chain_body and to the oracle's chain_step_.
template <int CTRL>
__device__ __forceinline__ float qdpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// lane k of each quad, to the whole quad (quad_perm [k, k, k, k])
template <int K>
__device__ __forceinline__ float qbc(float v) { return qdpp<K | (K << 2) | (K << 4) | (K << 6)>(v); }
template <int K>
__device__ __forceinline__ V3 qbc3(V3 v) { return v3(qbc<K>(v.x), qbc<K>(v.y), qbc<K>(v.z)); }
template <int K>
__device__ __forceinline__ SV qbcs(SV v) { return sv(qbc3<K>(v.w), qbc3<K>(v.v)); }
template <int K>
__device__ __forceinline__ RI qbci(const RI& I) {
    RI r;
    r.xx = qbc<K>(I.xx); r.yy = qbc<K>(I.yy); r.zz = qbc<K>(I.zz);
    r.xy = qbc<K>(I.xy); r.xz = qbc<K>(I.xz); r.yz = qbc<K>(I.yz);
    r.h = qbc3<K>(I.h);
    r.m = qbc<K>(I.m);
    return r;
}
template <int K>
__device__ __forceinline__ Q4 qbcq(Q4 q) { return q4(qbc<K>(q.x), qbc<K>(q.y), qbc<K>(q.z), qbc<K>(q.w)); }

// joint K's chain_rel from lane K (value selects: a ternary on Q4 / V3 objects
// selects their addresses and puts them in scratch)
template <int K>
__device__ __forceinline__ void chain_rel_bc(int jt, Q4 qo, V3 po, Q4 a, V3 b, Q4& qr, V3& rr) {
    qr = qo;
    rr = po;
    if (jt == MG_JOINT_REVOLUTE) qr = qbcq<K>(a);
    else if (jt == MG_JOINT_PRISMATIC) rr = qbc3<K>(b);
}
// every joint's chain_rel at DOF positions q: lane k of the quad forms joint
// k's (lanes 0 and k > D: joint 1's; its constants by per-lane loads: a
// register-array select by the lane's link becomes a scratch lookup), the quad
// broadcasts them
struct ChainJoint {
    int jt;
    V3 po, ax;
    Q4 qo;
};
__device__ __forceinline__ ChainJoint chain_joint(const MgArticArgs& AA, int l) {
    const float* lf = AA.link_f + l * MG_LINK_F_N;
    ChainJoint J;
    J.po = v3(lf[0], lf[1], lf[2]);
    J.qo = q4(lf[3], lf[4], lf[5], lf[6]);
    J.ax = v3(lf[7], lf[8], lf[9]);
    J.jt = AA.link_i[l * MG_LINK_I_N + 1];
    return J;
}
template <int NL>
__device__ __forceinline__ void chain_rels_q(const ChainJoint& Jm, int ml, const int (&jt)[NL], const V3 (&po)[NL],
                                             const Q4 (&qo)[NL], const float* q, Q4 (&qr)[NL], V3 (&rr)[NL]) {
    // the lane's DOF position: selects of register values (a select of two loads
    // from one array is folded into a load at a selected index, which sends the
    // array to LDS)
    float qs[NL - 1];
#pragma unroll
    for (int d = 0; d < NL - 1; ++d) {
        qs[d] = q[d];
        asm volatile("" : "+v"(qs[d]));
    }
    float qm = qs[0];
    if constexpr (NL > 2) qm = ml == 2 ? qs[1] : qm;
    if constexpr (NL > 3) qm = ml == 3 ? qs[2] : qm;
    Q4 a;
    V3 b;
    chain_rel(Jm.jt, Jm.po, Jm.qo, Jm.ax, qm, a, b);
    chain_rel_bc<1>(jt[1], qo[1], po[1], a, b, qr[1], rr[1]);
    if constexpr (NL > 2) chain_rel_bc<2>(jt[2], qo[2], po[2], a, b, qr[2], rr[2]);
    if constexpr (NL > 3) chain_rel_bc<3>(jt[3], qo[3], po[3], a, b, qr[3], rr[3]);
}
// link K's terms of the bias C and the joint-space inertia M (from lane K of
// the quad) added in link order: chain_body's accumulation, term for term
template <int K, int D>
__device__ __forceinline__ void chain_terms_q(const float (&ct)[D], const float (&mt)[D][D], float (&Cb)[D],
                                              float (&M)[D][D]) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float c = qbc<K>(ct[j]);
        Cb[j] = j == K - 1 ? c : Cb[j] + c;
#pragma unroll
        for (int i = 0; i <= j; ++i) {
            const float m = qbc<K>(mt[i][j]);
            M[i][j] = j == K - 1 ? m : M[i][j] + m;
        }
    }
}

template <int NL, bool EXT, bool UNI, bool UDOF>
__device__ __forceinline__ void chain_body_q(const MgStep& P, const MgArticArgs& AA) {
    constexpr int D = NL - 1;
    CSTAMP(0);
    const int t = blockIdx.x * 64 + threadIdx.x;
    const int qd = threadIdx.x & 3;             // lane in the quad: this lane's link
    const int a = t >> 2;
    const bool live = a < AA.na;
    int b0, d0, ls;
    chain_row(AA, live ? a : 0, NL, b0, d0, ls);
    const int nb = AA.nb, nd = AA.nd;
    float* St = AA.state;
    const float* pr = AA.dof_props;
    const float h = P.h;
    const int ml = qd >= 1 && qd <= D ? qd : 1;  // the link whose inertia / bias force this lane forms
    const ChainJoint Jm = chain_joint(AA, ml);

    V3 po[NL], ax[NL];
    Q4 qo[NL];
    int jt[NL];
#pragma unroll
    for (int l = 1; l < NL; ++l) {
        const float* lf = AA.link_f + l * MG_LINK_F_N;
        po[l] = v3(lf[0], lf[1], lf[2]);
        qo[l] = q4(lf[3], lf[4], lf[5], lf[6]);
        ax[l] = v3(lf[7], lf[8], lf[9]);
        jt[l] = AA.link_i[l * MG_LINK_I_N + 1];
    }
    const V3 x0 = v3(fld(St, 0, nb, b0), fld(St, 1, nb, b0), fld(St, 2, nb, b0));
    const Q4 q0 = qnormalize(q4(fld(St, 3, nb, b0), fld(St, 4, nb, b0), fld(St, 5, nb, b0), fld(St, 6, nb, b0)));
    const M3 R0 = qmat(q0);
    const float gflag = UNI ? AA.uni[MG_CHAIN_UNI_GRAV] : AA.tbf[fld(AA.body_tmpl, 0, 0, b0) * MG_TBODY_F_N + 4];
    const V3 gw = gflag != 0.0f ? v3(P.g[0], P.g[1], P.g[2]) : v3(0.0f, 0.0f, 0.0f);
    float qv[D], uv[D], arm[D];
    ChainDof dc[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int gd = d0 + d;
        qv[d] = fld(AA.dof_pos, 0, 0, gd);
        uv[d] = fld(AA.dof_vel, 0, 0, gd);
        if constexpr (UDOF) {
            const float* u = AA.uni + MG_CHAIN_UNI_DOF + 9 * d;
            dc[d].mode = (int)u[0]; dc[d].kp = u[1]; dc[d].kd = u[2]; dc[d].eff = u[3]; dc[d].maxv = u[4];
            dc[d].lo = u[5]; dc[d].hi = u[6]; dc[d].haslim = u[7] != 0.0f; arm[d] = u[8];
        } else {
            dc[d].mode = (int)fld(pr, 0, nd, gd); dc[d].kp = fld(pr, 1, nd, gd); dc[d].kd = fld(pr, 2, nd, gd);
            dc[d].eff = fld(pr, 3, nd, gd); dc[d].maxv = fld(pr, 4, nd, gd); dc[d].lo = fld(pr, 5, nd, gd);
            dc[d].hi = fld(pr, 6, nd, gd); dc[d].haslim = fld(pr, 7, nd, gd) != 0.0f; arm[d] = fld(pr, 8, nd, gd);
        }
        dc[d].tpos = fld(AA.dof_tpos, 0, 0, gd);
        dc[d].tvel = fld(AA.dof_tvel, 0, 0, gd);
        dc[d].force = fld(AA.dof_force, 0, 0, gd);
        if (live && qd == 0) {   // fused target sets: write through (one lane of the quad)
            if (AA.tpos_w) fld(AA.tpos_w, 0, 0, gd) = dc[d].tpos;
            if (AA.tvel_w) fld(AA.tvel_w, 0, 0, gd) = dc[d].tvel;
            if (AA.force_w) fld(AA.force_w, 0, 0, gd) = dc[d].force;
        }
    }
    // this lane's link's mass constants
    ChainLink lk;
    if constexpr (UNI) {
        const float* u = AA.uni + MG_CHAIN_UNI_LINK + 10 * (ml - 1);
        lk.m = u[0];
        lk.com = v3(u[1], u[2], u[3]);
#pragma unroll
        for (int k = 0; k < 6; ++k) lk.ib[k] = u[4 + k];
    } else {
        lk = load_chain_link(AA.mass, nb, b0 + ml * ls);
    }

    CUSE(x0.x); CUSE(q0.w); CUSE(qv[0]); CUSE(uv[D - 1]); CUSE(dc[D - 1].tpos); CUSE(lk.m);
    CSTAMP(1);   // inputs in registers
    for (int st = 0; st < P.substeps; ++st) {
        SV xi[D];
        // ---- the serial scan (every lane); the values of link ml kept aside
        M3 Rm = R0;
        V3 xm = x0;
        SV vm = svzero(), am = svzero();
        {
            Q4 qr[NL];
            V3 rr[NL];
            chain_rels_q<NL>(Jm, ml, jt, po, qo, qv, qr, rr);
            Q4 qp = q0;
            M3 Rp = R0;
            V3 xp = x0;
            SV vp = svzero();
            SV ap = sv(v3(0.0f, 0.0f, 0.0f), v3(-gw.x, -gw.y, -gw.z));
#pragma unroll
            for (int l = 1; l < NL; ++l) {
                Q4 ql;
                V3 xl;
                chain_fk_rel<false>(qr[l], rr[l], qp, Rp, xp, ql, xl);
                const M3 Rl = qmat(ql);
                const SV x = chain_axis(jt[l], ax[l], Rl, xl, x0);
                const SV vJ = svscale(x, uv[l - 1]);
                const SV v = svadd(vp, vJ);
                const SV acc = svadd(ap, crm_f(v, vJ));
                xi[l - 1] = x;
                if (l == ml) { Rm = Rl; xm = xl; vm = v; am = acc; }
                qp = ql;
                Rp = Rl;
                xp = xl;
                vp = v;
                ap = acc;
            }
        }
        // ---- link ml's rigid inertia about x0 and bias force (lane ml)
        V3 cm;
        const RI Im = world_ri(lk, Rm, xm, x0, cm);
        SV fm = svadd(ri_mul(Im, am), crf_f(vm, ri_mul(Im, vm)));
        if constexpr (EXT) {
            const int b = b0 + ml * ls;
            const V3 fe = v3(fld(AA.ext, 0, nb, b), fld(AA.ext, 1, nb, b), fld(AA.ext, 2, nb, b));
            const V3 te = v3(fld(AA.ext, 3, nb, b), fld(AA.ext, 4, nb, b), fld(AA.ext, 5, nb, b));
            fm = sv(vsub(fm.w, vadd(te, vcross(cm, fe))), vsub(fm.v, fe));
        }
        // ---- link ml's terms of C and M (lane ml; every j < D formed, j < ml used),
        // then every link's from its lane, added in link order
        float ct[D], mt[D][D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            ct[j] = sdot(xi[j], fm);
            const SV Fm = ri_mul(Im, xi[j]);
#pragma unroll
            for (int i = 0; i <= j; ++i) mt[i][j] = sdot(xi[i], Fm);
        }
        float Cb[D];
        float M[D][D];
        chain_terms_q<1, D>(ct, mt, Cb, M);
        if constexpr (D > 1) chain_terms_q<2, D>(ct, mt, Cb, M);
        if constexpr (D > 2) chain_terms_q<3, D>(ct, mt, Cb, M);
        // ---- drives and the solve; one re-solve with effort-limited drives
        float qdd[D], tau0[D], imp[D], rhs[D];
        bool xm_[D], xp_[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            xm_[d] = false;
            xp_[d] = false;
            chain_drive(dc[d], qv[d], uv[d], h, false, false, tau0[d], imp[d]);
            rhs[d] = tau0[d] - Cb[d];
        }
        chain_solve<D>(M, arm, imp, rhs, qdd);
        bool flip = false;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (dc[d].eff > 0.0f && imp[d] != 0.0f) {
                const float actf = tau0[d] - imp[d] * qdd[d];
                if (actf > dc[d].eff) { xm_[d] = true; xp_[d] = true; flip = true; }
                else if (actf < -dc[d].eff) { xm_[d] = true; flip = true; }
            }
        }
        if (__any(flip)) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                chain_drive(dc[d], qv[d], uv[d], h, xm_[d], xp_[d], tau0[d], imp[d]);
                rhs[d] = tau0[d] - Cb[d];
            }
            chain_solve<D>(M, arm, imp, rhs, qdd);
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            float w = uv[d] + h * qdd[d];
            if (dc[d].maxv > 0.0f) w = fminf(fmaxf(w, -dc[d].maxv), dc[d].maxv);
            float x = qv[d] + h * w;
            if (dc[d].haslim) {
                if (x < dc[d].lo) { x = dc[d].lo; if (w < 0.0f) w = 0.0f; }
                if (x > dc[d].hi) { x = dc[d].hi; if (w > 0.0f) w = 0.0f; }
            }
            qv[d] = x;
            uv[d] = w;
        }
        CUSE(qv[0]);
        if (st == 0) CSTAMP(2); else CSTAMP(3);
    }
    if (!live) return;   // whole quads
    // ---- outputs: DOF state (lane 0); link qd's state by forward kinematics (lane qd)
    Q4 qr[NL];
    V3 rr[NL];
    chain_rels_q<NL>(Jm, ml, jt, po, qo, qv, qr, rr);   // the whole quad, before lanes leave
    if (qd == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            fld(AA.dof_pos, 0, 0, d0 + d) = qv[d];
            fld(AA.dof_vel, 0, 0, d0 + d) = uv[d];
        }
        if (AA.out_dof) {
            float* R = AA.out_dof + (size_t)d0 * 2;
#pragma unroll
            for (int d = 0; d < D; ++d) { R[2 * d] = qv[d]; R[2 * d + 1] = uv[d]; }
        }
    }
    if (qd >= NL) return;
    float r[MG_STATE_N] = {x0.x, x0.y, x0.z, q0.x, q0.y, q0.z, q0.w, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    {
        Q4 qp = q0;
        M3 Rp = R0;
        V3 xp = x0;
        SV vp = svzero();
#pragma unroll
        for (int l = 1; l < NL; ++l) {
            Q4 ql;
            V3 xl;
            chain_fk_rel<true>(qr[l], rr[l], qp, Rp, xp, ql, xl);
            const M3 Rl = qmat(ql);
            const SV v = svadd(vp, svscale(chain_axis(jt[l], ax[l], Rl, xl, x0), uv[l - 1]));
            if (l == qd) {
                // COM velocity: v_O + w x (COM - x0) (lane qd's own link constants)
                const V3 cw = vadd(vsub(xl, x0), rmul(Rl, lk.com));
                const V3 vw = vadd(v.v, fcross(v.w, cw));
                r[0] = xl.x; r[1] = xl.y; r[2] = xl.z;
                r[3] = ql.x; r[4] = ql.y; r[5] = ql.z; r[6] = ql.w;
                r[7] = vw.x; r[8] = vw.y; r[9] = vw.z;
                r[10] = v.w.x; r[11] = v.w.y; r[12] = v.w.z;
            }
            qp = ql;
            Rp = Rl;
            xp = xl;
            vp = v;
        }
    }
    CUSE(r[0]); CUSE(r[12]);
    CSTAMP(4);   // output rows formed
    const int b = b0 + qd * ls;
    // the fused refresh's rows: computed when the upload found them affine
    // (loading the indices with the inputs instead measured the same as at the
    // end: 9.88 vs 9.89 us at 4096 gimbals)
    const bool oaff = MG_CHAIN_AFF && AA.aff && AA.out_aff;
    const int out_b = AA.out_rb ? (oaff ? AA.og0 + a * NL + qd : fld(AA.out_body, 0, 0, b)) : 0;
    const int out_r = AA.out_root ? (oaff ? AA.or0 + a : fld(AA.out_root_row, 0, 0, b0)) : -1;
#pragma unroll
    for (int k = 0; k < MG_STATE_N; ++k) fld(St, k, nb, b) = r[k];
    if (AA.out_rb) {
        float* R = AA.out_rb + (size_t)out_b * MG_STATE_N;
#pragma unroll
        for (int k = 0; k < MG_STATE_N; ++k) R[k] = r[k];
    }
    if (qd == 0 && AA.out_root) {
        const int rr = out_r;
        if (rr >= 0) {
            float* R = AA.out_root + (size_t)rr * MG_STATE_N;
#pragma unroll
            for (int k = 0; k < MG_STATE_N; ++k) R[k] = r[k];
        }
    }
    CSTAMP(5);   // stores issued
#ifdef MG_CHAIN_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CSTAMP(6);   // stores complete
#endif
}

template <int NL, bool EXT, bool UNI>
__global__ void __launch_bounds__(64, 2) k_artic_chain_q(MgStep P, MgArticArgs AA) {
    if constexpr (UNI) {
        if (AA.uni[MG_CHAIN_UNI_DOFOK] != 0.0f) chain_body_q<NL, EXT, true, true>(P, AA);
        else chain_body_q<NL, EXT, true, false>(P, AA);
    } else {
        chain_body_q<NL, EXT, false, false>(P, AA);
    }
}

// The DOF constants' uniformity is read at run time (AA.uni[MG_CHAIN_UNI_DOFOK],
// one scalar load, the same branch for the whole launch): a hipGraph captured
// while every instance shared them keeps stepping correctly after a
// set_actor_dof_properties makes one differ, as the per-lane
// path reads d_dof_props in place.
template <int NL, bool EXT, bool UNI, bool AFF>
__global__ void __launch_bounds__(64, MG_CHAIN_WAVES) k_artic_chain(MgStep P, MgArticArgs AA) {
    __shared__ __align__(16) float s_rows[64 * NL * MG_STATE_N];
    __shared__ __align__(16) float s_root[64 * MG_STATE_N];
    if constexpr (UNI) {
        if (AA.uni[MG_CHAIN_UNI_DOFOK] != 0.0f) chain_body<NL, EXT, true, true, AFF>(P, AA, s_rows, s_root);
        else chain_body<NL, EXT, true, false, AFF>(P, AA, s_rows, s_root);
    } else {
        chain_body<NL, EXT, false, false, false>(P, AA, s_rows, s_root);
    }
}

}  // namespace

// serial chains of 2..4 links (fixed base, link l driven by DOF l - 1)
hipError_t mg_launch_artic_chain(const MgStep& P, const MgArticArgs& A, hipStream_t s) {
    if (A.na <= 0) return hipSuccess;
    if (!A.chain || A.nl < 2 || A.nl > 4) return hipErrorNotSupported;
    const int cb = (A.na + 63) / 64;
#ifndef MG_CHAIN_QUAD_MAX
#define MG_CHAIN_QUAD_MAX (64 * 1024)   // four lanes per chain up to this many lanes (one resident round)
#endif
    if ((long)A.na * 4 <= MG_CHAIN_QUAD_MAX) {
        const int qb = (A.na * 4 + 63) / 64;
#define MG_KQ(NL)                                                                                   \
    do {                                                                                            \
        if (A.ext) {                                                                                \
            if (A.uni) MG_LAUNCH((k_artic_chain_q<NL, true, true>), dim3(qb), dim3(64), 0, s, P, A);  \
            else MG_LAUNCH((k_artic_chain_q<NL, true, false>), dim3(qb), dim3(64), 0, s, P, A);       \
        } else {                                                                                    \
            if (A.uni) MG_LAUNCH((k_artic_chain_q<NL, false, true>), dim3(qb), dim3(64), 0, s, P, A); \
            else MG_LAUNCH((k_artic_chain_q<NL, false, false>), dim3(qb), dim3(64), 0, s, P, A);      \
        }                                                                                           \
    } while (0)
        if (A.nl == 2) MG_KQ(2);
        else if (A.nl == 3) MG_KQ(3);
        else MG_KQ(4);
#undef MG_KQ
        return hipGetLastError();
    }
#define MG_KC(NL)                                                                                       \
    do {                                                                                                \
        if (A.ext) {                                                                                    \
            if (A.uni && aff) MG_LAUNCH((k_artic_chain<NL, true, true, true>), dim3(cb), dim3(64), 0, s, P, A);   \
            else if (A.uni) MG_LAUNCH((k_artic_chain<NL, true, true, false>), dim3(cb), dim3(64), 0, s, P, A);    \
            else MG_LAUNCH((k_artic_chain<NL, true, false, false>), dim3(cb), dim3(64), 0, s, P, A);              \
        } else {                                                                                        \
            if (A.uni && aff) MG_LAUNCH((k_artic_chain<NL, false, true, true>), dim3(cb), dim3(64), 0, s, P, A);  \
            else if (A.uni) MG_LAUNCH((k_artic_chain<NL, false, true, false>), dim3(cb), dim3(64), 0, s, P, A);   \
            else MG_LAUNCH((k_artic_chain<NL, false, false, false>), dim3(cb), dim3(64), 0, s, P, A);             \
        }                                                                                               \
    } while (0)
    // the computed-row form when the upload found the rows affine (and the
    // fused refresh's rows too, when it writes them)
    const bool aff = MG_CHAIN_AFF && A.aff && ((A.out_rb == nullptr && A.out_root == nullptr) || A.out_aff);
    if (A.nl == 2) MG_KC(2);
    else if (A.nl == 3) MG_KC(3);
    else MG_KC(4);
#undef MG_KC
    return hipGetLastError();
}
