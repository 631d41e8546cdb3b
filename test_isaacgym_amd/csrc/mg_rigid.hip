// mg_rigid.hip — fused free-body step: gym.simulate() for every single-body
// dynamic actor (the servo scene's UAV and ground vehicle).
//
// One lane = one free body for the whole frame: `substeps` TGS substeps, each
//   1. unconstrained velocity: gravity, external force, PhysX-style damping
//      v *= 1 - min(damping*h, 1), max-velocity clamp;
//   2. contact generation against the ground plane (box corners, sphere and
//      capsule end caps within contact_offset), at most MG_MAX_CONTACTS slots;
//   3. TGS: npos position iterations of length h/npos, each a Gauss-Seidel pass
//      over the normal rows (speculative / depenetration target) and the
//      friction rows (Coulomb pyramid, PhysX-style), followed by integrating the
//      body's motion delta; then nvel velocity iterations with the bias removed
//      (single-shape bodies: the patch's anchor rows then the normal rows, the
//      first and the velocity sweeps opening with the normal rows too);
//   4. pose update: com += sum of iteration deltas, q = exp(dtheta) q.
// Envs are independent and (test10_servo_vecenv.py:317,323: group=i, filter=-1)
// the two actors of an env do not collide, so lanes never communicate: no
// atomics, no grid sync. State is SoA [field][body] so every load and store of
// a wavefront is one coalesced 256-B transaction per field.
//
// At the headline size (4096 envs = 128 waves on 1024 SIMDs) the frame time is
// one wave's instruction stream plus its memory round trips
// (tools/kbench_rigid_phases.py: 7.2 us with no contacts, +5.9 us for 10 of the
// 14 solver iterations), so the single-shape kernel k_rigid_step1 is built for
// latency:
//   - template constants (damping, speed limits, gravity flag and the shape
//     record) are one compact MG_TREC_N-float record per template body, staged
//     in LDS by the workgroup while the lanes' state loads are in flight: one
//     HBM round trip instead of body -> template -> shape -> ...;
//   - the 4 static contact slots are processed without branches: an inactive
//     slot has zero effective masses and a zero lever arm, so its rows apply
//     exactly zero impulse; only a wave with no contact at all skips the
//     solver loops (wave-uniform);
//   - the row updates fuse the impulse accumulation (fmaf) and clamp the
//     friction impulse with one v_med3_f32;
//   - the +Z ground (make_step's basis n = z, t1 = y, t2 = -x) is a template
//     specialisation with the cross / dot products written out.
// Multi-shape bodies run k_rigid_step (8 shift-register slots, a second launch).
// The C restatement is oracle/migym_oracle.c:rigid_body_step (same slot order,
// same specialisation, same evaluation order).
#include "mg_internal.h"
#include "mg_math.h"

#ifdef MG_RIGID1_STAMPS
// diagnostic build only (tools/kbench_rigid_stamps.py): s_memtime stamps of
// each k_rigid_step1 wave at its phase boundaries, lane 0 -> g_rigid_stamp[wave]
#define MG_RIGID1_NSTAMP 18
__device__ unsigned long long g_rigid_stamp[4096][MG_RIGID1_NSTAMP];
extern "C" int mg_debug_rigid_stamps(unsigned long long* out, int nwaves) {
    if (nwaves > 4096) nwaves = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rigid_stamp), (size_t)nwaves * MG_RIGID1_NSTAMP * 8) == hipSuccess
               ? 0
               : -1;
}
__device__ __forceinline__ unsigned long long rigid_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define RSTAMP(k) do { const unsigned long long t_ = rigid_stamp(); \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_rigid_stamp[blockIdx.x][k] = t_; } while (0)
#define RUSE(v) asm volatile("" ::"v"(v))
#else
#define RSTAMP(k) do { } while (0)
#define RUSE(v) do { } while (0)
#endif

namespace {

// ---- ground basis: general (n, t1, t2) or the +Z specialisation -----------
// Row kernels of the Gauss-Seidel chain use explicit fused multiply-adds
// (fmaf, correctly rounded like the oracle's C fmaf); everything else is built
// with -ffp-contract=off. vn / v1 / v2: velocity of the contact point along the
// row direction d (d . v + w . (r x d)); ps: separation s0 + n . dx + dth . (r x n).
__device__ __forceinline__ float fdot3(V3 a, V3 b, float acc) {
    return fmaf(a.z, b.z, fmaf(a.y, b.y, fmaf(a.x, b.x, acc)));
}
__device__ __forceinline__ V3 fmad3(V3 v, V3 d, float s) {
    return v3(fmaf(d.x, s, v.x), fmaf(d.y, s, v.y), fmaf(d.z, s, v.z));
}
struct BasisGen {
    static constexpr bool kPacked = false;
    V3 n, t1, t2;
    __device__ __forceinline__ float dn(V3 v) const { return vdot(n, v); }
    __device__ __forceinline__ float d1(V3 v) const { return vdot(t1, v); }
    __device__ __forceinline__ float d2(V3 v) const { return vdot(t2, v); }
    __device__ __forceinline__ V3 cn(V3 r) const { return vcross(r, n); }
    __device__ __forceinline__ V3 c1(V3 r) const { return vcross(r, t1); }
    __device__ __forceinline__ V3 c2(V3 r) const { return vcross(r, t2); }
    __device__ __forceinline__ V3 addn(V3 v, float s) const { return vmad(v, n, s); }
    __device__ __forceinline__ V3 add1(V3 v, float s) const { return vmad(v, t1, s); }
    __device__ __forceinline__ V3 add2(V3 v, float s) const { return vmad(v, t2, s); }
    __device__ __forceinline__ float vn(V3 v, V3 w, V3 r) const { return fdot3(w, cn(r), vdot(n, v)); }
    __device__ __forceinline__ float v1(V3 v, V3 w, V3 r) const { return fdot3(w, c1(r), vdot(t1, v)); }
    __device__ __forceinline__ float v2(V3 v, V3 w, V3 r) const { return fdot3(w, c2(r), vdot(t2, v)); }
    __device__ __forceinline__ float ps(float s0, V3 dx, V3 dth, V3 r) const {
        return fdot3(dth, cn(r), s0 + vdot(n, dx));
    }
    __device__ __forceinline__ V3 fn(V3 v, float dl, float invm) const { return fmad3(v, n, dl * invm); }
    __device__ __forceinline__ V3 f1(V3 v, float dl, float invm) const { return fmad3(v, t1, dl * invm); }
    __device__ __forceinline__ V3 f2(V3 v, float dl, float invm) const { return fmad3(v, t2, dl * invm); }
    // Iw (r x d) and (r x d) . Iw (r x d) of the three row directions
    __device__ __forceinline__ V3 iwn(const S3& I, V3 r) const { return symmul(I, cn(r)); }
    __device__ __forceinline__ V3 iw1(const S3& I, V3 r) const { return symmul(I, c1(r)); }
    __device__ __forceinline__ V3 iw2(const S3& I, V3 r) const { return symmul(I, c2(r)); }
    __device__ __forceinline__ float kn(V3 r, V3 In) const { return vdot(cn(r), In); }
    __device__ __forceinline__ float k1(V3 r, V3 I1) const { return vdot(c1(r), I1); }
    __device__ __forceinline__ float k2(V3 r, V3 I2) const { return vdot(c2(r), I2); }
};
// n = (0,0,1), t1 = (0,1,0), t2 = (-1,0,0)
struct BasisZ {
    static constexpr bool kPacked = true;   // tgs_z applies (rigid_body1<..., PACK>)
    __device__ __forceinline__ float dn(V3 v) const { return v.z; }
    __device__ __forceinline__ float d1(V3 v) const { return v.y; }
    __device__ __forceinline__ float d2(V3 v) const { return -v.x; }
    __device__ __forceinline__ V3 cn(V3 r) const { return v3(r.y, -r.x, 0.0f); }
    __device__ __forceinline__ V3 c1(V3 r) const { return v3(-r.z, 0.0f, r.x); }
    __device__ __forceinline__ V3 c2(V3 r) const { return v3(0.0f, -r.z, r.y); }
    __device__ __forceinline__ V3 addn(V3 v, float s) const { return v3(v.x, v.y, v.z + s); }
    __device__ __forceinline__ V3 add1(V3 v, float s) const { return v3(v.x, v.y + s, v.z); }
    __device__ __forceinline__ V3 add2(V3 v, float s) const { return v3(v.x - s, v.y, v.z); }
    // r x n = (r.y, -r.x, 0), r x t1 = (-r.z, 0, r.x), r x t2 = (0, -r.z, r.y): zero terms dropped
    __device__ __forceinline__ float vn(V3 v, V3 w, V3 r) const { return fmaf(w.y, -r.x, fmaf(w.x, r.y, v.z)); }
    __device__ __forceinline__ float v1(V3 v, V3 w, V3 r) const { return fmaf(w.z, r.x, fmaf(w.x, -r.z, v.y)); }
    __device__ __forceinline__ float v2(V3 v, V3 w, V3 r) const { return fmaf(w.z, r.y, fmaf(w.y, -r.z, -v.x)); }
    __device__ __forceinline__ float ps(float s0, V3 dx, V3 dth, V3 r) const {
        return fmaf(dth.y, -r.x, fmaf(dth.x, r.y, s0 + dx.z));
    }
    __device__ __forceinline__ V3 fn(V3 v, float dl, float invm) const { return v3(v.x, v.y, fmaf(dl, invm, v.z)); }
    __device__ __forceinline__ V3 f1(V3 v, float dl, float invm) const { return v3(v.x, fmaf(dl, invm, v.y), v.z); }
    __device__ __forceinline__ V3 f2(V3 v, float dl, float invm) const { return v3(fmaf(-dl, invm, v.x), v.y, v.z); }
    // symmul / vdot with the zero component of r x d dropped (symmul's term order)
    __device__ __forceinline__ V3 iwn(const S3& I, V3 r) const {
        const float a = r.y, b = -r.x;   // r x n = (a, b, 0)
        return v3(I.xx * a + I.xy * b, I.xy * a + I.yy * b, I.xz * a + I.yz * b);
    }
    __device__ __forceinline__ V3 iw1(const S3& I, V3 r) const {
        const float a = -r.z, c = r.x;   // r x t1 = (a, 0, c)
        return v3(I.xx * a + I.xz * c, I.xy * a + I.yz * c, I.xz * a + I.zz * c);
    }
    __device__ __forceinline__ V3 iw2(const S3& I, V3 r) const {
        const float b = -r.z, c = r.y;   // r x t2 = (0, b, c)
        return v3(I.xy * b + I.xz * c, I.yy * b + I.yz * c, I.yz * b + I.zz * c);
    }
    __device__ __forceinline__ float kn(V3 r, V3 In) const { return r.y * In.x + -r.x * In.y; }
    __device__ __forceinline__ float k1(V3 r, V3 I1) const { return -r.z * I1.x + r.x * I1.z; }
    __device__ __forceinline__ float k2(V3 r, V3 I2) const { return -r.z * I2.y + r.y * I2.z; }
};

// clamp x to [-lim, lim] (lim >= 0): the median of three, one instruction
__device__ __forceinline__ float clamp_sym(float x, float lim) { return __builtin_amdgcn_fmed3f(x, -lim, lim); }

struct Slot {
    V3 r;        // contact point - centre of mass (world)
    float s0;    // separation minus rest offset at substep start
    float mu, e; // combined friction / restitution
    float kn, kt1, kt2;   // effective masses
    float ln, lt1, lt2;   // accumulated impulses
    float vn0;            // pre-solve normal velocity (restitution)
    V3 In, I1, I2;        // Iw (r x n), Iw (r x t1), Iw (r x t2): cached when CACHE
    bool on;
};

// The empty asm makes the lever arm opaque to loop-invariant code motion, so
// (r x n), Iw (r x n) ... are recomputed per row instead of being hoisted for all
// 8 slots out of the iteration loop (which spilled to scratch).
#define MG_OPAQUE3(v) asm volatile("" : "+v"((v).x), "+v"((v).y), "+v"((v).z))

template <bool CACHE, class B>
__device__ __forceinline__ void contact_normal(const B& G, Slot& c, V3& v, V3& w, float invm, const S3& Iw,
                                               float tgt) {
    if (!CACHE) MG_OPAQUE3(c.r);
    const float vn = G.vn(v, w, c.r);
    const float nl = fmaxf(fmaf(c.kn, tgt - vn, c.ln), 0.0f);
    const float dl = nl - c.ln;
    c.ln = nl;
    v = G.fn(v, dl, invm);
    w = fmad3(w, CACHE ? c.In : G.iwn(Iw, c.r), dl);
}

// Coulomb friction, PhysX-style pyramid: the two tangent rows are solved one
// after the other, each accumulated impulse clamped to [-mu ln, mu ln]
// (no sqrt / divide on the Gauss-Seidel chain).
template <bool CACHE, class B>
__device__ __forceinline__ void contact_friction(const B& G, Slot& c, V3& v, V3& w, float invm, const S3& Iw) {
    if (!CACHE) MG_OPAQUE3(c.r);
    const float lim = c.mu * c.ln;
    const float vt1 = G.v1(v, w, c.r);
    const float n1 = clamp_sym(fmaf(-c.kt1, vt1, c.lt1), lim);
    const float d1 = n1 - c.lt1;
    c.lt1 = n1;
    v = G.f1(v, d1, invm);
    w = fmad3(w, CACHE ? c.I1 : G.iw1(Iw, c.r), d1);
    const float vt2 = G.v2(v, w, c.r);
    const float n2 = clamp_sym(fmaf(-c.kt2, vt2, c.lt2), lim);
    const float d2 = n2 - c.lt2;
    c.lt2 = n2;
    v = G.f2(v, d2, invm);
    w = fmad3(w, CACHE ? c.I2 : G.iw2(Iw, c.r), d2);
}

// Row targets. Position iterations: v_n >= -s / sub, capped at the maximum
// depenetration velocity (the cap only binds while penetrating: for s >= 0 the
// target is <= 0 <= max_depen). Velocity iterations: v_n >= -s / h while
// separated, else 0, raised to the restitution bounce -e v_n0 above the
// bounce threshold.
__device__ __forceinline__ float pos_target(const MgStep& P, float s) { return fminf(-s * P.inv_sub, P.max_depen); }
__device__ __forceinline__ float vel_target(const MgStep& P, float s, float e, float vn0) {
    float tgt = fminf(-s * P.inv_h, 0.0f);
    if (e > 0.0f && vn0 < -P.bounce_thresh) tgt = fmaxf(tgt, -e * vn0);
    return tgt;
}

// Identity skips shared by both kernels and the oracle (the skipped
// composition with an identity pose / a zero offset returns its input up to
// the sign of zero terms).
__device__ __forceinline__ bool shape_pose_identity(const float* sh) {
    return sh[4] == 0.0f && sh[5] == 0.0f && sh[6] == 0.0f && sh[7] == 0.0f && sh[8] == 0.0f && sh[9] == 0.0f &&
           sh[10] == 1.0f;
}
// orientation of the principal inertia frame: q iq
__device__ __forceinline__ Q4 inertia_frame(Q4 q, Q4 iq) {
    if (iq.x == 0.0f && iq.y == 0.0f && iq.z == 0.0f && iq.w == 1.0f) return q;
    return qmul(q, iq);
}
// centre of mass in the world: x + q com
__device__ __forceinline__ V3 com_world(V3 x, Q4 q, V3 com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return x;
    return vadd(x, qrot(q, com));
}
// body origin from the centre of mass: xc - q com
__device__ __forceinline__ V3 origin_from_com(V3 xc, Q4 q, V3 com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return xc;
    return vsub(xc, qrot(q, com));
}

// Candidates of one shape: emit(k, point, separation, mu, e) with k the static
// candidate index within the shape (box corner bits zyx, capsule end 0/1, the
// k-th deepest hull vertex).
template <class B, class F>
__device__ __forceinline__ void shape_candidates(const B& G, const MgStep& P, const float* sh, Q4 q, V3 x,
                                                 const float* hulls, F&& emit) {
    const int type = (int)sh[0];
    // shape pose in the world: a shape at the body origin with the body's
    // orientation (the usual URDF box / sphere) skips the composition
    Q4 qs = q;
    V3 cs = x;
    if (!shape_pose_identity(sh)) {
        qs = qmul(q, q4(sh[7], sh[8], sh[9], sh[10]));
        cs = vadd(x, qrot(q, v3(sh[4], sh[5], sh[6])));
    }
    const float mu = 0.5f * (sh[11] + P.mu_ground);
    const float e = 0.5f * (sh[12] + P.e_ground);
    if (type == MG_SHAPE_BOX) {
        // the face whose outward normal is most opposed to n: axis i* maximises
        // |n . axis_i| (first index on ties), side s* = -sign(n . axis_i*); its 4
        // corners are the candidates k = 0..3 (signs of the two other axes)
        const M3 Rs = qmat(qs);
        const float d0 = G.dn(Rs.c0), d1 = G.dn(Rs.c1), d2 = G.dn(Rs.c2);
        const float ad0 = fabsf(d0), ad1 = fabsf(d1), ad2 = fabsf(d2);
        int ia = 0;
        float best = ad0;
        if (ad1 > best) { ia = 1; best = ad1; }
        if (ad2 > best) ia = 2;
        const V3 a0 = vscale(Rs.c0, sh[1]);
        const V3 a1 = vscale(Rs.c1, sh[2]);
        const V3 a2 = vscale(Rs.c2, sh[3]);
        const float di = ia == 0 ? d0 : (ia == 1 ? d1 : d2);
        const V3 ai = ia == 0 ? a0 : (ia == 1 ? a1 : a2);
        const V3 e1 = ia == 0 ? a1 : a0;
        const V3 e2 = ia == 2 ? a1 : a2;
        const V3 u = vscale(ai, di > 0.0f ? -1.0f : 1.0f);
        const V3 cu = vadd(cs, u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float sx = (k & 1) ? 1.0f : -1.0f;
            const float sy = (k & 2) ? 1.0f : -1.0f;
            const V3 p = vadd(vadd(cu, vscale(e1, sx)), vscale(e2, sy));
            emit(k, p, G.dn(p) + P.pd, mu, e);
        }
    } else if (type == MG_SHAPE_SPHERE) {
        const float rad = sh[1];
        emit(0, G.addn(cs, -rad), G.dn(cs) + P.pd - rad, mu, e);
    } else if (type == MG_SHAPE_CAPSULE) {
        const float rad = sh[1];
        const V3 ax = vscale(qrot(qs, v3(1.0f, 0.0f, 0.0f)), sh[2]);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const V3 c = k ? vadd(cs, ax) : vsub(cs, ax);
            emit(k, G.addn(c, -rad), G.dn(c) + P.pd - rad, mu, e);
        }
    } else if (type == MG_SHAPE_CONVEX) {
        // the 4 deepest hull vertices within the contact offset, ascending
        // separation, lower vertex index first on ties
        const float* hv = hulls + (int)sh[2];
        const int nv = (int)hv[0];
        float ks[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        V3 kp[4];
        int kn = 0;
        for (int i = 0; i < nv; ++i) {
            const float* v = hv + MG_HULL_HEADER + 3 * i;
            const V3 p = vadd(cs, qrot(qs, v3(v[0], v[1], v[2])));
            const float sep = G.dn(p) + P.pd;
            if (!(sep < P.contact_offset)) continue;
            if (kn == 4 && !(sep < ks[3])) continue;
            int at = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < kn && ks[k] <= sep) at = k + 1;
#pragma unroll
            for (int k = 3; k > 0; --k)
                if (k > at) { ks[k] = ks[k - 1]; kp[k] = kp[k - 1]; }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k == at) { ks[k] = sep; kp[k] = p; }
            if (kn < 4) kn = kn + 1;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < kn) emit(k, kp[k], ks[k], mu, e);
    }
}

// MULTI = false: bodies with one shape, static slots (candidate k -> slot k),
// cached inertia vectors; MULTI = true: several shapes, shift-register slots.
template <int MAXC, bool MULTI, class B>
__device__ __forceinline__ void rigid_body(const B& G, const MgStep& P, const MgRigidArgs& A, int b) {
    constexpr bool CACHE = !MULTI;
    const int nb = A.nb;
    float* S = A.state;

    V3 x = v3(S[0 * nb + b], S[1 * nb + b], S[2 * nb + b]);
    Q4 q = q4(S[3 * nb + b], S[4 * nb + b], S[5 * nb + b], S[6 * nb + b]);
    V3 v = v3(S[7 * nb + b], S[8 * nb + b], S[9 * nb + b]);
    V3 w = v3(S[10 * nb + b], S[11 * nb + b], S[12 * nb + b]);

    const float* M = A.mass;
    const float invm = M[0 * nb + b];
    const V3 invI = v3(M[1 * nb + b], M[2 * nb + b], M[3 * nb + b]);
    const Q4 iq = q4(M[4 * nb + b], M[5 * nb + b], M[6 * nb + b], M[7 * nb + b]);
    const V3 com = v3(M[8 * nb + b], M[9 * nb + b], M[10 * nb + b]);

    const int tb = A.body_tmpl[b];
    const float lin_damp = A.tbf[tb * MG_TBODY_F_N + 0];
    const float ang_damp = A.tbf[tb * MG_TBODY_F_N + 1];
    const float max_lv = A.tbf[tb * MG_TBODY_F_N + 2];
    const float max_av = A.tbf[tb * MG_TBODY_F_N + 3];
    const float grav_on = A.tbf[tb * MG_TBODY_F_N + 4];
    const int sh0 = A.tbi[tb * MG_TBODY_I_N + 0];
    const int nsh = A.tbi[tb * MG_TBODY_I_N + 1];

    V3 fext = v3(0.0f, 0.0f, 0.0f), text = v3(0.0f, 0.0f, 0.0f);
    if (A.ext) {
        fext = v3(A.ext[0 * nb + b], A.ext[1 * nb + b], A.ext[2 * nb + b]);
        text = v3(A.ext[3 * nb + b], A.ext[4 * nb + b], A.ext[5 * nb + b]);
    }

    const float h = P.h;
    const float lin_keep = 1.0f - fminf(lin_damp * h, 1.0f);
    const float ang_keep = 1.0f - fminf(ang_damp * h, 1.0f);
    const float max_lv2 = max_lv * max_lv;
    const float max_av2 = max_av * max_av;

    q = qnormalize(q);
    V3 fsum = v3(0.0f, 0.0f, 0.0f);

    for (int st = 0; st < P.substeps; ++st) {
        const S3 Iw = sym_rdrt(qmat(inertia_frame(q, iq)), invI);
        const V3 xc = com_world(x, q, com);

        // 1. unconstrained velocity
        if (grav_on != 0.0f) v = vmad(v, v3(P.g[0], P.g[1], P.g[2]), h);
        if (A.ext) {   // applied wrench this frame (uniform; none: no update, as the oracle)
            v = vmad(v, fext, invm * h);
            w = vmad(w, symmul(Iw, text), h);
        }
        v = vscale(v, lin_keep);
        w = vscale(w, ang_keep);
        {
            float v2 = vdot(v, v);
            if (v2 > max_lv2) v = vscale(v, sqrtf(max_lv2 / v2));
            float w2 = vdot(w, w);
            if (w2 > max_av2) w = vscale(w, sqrtf(max_av2 / w2));
        }

        // 2. contacts against the ground plane
        Slot sl[MAXC];
#pragma unroll
        for (int j = 0; j < MAXC; ++j) sl[j].on = false;
        if (P.has_ground) {
            if constexpr (!MULTI) {
                // static slots: candidate k of the only shape lives in slot k
                if (nsh == 1)
                shape_candidates(G, P, A.shapes + sh0 * MG_SHAPE_STRIDE, q, x, A.hulls,
                                 [&](int k, V3 p, float sep, float mu, float e) {
                                     if (sep < P.contact_offset) {
                                         sl[k].on = true;
                                         sl[k].r = vsub(p, xc);
                                         sl[k].s0 = sep - P.rest_offset;
                                         sl[k].mu = mu;
                                         sl[k].e = e;
                                     }
                                 });
            } else {
                // several shapes: shift-register insert, newest candidate in slot 0
                int nc = 0;
                for (int s = sh0; s < sh0 + nsh; ++s) {
                    shape_candidates(G, P, A.shapes + s * MG_SHAPE_STRIDE, q, x, A.hulls,
                                     [&](int, V3 p, float sep, float mu, float e) {
                                         if (sep < P.contact_offset && nc < MAXC) {
#pragma unroll
                                             for (int j = MAXC - 1; j > 0; --j) {
                                                 sl[j].r = sl[j - 1].r; sl[j].s0 = sl[j - 1].s0;
                                                 sl[j].mu = sl[j - 1].mu; sl[j].e = sl[j - 1].e;
                                                 sl[j].on = sl[j - 1].on;
                                             }
                                             sl[0].r = vsub(p, xc); sl[0].s0 = sep - P.rest_offset;
                                             sl[0].mu = mu; sl[0].e = e; sl[0].on = true;
                                             nc = nc + 1;
                                         }
                                     });
                }
            }
        }
        // contact constants
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
            if (sl[j].on) {
                const V3 In = G.iwn(Iw, sl[j].r), I1 = G.iw1(Iw, sl[j].r), I2 = G.iw2(Iw, sl[j].r);
                if (CACHE) { sl[j].In = In; sl[j].I1 = I1; sl[j].I2 = I2; }
                sl[j].kn = 1.0f / (invm + G.kn(sl[j].r, In));
                sl[j].kt1 = 1.0f / (invm + G.k1(sl[j].r, I1));
                sl[j].kt2 = 1.0f / (invm + G.k2(sl[j].r, I2));
                sl[j].ln = 0.0f; sl[j].lt1 = 0.0f; sl[j].lt2 = 0.0f;
                sl[j].vn0 = G.vn(v, w, sl[j].r);
            }
        }

        // 3. TGS position iterations: every normal row, then every friction row
        V3 dx = v3(0.0f, 0.0f, 0.0f), dth = v3(0.0f, 0.0f, 0.0f);
        for (int it = 0; it < P.npos; ++it) {
#pragma unroll
            for (int j = 0; j < MAXC; ++j) {
                if (sl[j].on) {
                    const float s = G.ps(sl[j].s0, dx, dth, sl[j].r);
                    contact_normal<CACHE>(G, sl[j], v, w, invm, Iw, pos_target(P, s));
                }
            }
#pragma unroll
            for (int j = 0; j < MAXC; ++j)
                if (sl[j].on) contact_friction<CACHE>(G, sl[j], v, w, invm, Iw);
            dx = fmad3(dx, v, P.sub);
            dth = fmad3(dth, w, P.sub);
        }
        // velocity iterations (bias removed)
        for (int it = 0; it < P.nvel; ++it) {
#pragma unroll
            for (int j = 0; j < MAXC; ++j) {
                if (sl[j].on) {
                    const float s = G.ps(sl[j].s0, dx, dth, sl[j].r);
                    contact_normal<CACHE>(G, sl[j], v, w, invm, Iw, vel_target(P, s, sl[j].e, sl[j].vn0));
                }
            }
#pragma unroll
            for (int j = 0; j < MAXC; ++j)
                if (sl[j].on) contact_friction<CACHE>(G, sl[j], v, w, invm, Iw);
        }
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
            if (sl[j].on) {
                fsum = G.addn(fsum, sl[j].ln);
                fsum = G.add1(fsum, sl[j].lt1);
                fsum = G.add2(fsum, sl[j].lt2);
            }
        }

        // 4. pose update (centre of mass moves by the integrated delta)
        const V3 xc1 = vadd(xc, dx);
        q = qintegrate(q, dth);
        x = origin_from_com(xc1, q, com);
    }

    S[0 * nb + b] = x.x; S[1 * nb + b] = x.y; S[2 * nb + b] = x.z;
    S[3 * nb + b] = q.x; S[4 * nb + b] = q.y; S[5 * nb + b] = q.z; S[6 * nb + b] = q.w;
    S[7 * nb + b] = v.x; S[8 * nb + b] = v.y; S[9 * nb + b] = v.z;
    S[10 * nb + b] = w.x; S[11 * nb + b] = w.y; S[12 * nb + b] = w.z;
    A.cforce[0 * nb + b] = fsum.x * P.inv_dt;
    A.cforce[1 * nb + b] = fsum.y * P.inv_dt;
    A.cforce[2 * nb + b] = fsum.z * P.inv_dt;
}

// ---- single-shape bodies: k_rigid_step1 ------------------------------------
#ifndef MG_RIGID1_SHAPE_REGS
#define MG_RIGID1_SHAPE_REGS 1
#endif
// Friction is PhysX's patch friction, as in the coupled
// step (§3.6.1): the body-ground pair's contacts form one patch whose friction
// acts at up to two anchors, each fixed on the body (body frame) and on the
// ground (world point), kept from substep to substep and from step to step
// while the body's copy stays within the correlation distance of the ground's
// and the normal holds (cos >= MG_FP_NORMAL_COS in the body frame); anchors grow
// from this substep's contacts in slot order and spread over the patch
// (ground_patch_update). The record (MG_FP_N floats, the coupled record's layout) lives in
// HBM, SoA [MG_FP_N][nf1]: field 0 (the anchor count) is written every step,
// the rest only while anchors are held; a body that cannot touch the ground at
// the step's start (the far skip below) does not read it — its first substep
// has no contact, which drops any patch.
struct GPatch {
    int cnt;
    bool dirty;     // anchors / normal differ from the stored record (written back at the step's end)
    V3 nA;          // patch normal in the body frame
    V3 aA[2];       // anchor on the body (body frame)
    V3 aB[2];       // anchor on the ground (world)
};
// Anchors are placed by candidate index during the scan and turned into body
// copies (qrot_inv(q, p - x)) once per slot after it, from the scan points w0 /
// w1 (the candidate each slot ended with): the oracle's gpatch_update_ values.
// The normal test takes only the normal component of the rotated patch normal
// (G.dn: for the +Z ground one component of qrot; the same value as the
// oracle's dot product).
// Branch-free: every candidate value is formed on every lane and the oracle's
// branches become selects (the lanes of a wave hold different contact states,
// so the branches diverged and the wave paid every side plus the exec-mask
// bookkeeping: ~2.9k cycles per substep of a vehicle wave, tools/
// kbench_rigid_stamps.py). The values selected are the ones the branches
// computed, by the same operations, so results are unchanged.
template <class B>
__device__ __forceinline__ void ground_patch_update(const B& G, GPatch& R, V3 x, Q4 q, V3 n0, const V3 (&p)[4],
                                                    const float (&s0)[4], const bool (&on)[4], float fot,
                                                    float corr) {
    const float c2 = corr * corr;
    const V3 z3 = v3(0.0f, 0.0f, 0.0f);
    int cnt = R.cnt;
    const float nd = G.dn(qrot(q, R.nA));
    if (cnt > 0 && nd < MG_FP_NORMAL_COS) cnt = 0;
    // held anchors: kept while the body's copy stays within the correlation
    // distance of the ground's
    const V3 wa0 = vadd(x, qrot(q, R.aA[0]));
    const V3 wa1 = vadd(x, qrot(q, R.aA[1]));
    const V3 d0v = vsub(wa0, R.aB[0]), d1v = vsub(wa1, R.aB[1]);
    const bool k0 = 0 < cnt && vdot(d0v, d0v) <= c2;
    const bool k1 = 1 < cnt && vdot(d1v, d1v) <= c2;
    GPatch N;
    N.aA[0] = vsel(k0, R.aA[0], vsel(k1, R.aA[1], z3));
    N.aB[0] = vsel(k0, R.aB[0], vsel(k1, R.aB[1], z3));
    N.aA[1] = vsel(k0 && k1, R.aA[1], z3);
    N.aB[1] = vsel(k0 && k1, R.aB[1], z3);
    V3 w0 = vsel(k0, wa0, vsel(k1, wa1, z3));
    V3 w1 = z3;
    const int kept = (k0 ? 1 : 0) + (k1 ? 1 : 0);
    // growth from this substep's contacts in slot order (only while fewer than
    // two anchors are held): the first, then one farther than the correlation
    // distance, then a candidate replacing whichever end spreads the pair most
    int nc = kept;
    float dd = 0.0f;
    bool set0 = false, set1 = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool c = kept < 2 && on[j] && s0[j] <= fot;
        const V3 pj = p[j];
        const V3 e0 = vsub(pj, w0), e1 = vsub(pj, w1);
        const float dj0 = vdot(e0, e0), dj1 = vdot(e1, e1);
        const bool a0 = c && nc == 0;
        const bool a1 = c && nc == 1 && dj0 > c2;
        const bool a2 = c && nc == 2 && dj0 > dj1 && dj0 > dd;
        const bool a3 = c && nc == 2 && !(dj0 > dj1) && dj1 > dd;
        const bool to0 = a0 || a3, to1 = a1 || a2;
        dd = (a1 || a2) ? dj0 : (a3 ? dj1 : dd);
        w0 = vsel(to0, pj, w0);
        w1 = vsel(to1, pj, w1);
        set0 = set0 || to0;
        set1 = set1 || to1;
        nc = a0 ? 1 : (a1 ? 2 : nc);
    }
    N.aA[0] = vsel(set0, qrot_inv(q, vsub(w0, x)), N.aA[0]);
    N.aB[0] = vsel(set0, w0, N.aB[0]);
    N.aA[1] = vsel(set1, qrot_inv(q, vsub(w1, x)), N.aA[1]);
    N.aB[1] = vsel(set1, w1, N.aB[1]);
    N.cnt = nc;
    N.nA = vsel(kept > 0, R.nA, qrot_inv(q, n0));
    // the stored record changes unless every held anchor was kept in place and
    // none was placed (a resting body: most steps)
    N.dirty = R.dirty || !(kept == R.cnt && nc == kept);
    R = N;
}

// Normal row of the branch-free solver: an inactive slot holds r = 0, s0 = 0
// and kn = 0, so it computes ln = max(0 + 0 (tgt - vn), 0) = 0 and applies a
// zero impulse. Anchor rows likewise (k = 0, r = 0: raw 0 within any bound).
struct NRow {
    V3 r, In;                 // contact point - COM; Iw (r x n)
    float s0, kn, ln, vn0;
};
struct ARow {
    V3 r, I1, I2;             // anchor (body copy) - COM; Iw (r x t1), Iw (r x t2)
    float k1, k2, l1, l2;     // effective masses, accumulated impulses along t1, t2
    float e1, e2;             // position-sweep target velocities (drift closing)
};

template <class B>
__device__ __forceinline__ void row_normal1(const B& G, NRow& c, V3& v, V3& w, float invm, float tgt) {
    const float vn = G.vn(v, w, c.r);
    const float nl = fmaxf(fmaf(c.kn, tgt - vn, c.ln), 0.0f);
    const float dl = nl - c.ln;
    c.ln = nl;
    v = G.fn(v, dl, invm);
    w = fmad3(w, c.In, dl);
}

// ---- +Z ground: the solver on packed f32 pairs -------------------------------
// The same sweeps as rigid_body1's scalar loop with BasisZ (normal rows, the
// patch's anchor rows t1 = +y, t2 = -x, the closing normal pass of the last
// position sweep and the velocity sweeps), but the velocity state lives in
// register pairs W = (w.x, w.y), Z = (w.z, v.z), V = (v.x, v.y) (the motion
// delta in DW = (dth.x, dth.y), DZ = (dth.z, dx.z), DV = (dx.x, dx.y)), so one
// v_pk_fma_f32 applies two of a row's impulse updates and the separations of two
// slots share one packed chain. Each half of a packed op is the same correctly
// rounded fma / add / mul as the scalar form, so results are bit-identical to
// the scalar loop and to the oracle; only the issue count drops. Used by
// launches that fit in one resident round (the latency regime: DESIGN.md §3.2).
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk2(float a, float b) { return f2{a, b}; }
__device__ __forceinline__ f2 bc2(float a) { return f2{a, a}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// lim1 = share * mu: an anchor row's bound per unit of the patch's normal impulse
__device__ __forceinline__ void tgs_zp(const MgStep& P, NRow (&sl)[4], ARow (&an)[2], float lim1, float e, V3& v,
                                       V3& w, V3& dx, V3& dth, float invm, bool& c01, bool& c02, bool& c11,
                                       bool& c12) {
    f2 W = pk2(w.x, w.y), Z = pk2(w.z, v.z), V = pk2(v.x, v.y);
    f2 DW = pk2(dth.x, dth.y), DZ = pk2(dth.z, dx.z), DV = pk2(dx.x, dx.y);
    // the packed operands are named values, not arrays: an array of pairs built
    // lane by lane was kept in scratch (a memory round trip per substep)
    float s0r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // register copies: the pairs of loads were built through scratch
        s0r[j] = sl[j].s0;
        asm volatile("" : "+v"(s0r[j]));
    }
    const f2 S0a = pk2(s0r[0], s0r[1]), S0b = pk2(s0r[2], s0r[3]);
    const f2 RYa = pk2(sl[0].r.y, sl[1].r.y), RYb = pk2(sl[2].r.y, sl[3].r.y);
    const f2 NRXa = pk2(-sl[0].r.x, -sl[1].r.x), NRXb = pk2(-sl[2].r.x, -sl[3].r.x);
    // separations of slots (2h, 2h+1): s0 + dx.z + dth.x r.y - dth.y r.x (BasisZ::ps)
    auto sep = [&](int h) {
        f2 a = (h ? S0b : S0a) + bc2(DZ.y);
        a = pfma(bc2(DW.x), h ? RYb : RYa, a);
        return pfma(bc2(DW.y), h ? NRXb : NRXa, a);
    };
    auto normal = [&](int j, float tgt) {
        const float nrx = -sl[j].r.x, ry = sl[j].r.y;
        const float vn = fmaf(W.y, nrx, fmaf(W.x, ry, Z.y));
        const float nl = fmaxf(fmaf(sl[j].kn, tgt - vn, sl[j].ln), 0.0f);
        const float dl = nl - sl[j].ln;
        sl[j].ln = nl;
        W = pfma(pk2(sl[j].In.x, sl[j].In.y), bc2(dl), W);
        Z = pfma(pk2(sl[j].In.z, invm), bc2(dl), Z);   // Z = (w.z, v.z): In.z and 1/m (BasisZ::fn)
    };
    // the anchors' rows: t1 = +y (BasisZ::v1 / f1), t2 = -x (v2 / f2)
    auto anchors = [&](bool pos, bool last) {
        const float lim = lim1 * (((sl[0].ln + sl[1].ln) + sl[2].ln) + sl[3].ln);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const float rx = an[a].r.x, ry = an[a].r.y, nrz = -an[a].r.z;
            {
                const float v1 = fmaf(Z.x, rx, fmaf(W.x, nrz, V.y));
                const float raw = fmaf(an[a].k1, (pos ? an[a].e1 : 0.0f) - v1, an[a].l1);
                const float nl = clamp_sym(raw, lim);
                const float dl = nl - an[a].l1;
                const bool cl = last && (raw > lim || raw < -lim);
                if (a == 0) c01 = cl; else c11 = cl;
                an[a].l1 = nl;
                V.y = fmaf(dl, invm, V.y);
                W = pfma(pk2(an[a].I1.x, an[a].I1.y), bc2(dl), W);
                Z.x = fmaf(an[a].I1.z, dl, Z.x);
            }
            {
                const float v2 = fmaf(Z.x, ry, fmaf(W.y, nrz, -V.x));
                const float raw = fmaf(an[a].k2, (pos ? an[a].e2 : 0.0f) - v2, an[a].l2);
                const float nl = clamp_sym(raw, lim);
                const float dl = nl - an[a].l2;
                const bool cl = last && (raw > lim || raw < -lim);
                if (a == 0) c02 = cl; else c12 = cl;
                an[a].l2 = nl;
                V.x = fmaf(-dl, invm, V.x);
                W = pfma(pk2(an[a].I2.x, an[a].I2.y), bc2(dl), W);
                Z.x = fmaf(an[a].I2.z, dl, Z.x);
            }
        }
    };
    const f2 nsub = bc2(-P.inv_sub), psub = bc2(P.sub);
    const int nit = P.npos + P.nvel;
    // sweep order (round 6, as the oracle): a position sweep is the anchors'
    // rows then the normal rows (non-penetration has the last word before the
    // velocity is integrated); only the first opens with the normal rows
    for (int it = 0; it < P.npos; ++it) {
        const f2 t0 = sep(0) * nsub, t1 = sep(1) * nsub;   // -s / sub of each slot
        const float tg[4] = {fminf(t0.x, P.max_depen), fminf(t0.y, P.max_depen), fminf(t1.x, P.max_depen),
                             fminf(t1.y, P.max_depen)};
        if (it == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) normal(j, tg[j]);
        }
        anchors(true, it == nit - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) normal(j, tg[j]);   // same targets: dx, dth unchanged
        DV = pfma(V, psub, DV);
        DW = pfma(W, psub, DW);
        DZ = pfma(Z, psub, DZ);
    }
    if (P.nvel > 0) {
        const f2 s01 = sep(0), s23 = sep(1);
        const float sj[4] = {s01.x, s01.y, s23.x, s23.y};
        float tg[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) tg[j] = vel_target(P, sj[j], e, sl[j].vn0);
        for (int it = P.npos; it < nit; ++it) {
#pragma unroll
            for (int j = 0; j < 4; ++j) normal(j, tg[j]);
            anchors(false, it == nit - 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) normal(j, tg[j]);
        }
    }
    v = v3(V.x, V.y, Z.y);
    w = v3(W.x, W.y, Z.x);
    dx = v3(DV.x, DV.y, DZ.y);
    dth = v3(DW.x, DW.y, DZ.x);
}

// T: this body's compact template record (MG_TREC_N floats: MG_TBODY_F_N
// template floats, then the shape record; shape type < 0 when it has none).
// R: the ground patch at the step's start (cnt 0: none), at its end on return.
template <bool PACK, class B>
__device__ __forceinline__ void rigid_body1(const B& G, const MgStep& P, const float* T, V3& x, Q4& q, V3& v,
                                            V3& w, V3& fsum, float invm, V3 invI, Q4 iq, V3 com, bool has_ext,
                                            V3 fext, V3 text, const float* hulls, float* gp, int gstride) {
    const float lin_damp = T[0], ang_damp = T[1], max_lv = T[2], max_av = T[3], grav_on = T[4];
    // the shape record: wide launches read it from the template record (LDS
    // when staged) in each substep's candidate search — registers are scarcer
    // than LDS reads at three waves per SIMD; a one-round launch (PACK) keeps it
    // in registers (the LDS reads were on each substep's dependency chain)
    float shr[MG_SHAPE_STRIDE];
    const float* sh = T + MG_TBODY_F_N;
    if constexpr (PACK && MG_RIGID1_SHAPE_REGS) {
#pragma unroll
        for (int k = 0; k < 14; ++k) shr[k] = sh[k];
        sh = shr;
    }
    const bool has_shape = P.has_ground && sh[0] >= 0.0f;
    const float rho = sh[13];   // bounding radius about the body origin (< 0: none)
    const float h = P.h;
    const float lin_keep = 1.0f - fminf(lin_damp * h, 1.0f);
    const float ang_keep = 1.0f - fminf(ang_damp * h, 1.0f);
    const float max_lv2 = max_lv * max_lv;
    const float max_av2 = max_av * max_av;
    const float mu = 0.5f * (sh[11] + P.mu_ground);
    const float e = 0.5f * (sh[12] + P.e_ground);
    const V3 n0 = v3(P.n[0], P.n[1], P.n[2]);
    // the ground patch kept from the last step: read only by a body that can
    // touch the ground at this step's start (otherwise its first substep has no
    // contact and drops the patch, whatever the record holds)
    GPatch R;
    R.cnt = 0;
    R.dirty = false;
    R.nA = R.aA[0] = R.aA[1] = R.aB[0] = R.aB[1] = v3(0.0f, 0.0f, 0.0f);
    {
        const float clear = G.dn(x) + P.pd;
        const bool far = rho >= 0.0f && clear - rho > P.contact_offset + 1e-3f * (1.0f + fabsf(clear) + rho);
        if (gp && has_shape && !far) {
            float r[MG_FP_N];
#pragma unroll
            for (int k = 0; k < MG_FP_N; ++k) r[k] = gp[(size_t)k * gstride];
            R.cnt = (int)r[0];
            R.nA = v3(r[1], r[2], r[3]);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                R.aA[k] = v3(r[4 + 6 * k], r[5 + 6 * k], r[6 + 6 * k]);
                R.aB[k] = v3(r[7 + 6 * k], r[8 + 6 * k], r[9 + 6 * k]);
            }
        }
    }

    RUSE(R.cnt); RUSE(R.aA[1].z);
    RSTAMP(2);   // patch record read
    q = qnormalize(q);
    for (int st = 0; st < P.substeps; ++st) {
        const S3 Iw = sym_rdrt(qmat(inertia_frame(q, iq)), invI);
        const V3 xc = com_world(x, q, com);

        // 1. unconstrained velocity
        if (grav_on != 0.0f) v = vmad(v, v3(P.g[0], P.g[1], P.g[2]), h);
        if (has_ext) {   // applied wrench this frame (uniform; none: no update, as the oracle)
            v = vmad(v, fext, invm * h);
            w = vmad(w, symmul(Iw, text), h);
        }
        v = vscale(v, lin_keep);
        w = vscale(w, ang_keep);
        {
            float v2 = vdot(v, v);
            if (v2 > max_lv2) v = vscale(v, sqrtf(max_lv2 / v2));
            float w2 = vdot(w, w);
            if (w2 > max_av2) w = vscale(w, sqrtf(max_av2 / w2));
        }

        RUSE(v.x); RUSE(w.z); RUSE(xc.x);
        if (st < 2) RSTAMP(3 + 6 * st);   // free-flight velocity, Iw, COM
        // 2. ground contacts: candidate k of the shape -> slot k
        NRow sl[4];
        bool on[4];
        V3 cp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            on[j] = false;
            sl[j].r = v3(0.0f, 0.0f, 0.0f);
            sl[j].s0 = 0.0f;
            cp[j] = v3(0.0f, 0.0f, 0.0f);
        }
        // a body clearing the plane by more than its bounding radius (plus a
        // rounding margin far above the candidates' own error) has no candidate
        // within contact_offset: a wave of only such bodies skips the search
        const float clear = G.dn(x) + P.pd;
        const bool far = rho >= 0.0f && clear - rho > P.contact_offset + 1e-3f * (1.0f + fabsf(clear) + rho);
        if (__any(has_shape && !far) && has_shape)
            shape_candidates(G, P, sh, q, x, hulls, [&](int k, V3 p, float sep, float, float) {
                // selects, not a branch: the candidates of a wave's bodies pass
                // the test on different lanes
                const bool c = sep < P.contact_offset;
                on[k] = on[k] || c;
                sl[k].r = vsel(c, vsub(p, xc), sl[k].r);
                sl[k].s0 = c ? sep - P.rest_offset : sl[k].s0;
                cp[k] = vsel(c, p, cp[k]);
            });
        RUSE(sl[0].s0); RUSE(sl[3].r.z);
        if (st < 2) RSTAMP(4 + 6 * st);   // candidates
        bool any = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) any = any || on[j];
        // the friction patch of this substep (no contact: none)
        if (any) {
            float cs0[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) cs0[j] = sl[j].s0;
            ground_patch_update(G, R, x, q, n0, cp, cs0, on, P.fric_offset, P.fric_corr);
        } else {
            R.cnt = 0;
        }

        RUSE(R.cnt);
        if (st < 2) RSTAMP(5 + 6 * st);   // patch update
        // 3. TGS (skipped by a wave in which no body touches the ground)
        V3 dx = v3(0.0f, 0.0f, 0.0f), dth = v3(0.0f, 0.0f, 0.0f);
        if (__any(any)) {
            // contact constants (inactive slots: r = 0, so In = 0, kn = 0)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sl[j].In = G.iwn(Iw, sl[j].r);
                sl[j].kn = on[j] ? 1.0f / (invm + G.kn(sl[j].r, sl[j].In)) : 0.0f;
                sl[j].ln = 0.0f;
                sl[j].vn0 = G.vn(v, w, sl[j].r);
            }
            // anchor rows at the anchors' body copies; the position sweeps close
            // 80 % of the substep-start drift of their two copies
            ARow an[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const bool act = a < R.cnt;
                // formed on every lane, selected (a divergent branch cost more)
                const V3 wa = vadd(x, qrot(q, R.aA[a]));
                const V3 dr = vsub(wa, R.aB[a]);
                const float kd = 0.8f * P.inv_h;
                const V3 r = vsel(act, vsub(wa, xc), v3(0.0f, 0.0f, 0.0f));
                const float e1 = act ? fminf(fmaxf(-G.d1(dr) * kd, -P.max_depen), P.max_depen) : 0.0f;
                const float e2 = act ? fminf(fmaxf(-G.d2(dr) * kd, -P.max_depen), P.max_depen) : 0.0f;
                an[a].r = r;
                an[a].I1 = G.iw1(Iw, r);
                an[a].I2 = G.iw2(Iw, r);
                an[a].k1 = act ? 1.0f / (invm + G.k1(r, an[a].I1)) : 0.0f;
                an[a].k2 = act ? 1.0f / (invm + G.k2(r, an[a].I2)) : 0.0f;
                an[a].l1 = 0.0f;
                an[a].l2 = 0.0f;
                an[a].e1 = e1;
                an[a].e2 = e2;
            }
            // the anchors whose bound clamped a row in the last iteration, per
            // anchor and direction: the patch slips when every anchor it holds is
            // clamped along one direction (the Gauss-Seidel sweep may leave one of
            // two anchors at its half budget while the other still holds)
            bool c01 = false, c02 = false, c11 = false, c12 = false;
            // each anchor of a two-anchor patch holds half of the patch's Coulomb
            // budget mu N per direction: symmetric (a box sliding on its diagonal
            // anchors exerts no yaw torque), and the two saturate at mu N together
            const float share = R.cnt == 2 ? 0.5f : 1.0f;
            const int nit = P.npos + P.nvel;
            RUSE(an[1].k2); RUSE(sl[3].kn);
            if (st < 2) RSTAMP(6 + 6 * st);   // row constants, anchor rows
            if constexpr (B::kPacked && PACK) {
                tgs_zp(P, sl, an, share * mu, e, v, w, dx, dth, invm, c01, c02, c11, c12);
            } else
            for (int it = 0; it < nit; ++it) {
                const bool pos = it < P.npos, last = it == nit - 1;
                auto normals = [&]() {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float sj = G.ps(sl[j].s0, dx, dth, sl[j].r);
                        row_normal1(G, sl[j], v, w, invm, pos ? pos_target(P, sj) : vel_target(P, sj, e, sl[j].vn0));
                    }
                };
                // sweep order (round 6, oracle rigid_body_step): a position
                // sweep is the anchors' rows then the normal rows; the first
                // and the velocity sweeps open with the normal rows as well
                if (it == 0 || !pos) normals();
                // the patch's normal impulse (slot order)
                const float mun = mu * (((sl[0].ln + sl[1].ln) + sl[2].ln) + sl[3].ln);
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    {
                        const float lim = share * mun;
                        const float raw = fmaf(an[a].k1, (pos ? an[a].e1 : 0.0f) - G.v1(v, w, an[a].r), an[a].l1);
                        const float nl = clamp_sym(raw, lim);
                        const float dl = nl - an[a].l1;
                        const bool cl = last && (raw > lim || raw < -lim);
                        if (a == 0) c01 = cl; else c11 = cl;
                        an[a].l1 = nl;
                        v = G.f1(v, dl, invm);
                        w = fmad3(w, an[a].I1, dl);
                    }
                    {
                        const float lim = share * mun;
                        const float raw = fmaf(an[a].k2, (pos ? an[a].e2 : 0.0f) - G.v2(v, w, an[a].r), an[a].l2);
                        const float nl = clamp_sym(raw, lim);
                        const float dl = nl - an[a].l2;
                        const bool cl = last && (raw > lim || raw < -lim);
                        if (a == 0) c02 = cl; else c12 = cl;
                        an[a].l2 = nl;
                        v = G.f2(v, dl, invm);
                        w = fmad3(w, an[a].I2, dl);
                    }
                }
                normals();   // every sweep ends with the normal rows
                if (pos) {
                    dx = fmad3(dx, v, P.sub);
                    dth = fmad3(dth, w, P.sub);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) fsum = G.addn(fsum, sl[j].ln);
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                fsum = G.add1(fsum, an[a].l1);
                fsum = G.add2(fsum, an[a].l2);
            }
            // a slipping patch lets go (regrown at the next substep)
            const bool one = R.cnt < 2;
            if ((c01 && (c11 || one)) || (c02 && (c12 || one))) R.cnt = 0;
        } else {
            // no solver pass: the motion delta is the substep's free flight
            for (int it = 0; it < P.npos; ++it) {
                dx = fmad3(dx, v, P.sub);
                dth = fmad3(dth, w, P.sub);
            }
        }

        RUSE(dx.x); RUSE(dth.z);
        if (st < 2) RSTAMP(7 + 6 * st);   // solver sweeps (or free flight)
        // 4. pose update (centre of mass moves by the integrated delta)
        const V3 xc1 = vadd(xc, dx);
        q = qintegrate(q, dth);
        x = origin_from_com(xc1, q, com);
        RUSE(x.x); RUSE(q.w);
        if (st < 2) RSTAMP(8 + 6 * st);   // pose update
    }
    // the patch for the next step: the anchor count always, the anchors while held
    if (gp && has_shape) {
        gp[0] = (float)R.cnt;
        if (R.cnt > 0 && R.dirty) {
            const float r[MG_FP_N] = {0.0f, R.nA.x, R.nA.y, R.nA.z,
                                      R.aA[0].x, R.aA[0].y, R.aA[0].z, R.aB[0].x, R.aB[0].y, R.aB[0].z,
                                      R.aA[1].x, R.aA[1].y, R.aA[1].z, R.aB[1].x, R.aB[1].y, R.aB[1].z};
#pragma unroll
            for (int k = 1; k < MG_FP_N; ++k) gp[(size_t)k * gstride] = r[k];
        }
    }
}

// Wide launches: __launch_bounds__(64, 3), at most 168 VGPRs, so three waves
// share a SIMD (the Gauss-Seidel chains are latency-bound: more resident waves,
// not more lanes, fill the SIMD); free of scratch at that budget. One-round
// launches (the packed solver, the shape record in registers): two waves, 175
// VGPRs and no scratch — at three waves the shape record spilled 36 B/lane
// (4096 envs: 13.2 us against 13.5 with the record in LDS and 13.5 at either
// budget, same-box A/B, profiles/r05_ab_rigid_shape_regs.jsonl). The general
// ground basis needs more registers: two waves.
#ifndef MG_RIGID1_ROUND_WAVES
#define MG_RIGID1_ROUND_WAVES 2
#endif
#ifndef MG_RIGID1_WIDE_WAVES
#define MG_RIGID1_WIDE_WAVES 3
#endif
template <bool UPZ, bool LDS_T, bool WIDE>
__global__ void __launch_bounds__(64, UPZ && WIDE ? MG_RIGID1_WIDE_WAVES : (UPZ ? MG_RIGID1_ROUND_WAVES : 2))
k_rigid_step1(MgStep P, MgRigidArgs A) {
    extern __shared__ float s_trec[];
    const int i = (WIDE ? gridDim.x - 1 - blockIdx.x : blockIdx.x) * 64 + threadIdx.x;
    RSTAMP(0);
    const bool live = i < A.nf;
    const int b = A.free_ids ? A.free_ids[live ? i : A.nf - 1] : (live ? i : A.nf - 1);
    const int nb = A.nb;
    // this lane's inputs first, so they are in flight with the template staging;
    // a fused root-state set (migym_capi.cpp) supplies them from the actor's row
    // of the user tensor instead (the scatter that would have written them)
    const float* Si = A.state + b;
    int si = nb;
    if (A.root_src) {
        const int rr = A.root_row[b];
        if (rr >= 0) {
            Si = A.root_src + (size_t)rr * MG_STATE_N;
            si = 1;
        }
    }
    V3 x = v3(Si[0 * si], Si[1 * si], Si[2 * si]);
    Q4 q = q4(Si[3 * si], Si[4 * si], Si[5 * si], Si[6 * si]);
    V3 v = v3(Si[7 * si], Si[8 * si], Si[9 * si]);
    V3 w = v3(Si[10 * si], Si[11 * si], Si[12 * si]);
    const int tb = A.body_tmpl[b];
#ifdef MG_RIGID1_PREFETCH_OUT
    // the fused refresh's row indices, in flight with the state loads (loaded at
    // the end they were one more memory round trip before the last stores)
    const bool fout = (A.out_rb || A.out_root) && !WIDE;
    const int pre_ob = fout && A.out_rb ? A.out_body[b] : -1;
    const int pre_or = fout && A.out_root ? A.out_root_row[b] : -1;
#endif
    V3 fext = v3(0.0f, 0.0f, 0.0f), text = v3(0.0f, 0.0f, 0.0f);
    if (A.ext) {
        fext = v3(A.ext[0 * nb + b], A.ext[1 * nb + b], A.ext[2 * nb + b]);
        text = v3(A.ext[3 * nb + b], A.ext[4 * nb + b], A.ext[5 * nb + b]);
    }
    const float* T;
    if constexpr (LDS_T) {
        for (int k = threadIdx.x; k < A.ntb * MG_TREC_N; k += 64) s_trec[k] = A.trec[k];
        __syncthreads();
        T = s_trec + tb * MG_TREC_N;
    } else {
        T = A.trec + tb * MG_TREC_N;
    }
    // mass row: the template's own when all its bodies share it (the servo scene:
    // no per-body loads), else the body's SoA row (migym_capi.cpp upload)
    float mr[11];
    if (T[5] != 0.0f) {
#pragma unroll
        for (int k = 0; k < 11; ++k) mr[k] = T[MG_TREC_MASS + k];
    } else {
#pragma unroll
        for (int k = 0; k < 11; ++k) mr[k] = A.mass[k * nb + b];
    }
    const float invm = mr[0];
    const V3 invI = v3(mr[1], mr[2], mr[3]);
    const Q4 iq = q4(mr[4], mr[5], mr[6], mr[7]);
    const V3 com = v3(mr[8], mr[9], mr[10]);
    V3 fsum = v3(0.0f, 0.0f, 0.0f);
    RUSE(x.x); RUSE(q.w); RUSE(w.z); RUSE(invm); RUSE(com.z); RUSE(T[4]);
    RSTAMP(1);   // state, template record, mass row in registers
    // this body's ground-patch record (slot b of the SoA [MG_FP_N][gstride] table)
    // and its LDS copy during the frame
    float* gp = live && A.gpatch ? A.gpatch + b : nullptr;
    if constexpr (UPZ) {
        rigid_body1<!WIDE>(BasisZ{}, P, T, x, q, v, w, fsum, invm, invI, iq, com, A.ext != nullptr, fext, text, A.hulls,
                           gp, A.gstride);
    } else {
        BasisGen G;
        G.n = v3(P.n[0], P.n[1], P.n[2]);
        G.t1 = v3(P.t1[0], P.t1[1], P.t1[2]);
        G.t2 = v3(P.t2[0], P.t2[1], P.t2[2]);
        rigid_body1<!WIDE>(G, P, T, x, q, v, w, fsum, invm, invI, iq, com, A.ext != nullptr, fext, text, A.hulls, gp,
                           A.gstride);
    }
    // the output addresses are recomputed here (an opaque copy of the slot)
    // rather than kept live in registers across the frame
    int bo = b;
    asm volatile("" : "+v"(bo));
    if (live) {
        float* So = A.state;
        So[0 * nb + bo] = x.x; So[1 * nb + bo] = x.y; So[2 * nb + bo] = x.z;
        So[3 * nb + bo] = q.x; So[4 * nb + bo] = q.y; So[5 * nb + bo] = q.z; So[6 * nb + bo] = q.w;
        So[7 * nb + bo] = v.x; So[8 * nb + bo] = v.y; So[9 * nb + bo] = v.z;
        So[10 * nb + bo] = w.x; So[11 * nb + bo] = w.y; So[12 * nb + bo] = w.z;
        A.cforce[0 * nb + bo] = fsum.x * P.inv_dt;
        A.cforce[1 * nb + bo] = fsum.y * P.inv_dt;
        A.cforce[2 * nb + bo] = fsum.z * P.inv_dt;
    }
    if ((A.out_rb || A.out_root) && !WIDE) {
        // the refresh fused into the step: the same 13 values into the bound
        // rigid-body row and, for a root body, its actor's root row (the rows the
        // paired gather k_gather_rb_root would write from the SoA state)
        if (live) {
            const float o[MG_STATE_N] = {x.x, x.y, x.z, q.x, q.y, q.z, q.w, v.x, v.y, v.z, w.x, w.y, w.z};
#ifdef MG_RIGID1_PREFETCH_OUT
            const int ob = pre_ob;
            const int rr = pre_or;
#else
            const int ob = A.out_rb ? A.out_body[bo] : -1;
            const int rr = A.out_root ? A.out_root_row[bo] : -1;
#endif
            if (A.out_rb) {
                float* R = A.out_rb + (size_t)ob * MG_STATE_N;
#pragma unroll
                for (int k = 0; k < MG_STATE_N; ++k) R[k] = o[k];
            }
            if (rr >= 0) {
                float* Ro = A.out_root + (size_t)rr * MG_STATE_N;
#pragma unroll
                for (int k = 0; k < MG_STATE_N; ++k) Ro[k] = o[k];
            }
        }
        RSTAMP(15);   // all stores issued
#ifdef MG_RIGID1_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        RSTAMP(16);   // stores complete
#endif
    } else if (A.out_rb || A.out_root) {   // launch-uniform
        // Wide launches are issue-bound, and the rows are 52-B AoS records, every
        // other one per wave (the wave holds one template: UAVs or cars): written
        // lane by lane, each store instruction touches 64 rows 104 B apart. The
        // wave's rows are transposed through LDS instead, so that store k writes
        // elements k*64 .. k*64+63 of the wave's 64 x 13 block — runs of
        // consecutive floats, five rows each (262k envs: 46.9 -> 45.6 us; a
        // one-round launch is latency-bound and pays the LDS round trip: 10.2 ->
        // 11.3 us at 4096, so it keeps the direct stores).
        __shared__ float s_out[64 * 16];
        __shared__ int s_dst[2][64];
        const int l = threadIdx.x;
        const float o[MG_STATE_N] = {x.x, x.y, x.z, q.x, q.y, q.z, q.w, v.x, v.y, v.z, w.x, w.y, w.z};
#pragma unroll
        for (int k = 0; k < MG_STATE_N; ++k) s_out[l * 16 + k] = o[k];
        s_dst[0][l] = live && A.out_rb ? A.out_body[bo] : -1;
        s_dst[1][l] = live && A.out_root ? A.out_root_row[bo] : -1;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < MG_STATE_N; ++k) {
            const int e = k * 64 + l;
            const int row = e / MG_STATE_N, col = e - row * MG_STATE_N;
            const float val = s_out[row * 16 + col];
            const int d0 = s_dst[0][row], d1 = s_dst[1][row];
            if (d0 >= 0) A.out_rb[(size_t)d0 * MG_STATE_N + col] = val;
            if (d1 >= 0) A.out_root[(size_t)d1 * MG_STATE_N + col] = val;
        }
    }
}

template <bool UPZ, int MAXC, bool MULTI>
__global__ void __launch_bounds__(64) k_rigid_step(MgStep P, MgRigidArgs A) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= A.nf) return;
    const int b = A.free_ids ? A.free_ids[i] : i;
    if constexpr (UPZ) {
        rigid_body<MAXC, MULTI>(BasisZ{}, P, A, b);
    } else {
        BasisGen G;
        G.n = v3(P.n[0], P.n[1], P.n[2]);
        G.t1 = v3(P.t1[0], P.t1[1], P.t1[2]);
        G.t2 = v3(P.t2[0], P.t2[1], P.t2[2]);
        rigid_body<MAXC, MULTI>(G, P, A, b);
    }
}

}  // namespace

bool mg_step_is_upz(const MgStep& P) {
    return P.n[0] == 0.0f && P.n[1] == 0.0f && P.n[2] == 1.0f && P.t1[0] == 0.0f && P.t1[1] == 1.0f &&
           P.t1[2] == 0.0f && P.t2[0] == -1.0f && P.t2[1] == 0.0f && P.t2[2] == 0.0f;
}

static int mg_cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] <= 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

// A.free_ids lists the single-shape bodies first (A.nf1 of them), then the
// multi-shape ones; each group is its own launch.
hipError_t mg_launch_rigid_step(const MgStep& P, const MgRigidArgs& A, hipStream_t s) {
    if (A.nf <= 0) return hipSuccess;
    const bool upz = mg_step_is_upz(P);
    MgRigidArgs A1 = A, A2 = A;
    A2.root_src = nullptr;   // fused root sets only with single-shape bodies (migym_capi.cpp)
    A2.out_rb = nullptr;     // so is the fused refresh (MG_FUSE_STEP_OUT)
    A2.out_root = nullptr;
    A2.gpatch = nullptr;     // ground patches: single-shape bodies (multi-shape ones keep per-point rows)
    A1.nf = A.nf1;
    A2.nf = A.nf - A.nf1;
    if (A.free_ids) {
        A2.free_ids = A.free_ids + A.nf1;
    } else {   // bodies in storage slots 0..nf-1: the second group starts at slot nf1
        A2.state = A.state + A.nf1;
        A2.mass = A.mass + A.nf1;
        A2.body_tmpl = A.body_tmpl + A.nf1;
        A2.ext = A.ext ? A.ext + A.nf1 : nullptr;
        A2.cforce = A.cforce + A.nf1;
    }
    if (A1.nf > 0) {
        const int blocks = (A1.nf + 63) / 64;
        // wide: more waves than one resident round (4 SIMDs x 3 or 2 waves per
        // CU). Such a launch is issue-bound, not latency-bound: it dispatches
        // longest-first (back to front: the free-body order, migym_capi.cpp) and
        // solves with the scalar rows (tgs_z's packed pairs save latency, not
        // issue slots: DESIGN.md §3.2).
        const bool wide = blocks > mg_cu_count() * 4 * (upz ? MG_RIGID1_ROUND_WAVES : 2);
        const size_t lds = (size_t)A.ntb * MG_TREC_N * sizeof(float);
#define MG_K1(U, L) \
    do { \
        if (wide) MG_LAUNCH((k_rigid_step1<U, L, true>), dim3(blocks), dim3(64), L ? lds : 0, s, P, A1); \
        else MG_LAUNCH((k_rigid_step1<U, L, false>), dim3(blocks), dim3(64), L ? lds : 0, s, P, A1); \
    } while (0)
        if (lds <= MG_TREC_LDS_MAX) {
            if (upz) MG_K1(true, true);
            else MG_K1(false, true);
        } else {
            if (upz) MG_K1(true, false);
            else MG_K1(false, false);
        }
#undef MG_K1
    }
    if (A2.nf > 0) {
        const int blocks = (A2.nf + 63) / 64;
        if (upz) MG_LAUNCH((k_rigid_step<true, MG_MAX_CONTACTS, true>), dim3(blocks), dim3(64), 0, s, P, A2);
        else MG_LAUNCH((k_rigid_step<false, MG_MAX_CONTACTS, true>), dim3(blocks), dim3(64), 0, s, P, A2);
    }
    return hipGetLastError();
}
