/*
 * migym_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the engine's
 * step, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * as the checker. Never linked into, or called by, the product path
 * (test_isaacgym_amd/), which fails loudly without its HIP library.
 *
 * What it restates. The reference engine behind gym.simulate() is NVIDIA Isaac
 * Gym / PhysX, a closed binary that is not in /root/reference (SURVEY.md §0.1,
 * §8c), so there is no reference source to follow line by line: PHYSICS PARITY
 * WITH PHYSX IS UNPINNED. This file restates the algorithm DESIGN.md §3 states,
 * fixed by the reference's call sites:
 *   - sim parameters: test10_servo_vecenv.py:117-144 (dt 1/60, 2 substeps, TGS
 *     solver_type=1, 6 position / 1 velocity iterations, contact_offset 0.01,
 *     rest_offset 0), ground plane :198-206;
 *   - teleport semantics of set_actor_root_state_tensor: :451-456;
 *   - drive law of set_actor_dof_properties: examples/dof_controls.py:89-150,
 *     test13_camera_spherical_joint.py:197-205;
 *   - the articulated-body algorithm: Featherstone, RBDA Table 7.1.
 * It is pinned to the device by construction of the test, not to PhysX: the
 * arithmetic is written in the same evaluation order as the HIP kernels
 * (test_isaacgym_amd/csrc/mg_rigid.hip, mg_artic.hip), and both sides are
 * compiled with -ffp-contract=off, so parity is expected bit for bit. Analytic
 * known-answer tests (tests/test_oracle_kat.py) pin it to physics.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/migym.h"

#define OR_MAXC 8
#define OR_MAXL 32

typedef struct { float x, y, z; } v3_t;
typedef struct { float x, y, z, w; } q4_t;
typedef struct { v3_t c0, c1, c2; } m3_t;

static v3_t V(float x, float y, float z) { v3_t r; r.x = x; r.y = y; r.z = z; return r; }
static v3_t add3(v3_t a, v3_t b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3_t sub3(v3_t a, v3_t b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3_t mul3(v3_t a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static float dot3(v3_t a, v3_t b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3_t cross3(v3_t a, v3_t b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static v3_t mad3(v3_t a, v3_t b, float s) { return V(a.x + b.x * s, a.y + b.y * s, a.z + b.z * s); }

static q4_t Q(float x, float y, float z, float w) { q4_t r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
static q4_t qmul_(q4_t a, q4_t b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
             a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
             a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w,
             a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
static q4_t qnorm_(q4_t a) {
    float n2 = a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    float inv;
    if (!(n2 > 0.0f)) return Q(0.0f, 0.0f, 0.0f, 1.0f);
    inv = 1.0f / sqrtf(n2);
    return Q(a.x * inv, a.y * inv, a.z * inv, a.w * inv);
}
static v3_t qrot_(q4_t q, v3_t v) {
    float tx = 2.0f * (q.y * v.z - q.z * v.y);
    float ty = 2.0f * (q.z * v.x - q.x * v.z);
    float tz = 2.0f * (q.x * v.y - q.y * v.x);
    return V(v.x + q.w * tx + (q.y * tz - q.z * ty),
             v.y + q.w * ty + (q.z * tx - q.x * tz),
             v.z + q.w * tz + (q.x * ty - q.y * tx));
}
static m3_t qmat_(q4_t q) {
    float xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    float xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z;
    float wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
    m3_t m;
    m.c0 = V(1.0f - 2.0f * (yy + zz), 2.0f * (xy + wz), 2.0f * (xz - wy));
    m.c1 = V(2.0f * (xy - wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz + wx));
    m.c2 = V(2.0f * (xz + wy), 2.0f * (yz - wx), 1.0f - 2.0f * (xx + yy));
    return m;
}
static v3_t mv_(m3_t m, v3_t u) {
    return V(m.c0.x * u.x + m.c1.x * u.y + m.c2.x * u.z,
             m.c0.y * u.x + m.c1.y * u.y + m.c2.y * u.z,
             m.c0.z * u.x + m.c1.z * u.y + m.c2.z * u.z);
}
static v3_t mtv_(m3_t m, v3_t v) { return V(dot3(m.c0, v), dot3(m.c1, v), dot3(m.c2, v)); }
/* symmetric world inverse inertia: Rp diag(d) Rp^T */
typedef struct { float xx, yy, zz, xy, xz, yz; } s3_t;
static s3_t sym_rdrt_(m3_t Rp, v3_t d) {
    v3_t u0 = mul3(Rp.c0, d.x), u1 = mul3(Rp.c1, d.y), u2 = mul3(Rp.c2, d.z);
    s3_t s;
    s.xx = u0.x * Rp.c0.x + u1.x * Rp.c1.x + u2.x * Rp.c2.x;
    s.yy = u0.y * Rp.c0.y + u1.y * Rp.c1.y + u2.y * Rp.c2.y;
    s.zz = u0.z * Rp.c0.z + u1.z * Rp.c1.z + u2.z * Rp.c2.z;
    s.xy = u0.x * Rp.c0.y + u1.x * Rp.c1.y + u2.x * Rp.c2.y;
    s.xz = u0.x * Rp.c0.z + u1.x * Rp.c1.z + u2.x * Rp.c2.z;
    s.yz = u0.y * Rp.c0.z + u1.y * Rp.c1.z + u2.y * Rp.c2.z;
    return s;
}
static v3_t symmul_(s3_t s, v3_t v) {
    return V(s.xx * v.x + s.xy * v.y + s.xz * v.z,
             s.xy * v.x + s.yy * v.y + s.yz * v.z,
             s.xz * v.x + s.yz * v.y + s.zz * v.z);
}
/* sin/cos by Taylor + double angle */
static void sincos_(float x, float* so, float* co) {
    int k = 0, i;
    float x2, s, c;
    while (x > 0.5f && k < 24) { x = x * 0.5f; k = k + 1; }
    x2 = x * x;
    s = x * (1.0f - x2 * (1.0f / 6.0f) * (1.0f - x2 * (1.0f / 20.0f) * (1.0f - x2 * (1.0f / 42.0f) * (1.0f - x2 * (1.0f / 72.0f)))));
    c = 1.0f - x2 * 0.5f * (1.0f - x2 * (1.0f / 12.0f) * (1.0f - x2 * (1.0f / 30.0f) * (1.0f - x2 * (1.0f / 56.0f) * (1.0f - x2 * (1.0f / 90.0f)))));
    for (i = 0; i < k; ++i) {
        float s2 = 2.0f * s * c;
        float c2 = c * c - s * s;
        s = s2; c = c2;
    }
    *so = s; *co = c;
}
static q4_t qint_(q4_t q, v3_t dth) {
    float th2 = dot3(dth, dth), th, s, c, k;
    if (!(th2 > 0.0f)) return q;
    th = sqrtf(th2);
    sincos_(0.5f * th, &s, &c);
    k = s / th;
    return qnorm_(qmul_(Q(dth.x * k, dth.y * k, dth.z * k, c), q));
}

/* ---- step constants ---------------------------------- */
typedef struct {
    float h, sub, inv_sub, inv_h, inv_dt, g[3];
    int substeps, npos, nvel;
    float co, ro, maxdep, bounce;
    int ground;
    v3_t n, t1, t2;
    float pd, mu_g, e_g;
    float fot, corr;   /* friction_offset_threshold, friction_correlation_distance (friction anchors) */
} step_t;

static step_t make_step_(const mg_sim_params* p) {
    step_t P;
    int ss = p->substeps > 0 ? p->substeps : 1;
    int np = p->num_position_iterations > 0 ? p->num_position_iterations : 1;
    float nx = p->ground_normal[0], ny = p->ground_normal[1], nz = p->ground_normal[2];
    float ax = 1.0f, ay = 0.0f, az = 0.0f, t1x, t1y, t1z, inv;
    memset(&P, 0, sizeof P);
    P.substeps = ss; P.npos = np;
    P.nvel = p->num_velocity_iterations > 0 ? p->num_velocity_iterations : 0;
    P.h = p->dt / (float)ss;
    P.sub = P.h / (float)np;
    P.inv_sub = 1.0f / P.sub;
    P.inv_h = 1.0f / P.h;
    P.inv_dt = 1.0f / p->dt;
    P.g[0] = p->gravity[0]; P.g[1] = p->gravity[1]; P.g[2] = p->gravity[2];
    P.co = p->contact_offset; P.ro = p->rest_offset;
    P.maxdep = p->max_depenetration_velocity; P.bounce = p->bounce_threshold_velocity;
    P.ground = p->has_ground;
    P.n = V(nx, ny, nz);
    P.pd = p->ground_distance;
    if (!(fabsf(nx) < 0.9f)) { ax = 0.0f; ay = 1.0f; }
    t1x = ny * az - nz * ay; t1y = nz * ax - nx * az; t1z = nx * ay - ny * ax;
    inv = 1.0f / sqrtf(t1x * t1x + t1y * t1y + t1z * t1z);
    t1x = t1x * inv; t1y = t1y * inv; t1z = t1z * inv;
    P.t1 = V(t1x, t1y, t1z);
    P.t2 = V(ny * t1z - nz * t1y, nz * t1x - nx * t1z, nx * t1y - ny * t1x);
    P.mu_g = p->ground_dynamic_friction;
    P.e_g = p->ground_restitution;
    P.fot = p->friction_offset_threshold;
    P.corr = p->friction_correlation_distance;
    return P;
}

/* ---- free body --------------------------------------- */
/* Ground basis: the general (n, t1, t2), or the +Z basis n = z, t1 = y, t2 = -x
 * written out explicitly (as the device's BasisZ specialisation). */
typedef struct { int upz; v3_t n, t1, t2; } basis_t;
static float b_dn(const basis_t* B, v3_t v) { return B->upz ? v.z : dot3(B->n, v); }
static float b_d1(const basis_t* B, v3_t v) { return B->upz ? v.y : dot3(B->t1, v); }
static float b_d2(const basis_t* B, v3_t v) { return B->upz ? -v.x : dot3(B->t2, v); }
static v3_t b_addn(const basis_t* B, v3_t v, float s) { return B->upz ? V(v.x, v.y, v.z + s) : mad3(v, B->n, s); }
static v3_t b_add1(const basis_t* B, v3_t v, float s) { return B->upz ? V(v.x, v.y + s, v.z) : mad3(v, B->t1, s); }
static v3_t b_add2(const basis_t* B, v3_t v, float s) { return B->upz ? V(v.x - s, v.y, v.z) : mad3(v, B->t2, s); }

/* Gauss-Seidel row kernels with explicit fused multiply-adds, as the device
 * (mg_rigid.hip BasisGen / BasisZ vn, v1, v2, ps, fn, f1, f2) */
static float fdot3_(v3_t a, v3_t b, float acc) { return fmaf(a.z, b.z, fmaf(a.y, b.y, fmaf(a.x, b.x, acc))); }
static v3_t fmad3_(v3_t v, v3_t d, float s) { return V(fmaf(d.x, s, v.x), fmaf(d.y, s, v.y), fmaf(d.z, s, v.z)); }
static float b_vn(const basis_t* B, v3_t v, v3_t w, v3_t r) {
    return B->upz ? fmaf(w.y, -r.x, fmaf(w.x, r.y, v.z)) : fdot3_(w, cross3(r, B->n), dot3(B->n, v));
}
static float b_v1(const basis_t* B, v3_t v, v3_t w, v3_t r) {
    return B->upz ? fmaf(w.z, r.x, fmaf(w.x, -r.z, v.y)) : fdot3_(w, cross3(r, B->t1), dot3(B->t1, v));
}
static float b_v2(const basis_t* B, v3_t v, v3_t w, v3_t r) {
    return B->upz ? fmaf(w.z, r.y, fmaf(w.y, -r.z, -v.x)) : fdot3_(w, cross3(r, B->t2), dot3(B->t2, v));
}
static float b_ps(const basis_t* B, float s0, v3_t dx, v3_t dth, v3_t r) {
    return B->upz ? fmaf(dth.y, -r.x, fmaf(dth.x, r.y, s0 + dx.z)) : fdot3_(dth, cross3(r, B->n), s0 + dot3(B->n, dx));
}
static v3_t b_fn(const basis_t* B, v3_t v, float dl, float invm) {
    return B->upz ? V(v.x, v.y, fmaf(dl, invm, v.z)) : fmad3_(v, B->n, dl * invm);
}
static v3_t b_f1(const basis_t* B, v3_t v, float dl, float invm) {
    return B->upz ? V(v.x, fmaf(dl, invm, v.y), v.z) : fmad3_(v, B->t1, dl * invm);
}
static v3_t b_f2(const basis_t* B, v3_t v, float dl, float invm) {
    return B->upz ? V(fmaf(-dl, invm, v.x), v.y, v.z) : fmad3_(v, B->t2, dl * invm);
}
/* Iw (r x d) and (r x d) . Iw (r x d) per row direction; the +Z basis drops the
 * zero component of r x d (mg_rigid.hip BasisZ iwn / iw1 / iw2 / kn / k1 / k2,
 * symmul's term order otherwise) */
static v3_t b_iwn(const basis_t* B, const s3_t* I, v3_t r) {
    if (!B->upz) return symmul_(*I, cross3(r, B->n));
    {
        const float a = r.y, b = -r.x;
        return V(I->xx * a + I->xy * b, I->xy * a + I->yy * b, I->xz * a + I->yz * b);
    }
}
static v3_t b_iw1(const basis_t* B, const s3_t* I, v3_t r) {
    if (!B->upz) return symmul_(*I, cross3(r, B->t1));
    {
        const float a = -r.z, c = r.x;
        return V(I->xx * a + I->xz * c, I->xy * a + I->yz * c, I->xz * a + I->zz * c);
    }
}
static v3_t b_iw2(const basis_t* B, const s3_t* I, v3_t r) {
    if (!B->upz) return symmul_(*I, cross3(r, B->t2));
    {
        const float b = -r.z, c = r.y;
        return V(I->xy * b + I->xz * c, I->yy * b + I->yz * c, I->yz * b + I->zz * c);
    }
}
static float b_kn(const basis_t* B, v3_t r, v3_t In) { return B->upz ? r.y * In.x + -r.x * In.y : dot3(cross3(r, B->n), In); }
static float b_k1(const basis_t* B, v3_t r, v3_t I1) { return B->upz ? -r.z * I1.x + r.x * I1.z : dot3(cross3(r, B->t1), I1); }
static float b_k2(const basis_t* B, v3_t r, v3_t I2) { return B->upz ? -r.z * I2.y + r.y * I2.z : dot3(cross3(r, B->t2), I2); }

typedef struct {
    v3_t r; float s0, mu, e, kn, kt1, kt2, ln, lt1, lt2, vn0; int on;
} slot_t;

/* x clamped to [-lim, lim], lim >= 0 (the device's v_med3_f32) */
static float clamp_sym_(float x, float lim) { return fminf(fmaxf(x, -lim), lim); }
/* Row targets (mg_rigid.hip pos_target / vel_target): position iterations
 * v_n >= -s / sub capped at the maximum depenetration velocity (binding only
 * while penetrating); velocity iterations v_n >= -s / h while separated, else
 * 0, raised to the restitution bounce above the bounce threshold. */
static float pos_target_(const step_t* P, float s) { return fminf(-s * P->inv_sub, P->maxdep); }
static float vel_target_(const step_t* P, float s, float e, float vn0) {
    float tgt = fminf(-s * P->inv_h, 0.0f);
    if (e > 0.0f && vn0 < -P->bounce) tgt = fmaxf(tgt, -e * vn0);
    return tgt;
}

static void contact_normal(const basis_t* B, slot_t* c, v3_t* v, v3_t* w, float invm, const s3_t* Iw, float tgt) {
    float vn = b_vn(B, *v, *w, c->r);
    float nl = fmaxf(fmaf(c->kn, tgt - vn, c->ln), 0.0f);
    float dl = nl - c->ln;
    c->ln = nl;
    *v = b_fn(B, *v, dl, invm);
    *w = fmad3_(*w, b_iwn(B, Iw, c->r), dl);
}

/* PhysX-style pyramid friction: tangent rows one after the other, each
 * accumulated impulse clamped to [-mu ln, mu ln] */
static void contact_friction(const basis_t* B, slot_t* c, v3_t* v, v3_t* w, float invm, const s3_t* Iw) {
    const float lim = c->mu * c->ln;
    float vt1 = b_v1(B, *v, *w, c->r), vt2, n1, n2, d1, d2;
    n1 = clamp_sym_(fmaf(-c->kt1, vt1, c->lt1), lim);
    d1 = n1 - c->lt1;
    c->lt1 = n1;
    *v = b_f1(B, *v, d1, invm);
    *w = fmad3_(*w, b_iw1(B, Iw, c->r), d1);
    vt2 = b_v2(B, *v, *w, c->r);
    n2 = clamp_sym_(fmaf(-c->kt2, vt2, c->lt2), lim);
    d2 = n2 - c->lt2;
    c->lt2 = n2;
    *v = b_f2(B, *v, d2, invm);
    *w = fmad3_(*w, b_iw2(B, Iw, c->r), d2);
}

/* Identity skips (mg_rigid.hip shape_pose_identity / inertia_frame / com_world
 * / origin_from_com): the composition with an identity pose or a zero offset
 * is skipped, as on the device. */
static int shape_pose_identity_(const float* sh) {
    return sh[4] == 0.0f && sh[5] == 0.0f && sh[6] == 0.0f && sh[7] == 0.0f && sh[8] == 0.0f && sh[9] == 0.0f &&
           sh[10] == 1.0f;
}
static q4_t inertia_frame_(q4_t q, q4_t iq) {
    if (iq.x == 0.0f && iq.y == 0.0f && iq.z == 0.0f && iq.w == 1.0f) return q;
    return qmul_(q, iq);
}
static v3_t com_world_(v3_t x, q4_t q, v3_t com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return x;
    return add3(x, qrot_(q, com));
}
static v3_t origin_from_com_(v3_t xc, q4_t q, v3_t com) {
    if (com.x == 0.0f && com.y == 0.0f && com.z == 0.0f) return xc;
    return sub3(xc, qrot_(q, com));
}

/* Contact candidates of one shape: (static index k, point, separation). */
typedef struct { int k; v3_t p; float sep; } cand_t;
static int shape_candidates(const step_t* P, const basis_t* B, const float* sh, q4_t q, v3_t x, cand_t* out,
                            float* mu, float* e, const float* hulls) {
    const int type = (int)sh[0];
    q4_t qs = q;
    v3_t cs = x;
    int k, n = 0;
    if (!shape_pose_identity_(sh)) {
        qs = qmul_(q, Q(sh[7], sh[8], sh[9], sh[10]));
        cs = add3(x, qrot_(q, V(sh[4], sh[5], sh[6])));
    }
    *mu = 0.5f * (sh[11] + P->mu_g);
    *e = 0.5f * (sh[12] + P->e_g);
    if (type == MG_SHAPE_BOX) {
        /* the 4 corners of the face most opposed to n (first axis on ties) */
        const m3_t Rs = qmat_(qs);
        const float d0 = b_dn(B, Rs.c0), d1 = b_dn(B, Rs.c1), d2 = b_dn(B, Rs.c2);
        const float ad0 = fabsf(d0), ad1 = fabsf(d1), ad2 = fabsf(d2);
        const v3_t a0 = mul3(Rs.c0, sh[1]), a1 = mul3(Rs.c1, sh[2]), a2 = mul3(Rs.c2, sh[3]);
        int ia = 0;
        float best = ad0, di;
        v3_t ai, e1, e2, u, cu;
        if (ad1 > best) { ia = 1; best = ad1; }
        if (ad2 > best) ia = 2;
        di = ia == 0 ? d0 : (ia == 1 ? d1 : d2);
        ai = ia == 0 ? a0 : (ia == 1 ? a1 : a2);
        e1 = ia == 0 ? a1 : a0;
        e2 = ia == 2 ? a1 : a2;
        u = mul3(ai, di > 0.0f ? -1.0f : 1.0f);
        cu = add3(cs, u);
        for (k = 0; k < 4; ++k) {
            const float sx = (k & 1) ? 1.0f : -1.0f;
            const float sy = (k & 2) ? 1.0f : -1.0f;
            const v3_t p = add3(add3(cu, mul3(e1, sx)), mul3(e2, sy));
            out[n].k = k; out[n].p = p; out[n].sep = b_dn(B, p) + P->pd; n++;
        }
    } else if (type == MG_SHAPE_SPHERE) {
        const float rad = sh[1];
        out[n].k = 0; out[n].p = b_addn(B, cs, -rad); out[n].sep = b_dn(B, cs) + P->pd - rad; n++;
    } else if (type == MG_SHAPE_CAPSULE) {
        const float rad = sh[1];
        const v3_t ax = mul3(qrot_(qs, V(1.0f, 0.0f, 0.0f)), sh[2]);
        for (k = 0; k < 2; ++k) {
            const v3_t c = k ? add3(cs, ax) : sub3(cs, ax);
            out[n].k = k; out[n].p = b_addn(B, c, -rad); out[n].sep = b_dn(B, c) + P->pd - rad; n++;
        }
    } else if (type == MG_SHAPE_CONVEX) {
        /* the 4 deepest hull vertices within the contact offset, ascending
         * separation, lower vertex index first on ties (as mg_rigid.hip) */
        const float* hv = hulls + (int)sh[2];
        const int nv = (int)hv[0];
        float ks[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        v3_t kp[4];
        int kn = 0, i, at;
        for (i = 0; i < nv; ++i) {
            const float* vv = hv + MG_HULL_HEADER + 3 * i;
            const v3_t p = add3(cs, qrot_(qs, V(vv[0], vv[1], vv[2])));
            const float sep = b_dn(B, p) + P->pd;
            if (!(sep < P->co)) continue;
            if (kn == 4 && !(sep < ks[3])) continue;
            at = 0;
            for (k = 0; k < kn; ++k) if (ks[k] <= sep) at = k + 1;
            for (k = 3; k > at; --k) { ks[k] = ks[k - 1]; kp[k] = kp[k - 1]; }
            ks[at] = sep; kp[at] = p;
            if (kn < 4) kn = kn + 1;
        }
        for (k = 0; k < kn; ++k) { out[n].k = k; out[n].p = kp[k]; out[n].sep = ks[k]; n++; }
    }
    return n;
}

/* ---- friction patch of a free body on the ground plane:
 * mg_rigid.hip ground_patch_update, op for op. PhysX patch friction as the
 * coupled step's (§3.6.1, migym_oracle_env.c patch_update_) with the ground as
 * the static second body (its copy of an anchor is a world point): up to two
 * anchors kept while the normal holds and the copies stay within the
 * correlation distance, grown from this substep's contacts in slot order. The
 * record (16 floats, the coupled record's layout) persists from step to step:
 * bcache[b]. */
#define OR_GP_N 16
#define OR_FP_COS 0.999f
typedef struct { int cnt; v3_t nA, aA[2], aB[2]; } gpatch_t;
static v3_t qrot_inv0_(q4_t q, v3_t v) { return qrot_(Q(-q.x, -q.y, -q.z, q.w), v); }
static void gpatch_load_(gpatch_t* R, const float* r) {
    int k;
    R->cnt = (int)r[0];
    R->nA = V(r[1], r[2], r[3]);
    for (k = 0; k < 2; ++k) {
        R->aA[k] = V(r[4 + 6 * k], r[5 + 6 * k], r[6 + 6 * k]);
        R->aB[k] = V(r[7 + 6 * k], r[8 + 6 * k], r[9 + 6 * k]);
    }
}
static void gpatch_store_(const gpatch_t* R, float* r) {
    int k;
    r[0] = (float)R->cnt;
    if (R->cnt == 0) return;   /* the device writes the rest only when anchors are held */
    r[1] = R->nA.x; r[2] = R->nA.y; r[3] = R->nA.z;
    for (k = 0; k < 2; ++k) {
        r[4 + 6 * k] = R->aA[k].x; r[5 + 6 * k] = R->aA[k].y; r[6 + 6 * k] = R->aA[k].z;
        r[7 + 6 * k] = R->aB[k].x; r[8 + 6 * k] = R->aB[k].y; r[9 + 6 * k] = R->aB[k].z;
    }
}
static void gpatch_update_(gpatch_t* R, v3_t x, q4_t q, v3_t n0, const v3_t* p, const float* s0, const int* on,
                           float fot, float corr) {
    const float c2 = corr * corr;
    int cnt = R->cnt, k, j, kept;
    gpatch_t N;
    if (cnt > 0 && dot3(qrot_(q, R->nA), n0) < OR_FP_COS) cnt = 0;
    N.cnt = 0;
    N.aA[0] = N.aA[1] = N.aB[0] = N.aB[1] = V(0.0f, 0.0f, 0.0f);
    for (k = 0; k < 2; ++k) {
        if (k < cnt) {
            const v3_t d = sub3(add3(x, qrot_(q, R->aA[k])), R->aB[k]);
            if (dot3(d, d) <= c2) {
                if (N.cnt == 0) { N.aA[0] = R->aA[k]; N.aB[0] = R->aB[k]; }
                else { N.aA[1] = R->aA[k]; N.aB[1] = R->aB[k]; }
                N.cnt = N.cnt + 1;
            }
        }
    }
    kept = N.cnt;   /* anchors kept from the last substep */
    /* growth (PhysX growPatches, as mg_rigid.hip ground_patch_update) */
    {
        const int grow = N.cnt < 2;
        v3_t w0 = N.cnt > 0 ? add3(x, qrot_(q, N.aA[0])) : V(0.0f, 0.0f, 0.0f), w1 = V(0.0f, 0.0f, 0.0f);
        float dd = 0.0f;
        for (j = 0; j < 4; ++j) {
            if (grow && on[j] && s0[j] <= fot) {
                const v3_t pj = p[j];
                int put = -1;
                if (N.cnt == 0) {
                    put = 0;
                } else if (N.cnt == 1) {
                    const v3_t d = sub3(pj, w0);
                    const float d2 = dot3(d, d);
                    if (d2 > c2) { put = 1; dd = d2; }
                } else {
                    const v3_t e0 = sub3(pj, w0), e1 = sub3(pj, w1);
                    const float d0 = dot3(e0, e0), d1 = dot3(e1, e1);
                    if (d0 > d1) {
                        if (d0 > dd) { put = 1; dd = d0; }
                    } else if (d1 > dd) {
                        put = 0;
                        dd = d1;
                    }
                }
                if (put >= 0) {
                    const v3_t la = qrot_inv0_(q, sub3(pj, x));
                    if (put == 0) { N.aA[0] = la; N.aB[0] = pj; w0 = pj; }
                    else { N.aA[1] = la; N.aB[1] = pj; w1 = pj; }
                    if (N.cnt <= put) N.cnt = put + 1;
                }
            }
        }
    }
    N.nA = kept > 0 ? R->nA : qrot_inv0_(q, n0);   /* the creation normal while an anchor is kept */
    *R = N;
}

/* pr: the body's ground-patch record (OR_GP_N floats), or NULL (none kept) */
static void rigid_body_step(const step_t* P, const mg_model* m, int b, float* st, const float* ext, float* cf,
                            float* pr) {
    const float* M = m->body_mass + (size_t)b * MG_MASS_N;
    const int tb = m->body_tmpl[b];
    const float* tf = m->tmpl_body_f + (size_t)tb * MG_TBODY_F_N;
    const int sh0 = m->tmpl_body_i[tb * MG_TBODY_I_N + 0], nsh = m->tmpl_body_i[tb * MG_TBODY_I_N + 1];
    v3_t x = V(st[0], st[1], st[2]);
    q4_t q = Q(st[3], st[4], st[5], st[6]);
    v3_t v = V(st[7], st[8], st[9]);
    v3_t w = V(st[10], st[11], st[12]);
    const float invm = M[0];
    const v3_t invI = V(M[1], M[2], M[3]);
    const q4_t iq = Q(M[4], M[5], M[6], M[7]);
    const v3_t com = V(M[8], M[9], M[10]);
    const float h = P->h;
    const float lin_keep = 1.0f - fminf(tf[0] * h, 1.0f);
    const float ang_keep = 1.0f - fminf(tf[1] * h, 1.0f);
    const float max_lv2 = tf[2] * tf[2], max_av2 = tf[3] * tf[3];
    v3_t fext = V(0.0f, 0.0f, 0.0f), text = V(0.0f, 0.0f, 0.0f), fsum = V(0.0f, 0.0f, 0.0f);
    basis_t B;
    int s_, st_;
    B.n = P->n; B.t1 = P->t1; B.t2 = P->t2;
    B.upz = P->n.x == 0.0f && P->n.y == 0.0f && P->n.z == 1.0f && P->t1.x == 0.0f && P->t1.y == 1.0f &&
            P->t1.z == 0.0f && P->t2.x == -1.0f && P->t2.y == 0.0f && P->t2.z == 0.0f;
    gpatch_t R;
    if (ext) { fext = V(ext[0], ext[1], ext[2]); text = V(ext[3], ext[4], ext[5]); }
    R.cnt = 0;
    if (pr && nsh == 1 && P->ground) gpatch_load_(&R, pr);
    q = qnorm_(q);
    for (st_ = 0; st_ < P->substeps; ++st_) {
        const s3_t Iw = sym_rdrt_(qmat_(inertia_frame_(q, iq)), invI);
        const v3_t xc = com_world_(x, q, com);
        slot_t sl[OR_MAXC];
        v3_t cp[4];   /* single-shape bodies: contact point of slot k */
        int j, it;
        v3_t dx = V(0.0f, 0.0f, 0.0f), dth = V(0.0f, 0.0f, 0.0f);
        if (tf[4] != 0.0f) v = mad3(v, V(P->g[0], P->g[1], P->g[2]), h);
        if (ext) {   /* an applied wrench this frame (the device: A.ext non-null) */
            v = mad3(v, fext, invm * h);
            w = mad3(w, symmul_(Iw, text), h);
        }
        v = mul3(v, lin_keep);
        w = mul3(w, ang_keep);
        {
            float v2 = dot3(v, v), w2;
            if (v2 > max_lv2) v = mul3(v, sqrtf(max_lv2 / v2));
            w2 = dot3(w, w);
            if (w2 > max_av2) w = mul3(w, sqrtf(max_av2 / w2));
        }
        for (j = 0; j < OR_MAXC; ++j) sl[j].on = 0;
        if (P->ground) {
            int nc = 0;
            for (s_ = sh0; s_ < sh0 + nsh; ++s_) {
                cand_t cd[8];
                float mu, e;
                int k, n = shape_candidates(P, &B, m->shapes + (size_t)s_ * MG_SHAPE_STRIDE, q, x, cd, &mu, &e,
                                             m->hulls);
                for (k = 0; k < n; ++k) {
                    slot_t ns;
                    if (!(cd[k].sep < P->co)) continue;
                    ns.r = sub3(cd[k].p, xc); ns.s0 = cd[k].sep - P->ro; ns.mu = mu; ns.e = e; ns.on = 1;
                    if (nsh == 1) {
                        sl[cd[k].k] = ns;          /* static slot: candidate k -> slot k (of 4) */
                        cp[cd[k].k] = cd[k].p;
                    } else if (nc < OR_MAXC) {     /* shift register: newest in slot 0 */
                        for (j = OR_MAXC - 1; j > 0; --j) sl[j] = sl[j - 1];
                        sl[0] = ns;
                        nc = nc + 1;
                    }
                }
            }
        }
        if (nsh <= 1) {
            /* single-shape bodies (k_rigid_step1): the ground patch (anchors kept
             * or grown from this substep's contacts), then — once any of the 4
             * static slots is in contact — all 4 normal rows are solved, an
             * inactive one with r = 0, s0 = 0 and zero effective masses (so its
             * rows apply zero impulse), with the patch's anchors as the friction
             * rows (an absent anchor likewise) */
            int any = 0;
            for (j = 0; j < 4; ++j) any = any || sl[j].on;
            if (any) {
                float s0c[4];
                int onc[4];
                for (j = 0; j < 4; ++j) { onc[j] = sl[j].on; s0c[j] = sl[j].on ? sl[j].s0 : 0.0f; }
                gpatch_update_(&R, x, q, B.n, cp, s0c, onc, P->fot, P->corr);
            } else {
                R.cnt = 0;
            }
            if (any) {
                float mu = 0.0f, e = 0.0f, ak[2][2], al[2][2], ae[2][2], share;
                int clamped[2][2] = {{0, 0}, {0, 0}}, a;
                v3_t arr[2];
                if (nsh == 1) {
                    const float* sh = m->shapes + (size_t)sh0 * MG_SHAPE_STRIDE;
                    mu = 0.5f * (sh[11] + P->mu_g);
                    e = 0.5f * (sh[12] + P->e_g);
                }
                for (j = 0; j < 4; ++j) {
                    const int act = sl[j].on;
                    if (!act) { sl[j].r = V(0.0f, 0.0f, 0.0f); sl[j].s0 = 0.0f; }
                    sl[j].mu = mu; sl[j].e = e;
                    {
                        const v3_t r = sl[j].r;
                        sl[j].kn = act ? 1.0f / (invm + b_kn(&B, r, b_iwn(&B, &Iw, r))) : 0.0f;
                    }
                    sl[j].ln = 0.0f;
                    sl[j].vn0 = b_vn(&B, v, w, sl[j].r);
                    sl[j].on = 1;
                }
                /* anchor rows: the anchor's body copy, tangents t1, t2; position
                 * sweeps close 80 % of the substep-start drift of its two copies */
                for (a = 0; a < 2; ++a) {
                    const int act = a < R.cnt;
                    v3_t r = V(0.0f, 0.0f, 0.0f);
                    float e1 = 0.0f, e2 = 0.0f;
                    if (act) {
                        const v3_t wa = add3(x, qrot_(q, R.aA[a]));
                        const v3_t dr = sub3(wa, R.aB[a]);
                        const float kd = 0.8f * P->inv_h;
                        r = sub3(wa, xc);
                        e1 = fminf(fmaxf(-b_d1(&B, dr) * kd, -P->maxdep), P->maxdep);
                        e2 = fminf(fmaxf(-b_d2(&B, dr) * kd, -P->maxdep), P->maxdep);
                    }
                    arr[a] = r;
                    ak[a][0] = act ? 1.0f / (invm + b_k1(&B, r, b_iw1(&B, &Iw, r))) : 0.0f;
                    ak[a][1] = act ? 1.0f / (invm + b_k2(&B, r, b_iw2(&B, &Iw, r))) : 0.0f;
                    ae[a][0] = e1; ae[a][1] = e2;
                    al[a][0] = 0.0f; al[a][1] = 0.0f;
                }
                /* each anchor of a two-anchor patch holds half of the patch's
                 * Coulomb budget mu N per direction (symmetric: a box sliding on
                 * its diagonal anchors exerts no yaw torque; the two saturate at
                 * mu N together) */
                share = R.cnt == 2 ? 0.5f : 1.0f;
                /* sweep order (round 6): a position sweep solves the anchors'
                 * rows, then the normal rows, so the velocity it integrates is the
                 * one non-penetration had the last word on; only the first one
                 * opens with the normal rows (the anchors' budget needs a normal
                 * impulse). A velocity sweep is normal, anchor, normal rows. With
                 * the normal rows first in every position sweep (rounds 3-5) the
                 * anchors' rows left a rotation about the line through the two
                 * anchors in the integrated velocity: a vehicle pushed at 0.9
                 * mu m g across that line crept at ~13 mm/s, held by anchors that
                 * never clamped (tests/test_ground_patch_kat.py, yawed pushes). */
                for (it = 0; it < P->npos + P->nvel; ++it) {
                    const int pos = it < P->npos, last = it == P->npos + P->nvel - 1;
                    float psum;
                    for (j = 0; j < 4 && (it == 0 || !pos); ++j) {
                        const float sj = b_ps(&B, sl[j].s0, dx, dth, sl[j].r);
                        contact_normal(&B, &sl[j], &v, &w, invm, &Iw,
                                       pos ? pos_target_(P, sj) : vel_target_(P, sj, sl[j].e, sl[j].vn0));
                    }
                    /* the patch's normal impulse, in slot order */
                    psum = sl[0].ln;
                    for (j = 1; j < 4; ++j) psum = psum + sl[j].ln;
                    for (a = 0; a < 2; ++a) {
                        const float mun = mu * psum;
                        int rw;
                        for (rw = 0; rw < 2; ++rw) {
                            const float lim = share * mun;
                            const float tgt = pos ? ae[a][rw] : 0.0f;
                            const float vt = rw == 0 ? b_v1(&B, v, w, arr[a]) : b_v2(&B, v, w, arr[a]);
                            const float raw = fmaf(ak[a][rw], tgt - vt, al[a][rw]);
                            const float nl = clamp_sym_(raw, lim);
                            const float dl = nl - al[a][rw];
                            clamped[a][rw] = last && (raw > lim || raw < -lim);
                            al[a][rw] = nl;
                            if (rw == 0) {
                                v = b_f1(&B, v, dl, invm);
                                w = fmad3_(w, b_iw1(&B, &Iw, arr[a]), dl);
                            } else {
                                v = b_f2(&B, v, dl, invm);
                                w = fmad3_(w, b_iw2(&B, &Iw, arr[a]), dl);
                            }
                        }
                    }
                    /* every sweep ends with the normal rows (same targets: dx, dth
                     * are unchanged within a sweep) */
                    {
                        for (j = 0; j < 4; ++j) {
                            const float sj = b_ps(&B, sl[j].s0, dx, dth, sl[j].r);
                            contact_normal(&B, &sl[j], &v, &w, invm, &Iw,
                                           pos ? pos_target_(P, sj) : vel_target_(P, sj, sl[j].e, sl[j].vn0));
                        }
                    }
                    if (pos) {
                        dx = fmad3_(dx, v, P->sub);
                        dth = fmad3_(dth, w, P->sub);
                    }
                }
                for (j = 0; j < 4; ++j) fsum = b_addn(&B, fsum, sl[j].ln);
                for (a = 0; a < 2; ++a) {
                    fsum = b_add1(&B, fsum, al[a][0]);
                    fsum = b_add2(&B, fsum, al[a][1]);
                }
                /* a slipping patch lets go (regrown at the next substep): every
                 * anchor it holds clamped along one direction in the last sweep
                 * (mg_rigid.hip) */
                {
                    const int one = R.cnt < 2;
                    if ((clamped[0][0] && (clamped[1][0] || one)) || (clamped[0][1] && (clamped[1][1] || one)))
                        R.cnt = 0;
                }
            } else {
                for (it = 0; it < P->npos; ++it) {
                    dx = fmad3_(dx, v, P->sub);
                    dth = fmad3_(dth, w, P->sub);
                }
            }
            {
                const v3_t xc1 = add3(xc, dx);
                q = qint_(q, dth);
                x = origin_from_com_(xc1, q, com);
            }
            continue;
        }
        for (j = 0; j < OR_MAXC; ++j) {
            if (!sl[j].on || nsh <= 1) continue;
            {
                const v3_t r = sl[j].r;
                sl[j].kn = 1.0f / (invm + b_kn(&B, r, b_iwn(&B, &Iw, r)));
                sl[j].kt1 = 1.0f / (invm + b_k1(&B, r, b_iw1(&B, &Iw, r)));
                sl[j].kt2 = 1.0f / (invm + b_k2(&B, r, b_iw2(&B, &Iw, r)));
                sl[j].ln = 0.0f; sl[j].lt1 = 0.0f; sl[j].lt2 = 0.0f;
                sl[j].vn0 = b_vn(&B, v, w, sl[j].r);
            }
        }
        for (it = 0; it < P->npos; ++it) {
            for (j = 0; j < OR_MAXC; ++j) {
                if (!sl[j].on) continue;
                contact_normal(&B, &sl[j], &v, &w, invm, &Iw, pos_target_(P, b_ps(&B, sl[j].s0, dx, dth, sl[j].r)));
            }
            for (j = 0; j < OR_MAXC; ++j)
                if (sl[j].on) contact_friction(&B, &sl[j], &v, &w, invm, &Iw);
            dx = fmad3_(dx, v, P->sub);
            dth = fmad3_(dth, w, P->sub);
        }
        for (it = 0; it < P->nvel; ++it) {
            for (j = 0; j < OR_MAXC; ++j) {
                if (!sl[j].on) continue;
                contact_normal(&B, &sl[j], &v, &w, invm, &Iw,
                               vel_target_(P, b_ps(&B, sl[j].s0, dx, dth, sl[j].r), sl[j].e, sl[j].vn0));
            }
            for (j = 0; j < OR_MAXC; ++j)
                if (sl[j].on) contact_friction(&B, &sl[j], &v, &w, invm, &Iw);
        }
        for (j = 0; j < OR_MAXC; ++j) {
            if (!sl[j].on) continue;
            fsum = b_addn(&B, fsum, sl[j].ln);
            fsum = b_add1(&B, fsum, sl[j].lt1);
            fsum = b_add2(&B, fsum, sl[j].lt2);
        }
        {
            const v3_t xc1 = add3(xc, dx);
            q = qint_(q, dth);
            x = origin_from_com_(xc1, q, com);
        }
    }
    st[0] = x.x; st[1] = x.y; st[2] = x.z;
    st[3] = q.x; st[4] = q.y; st[5] = q.z; st[6] = q.w;
    st[7] = v.x; st[8] = v.y; st[9] = v.z;
    st[10] = w.x; st[11] = w.y; st[12] = w.z;
    cf[0] = fsum.x * P->inv_dt; cf[1] = fsum.y * P->inv_dt; cf[2] = fsum.z * P->inv_dt;
    if (pr && nsh == 1 && P->ground) gpatch_store_(&R, pr);
}

/* ---- spatial algebra ----------------------------------- */
typedef struct { v3_t w, v; } sv_t;

static sv_t SVc(v3_t w, v3_t v) { sv_t r; r.w = w; r.v = v; return r; }
static sv_t sv0(void) { return SVc(V(0.0f, 0.0f, 0.0f), V(0.0f, 0.0f, 0.0f)); }
static sv_t svadd_(sv_t a, sv_t b) { return SVc(add3(a.w, b.w), add3(a.v, b.v)); }
static sv_t svmul_(sv_t a, float s) { return SVc(mul3(a.w, s), mul3(a.v, s)); }
static sv_t crm_(sv_t a, sv_t b) { return SVc(cross3(a.w, b.w), add3(cross3(a.w, b.v), cross3(a.v, b.w))); }
static sv_t crf_(sv_t a, sv_t f) { return SVc(add3(cross3(a.w, f.w), cross3(a.v, f.v)), cross3(a.w, f.v)); }
static m3_t M3c(v3_t c0, v3_t c1, v3_t c2) { m3_t m; m.c0 = c0; m.c1 = c1; m.c2 = c2; return m; }
static m3_t mt_(m3_t a) { return M3c(V(a.c0.x, a.c1.x, a.c2.x), V(a.c0.y, a.c1.y, a.c2.y), V(a.c0.z, a.c1.z, a.c2.z)); }
static sv_t xmot_(m3_t E, v3_t r, sv_t m) { return SVc(mv_(E, m.w), mv_(E, sub3(m.v, cross3(r, m.w)))); }
static q4_t qaxang_(v3_t a, float th) {
    float s, c, half = 0.5f * th, ah = half < 0.0f ? -half : half;
    sincos_(ah, &s, &c);
    if (half < 0.0f) s = -s;
    return Q(a.x * s, a.y * s, a.z * s, c);
}

/* ---- ball joints in exponential coordinates (mg_spatial.h q_exp / q_log /
 * ball_step / link_joint, op for op): DOF positions = the rotation vector of
 * the child joint frame, velocities = its angular velocity in the child frame
 * (test13_camera_spherical_joint.py:243-256, quat2expcoord) */
static q4_t qexp_(v3_t th) {
    const float t2 = dot3(th, th);
    float t, s, c, k;
    if (!(t2 > 0.0f)) return Q(0.0f, 0.0f, 0.0f, 1.0f);
    t = sqrtf(t2);
    sincos_(0.5f * t, &s, &c);
    k = s / t;
    return Q(th.x * k, th.y * k, th.z * k, c);
}
static float atan_small_(float u) {
    const float u2 = u * u;
    float p = 1.0f / 19.0f;
    p = 1.0f / 17.0f - u2 * p;
    p = 1.0f / 15.0f - u2 * p;
    p = 1.0f / 13.0f - u2 * p;
    p = 1.0f / 11.0f - u2 * p;
    p = 1.0f / 9.0f - u2 * p;
    p = 1.0f / 7.0f - u2 * p;
    p = 1.0f / 5.0f - u2 * p;
    p = 1.0f / 3.0f - u2 * p;
    p = 1.0f - u2 * p;
    return u * p;
}
static float atan01_(float t) {
    if (t > 0.41421356f) return 0.78539816f + atan_small_((t - 1.0f) / (t + 1.0f));
    return atan_small_(t);
}
static v3_t qlog_(q4_t q) {
    float v2, vn, ha, k;
    if (q.w < 0.0f) q = Q(-q.x, -q.y, -q.z, -q.w);
    v2 = q.x * q.x + q.y * q.y + q.z * q.z;
    if (!(v2 > 0.0f)) return V(0.0f, 0.0f, 0.0f);
    vn = sqrtf(v2);
    ha = vn <= q.w ? atan01_(vn / q.w) : 1.57079633f - atan01_(q.w / vn);
    k = (2.0f * ha) / vn;
    return V(q.x * k, q.y * k, q.z * k);
}
static v3_t ball_step_(v3_t th, v3_t dth) { return qlog_(qnorm_(qmul_(qexp_(th), qexp_(dth)))); }

/* joint transform of link l at (q, qd): relative rotation/translation, S, vJ.
 * q: the articulation's DOF positions (a ball joint's first link reads three) */
static void joint_(const float* lf, int jt, const float* q, int dj, q4_t* qrel, v3_t* rr, sv_t* S) {
    const v3_t po = V(lf[0], lf[1], lf[2]);
    const q4_t qo = Q(lf[3], lf[4], lf[5], lf[6]);
    const v3_t ax = V(lf[7], lf[8], lf[9]);
    const int ball = (int)lf[10];
    const float qj = dj >= 0 ? q[dj] : 0.0f;
    *qrel = qo; *rr = po; *S = sv0();
    if (jt == MG_JOINT_REVOLUTE) {
        if (ball == 1) *qrel = qmul_(qo, qexp_(V(q[dj], q[dj + 1], q[dj + 2])));
        else if (ball == 0) *qrel = qmul_(qo, qaxang_(ax, qj));
        *S = SVc(ax, V(0.0f, 0.0f, 0.0f));
    } else if (jt == MG_JOINT_PRISMATIC) {
        *rr = add3(po, qrot_(qo, mul3(ax, qj)));
        *S = SVc(V(0.0f, 0.0f, 0.0f), ax);
    }
}
/* place of DOF d in a ball joint (1, 2, 3; 0: not a ball DOF) */
static int dof_ball_(const float* LF, const int* LI, int L, int d) {
    int l;
    for (l = 0; l < L; ++l)
        if (LI[l * MG_LINK_I_N + 2] == d) return (int)LF[l * MG_LINK_F_N + 10];
    return 0;
}

#include "migym_oracle_env.c"
#include "migym_oracle_pile.c"
#include "migym_oracle_render.c"

/* ---- serial chains: mg_chain.hip k_artic_chain, op for
 * op — the joint-space form (composite inertias, recursive Newton-Euler bias,
 * LDL^T of M + diag(armature + implicit drive)), explicit fmaf where the kernel
 * has them. Templates: fixed base, 2..4 links, link l's parent l - 1 and DOF
 * l - 1 (revolute or prismatic), one body per link (migym_capi.cpp g.chain). */
typedef struct { float xx, yy, zz, xy, xz, yz; v3_t h; float m; } ri_t;
typedef struct { float m; v3_t com; float ib[6]; } clink_t;

static v3_t fcross_(v3_t a, v3_t b) {
    return V(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static sv_t ri_mul_(const ri_t* I, sv_t x) {
    const v3_t t = fcross_(I->h, x.v), s = fcross_(I->h, x.w);
    return SVc(V(fmaf(I->xx, x.w.x, fmaf(I->xy, x.w.y, fmaf(I->xz, x.w.z, t.x))),
                 fmaf(I->xy, x.w.x, fmaf(I->yy, x.w.y, fmaf(I->yz, x.w.z, t.y))),
                 fmaf(I->xz, x.w.x, fmaf(I->yz, x.w.y, fmaf(I->zz, x.w.z, t.z)))),
               V(fmaf(I->m, x.v.x, -s.x), fmaf(I->m, x.v.y, -s.y), fmaf(I->m, x.v.z, -s.z)));
}
static float sdot_(sv_t a, sv_t b) {
    return fmaf(a.v.z, b.v.z, fmaf(a.v.y, b.v.y, fmaf(a.v.x, b.v.x, fmaf(a.w.z, b.w.z, fmaf(a.w.y, b.w.y, a.w.x * b.w.x)))));
}
static sv_t crm_f_(sv_t a, sv_t b) { return SVc(fcross_(a.w, b.w), add3(fcross_(a.w, b.v), fcross_(a.v, b.w))); }
static sv_t crf_f_(sv_t a, sv_t f) { return SVc(add3(fcross_(a.w, f.w), fcross_(a.v, f.v)), fcross_(a.w, f.v)); }
static clink_t chain_link_(const float* M) {
    clink_t k;
    const m3_t R = qmat_(Q(M[4], M[5], M[6], M[7]));
    const v3_t u0 = mul3(R.c0, M[1] > 0.0f ? 1.0f / M[1] : 0.0f);
    const v3_t u1 = mul3(R.c1, M[2] > 0.0f ? 1.0f / M[2] : 0.0f);
    const v3_t u2 = mul3(R.c2, M[3] > 0.0f ? 1.0f / M[3] : 0.0f);
    k.m = M[11];
    k.com = V(M[8], M[9], M[10]);
    k.ib[0] = fmaf(u0.x, R.c0.x, fmaf(u1.x, R.c1.x, u2.x * R.c2.x));
    k.ib[1] = fmaf(u0.y, R.c0.y, fmaf(u1.y, R.c1.y, u2.y * R.c2.y));
    k.ib[2] = fmaf(u0.z, R.c0.z, fmaf(u1.z, R.c1.z, u2.z * R.c2.z));
    k.ib[3] = fmaf(u0.x, R.c0.y, fmaf(u1.x, R.c1.y, u2.x * R.c2.y));
    k.ib[4] = fmaf(u0.x, R.c0.z, fmaf(u1.x, R.c1.z, u2.x * R.c2.z));
    k.ib[5] = fmaf(u0.y, R.c0.z, fmaf(u1.y, R.c1.z, u2.y * R.c2.z));
    return k;
}
/* R v, one fused chain per component (mg_chain.hip rmul) */
static v3_t rmul_(const m3_t* R, v3_t v) {
    return V(fmaf(R->c2.x, v.z, fmaf(R->c1.x, v.y, R->c0.x * v.x)), fmaf(R->c2.y, v.z, fmaf(R->c1.y, v.y, R->c0.y * v.x)),
             fmaf(R->c2.z, v.z, fmaf(R->c1.z, v.y, R->c0.z * v.x)));
}
static ri_t world_ri_(const clink_t* K, const m3_t* Rm, v3_t xl, v3_t x0, v3_t* cout) {
    const m3_t R = *Rm;
    const float* b = K->ib;
    const float ib[3][3] = {{b[0], b[3], b[4]}, {b[3], b[1], b[5]}, {b[4], b[5], b[2]}};
    const float r[3][3] = {{R.c0.x, R.c1.x, R.c2.x}, {R.c0.y, R.c1.y, R.c2.y}, {R.c0.z, R.c1.z, R.c2.z}};
    float t[3][3];
    int i, j;
    v3_t c, h;
    ri_t I;
    for (i = 0; i < 3; ++i)
        for (j = 0; j < 3; ++j) t[i][j] = fmaf(r[i][2], ib[2][j], fmaf(r[i][1], ib[1][j], r[i][0] * ib[0][j]));
#define OR_IC(i, j) fmaf(t[i][2], r[j][2], fmaf(t[i][1], r[j][1], t[i][0] * r[j][0]))
    c = sub3(add3(xl, rmul_(Rm, K->com)), x0);
    h = mul3(c, K->m);
    I.xx = fmaf(h.y, c.y, fmaf(h.z, c.z, OR_IC(0, 0)));
    I.yy = fmaf(h.x, c.x, fmaf(h.z, c.z, OR_IC(1, 1)));
    I.zz = fmaf(h.x, c.x, fmaf(h.y, c.y, OR_IC(2, 2)));
    I.xy = fmaf(-h.x, c.y, OR_IC(0, 1));
    I.xz = fmaf(-h.x, c.z, OR_IC(0, 2));
    I.yz = fmaf(-h.y, c.z, OR_IC(1, 2));
#undef OR_IC
    I.h = h;
    I.m = K->m;
    *cout = c;
    return I;
}
/* link pose from the parent's (orientation qp, rotation matrix Rp, origin xp);
 * norm: renormalise (the output pass only, mg_chain.hip chain_fk<NORM>) */
static void chain_fk_(const float* lf, int jt, float qj, q4_t qp, const m3_t* Rp, v3_t xp, int norm, q4_t* ql,
                      v3_t* xl) {
    const v3_t po = V(lf[0], lf[1], lf[2]), ax = V(lf[7], lf[8], lf[9]);
    const q4_t qo = Q(lf[3], lf[4], lf[5], lf[6]);
    q4_t qrel = qo;
    v3_t rr = po;
    if (jt == MG_JOINT_REVOLUTE) qrel = qmul_(qo, qaxang_(ax, qj));
    else if (jt == MG_JOINT_PRISMATIC) rr = add3(po, qrot_(qo, mul3(ax, qj)));
    *ql = norm ? qnorm_(qmul_(qp, qrel)) : qmul_(qp, qrel);
    *xl = add3(xp, rmul_(Rp, rr));
}
static sv_t chain_axis_(const float* lf, int jt, const m3_t* R, v3_t xl, v3_t x0) {
    const v3_t z = rmul_(R, V(lf[7], lf[8], lf[9]));
    return jt == MG_JOINT_REVOLUTE ? SVc(z, fcross_(sub3(xl, x0), z)) : SVc(V(0.0f, 0.0f, 0.0f), z);
}
static void chain_drive_(const float* pr, const float* tg, float q, float u, float h, int xm, int xp,
                         float* tau0, float* imp) {
    const int mode = (int)pr[0];
    const float kp = pr[1], kd = pr[2], eff = pr[3];
    float tau = 0.0f, im = 0.0f;
    if (mode == MG_DOF_MODE_POS) {
        tau = kp * (tg[0] - q - h * u) + kd * (tg[1] - u);
        im = h * kd + h * h * kp;
    } else if (mode == MG_DOF_MODE_VEL) {
        tau = kd * (tg[1] - u);
        im = h * kd;
    } else if (mode == MG_DOF_MODE_EFFORT) {
        tau = tg[2];
    }
    if (eff > 0.0f) {
        if (xm) {
            tau = xp ? eff : -eff;
            im = 0.0f;
        } else if (im == 0.0f) {
            tau = fminf(fmaxf(tau, -eff), eff);
        }
    }
    *tau0 = tau;
    *imp = im;
}
/* (M + diag(arm + imp)) x = b, LDL^T, M by its upper triangle */
static void chain_solve_(int D, float M[3][3], const float* arm, const float* imp, const float* b, float* x) {
    float L[3][3], Ld[3][3], r[3], y[3];
    int i, j, k;
    for (j = 0; j < D; ++j) {
        float dj = M[j][j] + (arm[j] + imp[j]);
        for (k = 0; k < j; ++k) dj = fmaf(-L[j][k], Ld[j][k], dj);
        r[j] = 1.0f / dj;
        for (i = j + 1; i < D; ++i) {
            float sm = M[j][i];
            for (k = 0; k < j; ++k) sm = fmaf(-L[i][k], Ld[j][k], sm);
            Ld[i][j] = sm;
            L[i][j] = sm * r[j];
        }
    }
    for (i = 0; i < D; ++i) {
        float t = b[i];
        for (k = 0; k < i; ++k) t = fmaf(-L[i][k], y[k], t);
        y[i] = t;
    }
    for (i = D - 1; i >= 0; --i) {
        float t = y[i] * r[i];
        for (k = i + 1; k < D; ++k) t = fmaf(-L[k][i], x[k], t);
        x[i] = t;
    }
}
/* 1 when the template steps in k_artic_chain (migym_capi.cpp g.chain, 2..4 links) */
static int is_chain_(const int* LI, int L, int D, int fixed_base) {
    int l;
    if (!fixed_base || L < 2 || L > 4 || D != L - 1 || LI[0] != -1 || LI[3] != 0) return 0;
    for (l = 1; l < L; ++l) {
        const int* li = LI + l * MG_LINK_I_N;
        if (li[0] != l - 1 || li[2] != l - 1 || li[3] != l) return 0;
        if (li[1] != MG_JOINT_REVOLUTE && li[1] != MG_JOINT_PRISMATIC) return 0;
    }
    return 1;
}
static void chain_step_(const step_t* P, const mg_model* m, const float* LF, const int* LI, int L, int b0, int d0,
                        float* state, float* dof, const float* tgt, const float* props, const float* ext) {
    const int D = L - 1;
    const float h = P->h;
    const float* s0 = state + (size_t)b0 * MG_STATE_N;
    const v3_t x0 = V(s0[0], s0[1], s0[2]);
    const q4_t q0 = qnorm_(Q(s0[3], s0[4], s0[5], s0[6]));
    const m3_t R0 = qmat_(q0);
    const float grav_on = m->tmpl_body_f[(size_t)m->body_tmpl[b0] * MG_TBODY_F_N + 4];
    const v3_t gw = grav_on != 0.0f ? V(P->g[0], P->g[1], P->g[2]) : V(0.0f, 0.0f, 0.0f);
    float qv[3], uv[3], arm[3];
    clink_t lk[4];
    int l, d, st_, j, i;
    for (d = 0; d < D; ++d) {
        qv[d] = dof[(d0 + d) * 2 + 0];
        uv[d] = dof[(d0 + d) * 2 + 1];
        arm[d] = props[(size_t)(d0 + d) * MG_DOFPROP_N + 8];
    }
    for (l = 1; l < L; ++l) lk[l] = chain_link_(m->body_mass + (size_t)(b0 + l) * MG_MASS_N);
    for (st_ = 0; st_ < P->substeps; ++st_) {
        sv_t xi[3];
        float Cb[3], M[3][3], qdd[3], tau0[3], imp[3], rhs[3];
        int xm[3], xpl[3], flip = 0;
        {
            q4_t qp = q0;
            m3_t Rp = R0;
            v3_t xp = x0;
            sv_t vp = sv0(), ap = SVc(V(0.0f, 0.0f, 0.0f), V(-gw.x, -gw.y, -gw.z));
            for (l = 1; l < L; ++l) {
                const float* lf = LF + l * MG_LINK_F_N;
                const int jt = LI[l * MG_LINK_I_N + 1];
                q4_t ql;
                v3_t xl, c;
                sv_t x, vJ, v, acc, f;
                ri_t I;
                m3_t Rl;
                chain_fk_(lf, jt, qv[l - 1], qp, &Rp, xp, 0, &ql, &xl);
                Rl = qmat_(ql);
                x = chain_axis_(lf, jt, &Rl, xl, x0);
                vJ = svmul_(x, uv[l - 1]);
                v = svadd_(vp, vJ);
                acc = svadd_(ap, crm_f_(v, vJ));
                I = world_ri_(&lk[l], &Rl, xl, x0, &c);
                {
                    const sv_t Iv = ri_mul_(&I, v);
                    f = svadd_(ri_mul_(&I, acc), crf_f_(v, Iv));
                }
                if (ext) {
                    const float* e = ext + (size_t)(b0 + l) * 6;
                    const v3_t fe = V(e[0], e[1], e[2]), te = V(e[3], e[4], e[5]);
                    f = SVc(sub3(f.w, add3(te, cross3(c, fe))), sub3(f.v, fe));
                }
                xi[l - 1] = x;
                for (j = 0; j < l; ++j) Cb[j] = j == l - 1 ? sdot_(x, f) : Cb[j] + sdot_(xi[j], f);
                /* joint-space inertia accumulated link by link (mg_chain.hip):
                 * link l - 1 adds xi_i . (I xi_j) to M_ij for i <= j <= l - 1 */
                for (j = 0; j < l; ++j) {
                    const sv_t Fm = ri_mul_(&I, xi[j]);
                    for (i = 0; i <= j; ++i) {
                        const float mij = sdot_(xi[i], Fm);
                        M[i][j] = j == l - 1 ? mij : M[i][j] + mij;
                    }
                }
                qp = ql; Rp = Rl; xp = xl; vp = v; ap = acc;
            }
        }
        for (d = 0; d < D; ++d) {
            const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
            xm[d] = 0; xpl[d] = 0;
            chain_drive_(pr, tgt + (size_t)(d0 + d) * 3, qv[d], uv[d], h, 0, 0, &tau0[d], &imp[d]);
            rhs[d] = tau0[d] - Cb[d];
        }
        chain_solve_(D, M, arm, imp, rhs, qdd);
        for (d = 0; d < D; ++d) {
            const float eff = props[(size_t)(d0 + d) * MG_DOFPROP_N + 3];
            if (eff > 0.0f && imp[d] != 0.0f) {
                const float actf = tau0[d] - imp[d] * qdd[d];
                if (actf > eff) { xm[d] = 1; xpl[d] = 1; flip = 1; }
                else if (actf < -eff) { xm[d] = 1; flip = 1; }
            }
        }
        if (flip) {
            for (d = 0; d < D; ++d) {
                chain_drive_(props + (size_t)(d0 + d) * MG_DOFPROP_N, tgt + (size_t)(d0 + d) * 3, qv[d], uv[d], h,
                             xm[d], xpl[d], &tau0[d], &imp[d]);
                rhs[d] = tau0[d] - Cb[d];
            }
            chain_solve_(D, M, arm, imp, rhs, qdd);
        }
        for (d = 0; d < D; ++d) {
            const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
            const float maxv = pr[4];
            float wv = uv[d] + h * qdd[d], xv;
            if (maxv > 0.0f) wv = fminf(fmaxf(wv, -maxv), maxv);
            xv = qv[d] + h * wv;
            if (pr[7] != 0.0f) {
                if (xv < pr[5]) { xv = pr[5]; if (wv < 0.0f) wv = 0.0f; }
                if (xv > pr[6]) { xv = pr[6]; if (wv > 0.0f) wv = 0.0f; }
            }
            qv[d] = xv;
            uv[d] = wv;
        }
    }
    for (d = 0; d < D; ++d) { dof[(d0 + d) * 2 + 0] = qv[d]; dof[(d0 + d) * 2 + 1] = uv[d]; }
    {
        q4_t qp = q0;
        m3_t Rp = R0;
        v3_t xp = x0;
        sv_t vp = sv0();
        for (l = 0; l < L; ++l) {
            float* so = state + (size_t)(b0 + l) * MG_STATE_N;
            q4_t ql = q0;
            v3_t xl = x0, ww = V(0.0f, 0.0f, 0.0f), vw = V(0.0f, 0.0f, 0.0f);
            if (l > 0) {
                const float* lf = LF + l * MG_LINK_F_N;
                const int jt = LI[l * MG_LINK_I_N + 1];
                sv_t v;
                v3_t cw;
                m3_t Rl;
                chain_fk_(lf, jt, qv[l - 1], qp, &Rp, xp, 1, &ql, &xl);
                Rl = qmat_(ql);
                v = svadd_(vp, svmul_(chain_axis_(lf, jt, &Rl, xl, x0), uv[l - 1]));
                cw = add3(sub3(xl, x0), rmul_(&Rl, lk[l].com));
                ww = v.w;
                vw = add3(v.v, fcross_(v.w, cw));
                qp = ql; Rp = Rl; xp = xl; vp = v;
            }
            so[0] = xl.x; so[1] = xl.y; so[2] = xl.z;
            so[3] = ql.x; so[4] = ql.y; so[5] = ql.z; so[6] = ql.w;
            so[7] = vw.x; so[8] = vw.y; so[9] = vw.z;
            so[10] = ww.x; so[11] = ww.y; so[12] = ww.z;
        }
    }
}

/* ---- articulation: the world-frame articulated-body
 * algorithm (aba_world_, with the implicit drives and the effort-limit
 * re-solve), then the joint integration of an articulation without contacts
 * and the link states by forward kinematics — as mg_env.hip:k_artic_lanes. */
static int artic_step(const step_t* P, const mg_model* m, const int* ai, float* state /*[nb][13]*/,
                      float* dof /*[nd][2]*/, const float* tgt /*[nd][3]*/, const float* props /*[nd][12]*/,
                      const float* ext, float* cforce) {
    const int b0 = ai[0], d0 = ai[1], t = ai[2];
    const int* ti = m->artic_tmpl_i + (size_t)t * MG_ATMPL_I_N;
    const int fl = ti[0], L = ti[1], D = ti[2], fixed_base = ti[3];
    const float* LF = m->tmpl_link_f + (size_t)fl * MG_LINK_F_N;
    const int* LI = m->tmpl_link_i + (size_t)fl * MG_LINK_I_N;
    const float h = P->h;
    float q[OR_MAXL], qd[OR_MAXL], qdd[OR_MAXL];
    sv_t v[OR_MAXL];
    q4_t ql[OR_MAXL];
    v3_t xl[OR_MAXL];
    const float* s0 = state + (size_t)b0 * MG_STATE_N;
    const v3_t x0 = V(s0[0], s0[1], s0[2]);
    const q4_t q0 = qnorm_(Q(s0[3], s0[4], s0[5], s0[6]));
    const float grav_on = m->tmpl_body_f[(size_t)m->body_tmpl[b0] * MG_TBODY_F_N + 4];
    const v3_t gw = grav_on != 0.0f ? V(P->g[0], P->g[1], P->g[2]) : V(0.0f, 0.0f, 0.0f);
    int d, l, st_;
    if (!fixed_base || L > OR_MAXL) return -1;
    if (is_chain_(LI, L, D, fixed_base)) {   /* mg_chain.hip k_artic_chain */
        chain_step_(P, m, LF, LI, L, b0, d0, state, dof, tgt, props, ext);
        return 0;
    }
    for (d = 0; d < D; ++d) { q[d] = dof[(d0 + d) * 2 + 0]; qd[d] = dof[(d0 + d) * 2 + 1]; qdd[d] = 0.0f; }
    for (st_ = 0; st_ < P->substeps; ++st_) {
        float tau0d[OR_MAXL], impd[OR_MAXL], mdiag[OR_MAXL];
        static __thread aba_ws_t W;   /* per thread: oracle_step_mt */
        aba_world_(P, m, LF, LI, L, D, b0, d0, q, qd, props, tgt, x0, q0, gw, &W, qdd, mdiag, tau0d, impd, 0, ext,
                   (L > 16 || D > 16) ? 64 : 16);   /* k_artic_lanes' lane width (mg_env.hip mg_wide) */
        {
            float qn[OR_MAXL], wn[OR_MAXL];
            for (d = 0; d < D; ++d) {
                const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
                const float maxv = pr[4];
                float wv = qd[d] + h * qdd[d], xv;
                if (maxv > 0.0f) wv = fminf(fmaxf(wv, -maxv), maxv);
                xv = q[d] + h * wv;
                if (pr[7] != 0.0f) {
                    const float lo = pr[5], hi = pr[6];
                    if (xv < lo) { xv = lo; if (wv < 0.0f) wv = 0.0f; }
                    if (xv > hi) { xv = hi; if (wv > 0.0f) wv = 0.0f; }
                }
                qn[d] = xv; wn[d] = wv;
            }
            for (d = 0; d < D; ++d) {   /* ball joints: th <- log(exp(th) exp(h w)) */
                const int bk = dof_ball_(LF, LI, L, d);
                if (bk > 0) {
                    const int f = d - (bk - 1);
                    const v3_t tn = ball_step_(V(q[f], q[f + 1], q[f + 2]),
                                               V(h * wn[f], h * wn[f + 1], h * wn[f + 2]));
                    qn[d] = bk == 1 ? tn.x : (bk == 2 ? tn.y : tn.z);
                }
            }
            for (d = 0; d < D; ++d) { q[d] = qn[d]; qd[d] = wn[d]; }
        }
    }
    for (d = 0; d < D; ++d) { dof[(d0 + d) * 2 + 0] = q[d]; dof[(d0 + d) * 2 + 1] = qd[d]; }
    for (l = 0; l < L; ++l) {
        const int p = LI[l * MG_LINK_I_N + 0], jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
        const int bl = LI[l * MG_LINK_I_N + 3];          /* -1: virtual link of a ball joint */
        const float* M = link_mass_(m, LI, b0, l);
        float* so = bl >= 0 ? state + (size_t)(b0 + bl) * MG_STATE_N : NULL;
        v3_t ww, vw, com = V(M[8], M[9], M[10]);
        if (p < 0) {
            ql[l] = q0; xl[l] = x0; v[l] = sv0();
        } else {
            q4_t qrel; v3_t rr; sv_t s;
            const float qdj = dj >= 0 ? qd[dj] : 0.0f;
            joint_(LF + l * MG_LINK_F_N, jt, q, dj, &qrel, &rr, &s);
            ql[l] = qnorm_(qmul_(ql[p], qrel));
            xl[l] = add3(xl[p], qrot_(ql[p], rr));
            v[l] = svadd_(xmot_(mt_(qmat_(qrel)), rr, v[p]), svmul_(s, qdj));
        }
        if (!so) continue;
        ww = qrot_(ql[l], v[l].w);
        vw = qrot_(ql[l], add3(v[l].v, cross3(v[l].w, com)));
        so[0] = xl[l].x; so[1] = xl[l].y; so[2] = xl[l].z;
        so[3] = ql[l].x; so[4] = ql[l].y; so[5] = ql[l].z; so[6] = ql[l].w;
        so[7] = vw.x; so[8] = vw.y; so[9] = vw.z;
        so[10] = ww.x; so[11] = ww.y; so[12] = ww.z;
        cforce[(size_t)(b0 + bl) * 3 + 0] = 0.0f;
        cforce[(size_t)(b0 + bl) * 3 + 1] = 0.0f;
        cforce[(size_t)(b0 + bl) * 3 + 2] = 0.0f;
    }
    return 0;
}


/* ---- entry point --------------------------------------------------------
 * One gym.simulate() over the whole model, AoS host arrays:
 *   state [nb][13] in/out, dof [nd][2] in/out, tgt [nd][3] (target pos, target
 *   vel, actuation force), props [nd][12] (NULL = model->dof_props),
 *   ext [nb][6] world force/torque at the COM or NULL, cforce [nb][3] out,
 *   fcache: the coupled step's friction patches, [num_envs][OE_FC_N] floats
 *   kept by the caller from step to step (zeros: no patch yet; NULL: none kept),
 *   bcache: the free bodies' ground patches, [num_bodies][OR_GP_N], likewise.
 * Bodies in [body_begin, body_end) only (a bounded CPU-baseline sample);
 * articulations are stepped when their root lies in that range. Returns 0, or
 * -1 for an unsupported model. */
int oracle_step(const mg_sim_params* p, const mg_model* m, float* state, float* dof, const float* tgt,
                const float* props, const float* ext, float* cforce, float* fcache, float* bcache, int body_begin,
                int body_end) {
    step_t P = make_step_(p);
    int b, k, ne, rc = 0;
    oenv_t* envs = NULL;
    char* owned = NULL;
    if (!props) props = m->dof_props;
    if (body_end < 0 || body_end > m->num_bodies) body_end = m->num_bodies;
    envs = (oenv_t*)calloc((size_t)(m->num_envs > 0 ? m->num_envs : 1), sizeof(oenv_t));
    owned = (char*)calloc((size_t)(m->num_bodies > 0 ? m->num_bodies : 1), 1);
    if (!envs || !owned) { rc = -1; goto done; }
    ne = classify_envs_(m, envs, owned);
    if (ne < 0) { rc = -1; goto done; }
    for (k = 0; k < ne; ++k) {
        const int first = envs[k].art_body >= 0 ? envs[k].art_body : envs[k].free_b[0];
        if (first < body_begin || first >= body_end) continue;
        if ((envs[k].pile ? pile_step_(&P, m, &envs[k], state, ext, cforce)
                          : env_step_(&P, m, &envs[k], state, dof, tgt, props, ext, cforce, fcache)) != 0) {
            rc = -1;
            goto done;
        }
    }
    for (k = 0; k < m->num_artics; ++k) {
        const int* ai = m->artic_i + (size_t)k * MG_ARTIC_I_N;
        if (ai[0] < body_begin || ai[0] >= body_end || owned[ai[0]]) continue;
        if (artic_step(&P, m, ai, state, dof, tgt, props, ext, cforce) != 0) { rc = -1; goto done; }
    }
    for (b = body_begin; b < body_end; ++b) {
        if (m->body_kind[b] != MG_BODY_FREE || owned[b]) continue;
        rigid_body_step(&P, m, b, state + (size_t)b * MG_STATE_N, ext ? ext + (size_t)b * 6 : NULL,
                        cforce + (size_t)b * 3, bcache ? bcache + (size_t)b * OR_GP_N : NULL);
    }
done:
    free(envs);
    free(owned);
    return rc;
}

/* The same step on `nthreads` host threads (OpenMP, explicit num_threads: the
 * CPU baseline of bench.py, SURVEY.md §8d "CPU beside it"). Envs, articulations
 * and free bodies are independent, so each of the three loops is split across
 * the threads after one classification; results equal oracle_step's. */
int oracle_step_mt(const mg_sim_params* p, const mg_model* m, float* state, float* dof, const float* tgt,
                   const float* props, const float* ext, float* cforce, float* fcache, float* bcache, int nthreads) {
    step_t P = make_step_(p);
    int ne, rc = 0;
    oenv_t* envs = NULL;
    char* owned = NULL;
    if (!props) props = m->dof_props;
    if (nthreads < 1) nthreads = 1;
    envs = (oenv_t*)calloc((size_t)(m->num_envs > 0 ? m->num_envs : 1), sizeof(oenv_t));
    owned = (char*)calloc((size_t)(m->num_bodies > 0 ? m->num_bodies : 1), 1);
    if (!envs || !owned) { rc = -1; goto done; }
    ne = classify_envs_(m, envs, owned);
    if (ne < 0) { rc = -1; goto done; }
    {
        int bad = 0;
#pragma omp parallel num_threads(nthreads) reduction(| : bad)
        {
            int k, b;
#pragma omp for schedule(dynamic, 16)
            for (k = 0; k < ne; ++k)
                if ((envs[k].pile ? pile_step_(&P, m, &envs[k], state, ext, cforce)
                                  : env_step_(&P, m, &envs[k], state, dof, tgt, props, ext, cforce, fcache)) != 0)
                    bad = 1;
#pragma omp for schedule(static)
            for (k = 0; k < m->num_artics; ++k) {
                const int* ai = m->artic_i + (size_t)k * MG_ARTIC_I_N;
                if (owned[ai[0]]) continue;
                if (artic_step(&P, m, ai, state, dof, tgt, props, ext, cforce) != 0) bad = 1;
            }
#pragma omp for schedule(static)
            for (b = 0; b < m->num_bodies; ++b) {
                if (m->body_kind[b] != MG_BODY_FREE || owned[b]) continue;
                rigid_body_step(&P, m, b, state + (size_t)b * MG_STATE_N, ext ? ext + (size_t)b * 6 : NULL,
                                cforce + (size_t)b * 3, bcache ? bcache + (size_t)b * OR_GP_N : NULL);
            }
        }
        if (bad) rc = -1;
    }
done:
    free(envs);
    free(owned);
    return rc;
}

int oracle_abi_version(void) { return MG_ABI_VERSION; }
