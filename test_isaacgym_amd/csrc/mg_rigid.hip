// mg_rigid.hip — fused free-body step: gym.simulate() for every single-body
// dynamic actor (the servo scene's UAV and ground vehicle).
//
// One lane = one free body for the whole frame: `substeps` TGS substeps, each
//   1. unconstrained velocity: gravity, external force, PhysX-style damping
//      v *= 1 - min(damping*h, 1), max-velocity clamp;
//   2. contact generation against the ground plane (box corners, sphere and
//      capsule end caps within contact_offset), at most MG_MAX_CONTACTS slots;
//   3. TGS: npos position iterations of length h/npos, each a Gauss-Seidel pass
//      over the normal rows (speculative / depenetration target) then over the
//      friction rows (Coulomb, circular cone), followed by integrating the
//      body's motion delta; then nvel velocity iterations with the bias removed;
//   4. pose update: com += sum of iteration deltas, q = exp(dtheta) q.
// Envs are independent and (test10_servo_vecenv.py:317,323: group=i, filter=-1)
// the two actors of an env do not collide, so lanes never communicate: no
// atomics, no LDS, no grid sync. State is SoA [field][body] so every load and
// store of a wavefront is one coalesced 256-B transaction per field.
// The C restatement is oracle/migym_oracle.c:oracle_rigid_step.
#include "mg_internal.h"
#include "mg_math.h"

namespace {

// 14 floats per contact slot: the world inverse inertia is one symmetric matrix
// per substep, re-applied to (r x dir) in every row instead of being cached per
// slot, which keeps the 8 slots in VGPRs (no scratch spills).
struct Slot {
    V3 r;        // contact point - centre of mass (world)
    float s0;    // separation minus rest offset at substep start
    float mu, e; // combined friction / restitution
    float kn, kt1, kt2;   // effective masses
    float ln, lt1, lt2;   // accumulated impulses
    float vn0;            // pre-solve normal velocity (restitution)
};

// Insert a contact candidate at slot 0 and shift the others up (static indices
// only: a select chain on `j == nc` is folded by the compiler into a dynamically
// indexed store, which forces the slot array into scratch memory). Slots hold
// the candidates newest-first; once MG_MAX_CONTACTS are held, later candidates
// are dropped.
__device__ __forceinline__ void push_candidate(Slot (&sl)[MG_MAX_CONTACTS], int& nc, V3 r, float s0,
                                               float mu, float e) {
    if (nc >= MG_MAX_CONTACTS) return;
#pragma unroll
    for (int j = MG_MAX_CONTACTS - 1; j > 0; --j) {
        sl[j].r = sl[j - 1].r; sl[j].s0 = sl[j - 1].s0; sl[j].mu = sl[j - 1].mu; sl[j].e = sl[j - 1].e;
    }
    sl[0].r = r; sl[0].s0 = s0; sl[0].mu = mu; sl[0].e = e;
    nc = nc + 1;
}

// The empty asm makes the lever arm opaque to loop-invariant code motion, so
// (r x n), Iw (r x n) ... are recomputed per row instead of being hoisted for all
// 8 slots out of the iteration loop (which spilled 176 B/lane to scratch).
#define MG_OPAQUE3(v) asm volatile("" : "+v"((v).x), "+v"((v).y), "+v"((v).z))

__device__ __forceinline__ void contact_normal(Slot& c, V3 n, V3& v, V3& w, float invm, const S3& Iw, float tgt) {
    MG_OPAQUE3(c.r);
    const V3 rn = vcross(c.r, n);
    const float vn = vdot(n, v) + vdot(w, rn);
    float dl = c.kn * (tgt - vn);
    const float nl = fmaxf(c.ln + dl, 0.0f);
    dl = nl - c.ln;
    c.ln = nl;
    v = vmad(v, n, dl * invm);
    w = vmad(w, symmul(Iw, rn), dl);
}

// Coulomb friction on a circular cone |lt| <= mu * ln
__device__ __forceinline__ void contact_friction(Slot& c, V3 t1, V3 t2, V3& v, V3& w, float invm, const S3& Iw) {
    MG_OPAQUE3(c.r);
    const V3 r1 = vcross(c.r, t1);
    const V3 r2 = vcross(c.r, t2);
    const float vt1 = vdot(t1, v) + vdot(w, r1);
    const float vt2 = vdot(t2, v) + vdot(w, r2);
    float n1 = c.lt1 - c.kt1 * vt1;
    float n2 = c.lt2 - c.kt2 * vt2;
    const float lim = c.mu * c.ln;
    const float m2 = n1 * n1 + n2 * n2;
    if (m2 > lim * lim) {
        const float sc = lim / sqrtf(m2);
        n1 = n1 * sc; n2 = n2 * sc;
    }
    const float d1 = n1 - c.lt1, d2 = n2 - c.lt2;
    c.lt1 = n1; c.lt2 = n2;
    v = vmad(vmad(v, t1, d1 * invm), t2, d2 * invm);
    w = vmad(vmad(w, symmul(Iw, r1), d1), symmul(Iw, r2), d2);
}

__global__ void __launch_bounds__(64) k_rigid_step(MgStep P, MgRigidArgs A) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= A.nf) return;
    const int b = A.free_ids[i];
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

    const V3 n = v3(P.n[0], P.n[1], P.n[2]);
    const V3 t1 = v3(P.t1[0], P.t1[1], P.t1[2]);
    const V3 t2 = v3(P.t2[0], P.t2[1], P.t2[2]);
    const float h = P.h;
    const float lin_keep = 1.0f - fminf(lin_damp * h, 1.0f);
    const float ang_keep = 1.0f - fminf(ang_damp * h, 1.0f);
    const float max_lv2 = max_lv * max_lv;
    const float max_av2 = max_av * max_av;

    q = qnormalize(q);
    V3 fsum = v3(0.0f, 0.0f, 0.0f);

    for (int st = 0; st < P.substeps; ++st) {
        const S3 Iw = sym_rdrt(qmat(qmul(q, iq)), invI);
        const V3 xc = vadd(x, qrot(q, com));

        // 1. unconstrained velocity
        if (grav_on != 0.0f) v = vmad(v, v3(P.g[0], P.g[1], P.g[2]), h);
        v = vmad(v, fext, invm * h);
        w = vmad(w, symmul(Iw, text), h);
        v = vscale(v, lin_keep);
        w = vscale(w, ang_keep);
        {
            float v2 = vdot(v, v);
            if (v2 > max_lv2) v = vscale(v, sqrtf(max_lv2 / v2));
            float w2 = vdot(w, w);
            if (w2 > max_av2) w = vscale(w, sqrtf(max_av2 / w2));
        }

        // 2. contacts against the ground plane
        Slot sl[MG_MAX_CONTACTS];
        int nc = 0;
        if (P.has_ground) {
            for (int s = sh0; s < sh0 + nsh; ++s) {
                const float* sh = A.shapes + s * MG_SHAPE_STRIDE;
                const int type = (int)sh[0];
                const Q4 qs = qmul(q, q4(sh[7], sh[8], sh[9], sh[10]));
                const V3 cs = vadd(x, qrot(q, v3(sh[4], sh[5], sh[6])));
                const float mu = 0.5f * (sh[11] + P.mu_ground);
                const float e = 0.5f * (sh[12] + P.e_ground);
                if (type == MG_SHAPE_BOX) {
                    const M3 Rs = qmat(qs);
                    const V3 a0 = vscale(Rs.c0, sh[1]);
                    const V3 a1 = vscale(Rs.c1, sh[2]);
                    const V3 a2 = vscale(Rs.c2, sh[3]);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const float sx = (k & 1) ? 1.0f : -1.0f;
                        const float sy = (k & 2) ? 1.0f : -1.0f;
                        const float sz = (k & 4) ? 1.0f : -1.0f;
                        const V3 p = vadd(vadd(vadd(cs, vscale(a0, sx)), vscale(a1, sy)), vscale(a2, sz));
                        const float sep = vdot(n, p) + P.pd;
                        if (sep < P.contact_offset)
                            push_candidate(sl, nc, vsub(p, xc), sep - P.rest_offset, mu, e);
                    }
                } else if (type == MG_SHAPE_SPHERE) {
                    const float sep = vdot(n, cs) + P.pd - sh[1];
                    if (sep < P.contact_offset) {
                        const V3 p = vsub(cs, vscale(n, sh[1]));
                        push_candidate(sl, nc, vsub(p, xc), sep - P.rest_offset, mu, e);
                    }
                } else if (type == MG_SHAPE_CAPSULE) {
                    const V3 ax = vscale(qrot(qs, v3(1.0f, 0.0f, 0.0f)), sh[2]);
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const V3 c = k ? vadd(cs, ax) : vsub(cs, ax);
                        const float sep = vdot(n, c) + P.pd - sh[1];
                        if (sep < P.contact_offset) {
                            const V3 p = vsub(c, vscale(n, sh[1]));
                            push_candidate(sl, nc, vsub(p, xc), sep - P.rest_offset, mu, e);
                        }
                    }
                }
            }
        }
        // contact constants
#pragma unroll
        for (int j = 0; j < MG_MAX_CONTACTS; ++j) {
            if (j < nc) {
                const V3 rn = vcross(sl[j].r, n);
                const V3 r1 = vcross(sl[j].r, t1);
                const V3 r2 = vcross(sl[j].r, t2);
                sl[j].kn = 1.0f / (invm + vdot(rn, symmul(Iw, rn)));
                sl[j].kt1 = 1.0f / (invm + vdot(r1, symmul(Iw, r1)));
                sl[j].kt2 = 1.0f / (invm + vdot(r2, symmul(Iw, r2)));
                sl[j].ln = 0.0f; sl[j].lt1 = 0.0f; sl[j].lt2 = 0.0f;
                sl[j].vn0 = vdot(n, v) + vdot(w, rn);
            }
        }

        // 3. TGS position iterations: every normal row, then every friction row
        V3 dx = v3(0.0f, 0.0f, 0.0f), dth = v3(0.0f, 0.0f, 0.0f);
        for (int it = 0; it < P.npos; ++it) {
#pragma unroll
            for (int j = 0; j < MG_MAX_CONTACTS; ++j) {
                if (j < nc) {
                    const V3 rn = vcross(sl[j].r, n);
                    const float s = sl[j].s0 + vdot(n, dx) + vdot(dth, rn);
                    float tgt = -s * P.inv_sub;
                    if (s < 0.0f) tgt = fminf(tgt, P.max_depen);
                    contact_normal(sl[j], n, v, w, invm, Iw, tgt);
                }
            }
#pragma unroll
            for (int j = 0; j < MG_MAX_CONTACTS; ++j)
                if (j < nc) contact_friction(sl[j], t1, t2, v, w, invm, Iw);
            dx = vmad(dx, v, P.sub);
            dth = vmad(dth, w, P.sub);
        }
        // velocity iterations (bias removed)
        for (int it = 0; it < P.nvel; ++it) {
#pragma unroll
            for (int j = 0; j < MG_MAX_CONTACTS; ++j) {
                if (j < nc) {
                    const V3 rn = vcross(sl[j].r, n);
                    const float s = sl[j].s0 + vdot(n, dx) + vdot(dth, rn);
                    float tgt = s > 0.0f ? -s * P.inv_h : 0.0f;
                    if (sl[j].e > 0.0f && sl[j].vn0 < -P.bounce_thresh) tgt = fmaxf(tgt, -sl[j].e * sl[j].vn0);
                    contact_normal(sl[j], n, v, w, invm, Iw, tgt);
                }
            }
#pragma unroll
            for (int j = 0; j < MG_MAX_CONTACTS; ++j)
                if (j < nc) contact_friction(sl[j], t1, t2, v, w, invm, Iw);
        }
#pragma unroll
        for (int j = 0; j < MG_MAX_CONTACTS; ++j) {
            if (j < nc) {
                fsum = vmad(fsum, n, sl[j].ln);
                fsum = vmad(fsum, t1, sl[j].lt1);
                fsum = vmad(fsum, t2, sl[j].lt2);
            }
        }

        // 4. pose update (centre of mass moves by the integrated delta)
        const V3 xc1 = vadd(xc, dx);
        q = qintegrate(q, dth);
        x = vsub(xc1, qrot(q, com));
    }

    S[0 * nb + b] = x.x; S[1 * nb + b] = x.y; S[2 * nb + b] = x.z;
    S[3 * nb + b] = q.x; S[4 * nb + b] = q.y; S[5 * nb + b] = q.z; S[6 * nb + b] = q.w;
    S[7 * nb + b] = v.x; S[8 * nb + b] = v.y; S[9 * nb + b] = v.z;
    S[10 * nb + b] = w.x; S[11 * nb + b] = w.y; S[12 * nb + b] = w.z;
    A.cforce[0 * nb + b] = fsum.x * P.inv_dt;
    A.cforce[1 * nb + b] = fsum.y * P.inv_dt;
    A.cforce[2 * nb + b] = fsum.z * P.inv_dt;
}

}  // namespace

hipError_t mg_launch_rigid_step(const MgStep& P, const MgRigidArgs& A, hipStream_t s) {
    if (A.nf <= 0) return hipSuccess;
    const int blocks = (A.nf + 63) / 64;
    hipLaunchKernelGGL(k_rigid_step, dim3(blocks), dim3(64), 0, s, P, A);
    return hipGetLastError();
}
