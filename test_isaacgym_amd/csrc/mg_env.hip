// mg_env.hip — coupled per-env step: an env whose bodies touch each other
// (the Franka cube-pick scene of examples/franka_cube_ik_osc.py:111-285: a
// fixed-base arm, a table and a cube in one collision group).
//
// One lane = one env for the whole frame. The env holds at most one fixed-base
// articulation (reduced coordinates q, qd), up to MG_ENV_MAXF free bodies and
// MG_ENV_MAXS static bodies. Per substep:
//   1. articulation: ABA (as mg_artic.hip) gives the unconstrained qd + h qdd
//      with implicit drives; free bodies: gravity, external force, damping;
//   2. contacts (mg_collide.h) between every collidable pair — links and free
//      bodies vs the ground, vs static bodies, links vs free bodies, free vs
//      free — at most MG_ENV_MAXCT per env, in a fixed pair order;
//   3. rows n, t1, t2 per contact. A free participant's response is the usual
//      (m^-1 d, Iw (r x d)); an articulation link's is W = M_eff^-1 J^T with
//      J the row of the point Jacobian and M_eff = CRBA mass matrix + armature
//      + the implicit drive terms h kd + h^2 kp that ABA added to D, so the
//      contact sees exactly the drive stiffness the integrator applies
//      (Cholesky of M_eff once per substep, only if a link row exists);
//   4. TGS: npos position iterations (normal rows then friction rows, the
//      separation re-evaluated from the accumulated motion J . dq), nvel
//      velocity iterations; 5. integrate q += dq, clamp velocities / limits,
//      free bodies as in mg_rigid.hip.
// Static bodies and the fixed base link have infinite mass. Restated in C by
// oracle/migym_oracle_env.c (same pair order, row order and arithmetic).
#include "mg_internal.h"
#include "mg_spatial.h"
#include "mg_collide.h"

namespace {

struct Ct {
    int a, b;          // participants: -1 static, 0..MAXL-1 link, MG_ENV_FREE0 + k free body k
    V3 d[3];           // n (from b towards a), t1, t2
    V3 ra, rb;         // contact point - centre of mass (free participants)
    float s0, mu, e, vn0;
    float k[3], lam[3];
};

MG_HD void env_tangents(V3 n, V3* t1, V3* t2) {
    V3 a = v3(1.0f, 0.0f, 0.0f);
    if (!(fabsf(n.x) < 0.9f)) a = v3(0.0f, 1.0f, 0.0f);
    V3 t = vcross(n, a);
    const float inv = 1.0f / sqrtf(vdot(t, t));
    t = vscale(t, inv);
    *t1 = t;
    *t2 = vcross(n, t);
}

MG_HD CShape place_shape(const float* sh, V3 x, Q4 q) {
    CShape c;
    c.type = (int)sh[0];
    c.c = vadd(x, qrot(q, v3(sh[4], sh[5], sh[6])));
    c.R = qmat(qmul(q, q4(sh[7], sh[8], sh[9], sh[10])));
    c.h = v3(sh[1], sh[2], sh[3]);
    return c;
}

// contacts of a placed shape with the ground plane (as mg_rigid.hip: the four
// corners of the box face most opposed to n, sphere, capsule end caps)
MG_HD void ground_pair(const MgStep& P, const CShape& s, PairOut& o) {
    const V3 n = v3(P.n[0], P.n[1], P.n[2]);
    const float off = P.contact_offset;
    if (s.type == MG_SHAPE_BOX) {
        const float d0 = vdot(n, s.R.c0), d1 = vdot(n, s.R.c1), d2 = vdot(n, s.R.c2);
        const float ad0 = fabsf(d0), ad1 = fabsf(d1), ad2 = fabsf(d2);
        int ia = 0;
        float best = ad0;
        if (ad1 > best) { ia = 1; best = ad1; }
        if (ad2 > best) ia = 2;
        const V3 a0 = vscale(s.R.c0, s.h.x), a1 = vscale(s.R.c1, s.h.y), a2 = vscale(s.R.c2, s.h.z);
        const float di = ia == 0 ? d0 : (ia == 1 ? d1 : d2);
        const V3 ai = ia == 0 ? a0 : (ia == 1 ? a1 : a2);
        const V3 e1 = ia == 0 ? a1 : a0;
        const V3 e2 = ia == 2 ? a1 : a2;
        const V3 cu = vadd(s.c, vscale(ai, di > 0.0f ? -1.0f : 1.0f));
        for (int k = 0; k < 4; ++k) {
            const float sx = (k & 1) ? 1.0f : -1.0f;
            const float sy = (k & 2) ? 1.0f : -1.0f;
            const V3 p = vadd(vadd(cu, vscale(e1, sx)), vscale(e2, sy));
            const float sep = vdot(n, p) + P.pd;
            if (sep < off) pair_push(o, p, n, sep);
        }
    } else {
        const int ne = s.type == MG_SHAPE_CAPSULE ? 2 : 1;
        for (int k = 0; k < ne; ++k) {
            V3 c = s.c;
            if (s.type == MG_SHAPE_CAPSULE) c = k ? vadd(s.c, vscale(s.R.c0, s.h.y)) : vsub(s.c, vscale(s.R.c0, s.h.y));
            const float sep = vdot(n, c) + P.pd - s.h.x;
            if (sep < off) pair_push(o, vmad(c, n, -s.h.x), n, sep);
        }
    }
}

template <int MAXL, int MAXD>
__global__ void __launch_bounds__(64) k_env_step(MgStep P, MgEnvArgs A) {
    constexpr int MAXF = MG_ENV_MAXF, MAXCT = MG_ENV_MAXCT;
    constexpr int F0 = MG_ENV_FREE0;
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= A.ne) return;
    const int* ei = A.env_i + (size_t)e * MG_ENV_I_N;
    const int b0 = ei[0], d0 = ei[1], nfr = ei[2], nst = ei[7], cmask = ei[12];
    const int L = b0 >= 0 ? A.nl : 0;
    const int D = b0 >= 0 ? A.ndof : 0;
    const int nb = A.nb, nd = A.nd;
    float* S = A.state;
    const float* Ms = A.mass;
    const float h = P.h;
    const V3 gvec = v3(P.g[0], P.g[1], P.g[2]);
    const float* pr = A.dof_props;

    // ---- articulation state
    V3 x0 = v3(0.0f, 0.0f, 0.0f), gb = v3(0.0f, 0.0f, 0.0f);
    Q4 q0 = q4(0.0f, 0.0f, 0.0f, 1.0f);
    float q[MAXD], qd[MAXD], qdd[MAXD], dq[MAXD], mdiag[MAXD], tau0d[MAXD], impd[MAXD];
    if (L > 0) {
        x0 = v3(S[0 * nb + b0], S[1 * nb + b0], S[2 * nb + b0]);
        q0 = qnormalize(q4(S[3 * nb + b0], S[4 * nb + b0], S[5 * nb + b0], S[6 * nb + b0]));
        const float grav_on = A.tbf[A.body_tmpl[b0] * MG_TBODY_F_N + 4];
        gb = qrot_inv(q0, grav_on != 0.0f ? gvec : v3(0.0f, 0.0f, 0.0f));
    }
    for (int d = 0; d < D; ++d) {
        q[d] = A.dof_pos[d0 + d];
        qd[d] = A.dof_vel[d0 + d];
    }
    V3 lsum[MAXL];
    for (int l = 0; l < L; ++l) lsum[l] = v3(0.0f, 0.0f, 0.0f);

    // ---- free bodies
    V3 fx[MAXF], fv[MAXF], fw[MAXF], fcom[MAXF], finvI[MAXF], fsum[MAXF], fext[MAXF], text[MAXF];
    Q4 fq[MAXF], fiq[MAXF];
    float finvm[MAXF], lkeep[MAXF], akeep[MAXF], mlv2[MAXF], mav2[MAXF], gon[MAXF];
    for (int k = 0; k < nfr; ++k) {
        const int b = ei[3 + k];
        fx[k] = v3(S[0 * nb + b], S[1 * nb + b], S[2 * nb + b]);
        fq[k] = qnormalize(q4(S[3 * nb + b], S[4 * nb + b], S[5 * nb + b], S[6 * nb + b]));
        fv[k] = v3(S[7 * nb + b], S[8 * nb + b], S[9 * nb + b]);
        fw[k] = v3(S[10 * nb + b], S[11 * nb + b], S[12 * nb + b]);
        finvm[k] = Ms[0 * nb + b];
        finvI[k] = v3(Ms[1 * nb + b], Ms[2 * nb + b], Ms[3 * nb + b]);
        fiq[k] = q4(Ms[4 * nb + b], Ms[5 * nb + b], Ms[6 * nb + b], Ms[7 * nb + b]);
        fcom[k] = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
        const int tb = A.body_tmpl[b];
        const float* tf = A.tbf + tb * MG_TBODY_F_N;
        lkeep[k] = 1.0f - fminf(tf[0] * h, 1.0f);
        akeep[k] = 1.0f - fminf(tf[1] * h, 1.0f);
        mlv2[k] = tf[2] * tf[2];
        mav2[k] = tf[3] * tf[3];
        gon[k] = tf[4];
        fext[k] = v3(0.0f, 0.0f, 0.0f);
        text[k] = v3(0.0f, 0.0f, 0.0f);
        if (A.ext) {
            fext[k] = v3(A.ext[0 * nb + b], A.ext[1 * nb + b], A.ext[2 * nb + b]);
            text[k] = v3(A.ext[3 * nb + b], A.ext[4 * nb + b], A.ext[5 * nb + b]);
        }
        fsum[k] = v3(0.0f, 0.0f, 0.0f);
    }

    // per-substep scratch
    M3 E[MAXL];
    V3 r[MAXL];
    SV Sj[MAXL], vl[MAXL], cl[MAXL], pA[MAXL], U[MAXL], al[MAXL];
    SI IA[MAXL];
    float Dl[MAXL], ul[MAXL];
    Q4 ql[MAXL];
    V3 xl[MAXL], zl[MAXL];
    S3 fIw[MAXF];
    V3 fxc[MAXF], fdx[MAXF], fdth[MAXF];
    Ct ct[MAXCT];
    float Jr[MAXCT * 3][MAXD], Wr[MAXCT * 3][MAXD];
    float Mf[MAXD][MAXD], invd[MAXD];

    for (int st = 0; st < P.substeps; ++st) {
        // ================= 1a. articulation: ABA with implicit drives (effort
        // limit as in mg_artic.hip: one exact re-solve when a drive saturates)
        if (L > 0) {
          unsigned xmask = 0u, xpos = 0u;
          for (int att = 0; att < 2; ++att) {
            for (int l = 0; l < L; ++l) {
                const float* lf = A.link_f + l * MG_LINK_F_N;
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], jt = li[1], dof = li[2];
                const int b = b0 + l;
                if (p < 0) {
                    E[l] = m3cols(v3(1.0f, 0.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), v3(0.0f, 0.0f, 1.0f));
                    r[l] = v3(0.0f, 0.0f, 0.0f);
                    Sj[l] = svzero();
                    vl[l] = svzero();
                    cl[l] = svzero();
                    ql[l] = q0;
                    xl[l] = x0;
                    zl[l] = v3(0.0f, 0.0f, 0.0f);
                } else {
                    const V3 po = v3(lf[0], lf[1], lf[2]);
                    const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
                    const V3 ax = v3(lf[7], lf[8], lf[9]);
                    const float qj = dof >= 0 ? q[dof] : 0.0f;
                    const float qdj = dof >= 0 ? qd[dof] : 0.0f;
                    Q4 qrel = qo;
                    V3 rr = po;
                    SV s = svzero();
                    if (jt == MG_JOINT_REVOLUTE) {
                        qrel = qmul(qo, q_axis_angle(ax, qj));
                        s = sv(ax, v3(0.0f, 0.0f, 0.0f));
                    } else if (jt == MG_JOINT_PRISMATIC) {
                        rr = vadd(po, qrot(qo, vscale(ax, qj)));
                        s = sv(v3(0.0f, 0.0f, 0.0f), ax);
                    }
                    E[l] = m3t(qmat(qrel));
                    r[l] = rr;
                    Sj[l] = s;
                    const SV vJ = svscale(s, qdj);
                    vl[l] = svadd(x_motion(E[l], rr, vl[p]), vJ);
                    cl[l] = crm(vl[l], vJ);
                    ql[l] = qnormalize(qmul(ql[p], qrel));
                    xl[l] = vadd(xl[p], qrot(ql[p], rr));
                    zl[l] = qrot(ql[l], ax);
                }
                const float m = Ms[11 * nb + b];
                const V3 com = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
                const Q4 iq = q4(Ms[4 * nb + b], Ms[5 * nb + b], Ms[6 * nb + b], Ms[7 * nb + b]);
                const V3 invI = v3(Ms[1 * nb + b], Ms[2 * nb + b], Ms[3 * nb + b]);
                const V3 Id = v3(invI.x > 0.0f ? 1.0f / invI.x : 0.0f, invI.y > 0.0f ? 1.0f / invI.y : 0.0f,
                                 invI.z > 0.0f ? 1.0f / invI.z : 0.0f);
                const M3 Rq = qmat(iq);
                const M3 Ic = m3mul(m3mul(Rq, m3cols(v3(Id.x, 0.0f, 0.0f), v3(0.0f, Id.y, 0.0f), v3(0.0f, 0.0f, Id.z))),
                                    m3t(Rq));
                IA[l] = si_rigid(m, com, Ic);
                pA[l] = crf(vl[l], si_mul(IA[l], vl[l]));
            }
            for (int l = L - 1; l >= 1; --l) {
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], dof = li[2];
                SI Ia = IA[l];
                SV pa;
                if (dof >= 0) {
                    const int gd = d0 + dof;
                    const int mode = (int)pr[0 * nd + gd];
                    const float kp = pr[1 * nd + gd], kd = pr[2 * nd + gd], eff = pr[3 * nd + gd];
                    const float arm = pr[8 * nd + gd];
                    float tau = 0.0f, imp = 0.0f;
                    if (mode == MG_DOF_MODE_POS) {
                        tau = kp * (A.dof_tpos[gd] - q[dof] - h * qd[dof]) + kd * (A.dof_tvel[gd] - qd[dof]);
                        imp = h * kd + h * h * kp;
                    } else if (mode == MG_DOF_MODE_VEL) {
                        tau = kd * (A.dof_tvel[gd] - qd[dof]);
                        imp = h * kd;
                    } else if (mode == MG_DOF_MODE_EFFORT) {
                        tau = A.dof_force[gd];
                    }
                    if (eff > 0.0f) {
                        if ((xmask >> dof) & 1u) {
                            tau = ((xpos >> dof) & 1u) ? eff : -eff;
                            imp = 0.0f;
                        } else if (imp == 0.0f) {
                            tau = fminf(fmaxf(tau, -eff), eff);
                        }
                    }
                    tau0d[dof] = tau;
                    impd[dof] = imp;
                    mdiag[dof] = arm + imp;
                    U[l] = si_mul(Ia, Sj[l]);
                    Dl[l] = svdot(Sj[l], U[l]) + arm + imp;
                    ul[l] = tau - svdot(Sj[l], pA[l]);
                    const float invD = 1.0f / Dl[l];
                    Ia.A = m3sub(Ia.A, m3outer(U[l].w, U[l].w, invD));
                    Ia.B = m3sub(Ia.B, m3outer(U[l].w, U[l].v, invD));
                    Ia.C = m3sub(Ia.C, m3outer(U[l].v, U[l].v, invD));
                    pa = svadd(svadd(pA[l], si_mul(Ia, cl[l])), svscale(U[l], ul[l] * invD));
                } else {
                    pa = svadd(pA[l], si_mul(Ia, cl[l]));
                }
                if (p > 0) {
                    IA[p] = si_add(IA[p], x_inertia_t(E[l], r[l], Ia));
                    pA[p] = svadd(pA[p], x_force_t(E[l], r[l], pa));
                }
            }
            al[0] = sv(v3(0.0f, 0.0f, 0.0f), vscale(gb, -1.0f));
            for (int l = 1; l < L; ++l) {
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], dof = li[2];
                SV ap = svadd(x_motion(E[l], r[l], al[p]), cl[l]);
                if (dof >= 0) {
                    const float acc = (ul[l] - svdot(U[l], ap)) / Dl[l];
                    qdd[dof] = acc;
                    ap = svadd(ap, svscale(Sj[l], acc));
                }
                al[l] = ap;
            }
            unsigned nm = xmask;
            for (int d = 0; d < D; ++d) {
                const float eff = pr[3 * nd + d0 + d];
                if (eff > 0.0f && impd[d] != 0.0f) {
                    const float act = tau0d[d] - impd[d] * qdd[d];
                    if (act > eff) { nm |= 1u << d; xpos |= 1u << d; }
                    else if (act < -eff) nm |= 1u << d;
                }
            }
            if (nm == xmask) break;
            xmask = nm;
          }
            // unconstrained joint velocity, clamped to the joint speed limit
            for (int d = 0; d < D; ++d) {
                const float maxv = pr[4 * nd + d0 + d];
                float w = qd[d] + h * qdd[d];
                if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
                qd[d] = w;
                dq[d] = 0.0f;
            }
        }

        // ================= 1b. free bodies: unconstrained velocity
        for (int k = 0; k < nfr; ++k) {
            fIw[k] = sym_rdrt(qmat(qmul(fq[k], fiq[k])), finvI[k]);
            fxc[k] = vadd(fx[k], qrot(fq[k], fcom[k]));
            V3 v = fv[k], w = fw[k];
            if (gon[k] != 0.0f) v = vmad(v, gvec, h);
            v = vmad(v, fext[k], finvm[k] * h);
            w = vmad(w, symmul(fIw[k], text[k]), h);
            v = vscale(v, lkeep[k]);
            w = vscale(w, akeep[k]);
            const float v2 = vdot(v, v);
            if (v2 > mlv2[k]) v = vscale(v, sqrtf(mlv2[k] / v2));
            const float w2 = vdot(w, w);
            if (w2 > mav2[k]) w = vscale(w, sqrtf(mav2[k] / w2));
            fv[k] = v;
            fw[k] = w;
            fdx[k] = v3(0.0f, 0.0f, 0.0f);
            fdth[k] = v3(0.0f, 0.0f, 0.0f);
        }

        // ================= 2. contacts
        int nct = 0;
        auto add = [&](int a, int b, const PairOut& o, float mu, float rest) {
            for (int j = 0; j < o.n; ++j) {
                if (nct >= MAXCT) return;
                Ct& c = ct[nct];
                c.a = a;
                c.b = b;
                c.d[0] = o.nrm[j];
                env_tangents(o.nrm[j], &c.d[1], &c.d[2]);
                c.ra = a >= F0 ? vsub(o.p[j], fxc[a - F0]) : o.p[j];
                c.rb = b >= F0 ? vsub(o.p[j], fxc[b - F0]) : v3(0.0f, 0.0f, 0.0f);
                c.s0 = o.sep[j] - P.rest_offset;
                c.mu = mu;
                c.e = rest;
                nct = nct + 1;
            }
        };
        const float off = P.contact_offset;
        // free bodies: ground, static bodies, later free bodies, the fixed base link
        for (int k = 0; k < nfr; ++k) {
            const int bk = ei[3 + k];
            const int tk = A.body_tmpl[bk];
            const int s0k = A.tbi[tk * MG_TBODY_I_N + 0], nsk = A.tbi[tk * MG_TBODY_I_N + 1];
            for (int sa = s0k; sa < s0k + nsk; ++sa) {
                const float* sha = A.shapes + sa * MG_SHAPE_STRIDE;
                const CShape ca = place_shape(sha, fx[k], fq[k]);
                if (P.has_ground) {
                    PairOut o;
                    o.n = 0;
                    ground_pair(P, ca, o);
                    add(F0 + k, -1, o, 0.5f * (sha[11] + P.mu_ground), 0.5f * (sha[12] + P.e_ground));
                }
                for (int s = 0; s < nst; ++s) {
                    if (!((cmask >> (14 + k * 4 + s)) & 1)) continue;
                    const int bs = ei[8 + s];
                    const int ts = A.body_tmpl[bs];
                    const V3 xs = v3(S[0 * nb + bs], S[1 * nb + bs], S[2 * nb + bs]);
                    const Q4 qs = qnormalize(q4(S[3 * nb + bs], S[4 * nb + bs], S[5 * nb + bs], S[6 * nb + bs]));
                    const int s0s = A.tbi[ts * MG_TBODY_I_N + 0], nss = A.tbi[ts * MG_TBODY_I_N + 1];
                    for (int sb = s0s; sb < s0s + nss; ++sb) {
                        const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                        PairOut o;
                        o.n = 0;
                        collide(ca, place_shape(shb, xs, qs), off, o);
                        add(F0 + k, -1, o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                for (int j = k + 1; j < nfr; ++j) {
                    const int bit = k == 0 ? j - 1 : (k == 1 ? j + 1 : 5);
                    if (!((cmask >> (8 + bit)) & 1)) continue;
                    const int bj = ei[3 + j];
                    const int tj = A.body_tmpl[bj];
                    const int s0j = A.tbi[tj * MG_TBODY_I_N + 0], nsj = A.tbi[tj * MG_TBODY_I_N + 1];
                    for (int sb = s0j; sb < s0j + nsj; ++sb) {
                        const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                        PairOut o;
                        o.n = 0;
                        collide(ca, place_shape(shb, fx[j], fq[j]), off, o);
                        add(F0 + k, F0 + j, o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                if (L > 0 && ((cmask >> k) & 1)) {
                    const int t0 = A.body_tmpl[b0];
                    const int s00 = A.tbi[t0 * MG_TBODY_I_N + 0], ns0 = A.tbi[t0 * MG_TBODY_I_N + 1];
                    for (int sb = s00; sb < s00 + ns0; ++sb) {
                        const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                        PairOut o;
                        o.n = 0;
                        collide(ca, place_shape(shb, xl[0], ql[0]), off, o);
                        add(F0 + k, -1, o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
            }
        }
        // moving links: ground, static bodies, free bodies
        int first_link_row = nct;
        for (int l = 1; l < L; ++l) {
            const int bl = b0 + l;
            const int tl = A.body_tmpl[bl];
            const int s0l = A.tbi[tl * MG_TBODY_I_N + 0], nsl = A.tbi[tl * MG_TBODY_I_N + 1];
            for (int sa = s0l; sa < s0l + nsl; ++sa) {
                const float* sha = A.shapes + sa * MG_SHAPE_STRIDE;
                const CShape ca = place_shape(sha, xl[l], ql[l]);
                if (P.has_ground) {
                    PairOut o;
                    o.n = 0;
                    ground_pair(P, ca, o);
                    add(l, -1, o, 0.5f * (sha[11] + P.mu_ground), 0.5f * (sha[12] + P.e_ground));
                }
                for (int s = 0; s < nst; ++s) {
                    if (!((cmask >> (4 + s)) & 1)) continue;
                    const int bs = ei[8 + s];
                    const int ts = A.body_tmpl[bs];
                    const V3 xs = v3(S[0 * nb + bs], S[1 * nb + bs], S[2 * nb + bs]);
                    const Q4 qs = qnormalize(q4(S[3 * nb + bs], S[4 * nb + bs], S[5 * nb + bs], S[6 * nb + bs]));
                    const int s0s = A.tbi[ts * MG_TBODY_I_N + 0], nss = A.tbi[ts * MG_TBODY_I_N + 1];
                    for (int sb = s0s; sb < s0s + nss; ++sb) {
                        const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                        PairOut o;
                        o.n = 0;
                        collide(ca, place_shape(shb, xs, qs), off, o);
                        add(l, -1, o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                for (int k = 0; k < nfr; ++k) {
                    if (!((cmask >> k) & 1)) continue;
                    const int bk = ei[3 + k];
                    const int tk = A.body_tmpl[bk];
                    const int s0k = A.tbi[tk * MG_TBODY_I_N + 0], nsk = A.tbi[tk * MG_TBODY_I_N + 1];
                    for (int sb = s0k; sb < s0k + nsk; ++sb) {
                        const float* shb = A.shapes + sb * MG_SHAPE_STRIDE;
                        PairOut o;
                        o.n = 0;
                        collide(ca, place_shape(shb, fx[k], fq[k]), off, o);
                        add(l, F0 + k, o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
            }
        }

        // ================= 3. rows: Jacobians, responses, effective masses
        const bool link_rows = nct > first_link_row;
        if (link_rows) {
            // joint-space inertia (CRBA, link coordinates) + armature + implicit drive terms
            for (int l = 0; l < L; ++l) {
                const int b = b0 + l;
                const float m = Ms[11 * nb + b];
                const V3 com = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
                const Q4 iq = q4(Ms[4 * nb + b], Ms[5 * nb + b], Ms[6 * nb + b], Ms[7 * nb + b]);
                const V3 invI = v3(Ms[1 * nb + b], Ms[2 * nb + b], Ms[3 * nb + b]);
                const V3 Id = v3(invI.x > 0.0f ? 1.0f / invI.x : 0.0f, invI.y > 0.0f ? 1.0f / invI.y : 0.0f,
                                 invI.z > 0.0f ? 1.0f / invI.z : 0.0f);
                const M3 Rq = qmat(iq);
                IA[l] = si_rigid(m, com, m3mul(m3mul(Rq, m3cols(v3(Id.x, 0.0f, 0.0f), v3(0.0f, Id.y, 0.0f),
                                                               v3(0.0f, 0.0f, Id.z))), m3t(Rq)));
            }
            for (int i = 0; i < D; ++i)
                for (int j = 0; j < D; ++j) Mf[i][j] = 0.0f;
            for (int l = L - 1; l >= 1; --l) {
                const int p = A.link_i[l * MG_LINK_I_N + 0];
                if (p > 0) IA[p] = si_add(IA[p], x_inertia_t(E[l], r[l], IA[l]));
            }
            for (int l = 1; l < L; ++l) {
                const int di = A.link_i[l * MG_LINK_I_N + 2];
                if (di < 0) continue;
                SV Fv = si_mul(IA[l], Sj[l]);
                Mf[di][di] = svdot(Sj[l], Fv) + mdiag[di];
                int j = l;
                while (A.link_i[j * MG_LINK_I_N + 0] > 0) {
                    Fv = x_force_t(E[j], r[j], Fv);
                    j = A.link_i[j * MG_LINK_I_N + 0];
                    const int dj = A.link_i[j * MG_LINK_I_N + 2];
                    if (dj >= 0) {
                        const float hv = svdot(Fv, Sj[j]);
                        Mf[di][dj] = hv;
                        Mf[dj][di] = hv;
                    }
                }
            }
            // Cholesky, lower triangle in place
            for (int j = 0; j < D; ++j) {
                float s = Mf[j][j];
                for (int k = 0; k < j; ++k) s = s - Mf[j][k] * Mf[j][k];
                const float dj = sqrtf(s);
                invd[j] = 1.0f / dj;
                Mf[j][j] = dj;
                for (int i = j + 1; i < D; ++i) {
                    float t = Mf[i][j];
                    for (int k = 0; k < j; ++k) t = t - Mf[i][k] * Mf[j][k];
                    Mf[i][j] = t * invd[j];
                }
            }
        }
        for (int c = 0; c < nct; ++c) {
            Ct& C = ct[c];
            const V3 pw = C.a < F0 ? C.ra : vadd(C.ra, fxc[C.a - F0]);   // link rows keep the world point in ra
            for (int rw = 0; rw < 3; ++rw) {
                const V3 dir = C.d[rw];
                float wa = 0.0f, wb = 0.0f;
                if (C.a >= F0) {
                    const int k = C.a - F0;
                    const V3 rd = vcross(C.ra, dir);
                    wa = finvm[k] + vdot(rd, symmul(fIw[k], rd));
                } else {
                    float* J = Jr[c * 3 + rw];
                    float* W = Wr[c * 3 + rw];
                    for (int d = 0; d < D; ++d) J[d] = 0.0f;
                    int j = C.a;
                    while (j > 0) {
                        const int* lj = A.link_i + j * MG_LINK_I_N;
                        const int dof = lj[2];
                        if (dof >= 0) {
                            if (lj[1] == MG_JOINT_REVOLUTE) J[dof] = vdot(vcross(zl[j], vsub(pw, xl[j])), dir);
                            else J[dof] = vdot(zl[j], dir);
                        }
                        j = lj[0];
                    }
                    // W = M_eff^-1 J: forward then backward substitution
                    for (int i = 0; i < D; ++i) {
                        float t = J[i];
                        for (int k = 0; k < i; ++k) t = t - Mf[i][k] * W[k];
                        W[i] = t * invd[i];
                    }
                    for (int i = D - 1; i >= 0; --i) {
                        float t = W[i];
                        for (int k = i + 1; k < D; ++k) t = t - Mf[k][i] * W[k];
                        W[i] = t * invd[i];
                    }
                    for (int d = 0; d < D; ++d) wa = wa + J[d] * W[d];
                }
                if (C.b >= F0) {
                    const int k = C.b - F0;
                    const V3 rd = vcross(C.rb, dir);
                    wb = finvm[k] + vdot(rd, symmul(fIw[k], rd));
                }
                C.k[rw] = 1.0f / (wa + wb);
                C.lam[rw] = 0.0f;
            }
        }

        // relative velocity / motion of a row, and the impulse application
        auto rel = [&](const Ct& C, int c, int rw, bool motion) -> float {
            const V3 dir = C.d[rw];
            float va = 0.0f, vb = 0.0f;
            if (C.a >= F0) {
                const int k = C.a - F0;
                va = motion ? vdot(dir, fdx[k]) + vdot(fdth[k], vcross(C.ra, dir))
                            : vdot(dir, fv[k]) + vdot(fw[k], vcross(C.ra, dir));
            } else {
                const float* J = Jr[c * 3 + rw];
                for (int d = 0; d < D; ++d) va = va + J[d] * (motion ? dq[d] : qd[d]);
            }
            if (C.b >= F0) {
                const int k = C.b - F0;
                vb = motion ? vdot(dir, fdx[k]) + vdot(fdth[k], vcross(C.rb, dir))
                            : vdot(dir, fv[k]) + vdot(fw[k], vcross(C.rb, dir));
            }
            return va - vb;
        };
        auto apply = [&](const Ct& C, int c, int rw, float dl) {
            const V3 dir = C.d[rw];
            if (C.a >= F0) {
                const int k = C.a - F0;
                fv[k] = vmad(fv[k], dir, dl * finvm[k]);
                fw[k] = vmad(fw[k], symmul(fIw[k], vcross(C.ra, dir)), dl);
            } else {
                const float* W = Wr[c * 3 + rw];
                for (int d = 0; d < D; ++d) qd[d] = qd[d] + W[d] * dl;
            }
            if (C.b >= F0) {
                const int k = C.b - F0;
                fv[k] = vmad(fv[k], dir, -(dl * finvm[k]));
                fw[k] = vmad(fw[k], symmul(fIw[k], vcross(C.rb, dir)), -dl);
            }
        };
        auto normal_row = [&](Ct& C, int c, float tgt) {
            float dl = C.k[0] * (tgt - rel(C, c, 0, false));
            const float nl = fmaxf(C.lam[0] + dl, 0.0f);
            dl = nl - C.lam[0];
            C.lam[0] = nl;
            apply(C, c, 0, dl);
        };
        auto friction_rows = [&](Ct& C, int c) {
            const float lim = C.mu * C.lam[0];
            for (int rw = 1; rw < 3; ++rw) {
                const float nl = fminf(fmaxf(C.lam[rw] - C.k[rw] * rel(C, c, rw, false), -lim), lim);
                const float dl = nl - C.lam[rw];
                C.lam[rw] = nl;
                apply(C, c, rw, dl);
            }
        };
        for (int c = 0; c < nct; ++c) ct[c].vn0 = rel(ct[c], c, 0, false);

        // ================= 4. TGS
        for (int it = 0; it < P.npos; ++it) {
            for (int c = 0; c < nct; ++c) {
                const float s = ct[c].s0 + rel(ct[c], c, 0, true);
                float tgt = -s * P.inv_sub;
                if (s < 0.0f) tgt = fminf(tgt, P.max_depen);
                normal_row(ct[c], c, tgt);
            }
            for (int c = 0; c < nct; ++c) friction_rows(ct[c], c);
            for (int d = 0; d < D; ++d) dq[d] = dq[d] + qd[d] * P.sub;
            for (int k = 0; k < nfr; ++k) {
                fdx[k] = vmad(fdx[k], fv[k], P.sub);
                fdth[k] = vmad(fdth[k], fw[k], P.sub);
            }
        }
        for (int it = 0; it < P.nvel; ++it) {
            for (int c = 0; c < nct; ++c) {
                const float s = ct[c].s0 + rel(ct[c], c, 0, true);
                float tgt = s > 0.0f ? -s * P.inv_h : 0.0f;
                if (ct[c].e > 0.0f && ct[c].vn0 < -P.bounce_thresh) tgt = fmaxf(tgt, -ct[c].e * ct[c].vn0);
                normal_row(ct[c], c, tgt);
            }
            for (int c = 0; c < nct; ++c) friction_rows(ct[c], c);
        }
        // contact impulses -> forces on the participants
        for (int c = 0; c < nct; ++c) {
            const Ct& C = ct[c];
            V3 imp = vscale(C.d[0], C.lam[0]);
            imp = vmad(imp, C.d[1], C.lam[1]);
            imp = vmad(imp, C.d[2], C.lam[2]);
            if (C.a >= F0) fsum[C.a - F0] = vadd(fsum[C.a - F0], imp);
            else if (C.a >= 0) lsum[C.a] = vadd(lsum[C.a], imp);
            if (C.b >= F0) fsum[C.b - F0] = vsub(fsum[C.b - F0], imp);
        }

        // ================= 5. integrate
        for (int d = 0; d < D; ++d) {
            const int gd = d0 + d;
            const float maxv = pr[4 * nd + gd];
            float w = qd[d];
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            float x = q[d] + dq[d];
            if (pr[7 * nd + gd] != 0.0f) {
                const float lo = pr[5 * nd + gd], hi = pr[6 * nd + gd];
                if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
            }
            q[d] = x;
            qd[d] = w;
        }
        for (int k = 0; k < nfr; ++k) {
            const V3 xc1 = vadd(fxc[k], fdx[k]);
            fq[k] = qintegrate(fq[k], fdth[k]);
            fx[k] = vsub(xc1, qrot(fq[k], fcom[k]));
        }
    }

    // ---- outputs
    for (int k = 0; k < nfr; ++k) {
        const int b = ei[3 + k];
        S[0 * nb + b] = fx[k].x; S[1 * nb + b] = fx[k].y; S[2 * nb + b] = fx[k].z;
        S[3 * nb + b] = fq[k].x; S[4 * nb + b] = fq[k].y; S[5 * nb + b] = fq[k].z; S[6 * nb + b] = fq[k].w;
        S[7 * nb + b] = fv[k].x; S[8 * nb + b] = fv[k].y; S[9 * nb + b] = fv[k].z;
        S[10 * nb + b] = fw[k].x; S[11 * nb + b] = fw[k].y; S[12 * nb + b] = fw[k].z;
        A.cforce[0 * nb + b] = fsum[k].x * P.inv_dt;
        A.cforce[1 * nb + b] = fsum[k].y * P.inv_dt;
        A.cforce[2 * nb + b] = fsum[k].z * P.inv_dt;
    }
    if (L == 0) return;
    for (int d = 0; d < D; ++d) {
        A.dof_pos[d0 + d] = q[d];
        A.dof_vel[d0 + d] = qd[d];
    }
    for (int l = 0; l < L; ++l) {
        const float* lf = A.link_f + l * MG_LINK_F_N;
        const int* li = A.link_i + l * MG_LINK_I_N;
        const int p = li[0], jt = li[1], dof = li[2];
        const int b = b0 + l;
        if (p < 0) {
            ql[l] = q0; xl[l] = x0;
            vl[l] = svzero();
        } else {
            const V3 po = v3(lf[0], lf[1], lf[2]);
            const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
            const V3 ax = v3(lf[7], lf[8], lf[9]);
            const float qj = dof >= 0 ? q[dof] : 0.0f;
            const float qdj = dof >= 0 ? qd[dof] : 0.0f;
            Q4 qrel = qo;
            V3 rr = po;
            SV s = svzero();
            if (jt == MG_JOINT_REVOLUTE) {
                qrel = qmul(qo, q_axis_angle(ax, qj));
                s = sv(ax, v3(0.0f, 0.0f, 0.0f));
            } else if (jt == MG_JOINT_PRISMATIC) {
                rr = vadd(po, qrot(qo, vscale(ax, qj)));
                s = sv(v3(0.0f, 0.0f, 0.0f), ax);
            }
            ql[l] = qnormalize(qmul(ql[p], qrel));
            xl[l] = vadd(xl[p], qrot(ql[p], rr));
            vl[l] = svadd(x_motion(m3t(qmat(qrel)), rr, vl[p]), svscale(s, qdj));
        }
        const V3 com = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
        const V3 ww = qrot(ql[l], vl[l].w);
        const V3 vw = qrot(ql[l], vadd(vl[l].v, vcross(vl[l].w, com)));
        S[0 * nb + b] = xl[l].x; S[1 * nb + b] = xl[l].y; S[2 * nb + b] = xl[l].z;
        S[3 * nb + b] = ql[l].x; S[4 * nb + b] = ql[l].y; S[5 * nb + b] = ql[l].z; S[6 * nb + b] = ql[l].w;
        S[7 * nb + b] = vw.x; S[8 * nb + b] = vw.y; S[9 * nb + b] = vw.z;
        S[10 * nb + b] = ww.x; S[11 * nb + b] = ww.y; S[12 * nb + b] = ww.z;
        A.cforce[0 * nb + b] = lsum[l].x * P.inv_dt;
        A.cforce[1 * nb + b] = lsum[l].y * P.inv_dt;
        A.cforce[2 * nb + b] = lsum[l].z * P.inv_dt;
    }
}

}  // namespace

hipError_t mg_launch_env_step(const MgStep& P, const MgEnvArgs& A, hipStream_t s) {
    if (A.ne <= 0) return hipSuccess;
    const int blocks = (A.ne + 63) / 64;
    if (A.nl <= 4 && A.ndof <= 4)
        hipLaunchKernelGGL((k_env_step<4, 4>), dim3(blocks), dim3(64), 0, s, P, A);
    else if (A.nl <= MG_MAX_LINKS && A.ndof <= 12)
        hipLaunchKernelGGL((k_env_step<MG_MAX_LINKS, 12>), dim3(blocks), dim3(64), 0, s, P, A);
    else if (A.nl <= MG_MAX_LINKS && A.ndof <= MG_MAX_DOFS)
        hipLaunchKernelGGL((k_env_step<MG_MAX_LINKS, MG_MAX_DOFS>), dim3(blocks), dim3(64), 0, s, P, A);
    else
        return hipErrorNotSupported;
    return hipGetLastError();
}
