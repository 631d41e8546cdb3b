// mg_artic.hip — articulation step: Featherstone articulated-body algorithm
// (RBDA Table 7.1) with implicit PD/velocity drives, for fixed-base
// articulations (the 3-DOF camera gimbal `dof_test_camera.urdf` of
// test12_add_joint.py.py:69-98 and the Franka of examples/franka_cube_ik_osc.py).
//
// One lane = one articulation instance for the whole frame. Per substep:
//   pass 1 (outward): joint transforms X_l from q, link velocities v_l, bias c_l,
//           rigid inertia I_l and bias force pA_l = v_l x* (I_l v_l);
//   pass 2 (inward):  U = IA S, D = S^T U + armature + h kd + h^2 kp (implicit
//           drive), u = tau0 - S^T pA, articulated inertia/bias to the parent;
//   pass 3 (outward): a_0 = -g (base frame), qdd = (u - U^T a') / D;
//   semi-implicit Euler on (q, qd), joint-velocity clamp, joint-limit clamp.
// Drive law: POS tau0 = kp (q* - q - h qd) + kd (qd* - qd),
// VEL tau0 = kd (qd* - qd), EFFORT tau0 = u. Effort limit: EFFORT forces are
// clamped; a PD / velocity drive whose implicit force tau0 - (h kd + h^2 kp) qdd
// exceeds the limit is re-solved (once, exactly) as a constant force at the limit.
// Per-template link constants (parent, joint frame, axis) are read with
// wave-uniform addresses, so they come through the scalar cache once per wave.
// Restated in C by oracle/migym_oracle.c:oracle_artic_step.
#include "mg_internal.h"
#include "mg_spatial.h"
#include "mg_world.h"

namespace {

template <int MAXL>
__global__ void __launch_bounds__(64) k_artic_step(MgStep P, MgArticArgs A) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= A.na) return;
    const int b0 = A.artic_i[i * MG_ARTIC_I_N + 0];
    const int d0 = A.artic_i[i * MG_ARTIC_I_N + 1];
    const int nb = A.nb, nd = A.nd;
    const int L = A.nl, D = A.ndof;
    float* S = A.state;
    const float h = P.h;

    // base pose (fixed base: the root link never moves; set_actor_root_state teleports it)
    const V3 x0 = v3(S[0 * nb + b0], S[1 * nb + b0], S[2 * nb + b0]);
    const Q4 q0 = qnormalize(q4(S[3 * nb + b0], S[4 * nb + b0], S[5 * nb + b0], S[6 * nb + b0]));
    const float grav_on = A.tbf[A.body_tmpl[b0] * MG_TBODY_F_N + 4];
    const V3 gw = grav_on != 0.0f ? v3(P.g[0], P.g[1], P.g[2]) : v3(0.0f, 0.0f, 0.0f);
    const V3 gb = qrot_inv(q0, gw);

    float q[MAXL], qd[MAXL], qdd[MAXL];
    for (int d = 0; d < D; ++d) {
        q[d] = A.dof_pos[d0 + d];
        qd[d] = A.dof_vel[d0 + d];
        qdd[d] = 0.0f;
    }

    M3 E[MAXL];
    V3 r[MAXL];
    SV Sj[MAXL], v[MAXL], c[MAXL], pA[MAXL], U[MAXL], a[MAXL];
    SI IA[MAXL];
    float Dl[MAXL], ul[MAXL];

    for (int st = 0; st < P.substeps; ++st) {
      // Effort limit: a drive whose implicit force tau0 - imp qdd exceeds the
      // limit is re-solved as a constant force at the limit (xmask / xpos), one
      // exact ABA re-solve when any joint saturates.
      unsigned xmask = 0u, xpos = 0u;
      float tau0d[MAXL], impd[MAXL];
      for (int att = 0; att < 2; ++att) {
        // ---- pass 1: kinematics, velocities, bias forces
        for (int l = 0; l < L; ++l) {
            const float* lf = A.link_f + l * MG_LINK_F_N;
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], jt = li[1], dof = li[2];
            const int b = b0 + l;
            if (p < 0) {
                E[l] = m3cols(v3(1.0f, 0.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), v3(0.0f, 0.0f, 1.0f));
                r[l] = v3(0.0f, 0.0f, 0.0f);
                Sj[l] = svzero();
                v[l] = svzero();
                c[l] = svzero();
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
                v[l] = svadd(x_motion(E[l], rr, v[p]), vJ);
                c[l] = crm(v[l], vJ);
            }
            const float* M = A.mass;
            const float m = M[11 * nb + b];
            const V3 com = v3(M[8 * nb + b], M[9 * nb + b], M[10 * nb + b]);
            const Q4 iq = q4(M[4 * nb + b], M[5 * nb + b], M[6 * nb + b], M[7 * nb + b]);
            const V3 invI = v3(M[1 * nb + b], M[2 * nb + b], M[3 * nb + b]);
            const V3 Id = v3(invI.x > 0.0f ? 1.0f / invI.x : 0.0f, invI.y > 0.0f ? 1.0f / invI.y : 0.0f,
                             invI.z > 0.0f ? 1.0f / invI.z : 0.0f);
            const M3 Rq = qmat(iq);
            const M3 Ic = m3mul(m3mul(Rq, m3cols(v3(Id.x, 0.0f, 0.0f), v3(0.0f, Id.y, 0.0f), v3(0.0f, 0.0f, Id.z))), m3t(Rq));
            IA[l] = si_rigid(m, com, Ic);
            pA[l] = crf(v[l], si_mul(IA[l], v[l]));
        }
        // ---- pass 2: articulated inertias, inward
        for (int l = L - 1; l >= 1; --l) {
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], dof = li[2];
            SI Ia = IA[l];
            SV pa;
            if (dof >= 0) {
                const float* pr = A.dof_props;
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
                U[l] = si_mul(Ia, Sj[l]);
                Dl[l] = svdot(Sj[l], U[l]) + arm + imp;
                ul[l] = tau - svdot(Sj[l], pA[l]);
                const float invD = 1.0f / Dl[l];
                Ia.A = m3sub(Ia.A, m3outer(U[l].w, U[l].w, invD));
                Ia.B = m3sub(Ia.B, m3outer(U[l].w, U[l].v, invD));
                Ia.C = m3sub(Ia.C, m3outer(U[l].v, U[l].v, invD));
                pa = svadd(svadd(pA[l], si_mul(Ia, c[l])), svscale(U[l], ul[l] * invD));
            } else {
                pa = svadd(pA[l], si_mul(Ia, c[l]));
            }
            if (p > 0 || (p == 0 && !A.fixed_base)) {
                IA[p] = si_add(IA[p], x_inertia_t(E[l], r[l], Ia));
                pA[p] = svadd(pA[p], x_force_t(E[l], r[l], pa));
            }
        }
        // ---- pass 3: accelerations, outward
        a[0] = sv(v3(0.0f, 0.0f, 0.0f), vscale(gb, -1.0f));
        for (int l = 1; l < L; ++l) {
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], dof = li[2];
            SV ap = svadd(x_motion(E[l], r[l], a[p]), c[l]);
            if (dof >= 0) {
                const float acc = (ul[l] - svdot(U[l], ap)) / Dl[l];
                qdd[dof] = acc;
                ap = svadd(ap, svscale(Sj[l], acc));
            }
            a[l] = ap;
        }
        // ---- saturated implicit drives?
        unsigned nm = xmask;
        for (int d = 0; d < D; ++d) {
            const float eff = A.dof_props[3 * nd + d0 + d];
            if (eff > 0.0f && impd[d] != 0.0f) {
                const float act = tau0d[d] - impd[d] * qdd[d];
                if (act > eff) { nm |= 1u << d; xpos |= 1u << d; }
                else if (act < -eff) nm |= 1u << d;
            }
        }
        if (nm == xmask) break;
        xmask = nm;
      }
        // ---- integrate joints
        for (int d = 0; d < D; ++d) {
            const int gd = d0 + d;
            const float* pr = A.dof_props;
            const float maxv = pr[4 * nd + gd];
            float w = qd[d] + h * qdd[d];
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            float x = q[d] + h * w;
            if (pr[7 * nd + gd] != 0.0f) {
                const float lo = pr[5 * nd + gd], hi = pr[6 * nd + gd];
                if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
            }
            q[d] = x;
            qd[d] = w;
        }
    }

    // ---- outputs: DOF state and link states (forward kinematics at the new q, qd)
    for (int d = 0; d < D; ++d) {
        A.dof_pos[d0 + d] = q[d];
        A.dof_vel[d0 + d] = qd[d];
    }
    Q4 ql[MAXL];
    V3 xl[MAXL];
    for (int l = 0; l < L; ++l) {
        const float* lf = A.link_f + l * MG_LINK_F_N;
        const int* li = A.link_i + l * MG_LINK_I_N;
        const int p = li[0], jt = li[1], dof = li[2];
        const int b = b0 + l;
        if (p < 0) {
            ql[l] = q0; xl[l] = x0;
            v[l] = svzero();
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
            v[l] = svadd(x_motion(m3t(qmat(qrel)), rr, v[p]), svscale(s, qdj));
        }
        const V3 com = v3(A.mass[8 * nb + b], A.mass[9 * nb + b], A.mass[10 * nb + b]);
        const V3 ww = qrot(ql[l], v[l].w);
        const V3 vw = qrot(ql[l], vadd(v[l].v, vcross(v[l].w, com)));
        S[0 * nb + b] = xl[l].x; S[1 * nb + b] = xl[l].y; S[2 * nb + b] = xl[l].z;
        S[3 * nb + b] = ql[l].x; S[4 * nb + b] = ql[l].y; S[5 * nb + b] = ql[l].z; S[6 * nb + b] = ql[l].w;
        S[7 * nb + b] = vw.x; S[8 * nb + b] = vw.y; S[9 * nb + b] = vw.z;
        S[10 * nb + b] = ww.x; S[11 * nb + b] = ww.y; S[12 * nb + b] = ww.z;
        A.cforce[0 * nb + b] = 0.0f; A.cforce[1 * nb + b] = 0.0f; A.cforce[2 * nb + b] = 0.0f;
    }
}

// static-index access for register-resident per-link arrays (k_artic_world):
// the parent / DOF index is data, so reads are select chains and writes are
// guarded static stores — no private-memory (scratch) arrays
template <int N, class T>
__device__ __forceinline__ T sel(const T (&a)[N], int k) {
    T v = a[0];
#pragma unroll
    for (int j = 1; j < N; ++j)
        if (k == j) v = a[j];
    return v;
}
// parent of link l: index < l
template <int N, class T>
__device__ __forceinline__ T sel_lt(const T (&a)[N], int k, int l) {
    T v = a[0];
#pragma unroll
    for (int j = 1; j < N; ++j)
        if (j < l && k == j) v = a[j];
    return v;
}
template <int N, class T>
__device__ __forceinline__ void put(T (&a)[N], int k, const T& v) {
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (k == j) a[j] = v;
}

// One-lane world-frame articulated-body algorithm for templates of at most 4
// links (the S2 gimbal): every quantity about the base origin x0 in world axes
// (RBDA ch. 7), so the inward pass accumulates inertias by plain addition — no
// 6x6 spatial transforms, which dominate the body-frame k_artic_step. The
// arithmetic and its order are those of aba_world (mg_env.hip) as restated by
// oracle/migym_oracle_env.c:aba_world_ (the same function the oracle runs for
// these templates); per-link arrays are register-resident (static link loops,
// select chains for parent / DOF indices). Integration and outputs as
// k_artic_step.
template <int MAXL>
__global__ void __launch_bounds__(64) k_artic_world(MgStep P, MgArticArgs A) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= A.na) return;
    const int b0 = A.artic_i[i * MG_ARTIC_I_N + 0];
    const int d0 = A.artic_i[i * MG_ARTIC_I_N + 1];
    const int nb = A.nb, nd = A.nd;
    const int L = A.nl, D = A.ndof;
    float* S = A.state;
    const float* pr = A.dof_props;
    const float h = P.h;

    const V3 x0 = v3(S[0 * nb + b0], S[1 * nb + b0], S[2 * nb + b0]);
    const Q4 q0 = qnormalize(q4(S[3 * nb + b0], S[4 * nb + b0], S[5 * nb + b0], S[6 * nb + b0]));
    const float grav_on = A.tbf[A.body_tmpl[b0] * MG_TBODY_F_N + 4];
    const V3 gw = grav_on != 0.0f ? v3(P.g[0], P.g[1], P.g[2]) : v3(0.0f, 0.0f, 0.0f);

    float q[MAXL], qd[MAXL], qdd[MAXL];
#pragma unroll
    for (int d = 0; d < MAXL; ++d) {
        q[d] = d < D ? A.dof_pos[d0 + d] : 0.0f;
        qd[d] = d < D ? A.dof_vel[d0 + d] : 0.0f;
        qdd[d] = 0.0f;
    }
    LinkC lk[MAXL];
#pragma unroll
    for (int l = 1; l < MAXL; ++l)
        if (l < L) lk[l] = load_link(A.mass, nb, b0 + l);

    Q4 ql[MAXL], qrl[MAXL];
    V3 xl[MAXL], rrl[MAXL];
    float Iw[MAXL][36], xi[MAXL][6], va[MAXL][6], cc[MAXL][6], pa[MAXL][6], Ua[MAXL][6], Dd[MAXL], uu[MAXL];

    for (int st = 0; st < P.substeps; ++st) {
        unsigned xmask = 0u, xpos = 0u;
        float tau0d[MAXL], impd[MAXL];
#pragma unroll
        for (int d = 0; d < MAXL; ++d) { tau0d[d] = 0.0f; impd[d] = 0.0f; }
        for (int att = 0; att < 2; ++att) {
            // joint transforms, forward kinematics, motion axes, world inertias
            ql[0] = q0;
            xl[0] = x0;
#pragma unroll
            for (int l = 1; l < MAXL; ++l) {
                if (l >= L) break;
                const float* lf = A.link_f + l * MG_LINK_F_N;
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], jt = li[1], dj = li[2];
                const V3 po = v3(lf[0], lf[1], lf[2]);
                const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
                const V3 ax = v3(lf[7], lf[8], lf[9]);
                const float qj = dj >= 0 ? sel(q, dj) : 0.0f;
                qrl[l] = qo;
                rrl[l] = po;
                if (jt == MG_JOINT_REVOLUTE) qrl[l] = qmul(qo, q_axis_angle(ax, qj));
                else if (jt == MG_JOINT_PRISMATIC) rrl[l] = vadd(po, qrot(qo, vscale(ax, qj)));
                const Q4 qp = sel_lt(ql, p, l);
                ql[l] = qnormalize(qmul(qp, qrl[l]));
                xl[l] = vadd(sel_lt(xl, p, l), qrot(qp, rrl[l]));
                const V3 z = qrot(ql[l], ax);
                SV x = svzero();
                if (dj >= 0) {
                    if (jt == MG_JOINT_REVOLUTE) x = sv(z, vcross(vsub(xl[l], x0), z));
                    else x = sv(v3(0.0f, 0.0f, 0.0f), z);
                }
                put6(xi[l], x);
                world_inertia(lk[l], ql[l], xl[l], x0, Iw[l]);
            }
            // velocities, velocity-product accelerations, bias forces
#pragma unroll
            for (int k = 0; k < 6; ++k) va[0][k] = 0.0f;
#pragma unroll
            for (int l = 1; l < MAXL; ++l) {
                if (l >= L) break;
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], dj = li[2];
                const float qdl = dj >= 0 ? sel(qd, dj) : 0.0f;
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    float vp = va[0][k];
#pragma unroll
                    for (int j = 1; j < l; ++j)
                        if (p == j) vp = va[j][k];
                    va[l][k] = vp + xi[l][k] * qdl;
                }
                const SV v = sv6(va[l]);
                const SV vJ = svscale(sv6(xi[l]), qdl);
                float Iv[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) Iv[k] = dot6(&Iw[l][k * 6], va[l]);
                put6(cc[l], crm(v, vJ));
                put6(pa[l], crf(v, sv6(Iv)));
            }
            // inward pass: articulated inertias and bias forces
#pragma unroll
            for (int l = MAXL - 1; l >= 1; --l) {
                if (l >= L) continue;
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], dj = li[2];
                float uinvD = 0.0f;
                if (dj >= 0) {
                    const int gd = d0 + dj;
                    const int mode = (int)pr[0 * nd + gd];
                    const float kp = pr[1 * nd + gd], kd = pr[2 * nd + gd], eff = pr[3 * nd + gd];
                    const float arm = pr[8 * nd + gd];
                    const float qv = sel(q, dj), uv = sel(qd, dj);
#pragma unroll
                    for (int k = 0; k < 6; ++k) Ua[l][k] = dot6(&Iw[l][k * 6], xi[l]);
                    float tau = 0.0f, imp = 0.0f;
                    if (mode == MG_DOF_MODE_POS) {
                        tau = kp * (A.dof_tpos[gd] - qv - h * uv) + kd * (A.dof_tvel[gd] - uv);
                        imp = h * kd + h * h * kp;
                    } else if (mode == MG_DOF_MODE_VEL) {
                        tau = kd * (A.dof_tvel[gd] - uv);
                        imp = h * kd;
                    } else if (mode == MG_DOF_MODE_EFFORT) {
                        tau = A.dof_force[gd];
                    }
                    if (eff > 0.0f) {
                        if ((xmask >> dj) & 1u) {
                            tau = ((xpos >> dj) & 1u) ? eff : -eff;
                            imp = 0.0f;
                        } else if (imp == 0.0f) {
                            tau = fminf(fmaxf(tau, -eff), eff);
                        }
                    }
                    const float Dv = dot6(xi[l], Ua[l]) + arm + imp;
                    const float uvv = tau - dot6(xi[l], pa[l]);
                    const float invD = 1.0f / Dv;
                    uinvD = uvv * invD;
#pragma unroll
                    for (int e = 0; e < 36; ++e) Iw[l][e] = Iw[l][e] - Ua[l][e / 6] * (Ua[l][e % 6] * invD);
                    Dd[l] = Dv;
                    uu[l] = uvv;
                    put(tau0d, dj, tau);
                    put(impd, dj, imp);
                }
                if (p > 0) {
                    float pv[6];
#pragma unroll
                    for (int k = 0; k < 6; ++k) {
                        pv[k] = pa[l][k] + dot6(&Iw[l][k * 6], cc[l]);
                        if (dj >= 0) pv[k] = pv[k] + Ua[l][k] * uinvD;
                    }
#pragma unroll
                    for (int j = 1; j < l; ++j)
                        if (p == j) {
#pragma unroll
                            for (int k = 0; k < 6; ++k) pa[j][k] = pa[j][k] + pv[k];
#pragma unroll
                            for (int e = 0; e < 36; ++e) Iw[j][e] = Iw[j][e] + Iw[l][e];
                        }
                }
            }
            // outward pass: accelerations (gravity as a base acceleration -g)
            va[0][0] = 0.0f; va[0][1] = 0.0f; va[0][2] = 0.0f;
            va[0][3] = -gw.x; va[0][4] = -gw.y; va[0][5] = -gw.z;
#pragma unroll
            for (int l = 1; l < MAXL; ++l) {
                if (l >= L) break;
                const int* li = A.link_i + l * MG_LINK_I_N;
                const int p = li[0], dj = li[2];
                float a6[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    float ap = va[0][k];
#pragma unroll
                    for (int j = 1; j < l; ++j)
                        if (p == j) ap = va[j][k];
                    a6[k] = ap + cc[l][k];
                }
                if (dj >= 0) {
                    // the 16-lane reduction tree of aba_world over lanes 0..5 (the rest zero)
                    float t[6];
#pragma unroll
                    for (int k = 0; k < 6; ++k) t[k] = Ua[l][k] * a6[k] + 0.0f;
                    const float u0 = (t[0] + t[4]) + (t[2] + 0.0f);
                    const float u1 = (t[1] + t[5]) + (t[3] + 0.0f);
                    const float acc = (uu[l] - (u0 + u1)) / Dd[l];
#pragma unroll
                    for (int k = 0; k < 6; ++k) a6[k] = a6[k] + xi[l][k] * acc;
                    put(qdd, dj, acc);
                }
#pragma unroll
                for (int k = 0; k < 6; ++k) va[l][k] = a6[k];
            }
            // drives whose implicit force exceeds the effort limit: re-solve once
            unsigned nm = xmask;
#pragma unroll
            for (int d = 0; d < MAXL; ++d) {
                if (d >= D) break;
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
        // integrate joints
#pragma unroll
        for (int d = 0; d < MAXL; ++d) {
            if (d >= D) break;
            const int gd = d0 + d;
            const float maxv = pr[4 * nd + gd];
            float w = qd[d] + h * qdd[d];
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            float x = q[d] + h * w;
            if (pr[7 * nd + gd] != 0.0f) {
                const float lo = pr[5 * nd + gd], hi = pr[6 * nd + gd];
                if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
            }
            q[d] = x;
            qd[d] = w;
        }
    }

    // outputs: DOF state and link states (forward kinematics at the new q, qd)
#pragma unroll
    for (int d = 0; d < MAXL; ++d) {
        if (d >= D) break;
        A.dof_pos[d0 + d] = q[d];
        A.dof_vel[d0 + d] = qd[d];
    }
    SV v[MAXL];
#pragma unroll
    for (int l = 0; l < MAXL; ++l) {
        if (l >= L) break;
        const float* lf = A.link_f + l * MG_LINK_F_N;
        const int* li = A.link_i + l * MG_LINK_I_N;
        const int p = li[0], jt = li[1], dof = li[2];
        const int b = b0 + l;
        if (p < 0) {
            ql[l] = q0; xl[l] = x0;
            v[l] = svzero();
        } else {
            const V3 po = v3(lf[0], lf[1], lf[2]);
            const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
            const V3 ax = v3(lf[7], lf[8], lf[9]);
            const float qj = dof >= 0 ? sel(q, dof) : 0.0f;
            const float qdj = dof >= 0 ? sel(qd, dof) : 0.0f;
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
            const Q4 qp = sel_lt(ql, p, l);
            ql[l] = qnormalize(qmul(qp, qrel));
            xl[l] = vadd(sel_lt(xl, p, l), qrot(qp, rr));
            v[l] = svadd(x_motion(m3t(qmat(qrel)), rr, sel_lt(v, p, l)), svscale(s, qdj));
        }
        const V3 com = v3(A.mass[8 * nb + b], A.mass[9 * nb + b], A.mass[10 * nb + b]);
        const V3 ww = qrot(ql[l], v[l].w);
        const V3 vw = qrot(ql[l], vadd(v[l].v, vcross(v[l].w, com)));
        S[0 * nb + b] = xl[l].x; S[1 * nb + b] = xl[l].y; S[2 * nb + b] = xl[l].z;
        S[3 * nb + b] = ql[l].x; S[4 * nb + b] = ql[l].y; S[5 * nb + b] = ql[l].z; S[6 * nb + b] = ql[l].w;
        S[7 * nb + b] = vw.x; S[8 * nb + b] = vw.y; S[9 * nb + b] = vw.z;
        S[10 * nb + b] = ww.x; S[11 * nb + b] = ww.y; S[12 * nb + b] = ww.z;
        A.cforce[0 * nb + b] = 0.0f; A.cforce[1 * nb + b] = 0.0f; A.cforce[2 * nb + b] = 0.0f;
    }
}

// Lane-parallel Jacobian and mass matrix: JG = 16 lanes per articulation, 4
// articulations per wavefront, per-articulation kinematics staged in LDS.
// Lane l: joint transform, world motion axis xi_l (about the base origin x0)
// and world inertia of link l; lane 0: the forward-kinematics scan; lane d:
// Jacobian column d for every link (nonzero where joint d is on the link's
// path); composite inertias IC_l by subtree sums (lanes over the 36 entries);
// lane i: row i of M, M_ij = xi_j . IC_i xi_i for j on the path of i (RBDA
// Table 6.2 in one frame: no spatial transforms). Float64 textbook kinematics
// check it (tests/test_franka_gpu.py, tests/test_gimbal_*).
constexpr int JG = 16;
constexpr int JEPW = 64 / JG;

struct JacLds {
    Q4 qr[MG_MAX_LINKS], ql[MG_MAX_LINKS];
    V3 rr[MG_MAX_LINKS], xl[MG_MAX_LINKS], zl[MG_MAX_LINKS];
    float xi[MG_MAX_LINKS][6];
    float Iw[MG_MAX_LINKS][36];
    float M[JG][JG];
    int amask[MG_MAX_LINKS];
};

__global__ void __launch_bounds__(64) k_artic_jac_mm_g(MgArticArgs A, float* jac, float* mm) {
    __shared__ JacLds shm[JEPW];
    const int gi = threadIdx.x / JG, ln = threadIdx.x % JG;
    const int e = blockIdx.x * JEPW + gi;
    const bool live = e < A.na;
    JacLds& S = shm[gi];
    const int ei = live ? e : 0;
    const int b0 = A.artic_i[ei * MG_ARTIC_I_N + 0];
    const int d0 = A.artic_i[ei * MG_ARTIC_I_N + 1];
    const int nb = A.nb;
    const int L = A.nl, D = A.ndof;
    const float* St = A.state;
    const V3 x0 = v3(St[0 * nb + b0], St[1 * nb + b0], St[2 * nb + b0]);
    const Q4 q0 = qnormalize(q4(St[3 * nb + b0], St[4 * nb + b0], St[5 * nb + b0], St[6 * nb + b0]));
    // joint transforms (lane l)
    if (live && ln > 0 && ln < L) {
        const float* lf = A.link_f + ln * MG_LINK_F_N;
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        const V3 po = v3(lf[0], lf[1], lf[2]);
        const Q4 qo = q4(lf[3], lf[4], lf[5], lf[6]);
        const V3 ax = v3(lf[7], lf[8], lf[9]);
        const float qj = dof >= 0 ? A.dof_pos[d0 + dof] : 0.0f;
        Q4 qrel = qo;
        V3 rr = po;
        if (jt == MG_JOINT_REVOLUTE) qrel = qmul(qo, q_axis_angle(ax, qj));
        else if (jt == MG_JOINT_PRISMATIC) rr = vadd(po, qrot(qo, vscale(ax, qj)));
        S.qr[ln] = qrel;
        S.rr[ln] = rr;
    }
    __syncthreads();
    // forward kinematics and joint-path masks (lane 0)
    if (live && ln == 0) {
        for (int l = 0; l < L; ++l) {
            const int* li = A.link_i + l * MG_LINK_I_N;
            const int p = li[0], dof = li[2];
            if (p < 0) {
                S.ql[l] = q0;
                S.xl[l] = x0;
                S.amask[l] = 0;
            } else {
                const Q4 qp = S.ql[p];
                S.ql[l] = qnormalize(qmul(qp, S.qr[l]));
                S.xl[l] = vadd(S.xl[p], qrot(qp, S.rr[l]));
                S.amask[l] = S.amask[p] | (dof >= 0 ? (1 << dof) : 0);
            }
        }
    }
    __syncthreads();
    // world axes, motion subspaces, inertias (lane l)
    if (live && ln < L) {
        const int* li = A.link_i + ln * MG_LINK_I_N;
        const int jt = li[1], dof = li[2];
        const float* lf = A.link_f + ln * MG_LINK_F_N;
        const V3 z = ln > 0 ? qrot(S.ql[ln], v3(lf[7], lf[8], lf[9])) : v3(0.0f, 0.0f, 0.0f);
        S.zl[ln] = z;
        SV x = svzero();
        if (ln > 0 && dof >= 0) {
            if (jt == MG_JOINT_REVOLUTE) x = sv(z, vcross(vsub(S.xl[ln], x0), z));
            else x = sv(v3(0.0f, 0.0f, 0.0f), z);
        }
        put6(S.xi[ln], x);
        if (mm && ln > 0) world_inertia(load_link(A.mass, nb, b0 + ln), S.ql[ln], S.xl[ln], x0, S.Iw[ln]);
    }
    __syncthreads();
    // the link whose joint is DOF ln
    int jl = -1;
    bool jrev = false;
    for (int l = 1; l < L; ++l)
        if (A.link_i[l * MG_LINK_I_N + 2] == ln) {
            jl = l;
            jrev = A.link_i[l * MG_LINK_I_N + 1] == MG_JOINT_REVOLUTE;
        }
    if (jac && live && ln < D && jl > 0) {
        // column ln of every link's 6 x D block: [linear at the link origin; angular]
        float* J = jac + (size_t)e * (L - 1) * 6 * D;
        const V3 z = S.zl[jl], xj = S.xl[jl];
        for (int l = 1; l < L; ++l) {
            V3 lin = v3(0.0f, 0.0f, 0.0f), ang = v3(0.0f, 0.0f, 0.0f);
            if ((S.amask[l] >> ln) & 1) {
                if (jrev) { lin = vcross(z, vsub(S.xl[l], xj)); ang = z; }
                else lin = z;
            }
            float* Jl = J + (size_t)(l - 1) * 6 * D + ln;
            Jl[0 * D] = lin.x; Jl[1 * D] = lin.y; Jl[2 * D] = lin.z;
            Jl[3 * D] = ang.x; Jl[4 * D] = ang.y; Jl[5 * D] = ang.z;
        }
    }
    if (!mm) return;
    // composite inertias: subtree sums, deepest link first (links are in
    // topological order: a parent precedes its children)
    for (int l = L - 1; l >= 1; --l) {
        const int p = A.link_i[l * MG_LINK_I_N + 0];
        if (live && p > 0)
            for (int k = ln; k < 36; k += JG) S.Iw[p][k] = S.Iw[p][k] + S.Iw[l][k];
        __syncthreads();
    }
    for (int k = 0; k < JG; ++k) S.M[ln][k] = 0.0f;
    __syncthreads();
    if (live && ln < D && jl > 0) {
        float F[6];
        for (int r = 0; r < 6; ++r) F[r] = dot6(&S.Iw[jl][r * 6], S.xi[jl]);
        S.M[ln][ln] = dot6(S.xi[jl], F);
        int j = A.link_i[jl * MG_LINK_I_N + 0];
        while (j > 0) {
            const int dj = A.link_i[j * MG_LINK_I_N + 2];
            if (dj >= 0) {
                const float hv = dot6(S.xi[j], F);
                S.M[ln][dj] = hv;
                S.M[dj][ln] = hv;
            }
            j = A.link_i[j * MG_LINK_I_N + 0];
        }
    }
    __syncthreads();
    if (live) {
        float* Mo = mm + (size_t)e * D * D;
        for (int k = ln; k < D * D; k += JG) Mo[k] = S.M[k / D][k % D];
    }
}

}  // namespace

// refresh_jacobian_tensors / refresh_mass_matrix_tensors
// (examples/franka_cube_ik_osc.py:305-316,345-346): for a fixed base
//   J: (instances, L-1, 6, D): link l = 1..L-1, rows [linear xyz of the link
//      frame origin, angular xyz] in the world frame, column d = DOF d;
//   M: (instances, D, D): joint-space inertia without joint armature.
hipError_t mg_launch_jacobian(const MgArticArgs& A, float* jac, float* mm, hipStream_t s) {
    if (A.na <= 0) return hipSuccess;
    if (!A.fixed_base || A.nl > MG_MAX_LINKS || A.ndof > JG) return hipErrorNotSupported;
    hipLaunchKernelGGL(k_artic_jac_mm_g, dim3((A.na + JEPW - 1) / JEPW), dim3(64), 0, s, A, jac, mm);
    return hipGetLastError();
}

hipError_t mg_launch_artic_step(const MgStep& P, const MgArticArgs& A, hipStream_t s) {
    if (A.na <= 0) return hipSuccess;
    if (!A.fixed_base) return hipErrorNotSupported;
    const int blocks = (A.na + 63) / 64;
    if (A.nl <= 4)
        MG_LAUNCH(k_artic_world<4>, dim3(blocks), dim3(64), 0, s, P, A);
    else if (A.nl <= 8)
        MG_LAUNCH(k_artic_step<8>, dim3(blocks), dim3(64), 0, s, P, A);
    else if (A.nl <= MG_MAX_LINKS)
        MG_LAUNCH(k_artic_step<MG_MAX_LINKS>, dim3(blocks), dim3(64), 0, s, P, A);
    else
        return hipErrorNotSupported;
    return hipGetLastError();
}
