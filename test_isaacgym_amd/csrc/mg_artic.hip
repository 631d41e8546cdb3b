// mg_artic.hip — Jacobian and mass-matrix tensors of fixed-base articulations
// (refresh_jacobian_tensors / refresh_mass_matrix_tensors,
// examples/franka_cube_ik_osc.py:305-316,345-346), and the launcher of the
// articulation step.
//
// The step itself (Featherstone's articulated-body algorithm in the world frame
// about the base origin, implicit PD / velocity drives, the effort-limit
// re-solve, joint integration, forward kinematics of the link states) runs on
// 16 lanes per articulation in mg_env.hip:k_artic_lanes, sharing aba_world
// with the coupled per-env step. Drive law: POS
// tau0 = kp (q* - q - h qd) + kd (qd* - qd), VEL tau0 = kd (qd* - qd), EFFORT
// tau0 = u. Restated in C by oracle/migym_oracle.c:artic_step.
#include "mg_internal.h"
#include "mg_spatial.h"
#include "mg_world.h"

namespace {

// Lane-parallel Jacobian and mass matrix: JG = 16 lanes per articulation, 4
// articulations per wavefront (JG = 32, 2 per wavefront, for more than 16
// links — virtual links included — or generalized velocities: the MJCF
// humanoid's 21 DOFs + 6 root columns), per-articulation kinematics staged in LDS.
// Lane l: joint transform, world motion axis xi_l (about the base origin x0)
// and world inertia of link l; lane 0: the forward-kinematics scan; lane d:
// Jacobian column d for every link (nonzero where joint d is on the link's
// path); composite inertias IC_l by subtree sums (lanes over the 36 entries);
// lane i: row i of M, M_ij = xi_j . IC_i xi_i for j on the path of i (RBDA
// Table 6.2 in one frame: no spatial transforms). Float64 textbook kinematics
// check it (tests/test_franka_gpu.py, tests/test_gimbal_*).
template <int JG>
struct JacLds {
    Q4 qr[MG_MAX_LINKS], ql[MG_MAX_LINKS];
    V3 rr[MG_MAX_LINKS], xl[MG_MAX_LINKS], zl[MG_MAX_LINKS];
    float xi[MG_MAX_LINKS][6];
    float Iw[MG_MAX_LINKS][36];
    float M[JG][JG];
    unsigned amask[MG_MAX_LINKS];
};

template <int JG>
__global__ void __launch_bounds__(64) k_artic_jac_mm_g(MgArticArgs A, float* jac, float* mm) {
    constexpr int JEPW = 64 / JG;
    static_assert(JG >= 16 && JG <= 32 && MG_MAX_LINKS <= 32, "lanes own links, DOFs and M rows");
    __shared__ JacLds<JG> shm[JEPW];
    const int gi = threadIdx.x / JG, ln = threadIdx.x % JG;
    const int e = blockIdx.x * JEPW + gi;
    const bool live = e < A.na;
    JacLds<JG>& S = shm[gi];
    const int ei = live ? e : 0;
    const int b0 = A.artic_i[ei * MG_ARTIC_I_N + 0];
    const int d0 = A.artic_i[ei * MG_ARTIC_I_N + 1];
    const int ls = A.artic_i[ei * MG_ARTIC_I_N + 3];     // link stride (migym_capi.cpp)
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
        Q4 qrel;
        V3 rr;
        link_joint(jt, (int)lf[10], po, qo, ax, A.dof_pos + d0, dof, qrel, rr);
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
                S.amask[l] = 0u;
            } else {
                const Q4 qp = S.ql[p];
                S.ql[l] = qnormalize(qmul(qp, S.qr[l]));
                S.xl[l] = vadd(S.xl[p], qrot(qp, S.rr[l]));
                S.amask[l] = S.amask[p] | (dof >= 0 ? (1u << dof) : 0u);
            }
        }
    }
    __syncthreads();
    // world axes, motion subspaces, inertias (lane l)
    const bool fb = !A.fixed_base;
    const int R0 = fb ? 6 : 0;            // root columns (floating base) before the DOFs
    const int NC = D + R0;                // generalized velocities
    const int row0 = fb ? 0 : 1;          // first link row of the Jacobian
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
        // a virtual link (ball joint, body -1) has no mass
        if (mm && (ln > 0 || fb)) {
            if (li[3] >= 0) {
                world_inertia(load_link(A.mass, nb, b0 + li[3] * ls), S.ql[ln], S.xl[ln], x0, S.Iw[ln]);
            } else {
                for (int k = 0; k < 36; ++k) S.Iw[ln][k] = 0.0f;
            }
        }
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
    if (jac && live) {
        // rows: the template's bodies (virtual links of ball joints have none)
        float* J = jac + (size_t)e * (A.nbl - row0) * 6 * NC;
        if (ln < D && jl > 0) {
            // column R0 + ln of every link's 6 x NC block: [linear at the link origin; angular]
            const V3 z = S.zl[jl], xj = S.xl[jl];
            for (int l = row0; l < L; ++l) {
                const int bl = A.link_i[l * MG_LINK_I_N + 3];
                if (bl < 0) continue;
                V3 lin = v3(0.0f, 0.0f, 0.0f), ang = v3(0.0f, 0.0f, 0.0f);
                if ((S.amask[l] >> ln) & 1) {
                    if (jrev) { lin = vcross(z, vsub(S.xl[l], xj)); ang = z; }
                    else lin = z;
                }
                float* Jl = J + (size_t)(bl - row0) * 6 * NC + R0 + ln;
                Jl[0 * NC] = lin.x; Jl[1 * NC] = lin.y; Jl[2 * NC] = lin.z;
                Jl[3 * NC] = ang.x; Jl[4 * NC] = ang.y; Jl[5 * NC] = ang.z;
            }
        } else if (fb && ln >= D && ln < D + 6) {
            // root column k: linear velocity of x0 along e_k (k < 3), rotation
            // about e_(k-3) through x0
            const int k = ln - D;
            const V3 ek = v3(k % 3 == 0 ? 1.0f : 0.0f, k % 3 == 1 ? 1.0f : 0.0f, k % 3 == 2 ? 1.0f : 0.0f);
            for (int l = 0; l < L; ++l) {
                const int bl = A.link_i[l * MG_LINK_I_N + 3];
                if (bl < 0) continue;
                V3 lin = ek, ang = v3(0.0f, 0.0f, 0.0f);
                if (k >= 3) { lin = vcross(ek, vsub(S.xl[l], x0)); ang = ek; }
                float* Jl = J + (size_t)bl * 6 * NC + k;
                Jl[0 * NC] = lin.x; Jl[1 * NC] = lin.y; Jl[2 * NC] = lin.z;
                Jl[3 * NC] = ang.x; Jl[4 * NC] = ang.y; Jl[5 * NC] = ang.z;
            }
        }
    }
    if (!mm) return;
    // composite inertias: subtree sums, deepest link first (links are in
    // topological order: a parent precedes its children); a floating base also
    // folds the tree into link 0
    for (int l = L - 1; l >= 1; --l) {
        const int p = A.link_i[l * MG_LINK_I_N + 0];
        if (live && (p > 0 || (fb && p == 0)))
            for (int k = ln; k < 36; k += JG) S.Iw[p][k] = S.Iw[p][k] + S.Iw[l][k];
        __syncthreads();
    }
    for (int k = 0; k < JG; ++k) S.M[ln][k] = 0.0f;
    __syncthreads();
    if (live && ln < D && jl > 0) {
        float F[6];
        for (int r = 0; r < 6; ++r) F[r] = dot6(&S.Iw[jl][r * 6], S.xi[jl]);
        const int i = R0 + ln;
        S.M[i][i] = dot6(S.xi[jl], F);
        int j = A.link_i[jl * MG_LINK_I_N + 0];
        while (j > 0) {
            const int dj = A.link_i[j * MG_LINK_I_N + 2];
            if (dj >= 0) {
                const float hv = dot6(S.xi[j], F);
                S.M[i][R0 + dj] = hv;
                S.M[R0 + dj][i] = hv;
            }
            j = A.link_i[j * MG_LINK_I_N + 0];
        }
        if (fb)
            // DOF - root coupling: the force IC xi (moment about x0, force) paired
            // with the root's unit motions (linear e_k: force k; angular e_k: moment k)
            for (int k = 0; k < 3; ++k) {
                S.M[i][k] = F[3 + k];
                S.M[k][i] = F[3 + k];
                S.M[i][3 + k] = F[k];
                S.M[3 + k][i] = F[k];
            }
    }
    if (live && fb && ln == D) {
        // root block from the whole-tree composite inertia about x0 ([A B; B^T C],
        // rows / columns (w, v)) in the root's (linear, angular) order
        const float* I0 = S.Iw[0];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                S.M[a][b] = I0[(3 + a) * 6 + 3 + b];
                S.M[a][3 + b] = I0[(3 + a) * 6 + b];
                S.M[3 + a][b] = I0[a * 6 + 3 + b];
                S.M[3 + a][3 + b] = I0[a * 6 + b];
            }
    }
    __syncthreads();
    if (live) {
        float* Mo = mm + (size_t)e * NC * NC;
        for (int k = ln; k < NC * NC; k += JG) Mo[k] = S.M[k / NC][k % NC];
    }
}

}  // namespace

// refresh_jacobian_tensors / refresh_mass_matrix_tensors
// (examples/franka_cube_ik_osc.py:305-316,345-346): for a fixed base
//   J: (instances, B-1, 6, D): body l = 1..B-1 (B bodies: the template's links
//      minus the virtual links of ball joints), rows [linear xyz of the link
//      frame origin, angular xyz] in the world frame, column d = DOF d;
//   M: (instances, D, D): joint-space inertia without joint armature;
// for a floating base (D + 6 <= 32) the 6 root columns come first — linear
// velocity of the base-link origin, then angular velocity, world axes:
//   J: (instances, L, 6, D + 6), every link including the root;
//   M: (instances, D + 6, D + 6) in the same generalized velocities.
hipError_t mg_launch_jacobian(const MgArticArgs& A, float* jac, float* mm, hipStream_t s) {
    if (A.na <= 0) return hipSuccess;
    const int nc = A.ndof + (A.fixed_base ? 0 : 6);
    if (A.nl > MG_MAX_LINKS || nc > 32) return hipErrorNotSupported;
    if (A.nl <= 16 && nc <= 16)
        hipLaunchKernelGGL(k_artic_jac_mm_g<16>, dim3((A.na + 3) / 4), dim3(64), 0, s, A, jac, mm);
    else
        hipLaunchKernelGGL(k_artic_jac_mm_g<32>, dim3((A.na + 1) / 2), dim3(64), 0, s, A, jac, mm);
    return hipGetLastError();
}

hipError_t mg_launch_artic_step(const MgStep& P, const MgArticArgs& A, hipStream_t s) {
    return mg_launch_artic_lanes(P, A, s);
}
