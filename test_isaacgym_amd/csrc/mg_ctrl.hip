// mg_ctrl.hip — the S3 cube-pick controller (examples/franka_cube_ik_osc.py
// :348-410, restated in torch by test_isaacgym_amd/franka_control.py) as one
// kernel, one lane per env.
//
// The torch restatement is ~150 small launches per frame (gathers, quaternion
// algebra, two batched 7x7 / 6x6 inverses and their products): ~0.6 ms of the
// S3 frame's 1.07 ms on MI355X, every launch a few microseconds of a nearly
// empty GPU. Here each lane reads its env's cube and hand rows, its 9 DOF
// states, its 6x7 end-effector Jacobian and 7x7 mass matrix (strided views of
// the sim's tensors: no copies), runs the script's grasp state machine and the
// OSC (:59-79) or damped-least-squares IK (:51-56) law in registers, and
// writes the (n, 9) position-target / effort rows the script hands to
// set_dof_position_target_tensor / set_dof_actuation_force_tensor (:409-410).
//
// The linear algebra is the same law without explicit inverses: with X = J M^-1
// (Cholesky solves of M for the six Jacobian rows) and m_eef = (X J^T)^-1,
//   u = J^T m_eef (kp dpose - kd v) + (I - J^T m_eef X) M u_null
//     = J^T m_eef (kp dpose - kd v - X M u_null) + M u_null,
// one 6x6 Cholesky solve, in float64: J M^-1 J^T is badly conditioned near the
// arm's singular poses (a float32 factorisation broke down there, where the
// script's float32 LU inverse returns large but finite values), and MI355X runs
// these few hundred FP64 operations per lane at full rate. The result matches
// the torch restatement evaluated in float64 to ~1e-6 of the effort, and its
// float32 evaluation to that evaluation's own rounding (tests/
// test_franka_ctrl_gpu.py) — not bit for bit: the controller is the reference
// script's own torch code, not part of the engine the oracle restates.
#include "mg_internal.h"
#include "mg_math.h"

namespace {

// franka_control.quat_rotate (torch_utils.quat_rotate): v (2w^2 - 1) + 2 w
// (q x v) + 2 q (q . v)
__device__ __forceinline__ V3 tq_rotate(Q4 q, V3 v) {
    const V3 u = v3(q.x, q.y, q.z);
    const V3 a = vscale(v, 2.0f * q.w * q.w - 1.0f);
    const V3 b = vscale(vcross(u, v), q.w * 2.0f);
    const V3 c = vscale(u, vdot(u, v) * 2.0f);
    return vadd(vadd(a, b), c);
}
// torch_utils.quat_mul (xyzw)
__device__ __forceinline__ Q4 tq_mul(Q4 a, Q4 b) {
    return q4(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
              a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
// Python / torch float remainder: the result has the divisor's sign
__device__ __forceinline__ float py_mod(float x, float y) { return x - floorf(x / y) * y; }
__device__ __forceinline__ float tsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

// In-place Cholesky of the symmetric N x N matrix a (lower triangle used):
// a = L L^T, L in the lower triangle, 1 / L_jj in inv_d.
template <int N>
__device__ __forceinline__ void chol(double (&a)[N][N], double (&inv_d)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double s = a[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= a[j][k] * a[j][k];
        const double d = sqrt(fmax(s, 1e-300));
        a[j][j] = d;
        inv_d[j] = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double t = a[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= a[i][k] * a[j][k];
            a[i][j] = t * inv_d[j];
        }
    }
}
// x = (L L^T)^-1 b
template <int N>
__device__ __forceinline__ void chol_solve(const double (&l)[N][N], const double (&inv_d)[N], const double (&b)[N],
                                           double (&x)[N]) {
    double y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t -= l[i][k] * y[k];
        y[i] = t * inv_d[i];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double t = y[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) t -= l[k][i] * x[k];
        x[i] = t * inv_d[i];
    }
}

__global__ void __launch_bounds__(64) k_cube_pick(mg_cube_pick_args A) {
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= A.n) return;
    const float* rb = A.rb;
    const float* bx = rb + (size_t)A.box_row[e] * MG_STATE_N;
    const float* hd = rb + (size_t)A.hand_row[e] * MG_STATE_N;
    const V3 box_pos = v3(bx[0], bx[1], bx[2]);
    const Q4 box_rot = q4(bx[3], bx[4], bx[5], bx[6]);
    const V3 hand_pos = v3(hd[0], hd[1], hd[2]);
    const Q4 hand_rot = q4(hd[3], hd[4], hd[5], hd[6]);
    float hand_vel[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) hand_vel[k] = hd[7 + k];
    float q[9], qd[9];
    const float* ds = A.dof + (size_t)A.dof_row0[e] * 2;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        q[k] = ds[2 * k];
        qd[k] = ds[2 * k + 1];
    }
    const float go = A.grasp_offset;

    // :348-401, the grasp state machine
    const V3 to_box = vsub(box_pos, hand_pos);
    const float box_dist = sqrtf(vdot(to_box, to_box));
    const float box_dot = -(to_box.z / box_dist);                 // box_dir . (0, 0, -1)
    const float gripper_sep = q[7] + q[8];
    const bool gripped = gripper_sep < 0.045f && box_dist < go + 0.5f * A.box_size;
    // cube_grasping_yaw (:40-50)
    const float h = 0.5f * A.box_size;
    const V3 rc = tq_rotate(box_rot, v3(h, h, h));
    const float yaw = py_mod(atan2f(rc.y, rc.x) - 0.25f * 3.14159265358979f, 0.5f * 3.14159265358979f);
    const float theta = 0.5f * yaw;
    const Q4 yaw_q = q4(0.0f, 0.0f, sinf(theta), cosf(theta));
    const V3 box_yaw_dir = tq_rotate(yaw_q, v3(1.0f, 0.0f, 0.0f));
    const V3 hand_yaw_dir = tq_rotate(hand_rot, v3(1.0f, 0.0f, 0.0f));
    const float yaw_dot = vdot(box_yaw_dir, hand_yaw_dir);
    const V3 init_pos = v3(A.init_pos[3 * e], A.init_pos[3 * e + 1], A.init_pos[3 * e + 2]);
    const Q4 init_rot = q4(A.init_rot[4 * e], A.init_rot[4 * e + 1], A.init_rot[4 * e + 2], A.init_rot[4 * e + 3]);
    const V3 to_init = vsub(init_pos, hand_pos);
    const float init_dist = sqrtf(vdot(to_init, to_init));
    bool restart = A.hand_restart[e] != 0 && init_dist > 0.02f;
    const bool return_to_start = restart || gripped;
    const bool above_box = box_dot >= 0.99f && yaw_dot >= 0.95f && box_dist < go * 3.0f;
    V3 grasp_pos = box_pos;
    grasp_pos.z = above_box ? box_pos.z + go : box_pos.z + go * 2.5f;
    const V3 goal_pos = return_to_start ? init_pos : grasp_pos;
    const Q4 goal_rot = return_to_start ? init_rot : tq_mul(q4(1.0f, 0.0f, 0.0f, 0.0f), qconj(yaw_q));
    // orientation_error (:34-37)
    const Q4 qr = tq_mul(goal_rot, qconj(hand_rot));
    const float sg = tsign(qr.w);
    const V3 pos_err = vsub(goal_pos, hand_pos);
    const double dpose[6] = {pos_err.x, pos_err.y, pos_err.z, qr.x * sg, qr.y * sg, qr.z * sg};

    // the end-effector Jacobian (6 x 7: linear rows, then angular)
    double J[6][7];
    const float* jb = A.jac + (size_t)e * A.jac_se;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 7; ++c) J[r][c] = jb[r * A.jac_sr + c * A.jac_sc];
    float* pa = A.pos_action + (size_t)e * 9;
    float* ea = A.effort_action + (size_t)e * 9;
    if (A.osc) {
        // control_osc (:59-79)
        double M[7][7], L[7][7], inv_dm[7];
        const float* mb = A.mm + (size_t)e * A.mm_se;
#pragma unroll
        for (int r = 0; r < 7; ++r)
#pragma unroll
            for (int c = 0; c < 7; ++c) {
                M[r][c] = mb[r * A.mm_sr + c * A.mm_sc];
                L[r][c] = M[r][c];
            }
        chol<7>(L, inv_dm);
        double X[6][7];   // X = J M^-1: row r solves M x = J_r
#pragma unroll
        for (int r = 0; r < 6; ++r) chol_solve<7>(L, inv_dm, J[r], X[r]);
        double Ae[6][6], inv_da[6];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int s = 0; s <= r; ++s) {
                double t = 0.0;
#pragma unroll
                for (int c = 0; c < 7; ++c) t += X[r][c] * J[s][c];
                Ae[r][s] = t;
                Ae[s][r] = t;
            }
        chol<6>(Ae, inv_da);
        // null-space term: M (kd_null (-qd) + kp_null wrap(default - q)), first 7 DOFs
        double un[7], mun[7];
#pragma unroll
        for (int k = 0; k < 7; ++k)
            un[k] = A.kd_null * -qd[k] +
                    A.kp_null * (py_mod(A.default_dof_pos[k] - q[k] + 3.14159265358979f, 2.0f * 3.14159265358979f) -
                                 3.14159265358979f);
#pragma unroll
        for (int r = 0; r < 7; ++r) {
            double t = 0.0;
#pragma unroll
            for (int c = 0; c < 7; ++c) t += M[r][c] * un[c];
            mun[r] = t;
        }
        double f[6], tvec[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            double xm = 0.0;
#pragma unroll
            for (int c = 0; c < 7; ++c) xm += X[r][c] * mun[c];
            f[r] = (double)A.kp * dpose[r] - (double)A.kd * hand_vel[r] - xm;
        }
        chol_solve<6>(Ae, inv_da, f, tvec);
#pragma unroll
        for (int c = 0; c < 7; ++c) {
            double t = mun[c];
#pragma unroll
            for (int r = 0; r < 6; ++r) t += J[r][c] * tvec[r];
            ea[c] = (float)t;
        }
    } else {
        // control_ik (:51-56): J^T (J J^T + damping^2 I)^-1 dpose
        double B[6][6], inv_db[6], tvec[6];
        const double l2 = (double)A.damping * A.damping;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int s = 0; s <= r; ++s) {
                double t = 0.0;
#pragma unroll
                for (int c = 0; c < 7; ++c) t += J[r][c] * J[s][c];
                B[r][s] = t + (r == s ? l2 : 0.0);
                B[s][r] = B[r][s];
            }
        chol<6>(B, inv_db);
        chol_solve<6>(B, inv_db, dpose, tvec);
#pragma unroll
        for (int c = 0; c < 7; ++c) {
            double t = 0.0;
#pragma unroll
            for (int r = 0; r < 6; ++r) t += J[r][c] * tvec[r];
            pa[c] = (float)(q[c] + t);
        }
    }
    // gripper (:403-407) and the restart flag (:401)
    bool close = box_dist < go + 0.02f || gripped;
    restart = restart || box_pos.z > 0.6f;
    close = close && !restart;
    pa[7] = close ? 0.0f : 0.04f;
    pa[8] = close ? 0.0f : 0.04f;
    A.hand_restart[e] = restart ? 1 : 0;
}

}  // namespace

hipError_t mg_launch_cube_pick(const mg_cube_pick_args& A, hipStream_t s) {
    if (A.n <= 0) return hipSuccess;
    MG_LAUNCH(k_cube_pick, dim3((A.n + 63) / 64), dim3(64), 0, s, A);
    return hipGetLastError();
}
