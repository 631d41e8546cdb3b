// mg_spatial.h — 6-D spatial algebra (Featherstone, RBDA ch. 2) on 3x3 blocks.
//
// Motion vector m = (w, v): angular velocity and the velocity of the frame
// origin. Force vector f = (n, f): moment about the frame origin and force.
// Spatial inertia / articulated inertia I = [A B; B^T C] (A, C symmetric).
// Transform X = (E, r): E maps parent coordinates to child coordinates, r is
// the child origin in parent coordinates, so X m = (E w, E (v - r x w)).
// Fixed evaluation order, no FMA contraction: oracle/migym_oracle.c restates
// every function here in C with the same order.
#pragma once
#include "mg_math.h"
#include "migym.h"

struct SV { V3 w, v; };
struct SI { M3 A, B, C; };

MG_HD SV sv(V3 w, V3 v) { SV r; r.w = w; r.v = v; return r; }
MG_HD SV svzero() { return sv(v3(0.0f, 0.0f, 0.0f), v3(0.0f, 0.0f, 0.0f)); }
MG_HD SV svadd(SV a, SV b) { return sv(vadd(a.w, b.w), vadd(a.v, b.v)); }
MG_HD SV svscale(SV a, float s) { return sv(vscale(a.w, s), vscale(a.v, s)); }
MG_HD float svdot(SV a, SV b) { return vdot(a.w, b.w) + vdot(a.v, b.v); }
// motion x motion
MG_HD SV crm(SV a, SV b) { return sv(vcross(a.w, b.w), vadd(vcross(a.w, b.v), vcross(a.v, b.w))); }
// motion x force
MG_HD SV crf(SV a, SV f) { return sv(vadd(vcross(a.w, f.w), vcross(a.v, f.v)), vcross(a.w, f.v)); }

MG_HD M3 m3cols(V3 c0, V3 c1, V3 c2) { M3 m; m.c0 = c0; m.c1 = c1; m.c2 = c2; return m; }
MG_HD M3 m3zero() { V3 z = v3(0.0f, 0.0f, 0.0f); return m3cols(z, z, z); }
MG_HD M3 m3add(M3 a, M3 b) { return m3cols(vadd(a.c0, b.c0), vadd(a.c1, b.c1), vadd(a.c2, b.c2)); }
MG_HD M3 m3sub(M3 a, M3 b) { return m3cols(vsub(a.c0, b.c0), vsub(a.c1, b.c1), vsub(a.c2, b.c2)); }
MG_HD M3 m3mul(M3 a, M3 b) { return m3cols(mmul(a, b.c0), mmul(a, b.c1), mmul(a, b.c2)); }
MG_HD M3 m3t(M3 a) {
    return m3cols(v3(a.c0.x, a.c1.x, a.c2.x), v3(a.c0.y, a.c1.y, a.c2.y), v3(a.c0.z, a.c1.z, a.c2.z));
}
// skew(r) u = r x u
MG_HD M3 m3skew(V3 r) { return m3cols(v3(0.0f, r.z, -r.y), v3(-r.z, 0.0f, r.x), v3(r.y, -r.x, 0.0f)); }
// a b^T * s
MG_HD M3 m3outer(V3 a, V3 b, float s) {
    return m3cols(vscale(a, b.x * s), vscale(a, b.y * s), vscale(a, b.z * s));
}

// I m
MG_HD SV si_mul(SI I, SV m) {
    return sv(vadd(mmul(I.A, m.w), mmul(I.B, m.v)), vadd(mtmul(I.B, m.w), mmul(I.C, m.v)));
}
// X m
MG_HD SV x_motion(M3 E, V3 r, SV m) { return sv(mmul(E, m.w), mmul(E, vsub(m.v, vcross(r, m.w)))); }
// X^T f (child force -> parent coordinates)
MG_HD SV x_force_t(M3 E, V3 r, SV f) {
    V3 n = mtmul(E, f.w);
    V3 fo = mtmul(E, f.v);
    return sv(vadd(n, vcross(r, fo)), fo);
}
// X^T I X (child inertia -> parent coordinates)
MG_HD SI x_inertia_t(M3 E, V3 r, SI I) {
    M3 Et = m3t(E);
    M3 A = m3mul(m3mul(Et, I.A), E);
    M3 B = m3mul(m3mul(Et, I.B), E);
    M3 C = m3mul(m3mul(Et, I.C), E);
    M3 rx = m3skew(r);
    SI o;
    o.A = m3add(m3sub(A, m3mul(B, rx)), m3sub(m3mul(rx, m3t(B)), m3mul(m3mul(rx, C), rx)));
    o.B = m3add(B, m3mul(rx, C));
    o.C = C;
    return o;
}
MG_HD SI si_add(SI a, SI b) { SI o; o.A = m3add(a.A, b.A); o.B = m3add(a.B, b.B); o.C = m3add(a.C, b.C); return o; }
// rigid-body spatial inertia about the link origin: mass m, COM c, rotational
// inertia Ic about the COM (link coordinates)
MG_HD SI si_rigid(float m, V3 c, M3 Ic) {
    SI o;
    float cc = vdot(c, c);
    M3 ccT = m3outer(c, c, m);
    M3 diag = m3cols(v3(m * cc, 0.0f, 0.0f), v3(0.0f, m * cc, 0.0f), v3(0.0f, 0.0f, m * cc));
    o.A = m3add(Ic, m3sub(diag, ccT));
    o.B = m3skew(vscale(c, m));
    o.C = m3cols(v3(m, 0.0f, 0.0f), v3(0.0f, m, 0.0f), v3(0.0f, 0.0f, m));
    return o;
}
// rotation about unit axis a by angle th, as a quaternion (uses mg_sincos)
MG_HD Q4 q_axis_angle(V3 a, float th) {
    float s, c;
    float half = 0.5f * th;
    float ah = half < 0.0f ? -half : half;
    mg_sincos(ah, &s, &c);
    if (half < 0.0f) s = -s;
    return q4(a.x * s, a.y * s, a.z * s, c);
}

// ---- spherical (ball) joints in exponential coordinates ---------------------
// A ball joint's three DOF positions are the rotation vector th of the child
// joint frame relative to the parent's (test13_camera_spherical_joint.py:
// 243-256 feeds targets through quat2expcoord), its velocities the relative
// angular velocity in the child frame. It is packed as three revolute kernel
// links about x, y, z (include/migym.h MG_LINK_F_N: link_f[10] = 1, 2, 3 is the
// link's place in the ball): the first link's joint rotation is exp(th), the
// other two turn by nothing, so the three motion axes are the child frame's
// x, y, z and the three DOF rates its angular velocity components. No
// gimbal lock: the coordinates are never Euler angles.
// Only + - * / and sqrt (correctly rounded on both sides): oracle/migym_oracle.c
// restates each function op for op.
MG_HD Q4 q_exp(V3 th) {
    const float t2 = vdot(th, th);
    if (!(t2 > 0.0f)) return q4(0.0f, 0.0f, 0.0f, 1.0f);
    const float t = sqrtf(t2);
    float s, c;
    mg_sincos(0.5f * t, &s, &c);
    const float k = s / t;
    return q4(th.x * k, th.y * k, th.z * k, c);
}
// atan(u) on |u| <= tan(pi/8): odd Taylor series to u^19 (error < 5e-10)
MG_HD float mg_atan_small(float u) {
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
// atan(t) on [0, 1]: atan t = pi/4 + atan((t - 1) / (t + 1)) above tan(pi/8)
MG_HD float mg_atan01(float t) {
    if (t > 0.41421356f) return 0.78539816f + mg_atan_small((t - 1.0f) / (t + 1.0f));
    return mg_atan_small(t);
}
// rotation vector of a unit quaternion (the rotation angle in [0, pi])
MG_HD V3 q_log(Q4 q) {
    if (q.w < 0.0f) q = q4(-q.x, -q.y, -q.z, -q.w);
    const float v2 = q.x * q.x + q.y * q.y + q.z * q.z;
    if (!(v2 > 0.0f)) return v3(0.0f, 0.0f, 0.0f);
    const float vn = sqrtf(v2);
    // half angle = atan2(vn, w), vn > 0, w >= 0
    const float ha = vn <= q.w ? mg_atan01(vn / q.w) : 1.57079633f - mg_atan01(q.w / vn);
    const float k = (2.0f * ha) / vn;
    return v3(q.x * k, q.y * k, q.z * k);
}
// a ball joint turned by dth (child frame): log(exp(th) exp(dth))
MG_HD V3 ball_step(V3 th, V3 dth) { return q_log(qnormalize(qmul(q_exp(th), q_exp(dth)))); }
// link l's joint rotation qrel and offset rr from its origin (po, qo), axis ax
// and the DOF positions q (indexed by local DOF): revolute, prismatic, or a ball
// joint's first link (exp of its three DOFs) / later links (no turn)
MG_HD void link_joint(int jt, int ball, V3 po, Q4 qo, V3 ax, const float* q, int dof, Q4& qrel, V3& rr) {
    qrel = qo;
    rr = po;
    if (ball == 1) qrel = qmul(qo, q_exp(v3(q[dof], q[dof + 1], q[dof + 2])));
    else if (ball > 1) qrel = qo;
    else if (jt == MG_JOINT_REVOLUTE) qrel = qmul(qo, q_axis_angle(ax, dof >= 0 ? q[dof] : 0.0f));
    else if (jt == MG_JOINT_PRISMATIC) rr = vadd(po, qrot(qo, vscale(ax, dof >= 0 ? q[dof] : 0.0f)));
}
