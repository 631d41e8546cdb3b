// mg_math.h — fp32 vector/quaternion helpers for the HIP kernels.
//
// Every helper fixes its evaluation order (left-to-right sums, no FMA: the
// build uses -ffp-contract=off) so oracle/migym_oracle.c, which restates the
// same formulas in plain C, matches the device bit for bit.
// Quaternions are (x, y, z, w), as in Isaac Gym's tensors.
#pragma once
#include <hip/hip_runtime.h>

#define MG_HD __host__ __device__ __forceinline__

struct V3 { float x, y, z; };
struct Q4 { float x, y, z, w; };
struct M3 { V3 c0, c1, c2; };          // column-major 3x3

MG_HD V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
// c ? a : b per component: value selects (a ternary on V3 objects selects their
// addresses, which keeps them in scratch memory on the device)
MG_HD V3 vsel(bool c, V3 a, V3 b) { return v3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
MG_HD V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
MG_HD V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
MG_HD V3 vscale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
MG_HD float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
MG_HD V3 vcross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// a + b * s
MG_HD V3 vmad(V3 a, V3 b, float s) { return v3(a.x + b.x * s, a.y + b.y * s, a.z + b.z * s); }

MG_HD Q4 q4(float x, float y, float z, float w) { Q4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
MG_HD Q4 qmul(Q4 a, Q4 b) {
    return q4(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
              a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
              a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w,
              a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
MG_HD Q4 qconj(Q4 a) { return q4(-a.x, -a.y, -a.z, a.w); }
MG_HD Q4 qnormalize(Q4 a) {
    float n2 = a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    if (!(n2 > 0.0f)) return q4(0.0f, 0.0f, 0.0f, 1.0f);
    float inv = 1.0f / sqrtf(n2);
    return q4(a.x * inv, a.y * inv, a.z * inv, a.w * inv);
}
// rotate v by q: v + w t + u x t, t = 2 u x v
MG_HD V3 qrot(Q4 q, V3 v) {
    float tx = 2.0f * (q.y * v.z - q.z * v.y);
    float ty = 2.0f * (q.z * v.x - q.x * v.z);
    float tz = 2.0f * (q.x * v.y - q.y * v.x);
    return v3(v.x + q.w * tx + (q.y * tz - q.z * ty),
              v.y + q.w * ty + (q.z * tx - q.x * tz),
              v.z + q.w * tz + (q.x * ty - q.y * tx));
}
MG_HD V3 qrot_inv(Q4 q, V3 v) { return qrot(qconj(q), v); }
MG_HD M3 qmat(Q4 q) {
    float xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    float xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z;
    float wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
    M3 m;
    m.c0 = v3(1.0f - 2.0f * (yy + zz), 2.0f * (xy + wz), 2.0f * (xz - wy));
    m.c1 = v3(2.0f * (xy - wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz + wx));
    m.c2 = v3(2.0f * (xz + wy), 2.0f * (yz - wx), 1.0f - 2.0f * (xx + yy));
    return m;
}
MG_HD V3 mmul(M3 m, V3 u) {
    return v3(m.c0.x * u.x + m.c1.x * u.y + m.c2.x * u.z,
              m.c0.y * u.x + m.c1.y * u.y + m.c2.y * u.z,
              m.c0.z * u.x + m.c1.z * u.y + m.c2.z * u.z);
}
MG_HD V3 mtmul(M3 m, V3 v) { return v3(vdot(m.c0, v), vdot(m.c1, v), vdot(m.c2, v)); }
// world inverse inertia applied to v: Rp diag(invI) Rp^T v
MG_HD V3 inv_inertia_w(M3 Rp, V3 invI, V3 v) {
    V3 u = mtmul(Rp, v);
    u = v3(u.x * invI.x, u.y * invI.y, u.z * invI.z);
    return mmul(Rp, u);
}

// symmetric 3x3 (world inverse inertia)
struct S3 { float xx, yy, zz, xy, xz, yz; };
// Rp diag(d) Rp^T, Rp given by its columns
MG_HD S3 sym_rdrt(M3 Rp, V3 d) {
    const V3 u0 = vscale(Rp.c0, d.x), u1 = vscale(Rp.c1, d.y), u2 = vscale(Rp.c2, d.z);
    S3 s;
    s.xx = u0.x * Rp.c0.x + u1.x * Rp.c1.x + u2.x * Rp.c2.x;
    s.yy = u0.y * Rp.c0.y + u1.y * Rp.c1.y + u2.y * Rp.c2.y;
    s.zz = u0.z * Rp.c0.z + u1.z * Rp.c1.z + u2.z * Rp.c2.z;
    s.xy = u0.x * Rp.c0.y + u1.x * Rp.c1.y + u2.x * Rp.c2.y;
    s.xz = u0.x * Rp.c0.z + u1.x * Rp.c1.z + u2.x * Rp.c2.z;
    s.yz = u0.y * Rp.c0.z + u1.y * Rp.c1.z + u2.y * Rp.c2.z;
    return s;
}
MG_HD V3 symmul(S3 s, V3 v) {
    return v3(s.xx * v.x + s.xy * v.y + s.xz * v.z,
              s.xy * v.x + s.yy * v.y + s.yz * v.z,
              s.xz * v.x + s.yz * v.y + s.zz * v.z);
}

// sin / cos of a half angle by Taylor series on |x| <= 0.5 with double-angle
// reconstruction: only + - * / so host and device round identically.
MG_HD void mg_sincos(float x, float* s_out, float* c_out) {
    int k = 0;
    while (x > 0.5f && k < 24) { x = x * 0.5f; k = k + 1; }
    float x2 = x * x;
    float s = x * (1.0f - x2 * (1.0f / 6.0f) * (1.0f - x2 * (1.0f / 20.0f) * (1.0f - x2 * (1.0f / 42.0f) * (1.0f - x2 * (1.0f / 72.0f)))));
    float c = 1.0f - x2 * 0.5f * (1.0f - x2 * (1.0f / 12.0f) * (1.0f - x2 * (1.0f / 30.0f) * (1.0f - x2 * (1.0f / 56.0f) * (1.0f - x2 * (1.0f / 90.0f)))));
    for (int i = 0; i < k; ++i) {
        float s2 = 2.0f * s * c;
        float c2 = c * c - s * s;
        s = s2; c = c2;
    }
    *s_out = s; *c_out = c;
}
// q' = exp(dtheta) * q  (dtheta = rotation vector in world frame), normalised
MG_HD Q4 qintegrate(Q4 q, V3 dth) {
    float th2 = vdot(dth, dth);
    if (!(th2 > 0.0f)) return q;
    float th = sqrtf(th2);
    float s, c;
    mg_sincos(0.5f * th, &s, &c);
    float k = s / th;
    Q4 dq = q4(dth.x * k, dth.y * k, dth.z * k, c);
    return qnormalize(qmul(dq, q));
}
