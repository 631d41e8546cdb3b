// mg_world.h — world-frame spatial quantities shared by the articulated-body
// kernels (mg_env.hip k_env_step / k_artic_lanes / k_artic_chain, mg_artic.hip k_artic_jac_mm): 6-vectors as
// float[6] (angular, linear), link mass constants, and the world-frame spatial
// inertia of a link about a point. Restated in oracle/migym_oracle_env.c.
#pragma once
#include "mg_internal.h"
#include "mg_spatial.h"

// link l's mass properties, loaded once per kernel (principal inertia inverted)
struct LinkC {
    float m, Idx, Idy, Idz;
    V3 com;
    Q4 iq;
};

// fused multiply-add chain (fmaf is correctly rounded on both sides: the
// oracle's dot6_ is the same chain)
MG_HD float dot6(const float* a, const float* b) {
    return fmaf(a[5], b[5], fmaf(a[4], b[4], fmaf(a[3], b[3], fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])))));
}
MG_HD SV sv6(const float* a) { return sv(v3(a[0], a[1], a[2]), v3(a[3], a[4], a[5])); }
MG_HD void put6(float* a, SV s) { a[0] = s.w.x; a[1] = s.w.y; a[2] = s.w.z; a[3] = s.v.x; a[4] = s.v.y; a[5] = s.v.z; }

__device__ __forceinline__ LinkC load_link(const float* Ms, int nb, int b) {
    LinkC k;
    k.m = Ms[11 * nb + b];
    k.com = v3(Ms[8 * nb + b], Ms[9 * nb + b], Ms[10 * nb + b]);
    k.iq = q4(Ms[4 * nb + b], Ms[5 * nb + b], Ms[6 * nb + b], Ms[7 * nb + b]);
    const float ix = Ms[1 * nb + b], iy = Ms[2 * nb + b], iz = Ms[3 * nb + b];
    k.Idx = ix > 0.0f ? 1.0f / ix : 0.0f;
    k.Idy = iy > 0.0f ? 1.0f / iy : 0.0f;
    k.Idz = iz > 0.0f ? 1.0f / iz : 0.0f;
    return k;
}

// world-frame spatial inertia of link body b about the point O: row-major 6x6
// [A B; B^T C] with A = Ic + m (|c|^2 1 - c c^T), B = [m c]x, C = m 1
// (c = COM - O, Ic the rotational inertia about the COM in world axes)
MG_HD void world_inertia(const LinkC& K, Q4 ql, V3 xl, V3 O, float* I) {
    const float m = K.m;
    const V3 com = K.com;
    const Q4 iq = K.iq;
    const V3 Id = v3(K.Idx, K.Idy, K.Idz);
    const S3 Ic = sym_rdrt(qmat(qmul(ql, iq)), Id);
    const V3 c = vsub(vadd(xl, qrot(ql, com)), O);
    const float cc2 = vdot(c, c);
    const float ic[9] = {Ic.xx, Ic.xy, Ic.xz, Ic.xy, Ic.yy, Ic.yz, Ic.xz, Ic.yz, Ic.zz};
    const float cv[3] = {c.x, c.y, c.z};
    const V3 mc = vscale(c, m);
    const float sk[9] = {0.0f, -mc.z, mc.y, mc.z, 0.0f, -mc.x, -mc.y, mc.x, 0.0f};   // [m c]x, row-major
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
            const float dg = i == k ? m * cc2 : 0.0f;
            I[i * 6 + k] = ic[i * 3 + k] + (dg - cv[i] * (cv[k] * m));
            I[i * 6 + 3 + k] = sk[i * 3 + k];
            I[(3 + i) * 6 + k] = sk[k * 3 + i];
            I[(3 + i) * 6 + 3 + k] = i == k ? m : 0.0f;
        }
}

