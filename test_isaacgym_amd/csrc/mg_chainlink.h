// mg_chainlink.h — a chain link's mass constants (k_artic_chain, mg_chain.hip):
// mass, COM and the rotational inertia about the COM in link axes (symmetric:
// xx, yy, zz, xy, xz, yz), from a body's MG_MASS_N row (inverse principal
// moments, principal frame iq, COM, mass). Host and device: migym_capi.cpp
// builds a template's constants once when all its instances share them (the
// kernel then reads them as wave-uniform scalars), the kernel per lane
// otherwise — the same expressions, so the same bits (oracle/migym_oracle.c
// chain_step_ restates them).
#pragma once
#include "mg_math.h"

#define MG_CHAIN_UNI_N    64   // uniform constants of a chain group: 3 links x 10, 3 DOFs x 9, gravity flag
#define MG_CHAIN_UNI_LINK 0    // + (l - 1) * 10: m, com.xyz, ib[6]
#define MG_CHAIN_UNI_DOF  30   // + d * 9: mode, kp, kd, effort, max_vel, lower, upper, has_limits, armature
#define MG_CHAIN_UNI_DOFOK 62  // 1: the DOF constants above are valid (every instance shares them);
                               // cleared by a later set_actor_dof_properties that makes them differ
#define MG_CHAIN_UNI_GRAV 63   // the base body's gravity flag

struct ChainLink {
    float m;
    V3 com;
    float ib[6];
};

MG_HD ChainLink chain_link_make(float m, V3 com, float ix, float iy, float iz, Q4 iq) {
    ChainLink k;
    k.m = m;
    k.com = com;
    const M3 R = qmat(iq);
    const V3 u0 = vscale(R.c0, ix > 0.0f ? 1.0f / ix : 0.0f);
    const V3 u1 = vscale(R.c1, iy > 0.0f ? 1.0f / iy : 0.0f);
    const V3 u2 = vscale(R.c2, iz > 0.0f ? 1.0f / iz : 0.0f);
    k.ib[0] = fmaf(u0.x, R.c0.x, fmaf(u1.x, R.c1.x, u2.x * R.c2.x));
    k.ib[1] = fmaf(u0.y, R.c0.y, fmaf(u1.y, R.c1.y, u2.y * R.c2.y));
    k.ib[2] = fmaf(u0.z, R.c0.z, fmaf(u1.z, R.c1.z, u2.z * R.c2.z));
    k.ib[3] = fmaf(u0.x, R.c0.y, fmaf(u1.x, R.c1.y, u2.x * R.c2.y));
    k.ib[4] = fmaf(u0.x, R.c0.z, fmaf(u1.x, R.c1.z, u2.x * R.c2.z));
    k.ib[5] = fmaf(u0.y, R.c0.z, fmaf(u1.y, R.c1.z, u2.y * R.c2.z));
    return k;
}
