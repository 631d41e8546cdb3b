// mg_pairs.h — shape placement, the ground plane's contacts and the pair
// screen shared by the coupled per-env step (mg_env.hip) and the free-body
// pile step (mg_pile.hip). Part of the narrow phase's definition: restated
// by oracle/migym_oracle_env.c (place_, ground_pair_, pair_near_, tangents_).
#pragma once
#include "mg_internal.h"
#include "mg_collide.h"

// the pairs convex_convex handles (collide's dispatch): box / hull against box /
// hull, at least one hull (box-box is SAT)
MG_HD bool cvx_pair(int ta, int tb) {
    const bool pa = ta == MG_SHAPE_BOX || ta == MG_SHAPE_CONVEX, pb = tb == MG_SHAPE_BOX || tb == MG_SHAPE_CONVEX;
    return pa && pb && (ta == MG_SHAPE_CONVEX || tb == MG_SHAPE_CONVEX);
}

MG_HD void env_tangents(V3 n, V3* t1, V3* t2) {
    V3 a = v3(1.0f, 0.0f, 0.0f);
    if (!(fabsf(n.x) < 0.9f)) a = v3(0.0f, 1.0f, 0.0f);
    V3 t = vcross(n, a);
    const float inv = 1.0f / sqrtf(vdot(t, t));
    t = vscale(t, inv);
    *t1 = t;
    *t2 = vcross(n, t);
}

MG_HD CShape place_shape(const float* sh, V3 x, Q4 q, const float* hulls) {
    CShape c;
    c.type = (int)sh[0];
    c.c = vadd(x, qrot(q, v3(sh[4], sh[5], sh[6])));
    c.R = qmat(qmul(q, q4(sh[7], sh[8], sh[9], sh[10])));
    c.h = v3(sh[1], sh[2], sh[3]);
    c.hv = c.type == MG_SHAPE_CONVEX ? hulls + (int)sh[2] : nullptr;
    return c;
}

// contacts of a placed shape with the ground plane (as mg_rigid.hip: the four
// corners of the box face most opposed to n, sphere, capsule end caps, the 4
// deepest hull vertices)
MG_HD void ground_pair(const MgStep& P, const CShape& s, PairOut& o) {
    const V3 n = v3(P.n[0], P.n[1], P.n[2]);
    const float off = P.contact_offset;
    if (s.type == MG_SHAPE_CONVEX) {
        Deep4 D;
        D.n = 0;
        const int nv = cvx_nv(s);
        const float* V = s.hv + MG_HULL_HEADER;           // vertices streamed 4 ahead
        V3 r0 = hull_vl(V, nv, 0), r1 = hull_vl(V, nv, 1), r2 = hull_vl(V, nv, 2), r3 = hull_vl(V, nv, 3);
        for (int i = 0; i < nv; ++i) {
            const V3 l = r0;
            r0 = r1; r1 = r2; r2 = r3;
            r3 = hull_vl(V, nv, i + 4);
            const V3 p = vadd(s.c, mmul(s.R, l));          // cvx_vertex(s, i)
            const float sep = vdot(n, p) + P.pd;
            if (sep < off) deep4_add(D, sep, p, n);
        }
        deep4_emit(D, o);
    } else if (s.type == MG_SHAPE_BOX) {
        const float d0 = vdot(n, s.R.c0), d1 = vdot(n, s.R.c1), d2 = vdot(n, s.R.c2);
        const float ad0 = fabsf(d0), ad1 = fabsf(d1), ad2 = fabsf(d2);
        int ia = 0;
        float best = ad0;
        if (ad1 > best) { ia = 1; best = ad1; }
        if (ad2 > best) ia = 2;
        const V3 a0 = vscale(s.R.c0, s.h.x), a1 = vscale(s.R.c1, s.h.y), a2 = vscale(s.R.c2, s.h.z);
        const float di = ia == 0 ? d0 : (ia == 1 ? d1 : d2);
        const V3 ai = vsel(ia == 0, a0, vsel(ia == 1, a1, a2));
        const V3 e1 = vsel(ia == 0, a1, a0);
        const V3 e2 = vsel(ia == 2, a1, a2);
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

// radius of a sphere around the shape centre enclosing the shape
MG_HD float bound_radius(const float* sh) {
    const int t = (int)sh[0];
    if (t == MG_SHAPE_BOX) return sqrtf(sh[1] * sh[1] + sh[2] * sh[2] + sh[3] * sh[3]);
    if (t == MG_SHAPE_CAPSULE) return sh[1] + sh[2];
    return sh[1];
}


// Pair screen (part of the narrow phase's definition; the oracle applies the
// same test): a pair can only produce contacts when the bounding sphere of A
// (centre cA, radius rA) comes within the contact offset of the ground plane,
// of B's bounding sphere, and — when B (or A) is a box — of that box itself.
MG_HD bool sphere_near_box(V3 c, float r, const float* shb, V3 xb, Q4 qb, float off) {
    const V3 cb = vadd(xb, qrot(qb, v3(shb[4], shb[5], shb[6])));
    const M3 Rb = qmat(qmul(qb, q4(shb[7], shb[8], shb[9], shb[10])));
    const V3 loc = mtmul(Rb, vsub(c, cb));
    const V3 e = v3(loc.x - fminf(fmaxf(loc.x, -shb[1]), shb[1]), loc.y - fminf(fmaxf(loc.y, -shb[2]), shb[2]),
                    loc.z - fminf(fmaxf(loc.z, -shb[3]), shb[3]));
    const float rr = r + off;
    return vdot(e, e) < rr * rr * 1.0001f + 1e-6f;
}
// Oriented boxes of two box / hull shapes (ob: the shape-frame box of the
// shape, centre then half extents, migym_capi.cpp shape_obb) separated along one
// of their six face axes by more than the contact offset (plus a rounding
// slack): no point of one comes within the offset of the other, so neither
// convex_convex's vertex nor its edge pass can place a contact. A bounding
// sphere is loose around a long Franka link hull; half of the hull pairs that
// passed the sphere screens had no contact (profiles/r03_env_phase_p.json).
MG_HD bool obb_apart(const float* sha, V3 xa, Q4 qa, const float* oa, const float* shb, V3 xb, Q4 qb,
                     const float* ob, float off) {
    const M3 Ra = qmat(qmul(qa, q4(sha[7], sha[8], sha[9], sha[10])));
    const M3 Rb = qmat(qmul(qb, q4(shb[7], shb[8], shb[9], shb[10])));
    const V3 ca = vadd(vadd(xa, qrot(qa, v3(sha[4], sha[5], sha[6]))), mmul(Ra, v3(oa[0], oa[1], oa[2])));
    const V3 cb = vadd(vadd(xb, qrot(qb, v3(shb[4], shb[5], shb[6]))), mmul(Rb, v3(ob[0], ob[1], ob[2])));
    const V3 ea = v3(oa[3], oa[4], oa[5]), eb = v3(ob[3], ob[4], ob[5]);
    const V3 d = vsub(cb, ca);
    const float slack = off + 1e-5f * (1.0f + (ea.x + ea.y + ea.z) + (eb.x + eb.y + eb.z) +
                                       (fabsf(d.x) + fabsf(d.y) + fabsf(d.z)));
    const V3 A3[3] = {Ra.c0, Ra.c1, Ra.c2}, B3[3] = {Rb.c0, Rb.c1, Rb.c2};
    const float eA[3] = {ea.x, ea.y, ea.z}, eB[3] = {eb.x, eb.y, eb.z};
    float C[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[i][j] = fabsf(vdot(A3[i], B3[j]));
    bool apart = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float rb = eB[0] * C[i][0] + eB[1] * C[i][1] + eB[2] * C[i][2];
        apart = apart || fabsf(vdot(d, A3[i])) > eA[i] + rb + slack;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float ra = eA[0] * C[0][j] + eA[1] * C[1][j] + eA[2] * C[2][j];
        apart = apart || fabsf(vdot(d, B3[j])) > eB[j] + ra + slack;
    }
    return apart;
}
MG_HD bool pair_near(const MgStep& P, const float* sha, V3 xa, Q4 qa, const float* shb, V3 xb, Q4 qb, bool ground,
                     const float* oa, const float* ob) {
    const V3 cA = vadd(xa, qrot(qa, v3(sha[4], sha[5], sha[6])));
    const float rA = bound_radius(sha);
    if (ground) return vdot(v3(P.n[0], P.n[1], P.n[2]), cA) + P.pd - rA < P.contact_offset;
    const V3 cB = vadd(xb, qrot(qb, v3(shb[4], shb[5], shb[6])));
    const float rB = bound_radius(shb);
    const V3 d = vsub(cB, cA);
    const float rr = rA + rB + P.contact_offset;
    if (!(vdot(d, d) < rr * rr * 1.0001f + 1e-6f)) return false;
    if ((int)shb[0] == MG_SHAPE_BOX && !sphere_near_box(cA, rA, shb, xb, qb, P.contact_offset)) return false;
    if ((int)sha[0] == MG_SHAPE_BOX && !sphere_near_box(cB, rB, sha, xa, qa, P.contact_offset)) return false;
    if (oa && cvx_pair((int)sha[0], (int)shb[0]) && obb_apart(sha, xa, qa, oa, shb, xb, qb, ob, P.contact_offset))
        return false;
    return true;
}
