// mg_collide.h — narrow phase for the per-env step (mg_env.hip): contacts
// between two convex primitives (box, sphere, capsule) in world space.
//
// Output convention: each contact is (point p on shape A, unit normal n pointing
// from B towards A, separation sep — negative when penetrating). Boxes are
// (centre, rotation columns, half extents); spheres (centre, radius); capsules
// (centre, axis = local x, radius, half height): their two end-cap spheres plus,
// against a box or hull, the axis segment clipped by the shape's planes pushed
// out by radius + margin (one contact at the chord — at a box edge the
// edge-edge contact), against a sphere or capsule the closest points of the
// axis segments (round 4; round 3 had the caps only).
// Convex hulls (MG_SHAPE_CONVEX, the importer's hull of a mesh, at most
// MG_HULL_MAX_VERTS vertices) against boxes and hulls: vertex penetration both
// ways — every vertex of one shape within the margin of the other, by the
// other's face planes (signed distance = the largest plane distance, the face
// attaining it gives the normal) — the 4 deepest kept; against spheres /
// capsule caps: the centre's plane distance. With no vertex within the margin:
// edge crossings, the non-box shape's edges clipped against the other's planes,
// one candidate per chord — the edge-edge contact near a box edge, else the
// chord's midpoint by the planes (cvx_edges_vs).
// Box–box is SAT over the 15 axes (face axes preferred unless an edge axis
// separates by more than 1e-3 m), then Sutherland–Hodgman clipping of the
// incident face against the reference face (at most 8 points, the 4 deepest
// kept, ties by index); edge–edge gives one contact at the closest points.
// Fixed evaluation order, no FMA: oracle/migym_oracle_env.c restates it.
#pragma once
#include "mg_math.h"

#define MG_PAIR_MAXC 4

struct CShape {      // a primitive placed in the world
    int type;        // MG_SHAPE_*
    V3 c;            // centre
    M3 R;            // orientation (columns = local axes)
    V3 h;            // box half extents | (radius, half height, -) for sphere / capsule
    const float* hv; // convex: its hull record (MG_HULL_HEADER + 3 nv + 4 nf floats), else null
};

struct PairOut {
    int n;
    V3 p[MG_PAIR_MAXC];
    V3 nrm[MG_PAIR_MAXC];
    float sep[MG_PAIR_MAXC];
};

MG_HD V3 m3col(const M3& R, int i) { return vsel(i == 0, R.c0, vsel(i == 1, R.c1, R.c2)); }
MG_HD float m3c(const M3& R, int i, int k) {      // component k of column i
    const V3 c = m3col(R, i);
    return k == 0 ? c.x : (k == 1 ? c.y : c.z);
}
MG_HD float v3c(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// static slot writes (no dynamic indexing: the record stays in registers)
MG_HD void pair_push(PairOut& o, V3 p, V3 n, float sep) {
#pragma unroll
    for (int k = 0; k < MG_PAIR_MAXC; ++k) {
        const bool put = o.n == k;
        o.p[k] = vsel(put, p, o.p[k]);
        o.nrm[k] = vsel(put, n, o.nrm[k]);
        o.sep[k] = put ? sep : o.sep[k];
    }
    if (o.n < MG_PAIR_MAXC) o.n = o.n + 1;
}

// sphere A (centre a, radius ra) vs sphere B
MG_HD void sphere_sphere(V3 a, float ra, V3 b, float rb, float margin, PairOut& o) {
    const V3 d = vsub(a, b);
    const float l2 = vdot(d, d);
    const float l = sqrtf(l2);
    const float sep = l - ra - rb;
    if (!(sep < margin)) return;
    V3 n = l > 1e-9f ? vscale(d, 1.0f / l) : v3(0.0f, 0.0f, 1.0f);
    pair_push(o, vsub(a, vscale(n, ra)), n, sep);
}

// sphere A vs box B
MG_HD void sphere_box(V3 s, float r, const CShape& B, float margin, PairOut& o) {
    const V3 d = vsub(s, B.c);
    const V3 loc = mtmul(B.R, d);
    const float hx = B.h.x, hy = B.h.y, hz = B.h.z;
    const float qx = fminf(fmaxf(loc.x, -hx), hx);
    const float qy = fminf(fmaxf(loc.y, -hy), hy);
    const float qz = fminf(fmaxf(loc.z, -hz), hz);
    const bool inside = loc.x == qx && loc.y == qy && loc.z == qz;
    V3 n;
    float sep;
    if (!inside) {
        const V3 dq = mmul(B.R, v3(loc.x - qx, loc.y - qy, loc.z - qz));
        const float l = sqrtf(vdot(dq, dq));
        sep = l - r;
        if (!(sep < margin)) return;
        n = vscale(dq, 1.0f / l);
    } else {
        // centre inside: leave through the nearest face
        const float px = hx - fabsf(loc.x), py = hy - fabsf(loc.y), pz = hz - fabsf(loc.z);
        int ax = 0;
        float pen = px;
        if (py < pen) { ax = 1; pen = py; }
        if (pz < pen) { ax = 2; pen = pz; }
        const float sg = v3c(loc, ax) < 0.0f ? -1.0f : 1.0f;
        n = vscale(m3col(B.R, ax), sg);
        sep = -pen - r;
    }
    pair_push(o, vsub(s, vscale(n, r)), n, sep);
}

// box A vs box B
MG_HD void box_box(const CShape& A, const CShape& B, float margin, PairOut& o) {
    const V3 d = vsub(B.c, A.c);               // A -> B
    float Rm[3][3], AbsR[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Rm[i][j] = vdot(m3col(A.R, i), m3col(B.R, j));
            AbsR[i][j] = fabsf(Rm[i][j]) + 1e-6f;
        }
    const float ha[3] = {A.h.x, A.h.y, A.h.z};
    const float hb[3] = {B.h.x, B.h.y, B.h.z};
    const float t[3] = {vdot(d, A.R.c0), vdot(d, A.R.c1), vdot(d, A.R.c2)};
    // face axes
    float best_face = -1e30f;
    int face = 0;
    for (int i = 0; i < 3; ++i) {
        const float rb = hb[0] * AbsR[i][0] + hb[1] * AbsR[i][1] + hb[2] * AbsR[i][2];
        const float sep = fabsf(t[i]) - ha[i] - rb;
        if (sep > best_face) { best_face = sep; face = i; }
    }
    for (int j = 0; j < 3; ++j) {
        const float ra = ha[0] * AbsR[0][j] + ha[1] * AbsR[1][j] + ha[2] * AbsR[2][j];
        const float tb = t[0] * Rm[0][j] + t[1] * Rm[1][j] + t[2] * Rm[2][j];
        const float sep = fabsf(tb) - hb[j] - ra;
        if (sep > best_face) { best_face = sep; face = 3 + j; }
    }
    if (!(best_face < margin)) return;
    // edge axes
    float best_edge = -1e30f;
    int ei = -1, ej = -1;
    V3 eaxis = v3(0.0f, 0.0f, 0.0f);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            V3 ax = vcross(m3col(A.R, i), m3col(B.R, j));
            const float l2 = vdot(ax, ax);
            if (!(l2 > 1e-6f)) continue;
            ax = vscale(ax, 1.0f / sqrtf(l2));
            const float ra = ha[0] * fabsf(vdot(ax, A.R.c0)) + ha[1] * fabsf(vdot(ax, A.R.c1)) + ha[2] * fabsf(vdot(ax, A.R.c2));
            const float rb = hb[0] * fabsf(vdot(ax, B.R.c0)) + hb[1] * fabsf(vdot(ax, B.R.c1)) + hb[2] * fabsf(vdot(ax, B.R.c2));
            const float sep = fabsf(vdot(d, ax)) - ra - rb;
            if (!(sep < margin)) return;         // a separating axis: no contact
            if (sep > best_edge) { best_edge = sep; ei = i; ej = j; eaxis = ax; }
        }
    if (ei >= 0 && best_edge > best_face + 1e-3f) {
        // edge-edge: closest points of the two supporting edges
        V3 ax = eaxis;
        if (vdot(ax, d) < 0.0f) ax = vscale(ax, -1.0f);      // A -> B
        V3 pa = A.c, pb = B.c;
        for (int k = 0; k < 3; ++k) {
            if (k != ei) pa = vadd(pa, vscale(m3col(A.R, k), vdot(ax, m3col(A.R, k)) > 0.0f ? ha[k] : -ha[k]));
            if (k != ej) pb = vadd(pb, vscale(m3col(B.R, k), vdot(ax, m3col(B.R, k)) > 0.0f ? -hb[k] : hb[k]));
        }
        const V3 ua = m3col(A.R, ei), ub = m3col(B.R, ej);
        const V3 w = vsub(pa, pb);
        const float b = vdot(ua, ub), dd = vdot(ua, w), e = vdot(ub, w);
        const float den = 1.0f - b * b;
        float sa = 0.0f, sb = 0.0f;
        if (den > 1e-6f) {
            sa = (b * e - dd) / den;
            sb = (e - b * dd) / den;
        }
        const float hae = v3c(A.h, ei), hbe = v3c(B.h, ej);
        sa = fminf(fmaxf(sa, -hae), hae);
        sb = fminf(fmaxf(sb, -hbe), hbe);
        const V3 ca = vadd(pa, vscale(ua, sa));
        const V3 cb = vadd(pb, vscale(ub, sb));
        pair_push(o, vscale(vadd(ca, cb), 0.5f), vscale(ax, -1.0f), best_edge);
        return;
    }
    // face contact: reference box / axis, incident box. The contact polygon is
    // the intersection of the incident face with the reference face, taken from a
    // fixed candidate set in the reference face's (u, v) frame: the incident
    // quad's corners inside the reference rectangle (0..3), the rectangle's
    // corners inside the quad (4..7), the crossings of quad edge k with
    // rectangle side j (8 + 4k + j); the 4 deepest within the margin are kept,
    // lowest index first on ties.
    const bool refA = face < 3;
    const CShape& Rf = refA ? A : B;
    const CShape& In = refA ? B : A;
    const int fa = refA ? face : face - 3;
    V3 nref = m3col(Rf.R, fa);                         // outward normal of the reference face, towards In
    if (vdot(vsub(In.c, Rf.c), nref) < 0.0f) nref = vscale(nref, -1.0f);
    int ik = 0;
    float bestd = 1e30f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float dk = -fabsf(vdot(nref, m3col(In.R, k)));
        if (dk < bestd) { bestd = dk; ik = k; }
    }
    const V3 iax = m3col(In.R, ik);
    const float hik = v3c(In.h, ik);
    const V3 ifc = vadd(In.c, vscale(iax, vdot(nref, iax) > 0.0f ? -hik : hik));
    const int iu = ik == 0 ? 1 : 0, iv = ik == 2 ? 1 : 2;
    const V3 eu = vscale(m3col(In.R, iu), v3c(In.h, iu)), ev = vscale(m3col(In.R, iv), v3c(In.h, iv));
    const int ru = fa == 0 ? 1 : 0, rv = fa == 2 ? 1 : 2;
    const V3 U = m3col(Rf.R, ru), W = m3col(Rf.R, rv);
    const float hu = v3c(Rf.h, ru), hv = v3c(Rf.h, rv);
    const V3 rc = vadd(Rf.c, vscale(nref, v3c(Rf.h, fa)));     // reference face centre
    float qx[4], qy[4];
    {
        const V3 q0 = vsub(vsub(ifc, eu), ev), q1 = vsub(vadd(ifc, eu), ev);
        const V3 q2 = vadd(vadd(ifc, eu), ev), q3 = vadd(vsub(ifc, eu), ev);
        qx[0] = vdot(vsub(q0, rc), U); qy[0] = vdot(vsub(q0, rc), W);
        qx[1] = vdot(vsub(q1, rc), U); qy[1] = vdot(vsub(q1, rc), W);
        qx[2] = vdot(vsub(q2, rc), U); qy[2] = vdot(vsub(q2, rc), W);
        qx[3] = vdot(vsub(q3, rc), U); qy[3] = vdot(vsub(q3, rc), W);
    }
    float cx[24], cy[24];
    unsigned cvalid = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        cx[k] = qx[k];
        cy[k] = qy[k];
        if (fabsf(qx[k]) <= hu && fabsf(qy[k]) <= hv) cvalid |= 1u << k;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const float X = (m & 1) ? hu : -hu, Y = (m & 2) ? hv : -hv;
        bool pos = true, neg = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int k2 = (k + 1) & 3;
            const float sk = (qx[k2] - qx[k]) * (Y - qy[k]) - (qy[k2] - qy[k]) * (X - qx[k]);
            pos = pos && sk >= 0.0f;
            neg = neg && sk <= 0.0f;
        }
        cx[4 + m] = X;
        cy[4 + m] = Y;
        if (pos || neg) cvalid |= 1u << (4 + m);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int k2 = (k + 1) & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 8 + 4 * k + j;
            const bool xs = j < 2;
            const float lim = xs ? (j == 0 ? hu : -hu) : (j == 2 ? hv : -hv);
            const float a0 = xs ? qx[k] : qy[k], a1 = xs ? qx[k2] : qy[k2];
            const float o0 = xs ? qy[k] : qx[k], o1 = xs ? qy[k2] : qx[k2];
            const float da = a0 - lim, db = a1 - lim;
            const bool ok = (da < 0.0f) != (db < 0.0f);
            const float t = ok ? da / (da - db) : 0.0f;
            const float ov = o0 + (o1 - o0) * t;
            cx[c] = xs ? lim : ov;
            cy[c] = xs ? ov : lim;
            if (ok && fabsf(ov) <= (xs ? hv : hu)) cvalid |= 1u << c;
        }
    }
    // depth of each candidate below the reference face (along nref, to the incident plane)
    const V3 inrm = vscale(iax, vdot(nref, iax) > 0.0f ? -1.0f : 1.0f);
    const float den = vdot(inrm, nref);
    const float iden = fabsf(den) > 1e-6f ? 1.0f / den : 0.0f;
    float cdep[24];
#pragma unroll
    for (int c = 0; c < 24; ++c) {
        const V3 q = vadd(vadd(rc, vscale(U, cx[c])), vscale(W, cy[c]));
        cdep[c] = vdot(vsub(ifc, q), inrm) * iden;
    }
    const V3 n = refA ? vscale(nref, -1.0f) : nref;    // from B towards A
    unsigned used = 0u;
#pragma unroll
    for (int m = 0; m < MG_PAIR_MAXC; ++m) {
        int bk = -1;
        float bd = margin, x = 0.0f, y = 0.0f;
#pragma unroll
        for (int c = 0; c < 24; ++c)
            if (((cvalid & ~used) >> c) & 1u)
                if (cdep[c] < bd) { bd = cdep[c]; bk = c; x = cx[c]; y = cy[c]; }
        if (bk >= 0) {
            used |= 1u << bk;
            const V3 q = vadd(vadd(rc, vscale(U, x)), vscale(W, y));     // on the reference plane
            const V3 pt = vadd(q, vscale(nref, bd));                    // on the incident face
            // the point lies on the incident box: on B when A is the reference, on A otherwise
            pair_push(o, refA ? vsub(pt, vscale(nref, bd)) : pt, n, bd);
        }
    }
}

// ---- convex shapes as vertices + face planes (a box: 8 corners, 6 faces)
MG_HD int cvx_nv(const CShape& S) { return S.type == MG_SHAPE_BOX ? 8 : (int)S.hv[0]; }
MG_HD int cvx_nf(const CShape& S) { return S.type == MG_SHAPE_BOX ? 6 : (int)S.hv[1]; }
MG_HD V3 cvx_vertex(const CShape& S, int i) {
    V3 l;
    if (S.type == MG_SHAPE_BOX) {
        l = v3((i & 1) ? S.h.x : -S.h.x, (i & 2) ? S.h.y : -S.h.y, (i & 4) ? S.h.z : -S.h.z);
    } else {
        const float* v = S.hv + MG_HULL_HEADER + 3 * i;
        l = v3(v[0], v[1], v[2]);
    }
    return vadd(S.c, mmul(S.R, l));
}
// local face plane f: outward unit normal nl, offset dl (n . x <= d inside)
MG_HD void cvx_plane_l(const CShape& S, int f, V3& nl, float& dl) {
    if (S.type == MG_SHAPE_BOX) {
        const int ax = f >> 1;
        const float sg = (f & 1) ? -1.0f : 1.0f;
        nl = v3(ax == 0 ? sg : 0.0f, ax == 1 ? sg : 0.0f, ax == 2 ? sg : 0.0f);
        dl = v3c(S.h, ax);
    } else {
        const float* pl = S.hv + MG_HULL_HEADER + 3 * (int)S.hv[0] + 4 * f;
        nl = v3(pl[0], pl[1], pl[2]);
        dl = pl[3];
    }
}
// signed distance of world point p to S by its face planes (largest plane
// distance; first face on ties), and that face. Callers only use a result with
// best - r < margin: the scan stops at the first face that makes that false
// (the maximum can only grow), which leaves every used result unchanged.
MG_HD float cvx_sd(const CShape& S, V3 p, int& fbest, float r, float margin) {
    const V3 pl = mtmul(S.R, vsub(p, S.c));
    const int nf = cvx_nf(S);
    float best = -1e30f;
    fbest = 0;
    if (S.type == MG_SHAPE_CONVEX) {
        // hull planes in batches of 4: the batch's loads are all in flight
        // before the in-order scan of its faces
        const float* P = S.hv + MG_HULL_HEADER + 3 * (int)S.hv[0];
        for (int f0 = 0; f0 < nf; f0 += 4) {
            float c[4][4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float* q = P + 4 * (f0 + k < nf ? f0 + k : nf - 1);
                c[k][0] = q[0]; c[k][1] = q[1]; c[k][2] = q[2]; c[k][3] = q[3];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (f0 + k < nf) {
                    const float s = vdot(v3(c[k][0], c[k][1], c[k][2]), pl) - c[k][3];
                    if (s > best) {
                        best = s;
                        fbest = f0 + k;
                        if (!(best - r < margin)) return best;
                    }
                }
            }
        }
        return best;
    }
    for (int f = 0; f < nf; ++f) {
        V3 nl;
        float dl;
        cvx_plane_l(S, f, nl, dl);
        const float s = vdot(nl, pl) - dl;
        if (s > best) {
            best = s;
            fbest = f;
            if (!(best - r < margin)) break;
        }
    }
    return best;
}
MG_HD V3 cvx_normal(const CShape& S, int f) {
    V3 nl;
    float dl;
    cvx_plane_l(S, f, nl, dl);
    return mmul(S.R, nl);
}

// the MG_PAIR_MAXC deepest candidates, ascending separation, earlier first on ties
struct Deep4 {
    int n;
    float s[MG_PAIR_MAXC];
    V3 p[MG_PAIR_MAXC], nrm[MG_PAIR_MAXC];
};
MG_HD void deep4_add(Deep4& D, float s, V3 p, V3 n) {
    if (D.n == MG_PAIR_MAXC && !(s < D.s[MG_PAIR_MAXC - 1])) return;
    int at = 0;
#pragma unroll
    for (int k = 0; k < MG_PAIR_MAXC; ++k)
        if (k < D.n && D.s[k] <= s) at = k + 1;
    // every slot through selects, top down (an indexed insert kept the record
    // in scratch)
#pragma unroll
    for (int k = MG_PAIR_MAXC - 1; k >= 0; --k) {
        const int km = k > 0 ? k - 1 : 0;
        const bool sh = k > at, put = k == at;
        D.s[k] = sh ? D.s[km] : (put ? s : D.s[k]);
        D.p[k] = vsel(sh, D.p[km], vsel(put, p, D.p[k]));
        D.nrm[k] = vsel(sh, D.nrm[km], vsel(put, n, D.nrm[k]));
    }
    if (D.n < MG_PAIR_MAXC) D.n = D.n + 1;
}
MG_HD void deep4_emit(const Deep4& D, PairOut& o) {
#pragma unroll
    for (int k = 0; k < MG_PAIR_MAXC; ++k)
        if (k < D.n) pair_push(o, D.p[k], D.nrm[k], D.s[k]);
}

// local vertex i of a hull (clamped to the last vertex: prefetch beyond the end)
MG_HD V3 hull_vl(const float* V, int n, int i) {
    const int j = i < n ? i : n - 1;
    return v3(V[3 * j], V[3 * j + 1], V[3 * j + 2]);
}

// the candidates of X's vertices against Y's face planes, in vertex order, into
// D: a vertex v within the margin (cvx_sd: the largest plane distance s, first
// face f on ties) gives (s, v, n_f) when the point is taken on X (onY false), or
// (s, v - n_f s, -n_f) on Y's face. A hull X streams its vertices 4 ahead.
// Also the bounds (lo, hi) of X's vertices in Y's frame (the face-axis test of
// the edge pass).
MG_HD void aabb_add(V3& lo, V3& hi, V3 v) {
    lo = v3(fminf(lo.x, v.x), fminf(lo.y, v.y), fminf(lo.z, v.z));
    hi = v3(fmaxf(hi.x, v.x), fmaxf(hi.y, v.y), fmaxf(hi.z, v.z));
}
MG_HD void cvx_vertices_vs(const CShape& X, const CShape& Y, float margin, bool onY, Deep4& D, V3& lo, V3& hi) {
    const int nx = cvx_nv(X);
    lo = v3(1e30f, 1e30f, 1e30f);
    hi = v3(-1e30f, -1e30f, -1e30f);
    if (X.type == MG_SHAPE_CONVEX) {
        const float* V = X.hv + MG_HULL_HEADER;
        V3 r0 = hull_vl(V, nx, 0), r1 = hull_vl(V, nx, 1), r2 = hull_vl(V, nx, 2), r3 = hull_vl(V, nx, 3);
        for (int i = 0; i < nx; ++i) {
            const V3 l = r0;
            r0 = r1; r1 = r2; r2 = r3;
            r3 = hull_vl(V, nx, i + 4);
            const V3 v = vadd(X.c, mmul(X.R, l));            // cvx_vertex(X, i)
            aabb_add(lo, hi, mtmul(Y.R, vsub(v, Y.c)));
            int f;
            const float sv = cvx_sd(Y, v, f, 0.0f, margin);
            if (sv < margin) {
                const V3 n = cvx_normal(Y, f);
                if (onY) deep4_add(D, sv, vsub(v, vscale(n, sv)), vscale(n, -1.0f));
                else deep4_add(D, sv, v, n);
            }
        }
        return;
    }
    for (int i = 0; i < nx; ++i) {
        const V3 v = cvx_vertex(X, i);
        aabb_add(lo, hi, mtmul(Y.R, vsub(v, Y.c)));
        int f;
        const float sv = cvx_sd(Y, v, f, 0.0f, margin);
        if (sv < margin) {
            const V3 n = cvx_normal(Y, f);
            if (onY) deep4_add(D, sv, vsub(v, vscale(n, sv)), vscale(n, -1.0f));
            else deep4_add(D, sv, v, n);
        }
    }
}

// edges: a box's 12 (axis k = e / 4, the other two axes' signs from e % 4); a
// hull's from its record (MG_HULL_HEADER + 3 nv + 4 nf: vertex index pairs,
// hv[2] of them, the importer's Hull.record). Local vertex indices.
MG_HD int cvx_ne(const CShape& S) { return S.type == MG_SHAPE_BOX ? 12 : (int)S.hv[2]; }
MG_HD void cvx_edge_ids(const CShape& S, int e, int& ia, int& ib) {
    if (S.type == MG_SHAPE_BOX) {
        const int k = e >> 2, r = e & 3;
        const int k1 = k == 2 ? 0 : k + 1, k2 = k == 0 ? 2 : k - 1;
        ia = ((r & 1) << k1) | (((r >> 1) & 1) << k2);
        ib = ia | (1 << k);
    } else {
        const float* E = S.hv + MG_HULL_HEADER + 3 * (int)S.hv[0] + 4 * (int)S.hv[1] + 2 * e;
        ia = (int)E[0];
        ib = (int)E[1];
    }
}
MG_HD V3 cvx_vertex_l(const CShape& S, int i) {      // shape-local vertex i
    if (S.type == MG_SHAPE_BOX)
        return v3((i & 1) ? S.h.x : -S.h.x, (i & 2) ? S.h.y : -S.h.y, (i & 4) ? S.h.z : -S.h.z);
    const float* v = S.hv + MG_HULL_HEADER + 3 * i;
    return v3(v[0], v[1], v[2]);
}
MG_HD float cvx_radius(const CShape& S) { return S.type == MG_SHAPE_BOX ? sqrtf(vdot(S.h, S.h)) : S.h.x; }

// edge crossings (run when no vertex of either shape is within the margin of
// the other), in Y's frame: nothing unless X's bounding sphere reaches Y's box
// (or Y's bounding sphere); an edge farther from Y's centre than Y's bounding
// radius + margin is skipped; the rest are clipped against Y's face planes
// pushed out by the margin (Cyrus-Beck), and a non-empty chord [t0, t1] gives
// one candidate at its midpoint, by Y's planes like a vertex (cvx_sd:
// separation and face normal; onY: the point on Y's face).
// cvx_edges_gate: the gates shared by every edge; t = X's centre and M = X's
// axes in Y's frame, ry = Y's bounding radius + margin. cvx_edge_one: one edge
// (X-local endpoints la, lb) -> at most one candidate. The sequential pass
// (cvx_edges_vs) and mg_env.hip's 16-lane pass (edges spread over the lanes)
// run the same two functions.
MG_HD bool cvx_edges_gate(const CShape& X, const CShape& Y, float margin, V3 lo, V3 hi, V3& t, M3& M, float& ry) {
    t = mtmul(Y.R, vsub(X.c, Y.c));                         // X's centre in Y's frame
    const float rx = cvx_radius(X) + margin;
    ry = cvx_radius(Y) + margin;
    if (Y.type == MG_SHAPE_BOX) {
        const V3 dq = v3(t.x - fminf(fmaxf(t.x, -Y.h.x), Y.h.x), t.y - fminf(fmaxf(t.y, -Y.h.y), Y.h.y),
                         t.z - fminf(fmaxf(t.z, -Y.h.z), Y.h.z));
        if (vdot(dq, dq) > rx * rx) return false;
    } else if (vdot(t, t) > (rx + ry) * (rx + ry)) {
        return false;
    }
    M.c0 = mtmul(Y.R, X.R.c0);                              // X's axes in Y's frame
    M.c1 = mtmul(Y.R, X.R.c1);
    M.c2 = mtmul(Y.R, X.R.c2);
    if (Y.type == MG_SHAPE_BOX) {
        // Y's face axes separate X (X's vertex bounds from the vertex pass beyond
        // one face plus the margin): no crossing (a link hull just above a table)
        if (lo.x > Y.h.x + margin || hi.x < -Y.h.x - margin || lo.y > Y.h.y + margin || hi.y < -Y.h.y - margin ||
            lo.z > Y.h.z + margin || hi.z < -Y.h.z - margin)
            return false;
    }
    return cvx_ne(X) > 0;
}
// etol (>= 0): the band within which the chord's midpoint counts as near a box
// edge, when it is not the clip margin (a capsule's segment is clipped with its
// radius added to the margin, but is near an edge only within the margin)
MG_HD void cvx_edge_one(const CShape& Y, float margin, bool onY, V3 t, const M3& M, float ry, V3 la, V3 lb,
                        Deep4& D, float etol = -1.0f) {
    const int nf = cvx_nf(Y);
    const V3 al = vadd(t, mmul(M, la));
    const V3 ab = vsub(vadd(t, mmul(M, lb)), al);
    const float tc = fminf(fmaxf(-vdot(al, ab) / vdot(ab, ab), 0.0f), 1.0f);
    const V3 dc = vadd(al, vscale(ab, tc));
    if (vdot(dc, dc) > ry * ry) return;
    float t0 = 0.0f, t1 = 1.0f;
    for (int f = 0; f < nf; ++f) {
        V3 nl;
        float dl;
        cvx_plane_l(Y, f, nl, dl);
        const float sa = (vdot(nl, al) - dl) - margin, sb = (vdot(nl, vadd(al, ab)) - dl) - margin;
        if (sa >= 0.0f && sb >= 0.0f) { t0 = 1.0f; t1 = 0.0f; }
        else if (sa >= 0.0f) t0 = fmaxf(t0, sa / (sa - sb));
        else if (sb >= 0.0f) t1 = fminf(t1, sa / (sa - sb));
        if (!(t0 < t1)) break;
    }
    if (!(t0 < t1)) return;
    const float tm = 0.5f * (t0 + t1);
    if (Y.type == MG_SHAPE_BOX) {
        // the chord's midpoint m near a box edge (its two other coordinates
        // within the margin of their faces, along the axis k it is deepest
        // inside): an edge-edge contact — normal along the cross product of
        // the two edges, pointing out of the box, separation the distance of
        // the two lines along it, the point the closest one on X's edge
        const V3 m = vadd(al, vscale(ab, tm));
        const float ex = fabsf(m.x) - Y.h.x, ey = fabsf(m.y) - Y.h.y, ez = fabsf(m.z) - Y.h.z;
        int k = 0;
        float ek = ex;
        if (ey < ek) { k = 1; ek = ey; }
        if (ez < ek) k = 2;
        const float e1 = k == 0 ? ey : ex, e2 = k == 2 ? ey : ez;
        const float et = etol >= 0.0f ? etol : margin;
        if (e1 > -et && e2 > -et) {
            const V3 dk = v3(k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f, k == 2 ? 1.0f : 0.0f);
            const V3 p0 = v3(k == 0 ? 0.0f : (m.x < 0.0f ? -Y.h.x : Y.h.x),
                             k == 1 ? 0.0f : (m.y < 0.0f ? -Y.h.y : Y.h.y),
                             k == 2 ? 0.0f : (m.z < 0.0f ? -Y.h.z : Y.h.z));
            const V3 nn = vcross(ab, dk);
            const float l2 = vdot(nn, nn);
            if (l2 > 1e-12f * vdot(ab, ab)) {
                V3 n = vscale(nn, 1.0f / sqrtf(l2));
                if (vdot(n, p0) < 0.0f) n = vscale(n, -1.0f);
                const V3 r = vsub(al, p0);
                const float sv = vdot(n, r);
                if (sv < margin) {
                    const float bq = vdot(ab, dk), aq = vdot(ab, ab);
                    const float den = aq - bq * bq;
                    const float ts = fminf(fmaxf((bq * vdot(dk, r) - vdot(ab, r)) / den, 0.0f), 1.0f);
                    const V3 p = vadd(Y.c, mmul(Y.R, vadd(al, vscale(ab, ts))));
                    const V3 nw = mmul(Y.R, n);
                    if (onY) deep4_add(D, sv, vsub(p, vscale(nw, sv)), vscale(nw, -1.0f));
                    else deep4_add(D, sv, p, nw);
                }
                return;
            }
        }
    }
    const V3 p = vadd(Y.c, mmul(Y.R, vadd(al, vscale(ab, tm))));
    int f;
    const float sv = cvx_sd(Y, p, f, 0.0f, margin);
    if (sv < margin) {
        const V3 n = cvx_normal(Y, f);
        if (onY) deep4_add(D, sv, vsub(p, vscale(n, sv)), vscale(n, -1.0f));
        else deep4_add(D, sv, p, n);
    }
}
MG_HD void cvx_edges_vs(const CShape& X, const CShape& Y, float margin, bool onY, Deep4& D, V3 lo, V3 hi) {
    V3 t;
    M3 M;
    float ry;
    if (!cvx_edges_gate(X, Y, margin, lo, hi, t, M, ry)) return;
    const int ne = cvx_ne(X);
    // a hull's edge ids and endpoints are streamed ahead (ids two edges, the
    // endpoints one edge): the loads of the next edge are in flight while this
    // one is tested
    int ia1, ib1, ia2, ib2;
    cvx_edge_ids(X, 0, ia1, ib1);
    V3 la1 = cvx_vertex_l(X, ia1), lb1 = cvx_vertex_l(X, ib1);
    cvx_edge_ids(X, ne > 1 ? 1 : 0, ia2, ib2);
    for (int e = 0; e < ne; ++e) {
        const V3 la = la1, lb = lb1;
        la1 = cvx_vertex_l(X, ia2);
        lb1 = cvx_vertex_l(X, ib2);
        cvx_edge_ids(X, e + 2 < ne ? e + 2 : ne - 1, ia2, ib2);
        cvx_edge_one(Y, margin, onY, t, M, ry, la, lb, D);
    }
}

// vertex i of X against Y's planes: the candidate cvx_vertices_vs makes of it
// (and v, X's vertex in the world)
MG_HD void cvx_vertex_one(const CShape& X, const CShape& Y, float margin, bool onY, int i, Deep4& D, V3& lo,
                          V3& hi) {
    const V3 v = cvx_vertex(X, i);
    aabb_add(lo, hi, mtmul(Y.R, vsub(v, Y.c)));
    int f;
    const float sv = cvx_sd(Y, v, f, 0.0f, margin);
    if (sv < margin) {
        const V3 n = cvx_normal(Y, f);
        if (onY) deep4_add(D, sv, vsub(v, vscale(n, sv)), vscale(n, -1.0f));
        else deep4_add(D, sv, v, n);
    }
}

// convex A vs convex B (box or hull), vertex penetration both ways: A's vertices
// by B's planes (normal = B's face normal), then B's vertices by A's planes
// (point on A's face, normal = -A's); with no vertex candidate, edge crossings
MG_HD void convex_convex(const CShape& A, const CShape& B, float margin, PairOut& o) {
    Deep4 D;
    D.n = 0;
    V3 loA, hiA, loB, hiB;              // A's vertices in B's frame, B's in A's
    cvx_vertices_vs(A, B, margin, false, D, loA, hiA);
    cvx_vertices_vs(B, A, margin, true, D, loB, hiB);
    if (D.n == 0) {
        // edge crossings: the edges of the shape that is not a box, clipped by
        // the box's 6 planes behind its face-axis test; two hulls: A's edges by
        // B's planes, and when they find nothing B's by A's (a thin hull through
        // the middle of a larger one's face crosses only B's edges: the result
        // must not depend on the pair order)
        if (A.type == MG_SHAPE_BOX && B.type != MG_SHAPE_BOX) {
            cvx_edges_vs(B, A, margin, true, D, loB, hiB);
        } else {
            cvx_edges_vs(A, B, margin, false, D, loA, hiA);
            if (D.n == 0 && B.type != MG_SHAPE_BOX) cvx_edges_vs(B, A, margin, true, D, loB, hiB);
        }
    }
    deep4_emit(D, o);
}

// sphere A (centre s, radius r) vs convex B
MG_HD void sphere_convex(V3 s, float r, const CShape& B, float margin, PairOut& o) {
    int f;
    const float sep = cvx_sd(B, s, f, r, margin) - r;
    if (!(sep < margin)) return;
    const V3 n = cvx_normal(B, f);
    pair_push(o, vsub(s, vscale(n, r)), n, sep);
}

// a capsule's axis segment against a box or hull Y (capsule C: axis C.R.c0,
// radius C.h.x, half height C.h.y): the segment as an edge of C, clipped by Y's
// planes pushed out by radius + margin (cvx_edge_one) — a capsule lying across
// a box edge midway between its caps, which its cap spheres miss — giving at
// most one candidate, moved to the capsule's surface (point - n r, sep - r)
MG_HD void capsule_segment_convex(const CShape& C, const CShape& Y, float margin, PairOut& o) {
    if (!(C.h.y > 0.0f)) return;
    const float r = C.h.x, mr = margin + r;
    const V3 t = mtmul(Y.R, vsub(C.c, Y.c));
    M3 M;
    M.c0 = mtmul(Y.R, C.R.c0);
    M.c1 = mtmul(Y.R, C.R.c1);
    M.c2 = mtmul(Y.R, C.R.c2);
    Deep4 D;
    D.n = 0;
    cvx_edge_one(Y, mr, false, t, M, cvx_radius(Y) + mr, v3(-C.h.y, 0.0f, 0.0f), v3(C.h.y, 0.0f, 0.0f), D, margin);
    if (D.n > 0) pair_push(o, vsub(D.p[0], vscale(D.nrm[0], r)), D.nrm[0], D.s[0] - r);
}
// the point of segment [a, b] closest to p
MG_HD V3 seg_closest(V3 a, V3 b, V3 p) {
    const V3 ab = vsub(b, a);
    const float l2 = vdot(ab, ab);
    const float t = l2 > 0.0f ? fminf(fmaxf(vdot(vsub(p, a), ab) / l2, 0.0f), 1.0f) : 0.0f;
    return vadd(a, vscale(ab, t));
}
// closest points of segments [a0, a1] and [b0, b1] (clamped line parameters:
// s from the lines' closest points, t for that point, s again for that t)
MG_HD void seg_seg_closest(V3 a0, V3 a1, V3 b0, V3 b1, V3& pa, V3& pb) {
    const V3 d1 = vsub(a1, a0), d2 = vsub(b1, b0), r = vsub(a0, b0);
    const float a = vdot(d1, d1), e = vdot(d2, d2), f = vdot(d2, r);
    const float c = vdot(d1, r), b = vdot(d1, d2);
    const float den = a * e - b * b;
    float s = 0.0f;
    if (a > 0.0f && den > 1e-12f * a * e) s = fminf(fmaxf((b * f - c * e) / den, 0.0f), 1.0f);
    float t = e > 0.0f ? (b * s + f) / e : 0.0f;
    if (t < 0.0f || t > 1.0f) {
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        s = a > 0.0f ? fminf(fmaxf((b * t - c) / a, 0.0f), 1.0f) : 0.0f;
    }
    pa = vadd(a0, vscale(d1, s));
    pb = vadd(b0, vscale(d2, t));
}

// generic dispatch
MG_HD void collide(const CShape& A, const CShape& B, float margin, PairOut& o) {
    V3 ca[2], cb[2];
    float ra, rb;
    int na, nbs;
    if (A.type == MG_SHAPE_BOX && B.type == MG_SHAPE_BOX) { box_box(A, B, margin, o); return; }
    // sphere-like decomposition
    na = A.type == MG_SHAPE_CAPSULE ? 2 : 1;
    nbs = B.type == MG_SHAPE_CAPSULE ? 2 : 1;
    ra = A.h.x; rb = B.h.x;
    ca[0] = vsel(A.type == MG_SHAPE_CAPSULE, vsub(A.c, vscale(A.R.c0, A.h.y)), A.c);
    ca[1] = vadd(A.c, vscale(A.R.c0, A.h.y));
    cb[0] = vsel(B.type == MG_SHAPE_CAPSULE, vsub(B.c, vscale(B.R.c0, B.h.y)), B.c);
    cb[1] = vadd(B.c, vscale(B.R.c0, B.h.y));
    if (A.type == MG_SHAPE_CONVEX || B.type == MG_SHAPE_CONVEX) {
        const bool pa = A.type == MG_SHAPE_BOX || A.type == MG_SHAPE_CONVEX;
        const bool pb = B.type == MG_SHAPE_BOX || B.type == MG_SHAPE_CONVEX;
        if (pa && pb) { convex_convex(A, B, margin, o); return; }
        if (pb) {                            // sphere / capsule A vs convex B
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (k < na) sphere_convex(ca[k], ra, B, margin, o);
            if (A.type == MG_SHAPE_CAPSULE) capsule_segment_convex(A, B, margin, o);
            return;
        }
        PairOut t;                           // convex A vs sphere / capsule B: swap roles
        t.n = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (k < nbs) sphere_convex(cb[k], rb, A, margin, t);
        if (B.type == MG_SHAPE_CAPSULE) capsule_segment_convex(B, A, margin, t);
#pragma unroll
        for (int k = 0; k < MG_PAIR_MAXC; ++k)
            if (k < t.n) pair_push(o, vadd(t.p[k], vscale(t.nrm[k], t.sep[k])), vscale(t.nrm[k], -1.0f), t.sep[k]);
        return;
    }
    if (B.type == MG_SHAPE_BOX) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (k < na) sphere_box(ca[k], ra, B, margin, o);
        if (A.type == MG_SHAPE_CAPSULE) capsule_segment_convex(A, B, margin, o);
        return;
    }
    if (A.type == MG_SHAPE_BOX) {
        PairOut t;
        t.n = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (k < nbs) sphere_box(cb[k], rb, A, margin, t);
        if (B.type == MG_SHAPE_CAPSULE) capsule_segment_convex(B, A, margin, t);
#pragma unroll
        for (int k = 0; k < MG_PAIR_MAXC; ++k)     // swap roles: point on A, normal from B to A
            if (k < t.n) pair_push(o, vadd(t.p[k], vscale(t.nrm[k], t.sep[k])), vscale(t.nrm[k], -1.0f), t.sep[k]);
        return;
    }
    // spheres and capsules: the closest points of the axis segments (a sphere's
    // is its centre), one contact
    V3 pa = A.c, pb = B.c;
    if (A.type == MG_SHAPE_CAPSULE && B.type == MG_SHAPE_CAPSULE) seg_seg_closest(ca[0], ca[1], cb[0], cb[1], pa, pb);
    else if (A.type == MG_SHAPE_CAPSULE) pa = seg_closest(ca[0], ca[1], B.c);
    else if (B.type == MG_SHAPE_CAPSULE) pb = seg_closest(cb[0], cb[1], A.c);
    sphere_sphere(pa, ra, pb, rb, margin, o);
}
