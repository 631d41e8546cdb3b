/*
 * migym_oracle_env.c — TEST INFRASTRUCTURE ONLY (included by migym_oracle.c).
 * CPU restatement of the coupled per-env step (test_isaacgym_amd/csrc/mg_env.hip)
 * and its narrow phase (mg_collide.h): the Franka cube-pick scene of
 * examples/franka_cube_ik_osc.py:111-285 (arm, table and cube in one collision
 * group). Same pair order, row order and evaluation order as the device, so
 * parity is expected bit for bit; PHYSICS PARITY WITH PHYSX IS UNPINNED (see
 * migym_oracle.c). Env classification (which envs are coupled) is restated from
 * the rule in include/migym.h (actor_coll), independently of the library.
 */

#define OE_MAXF 2
#define OE_MAXS 4
#define OE_MAXCT 48   /* storage; an env uses MAXCT = 16, or 48 when 64 lanes wide (MG_ENV_MAXCT[_WIDE]) */
#define OE_F0 64      /* participant ids (mg_internal.h MG_ENV_FREE0 ...) */
#define OE_PMAX 4
/* friction patches (mg_internal.h MG_FP_*): record floats, pairs per env that
 * keep theirs, normal tolerance; the cache row of an env holds OE_FPP records
 * of OE_FP_N floats plus a held flag each */
#define OE_FP_N 16
#define OE_FPP 128
#define OE_FP_COS 0.999f
#define OE_FC_N (OE_FPP * (OE_FP_N + 1))

typedef struct { int type; v3_t c; m3_t R; v3_t h; const float* hv; } cshape_t;
typedef struct { int n; v3_t p[OE_PMAX]; v3_t nrm[OE_PMAX]; float sep[OE_PMAX]; } pair_t;

static v3_t mcol_(m3_t R, int i) { return i == 0 ? R.c0 : (i == 1 ? R.c1 : R.c2); }
static float vc_(v3_t v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

static void ppush_(pair_t* o, v3_t p, v3_t n, float sep) {
    if (o->n < OE_PMAX) { o->p[o->n] = p; o->nrm[o->n] = n; o->sep[o->n] = sep; o->n = o->n + 1; }
}

static void sph_sph_(v3_t a, float ra, v3_t b, float rb, float margin, pair_t* o) {
    const v3_t d = sub3(a, b);
    const float l = sqrtf(dot3(d, d));
    const float sep = l - ra - rb;
    v3_t n;
    if (!(sep < margin)) return;
    n = l > 1e-9f ? mul3(d, 1.0f / l) : V(0.0f, 0.0f, 1.0f);
    ppush_(o, sub3(a, mul3(n, ra)), n, sep);
}

static void sph_box_(v3_t s, float r, const cshape_t* B, float margin, pair_t* o) {
    const v3_t loc = mtv_(B->R, sub3(s, B->c));
    const float hx = B->h.x, hy = B->h.y, hz = B->h.z;
    const float qx = fminf(fmaxf(loc.x, -hx), hx);
    const float qy = fminf(fmaxf(loc.y, -hy), hy);
    const float qz = fminf(fmaxf(loc.z, -hz), hz);
    const int inside = loc.x == qx && loc.y == qy && loc.z == qz;
    v3_t n;
    float sep;
    if (!inside) {
        const v3_t dq = mv_(B->R, V(loc.x - qx, loc.y - qy, loc.z - qz));
        const float l = sqrtf(dot3(dq, dq));
        sep = l - r;
        if (!(sep < margin)) return;
        n = mul3(dq, 1.0f / l);
    } else {
        const float px = hx - fabsf(loc.x), py = hy - fabsf(loc.y), pz = hz - fabsf(loc.z);
        int ax = 0;
        float pen = px, sg;
        if (py < pen) { ax = 1; pen = py; }
        if (pz < pen) { ax = 2; pen = pz; }
        sg = vc_(loc, ax) < 0.0f ? -1.0f : 1.0f;
        n = mul3(mcol_(B->R, ax), sg);
        sep = -pen - r;
    }
    ppush_(o, sub3(s, mul3(n, r)), n, sep);
}

static void box_box_(const cshape_t* A, const cshape_t* B, float margin, pair_t* o) {
    const v3_t d = sub3(B->c, A->c);
    float Rm[3][3], AbsR[3][3], best_face = -1e30f, best_edge = -1e30f;
    const float ha[3] = {A->h.x, A->h.y, A->h.z}, hb[3] = {B->h.x, B->h.y, B->h.z};
    const float t[3] = {dot3(d, A->R.c0), dot3(d, A->R.c1), dot3(d, A->R.c2)};
    int i, j, k, face = 0, ei = -1, ej = -1;
    v3_t eaxis = V(0.0f, 0.0f, 0.0f);
    for (i = 0; i < 3; ++i)
        for (j = 0; j < 3; ++j) {
            Rm[i][j] = dot3(mcol_(A->R, i), mcol_(B->R, j));
            AbsR[i][j] = fabsf(Rm[i][j]) + 1e-6f;
        }
    for (i = 0; i < 3; ++i) {
        const float rb = hb[0] * AbsR[i][0] + hb[1] * AbsR[i][1] + hb[2] * AbsR[i][2];
        const float sep = fabsf(t[i]) - ha[i] - rb;
        if (sep > best_face) { best_face = sep; face = i; }
    }
    for (j = 0; j < 3; ++j) {
        const float ra = ha[0] * AbsR[0][j] + ha[1] * AbsR[1][j] + ha[2] * AbsR[2][j];
        const float tb = t[0] * Rm[0][j] + t[1] * Rm[1][j] + t[2] * Rm[2][j];
        const float sep = fabsf(tb) - hb[j] - ra;
        if (sep > best_face) { best_face = sep; face = 3 + j; }
    }
    if (!(best_face < margin)) return;
    for (i = 0; i < 3; ++i)
        for (j = 0; j < 3; ++j) {
            v3_t ax = cross3(mcol_(A->R, i), mcol_(B->R, j));
            const float l2 = dot3(ax, ax);
            float ra, rb, sep;
            if (!(l2 > 1e-6f)) continue;
            ax = mul3(ax, 1.0f / sqrtf(l2));
            ra = ha[0] * fabsf(dot3(ax, A->R.c0)) + ha[1] * fabsf(dot3(ax, A->R.c1)) + ha[2] * fabsf(dot3(ax, A->R.c2));
            rb = hb[0] * fabsf(dot3(ax, B->R.c0)) + hb[1] * fabsf(dot3(ax, B->R.c1)) + hb[2] * fabsf(dot3(ax, B->R.c2));
            sep = fabsf(dot3(d, ax)) - ra - rb;
            if (!(sep < margin)) return;
            if (sep > best_edge) { best_edge = sep; ei = i; ej = j; eaxis = ax; }
        }
    if (ei >= 0 && best_edge > best_face + 1e-3f) {
        v3_t ax = eaxis, pa = A->c, pb = B->c, ua, ub, w, ca, cb;
        float b, dd, e, den, sa = 0.0f, sb = 0.0f;
        if (dot3(ax, d) < 0.0f) ax = mul3(ax, -1.0f);
        for (k = 0; k < 3; ++k) {
            if (k != ei) pa = add3(pa, mul3(mcol_(A->R, k), dot3(ax, mcol_(A->R, k)) > 0.0f ? ha[k] : -ha[k]));
            if (k != ej) pb = add3(pb, mul3(mcol_(B->R, k), dot3(ax, mcol_(B->R, k)) > 0.0f ? -hb[k] : hb[k]));
        }
        ua = mcol_(A->R, ei); ub = mcol_(B->R, ej);
        w = sub3(pa, pb);
        b = dot3(ua, ub); dd = dot3(ua, w); e = dot3(ub, w);
        den = 1.0f - b * b;
        if (den > 1e-6f) {
            sa = (b * e - dd) / den;
            sb = (e - b * dd) / den;
        }
        sa = fminf(fmaxf(sa, -vc_(A->h, ei)), vc_(A->h, ei));
        sb = fminf(fmaxf(sb, -vc_(B->h, ej)), vc_(B->h, ej));
        ca = add3(pa, mul3(ua, sa));
        cb = add3(pb, mul3(ub, sb));
        ppush_(o, mul3(add3(ca, cb), 0.5f), mul3(ax, -1.0f), best_edge);
        return;
    }
    {
        /* face contact (mg_collide.h): candidate set in the reference face's
         * (u, v) frame — incident corners inside the rectangle (0..3), rectangle
         * corners inside the quad (4..7), edge k x side j crossings (8 + 4k + j);
         * the 4 deepest within the margin, lowest index on ties */
        const int refA = face < 3;
        const cshape_t* Rf = refA ? A : B;
        const cshape_t* In = refA ? B : A;
        const int fa = refA ? face : face - 3;
        v3_t nref = mcol_(Rf->R, fa), iax, ifc, eu, ev, U, W, rc, inrm, nn;
        int ik = 0, iu, iv, ru, rv, m, c;
        float bestd = 1e30f, hik, hu, hv, qx[4], qy[4], cx[24], cy[24], cdep[24], den, iden;
        unsigned cvalid = 0u, used = 0u;
        if (dot3(sub3(In->c, Rf->c), nref) < 0.0f) nref = mul3(nref, -1.0f);
        for (k = 0; k < 3; ++k) {
            const float dk = -fabsf(dot3(nref, mcol_(In->R, k)));
            if (dk < bestd) { bestd = dk; ik = k; }
        }
        iax = mcol_(In->R, ik);
        hik = vc_(In->h, ik);
        ifc = add3(In->c, mul3(iax, dot3(nref, iax) > 0.0f ? -hik : hik));
        iu = ik == 0 ? 1 : 0; iv = ik == 2 ? 1 : 2;
        eu = mul3(mcol_(In->R, iu), vc_(In->h, iu)); ev = mul3(mcol_(In->R, iv), vc_(In->h, iv));
        ru = fa == 0 ? 1 : 0; rv = fa == 2 ? 1 : 2;
        U = mcol_(Rf->R, ru); W = mcol_(Rf->R, rv);
        hu = vc_(Rf->h, ru); hv = vc_(Rf->h, rv);
        rc = add3(Rf->c, mul3(nref, vc_(Rf->h, fa)));
        {
            const v3_t q0 = sub3(sub3(ifc, eu), ev), q1 = sub3(add3(ifc, eu), ev);
            const v3_t q2 = add3(add3(ifc, eu), ev), q3 = add3(sub3(ifc, eu), ev);
            qx[0] = dot3(sub3(q0, rc), U); qy[0] = dot3(sub3(q0, rc), W);
            qx[1] = dot3(sub3(q1, rc), U); qy[1] = dot3(sub3(q1, rc), W);
            qx[2] = dot3(sub3(q2, rc), U); qy[2] = dot3(sub3(q2, rc), W);
            qx[3] = dot3(sub3(q3, rc), U); qy[3] = dot3(sub3(q3, rc), W);
        }
        for (k = 0; k < 4; ++k) {
            cx[k] = qx[k]; cy[k] = qy[k];
            if (fabsf(qx[k]) <= hu && fabsf(qy[k]) <= hv) cvalid |= 1u << k;
        }
        for (m = 0; m < 4; ++m) {
            const float X = (m & 1) ? hu : -hu, Y = (m & 2) ? hv : -hv;
            int pos = 1, neg = 1;
            for (k = 0; k < 4; ++k) {
                const int k2 = (k + 1) & 3;
                const float sk = (qx[k2] - qx[k]) * (Y - qy[k]) - (qy[k2] - qy[k]) * (X - qx[k]);
                pos = pos && sk >= 0.0f;
                neg = neg && sk <= 0.0f;
            }
            cx[4 + m] = X; cy[4 + m] = Y;
            if (pos || neg) cvalid |= 1u << (4 + m);
        }
        for (k = 0; k < 4; ++k) {
            const int k2 = (k + 1) & 3;
            int j;
            for (j = 0; j < 4; ++j) {
                const int ci = 8 + 4 * k + j;
                const int xs = j < 2;
                const float lim = xs ? (j == 0 ? hu : -hu) : (j == 2 ? hv : -hv);
                const float a0 = xs ? qx[k] : qy[k], a1 = xs ? qx[k2] : qy[k2];
                const float o0 = xs ? qy[k] : qx[k], o1 = xs ? qy[k2] : qx[k2];
                const float da = a0 - lim, db = a1 - lim;
                const int ok = (da < 0.0f) != (db < 0.0f);
                const float t = ok ? da / (da - db) : 0.0f;
                const float ov = o0 + (o1 - o0) * t;
                cx[ci] = xs ? lim : ov;
                cy[ci] = xs ? ov : lim;
                if (ok && fabsf(ov) <= (xs ? hv : hu)) cvalid |= 1u << ci;
            }
        }
        inrm = mul3(iax, dot3(nref, iax) > 0.0f ? -1.0f : 1.0f);
        den = dot3(inrm, nref);
        iden = fabsf(den) > 1e-6f ? 1.0f / den : 0.0f;
        for (c = 0; c < 24; ++c) {
            const v3_t qq = add3(add3(rc, mul3(U, cx[c])), mul3(W, cy[c]));
            cdep[c] = dot3(sub3(ifc, qq), inrm) * iden;
        }
        nn = refA ? mul3(nref, -1.0f) : nref;
        for (m = 0; m < OE_PMAX; ++m) {
            int bk = -1;
            float bd = margin, x = 0.0f, y = 0.0f;
            for (c = 0; c < 24; ++c)
                if (((cvalid & ~used) >> c) & 1u)
                    if (cdep[c] < bd) { bd = cdep[c]; bk = c; x = cx[c]; y = cy[c]; }
            if (bk >= 0) {
                const v3_t qq = add3(add3(rc, mul3(U, x)), mul3(W, y));
                const v3_t pt = add3(qq, mul3(nref, bd));
                used |= 1u << bk;
                ppush_(o, refA ? sub3(pt, mul3(nref, bd)) : pt, nn, bd);
            }
        }
    }
}

/* ---- convex shapes as vertices + face planes (a box: 8 corners, 6 faces),
 * vertex penetration both ways (mg_collide.h convex_convex) */
static int cvx_nv_(const cshape_t* S) { return S->type == MG_SHAPE_BOX ? 8 : (int)S->hv[0]; }
static int cvx_nf_(const cshape_t* S) { return S->type == MG_SHAPE_BOX ? 6 : (int)S->hv[1]; }
static v3_t cvx_vertex_(const cshape_t* S, int i) {
    v3_t l;
    if (S->type == MG_SHAPE_BOX) {
        l = V((i & 1) ? S->h.x : -S->h.x, (i & 2) ? S->h.y : -S->h.y, (i & 4) ? S->h.z : -S->h.z);
    } else {
        const float* v = S->hv + MG_HULL_HEADER + 3 * i;
        l = V(v[0], v[1], v[2]);
    }
    return add3(S->c, mv_(S->R, l));
}
static void cvx_plane_l_(const cshape_t* S, int f, v3_t* nl, float* dl) {
    if (S->type == MG_SHAPE_BOX) {
        const int ax = f >> 1;
        const float sg = (f & 1) ? -1.0f : 1.0f;
        *nl = V(ax == 0 ? sg : 0.0f, ax == 1 ? sg : 0.0f, ax == 2 ? sg : 0.0f);
        *dl = vc_(S->h, ax);
    } else {
        const float* pl = S->hv + MG_HULL_HEADER + 3 * (int)S->hv[0] + 4 * f;
        *nl = V(pl[0], pl[1], pl[2]);
        *dl = pl[3];
    }
}
static float cvx_sd_(const cshape_t* S, v3_t p, int* fbest) {
    const v3_t pl = mtv_(S->R, sub3(p, S->c));
    const int nf = cvx_nf_(S);
    float best = -1e30f;
    int f;
    *fbest = 0;
    for (f = 0; f < nf; ++f) {
        v3_t nl;
        float dl, sd;
        cvx_plane_l_(S, f, &nl, &dl);
        sd = dot3(nl, pl) - dl;
        if (sd > best) { best = sd; *fbest = f; }
    }
    return best;
}
static v3_t cvx_normal_(const cshape_t* S, int f) {
    v3_t nl;
    float dl;
    cvx_plane_l_(S, f, &nl, &dl);
    return mv_(S->R, nl);
}
/* the OE_PMAX deepest candidates, ascending separation, earlier first on ties */
static void deep4_add_(pair_t* D, float sep, v3_t p, v3_t n) {
    int at = 0, k;
    if (D->n == OE_PMAX && !(sep < D->sep[OE_PMAX - 1])) return;
    for (k = 0; k < D->n; ++k) if (D->sep[k] <= sep) at = k + 1;
    for (k = OE_PMAX - 1; k > at; --k) { D->sep[k] = D->sep[k - 1]; D->p[k] = D->p[k - 1]; D->nrm[k] = D->nrm[k - 1]; }
    D->sep[at] = sep; D->p[at] = p; D->nrm[at] = n;
    if (D->n < OE_PMAX) D->n = D->n + 1;
}
static void deep4_emit_(const pair_t* D, pair_t* o) {
    int k;
    for (k = 0; k < D->n; ++k) ppush_(o, D->p[k], D->nrm[k], D->sep[k]);
}
/* edges (mg_collide.h cvx_edge_ids): a box's 12, a hull's index pairs after its planes */
static int cvx_ne_(const cshape_t* S) { return S->type == MG_SHAPE_BOX ? 12 : (int)S->hv[2]; }
static void cvx_edge_ids_(const cshape_t* S, int e, int* ia, int* ib) {
    if (S->type == MG_SHAPE_BOX) {
        const int k = e >> 2, r = e & 3;
        const int k1 = k == 2 ? 0 : k + 1, k2 = k == 0 ? 2 : k - 1;
        *ia = ((r & 1) << k1) | (((r >> 1) & 1) << k2);
        *ib = *ia | (1 << k);
    } else {
        const float* E = S->hv + MG_HULL_HEADER + 3 * (int)S->hv[0] + 4 * (int)S->hv[1] + 2 * e;
        *ia = (int)E[0];
        *ib = (int)E[1];
    }
}
static v3_t cvx_vertex_l_(const cshape_t* S, int i) {
    if (S->type == MG_SHAPE_BOX)
        return V((i & 1) ? S->h.x : -S->h.x, (i & 2) ? S->h.y : -S->h.y, (i & 4) ? S->h.z : -S->h.z);
    return V(S->hv[MG_HULL_HEADER + 3 * i], S->hv[MG_HULL_HEADER + 3 * i + 1], S->hv[MG_HULL_HEADER + 3 * i + 2]);
}
static float cvx_radius_(const cshape_t* S) { return S->type == MG_SHAPE_BOX ? sqrtf(dot3(S->h, S->h)) : S->h.x; }
/* edge crossings, X's edges by Y's planes in Y's frame (mg_collide.h
 * cvx_edges_vs): sphere gate, per-edge distance prefilter, Cyrus-Beck clip
 * against the planes pushed out by the margin, one candidate at the chord's
 * midpoint */
static void aabb_add_(v3_t* lo, v3_t* hi, v3_t v) {
    *lo = V(fminf(lo->x, v.x), fminf(lo->y, v.y), fminf(lo->z, v.z));
    *hi = V(fmaxf(hi->x, v.x), fmaxf(hi->y, v.y), fmaxf(hi->z, v.z));
}
/* one edge (X-local endpoints la, lb; t, M: X's centre and axes in Y's frame,
 * ry: Y's bounding radius + margin) -> at most one candidate (mg_collide.h
 * cvx_edge_one) */
static void cvx_edge_one_(const cshape_t* Y, float margin, int onY, v3_t t, m3_t M, float ry, v3_t la, v3_t lb,
                          pair_t* D, float etol) {
    const int nf = cvx_nf_(Y);
    int f;
    v3_t al, ab, dc, p;
    float t0 = 0.0f, t1 = 1.0f, tm, sv, tc;
    al = add3(t, mv_(M, la));
    ab = sub3(add3(t, mv_(M, lb)), al);
    tc = fminf(fmaxf(-dot3(al, ab) / dot3(ab, ab), 0.0f), 1.0f);
    dc = add3(al, mul3(ab, tc));
    if (dot3(dc, dc) > ry * ry) return;
    for (f = 0; f < nf; ++f) {
        v3_t nl;
        float dl, sa, sb;
        cvx_plane_l_(Y, f, &nl, &dl);
        sa = (dot3(nl, al) - dl) - margin;
        sb = (dot3(nl, add3(al, ab)) - dl) - margin;
        if (sa >= 0.0f && sb >= 0.0f) { t0 = 1.0f; t1 = 0.0f; }
        else if (sa >= 0.0f) t0 = fmaxf(t0, sa / (sa - sb));
        else if (sb >= 0.0f) t1 = fminf(t1, sa / (sa - sb));
        if (!(t0 < t1)) break;
    }
    if (!(t0 < t1)) return;
    tm = 0.5f * (t0 + t1);
    if (Y->type == MG_SHAPE_BOX) {   /* near a box edge: edge-edge normal (mg_collide.h) */
        const v3_t mm = add3(al, mul3(ab, tm));
        const float ex = fabsf(mm.x) - Y->h.x, ey = fabsf(mm.y) - Y->h.y, ez = fabsf(mm.z) - Y->h.z;
        int k = 0;
        float ek = ex, e1, e2;
        if (ey < ek) { k = 1; ek = ey; }
        if (ez < ek) k = 2;
        e1 = k == 0 ? ey : ex;
        e2 = k == 2 ? ey : ez;
        if (e1 > -etol && e2 > -etol) {   /* etol: the near-edge band (the margin but for capsules) */
            const v3_t dk = V(k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f, k == 2 ? 1.0f : 0.0f);
            const v3_t p0 = V(k == 0 ? 0.0f : (mm.x < 0.0f ? -Y->h.x : Y->h.x),
                              k == 1 ? 0.0f : (mm.y < 0.0f ? -Y->h.y : Y->h.y),
                              k == 2 ? 0.0f : (mm.z < 0.0f ? -Y->h.z : Y->h.z));
            const v3_t nn = cross3(ab, dk);
            const float l2 = dot3(nn, nn);
            if (l2 > 1e-12f * dot3(ab, ab)) {
                v3_t n = mul3(nn, 1.0f / sqrtf(l2));
                v3_t r;
                float svv;
                if (dot3(n, p0) < 0.0f) n = mul3(n, -1.0f);
                r = sub3(al, p0);
                svv = dot3(n, r);
                if (svv < margin) {
                    const float bq = dot3(ab, dk), aq = dot3(ab, ab);
                    const float den = aq - bq * bq;
                    const float ts = fminf(fmaxf((bq * dot3(dk, r) - dot3(ab, r)) / den, 0.0f), 1.0f);
                    const v3_t pp = add3(Y->c, mv_(Y->R, add3(al, mul3(ab, ts))));
                    const v3_t nw = mv_(Y->R, n);
                    if (onY) deep4_add_(D, svv, sub3(pp, mul3(nw, svv)), mul3(nw, -1.0f));
                    else deep4_add_(D, svv, pp, nw);
                }
                return;
            }
        }
    }
    p = add3(Y->c, mv_(Y->R, add3(al, mul3(ab, tm))));
    sv = cvx_sd_(Y, p, &f);
    if (sv < margin) {
        const v3_t n = cvx_normal_(Y, f);
        if (onY) deep4_add_(D, sv, sub3(p, mul3(n, sv)), mul3(n, -1.0f));
        else deep4_add_(D, sv, p, n);
    }
}
static void cvx_edges_vs_(const cshape_t* X, const cshape_t* Y, float margin, int onY, pair_t* D, v3_t lo, v3_t hi) {
    const v3_t t = mtv_(Y->R, sub3(X->c, Y->c));
    const float rx = cvx_radius_(X) + margin, ry = cvx_radius_(Y) + margin;
    m3_t M;
    int e, ne;
    if (Y->type == MG_SHAPE_BOX) {
        const v3_t dq = V(t.x - fminf(fmaxf(t.x, -Y->h.x), Y->h.x), t.y - fminf(fmaxf(t.y, -Y->h.y), Y->h.y),
                          t.z - fminf(fmaxf(t.z, -Y->h.z), Y->h.z));
        if (dot3(dq, dq) > rx * rx) return;
    } else if (dot3(t, t) > (rx + ry) * (rx + ry)) {
        return;
    }
    M.c0 = mtv_(Y->R, X->R.c0);
    M.c1 = mtv_(Y->R, X->R.c1);
    M.c2 = mtv_(Y->R, X->R.c2);
    if (Y->type == MG_SHAPE_BOX) {   /* Y's face axes separate X (vertex-pass bounds): no crossing */
        if (lo.x > Y->h.x + margin || hi.x < -Y->h.x - margin || lo.y > Y->h.y + margin || hi.y < -Y->h.y - margin ||
            lo.z > Y->h.z + margin || hi.z < -Y->h.z - margin)
            return;
    }
    ne = cvx_ne_(X);
    for (e = 0; e < ne; ++e) {
        int ia, ib;
        cvx_edge_ids_(X, e, &ia, &ib);
        cvx_edge_one_(Y, margin, onY, t, M, ry, cvx_vertex_l_(X, ia), cvx_vertex_l_(X, ib), D, margin);
    }
}
static void convex_convex_(const cshape_t* A, const cshape_t* B, float margin, pair_t* o) {
    pair_t D;
    int i, f;
    const int na = cvx_nv_(A), nb = cvx_nv_(B);
    v3_t loA = V(1e30f, 1e30f, 1e30f), hiA = V(-1e30f, -1e30f, -1e30f), loB = loA, hiB = hiA;
    D.n = 0;
    for (i = 0; i < na; ++i) {
        const v3_t v = cvx_vertex_(A, i);
        const float sd = cvx_sd_(B, v, &f);
        aabb_add_(&loA, &hiA, mtv_(B->R, sub3(v, B->c)));
        if (sd < margin) deep4_add_(&D, sd, v, cvx_normal_(B, f));
    }
    for (i = 0; i < nb; ++i) {
        const v3_t v = cvx_vertex_(B, i);
        const float sd = cvx_sd_(A, v, &f);
        aabb_add_(&loB, &hiB, mtv_(A->R, sub3(v, A->c)));
        if (sd < margin) {
            const v3_t nA = cvx_normal_(A, f);
            deep4_add_(&D, sd, sub3(v, mul3(nA, sd)), mul3(nA, -1.0f));
        }
    }
    if (D.n == 0) {      /* no vertex candidate: edge crossings (mg_collide.h convex_convex) */
        if (A->type == MG_SHAPE_BOX && B->type != MG_SHAPE_BOX) {
            cvx_edges_vs_(B, A, margin, 1, &D, loB, hiB);
        } else {
            cvx_edges_vs_(A, B, margin, 0, &D, loA, hiA);
            if (D.n == 0 && B->type != MG_SHAPE_BOX) cvx_edges_vs_(B, A, margin, 1, &D, loB, hiB);
        }
    }
    deep4_emit_(&D, o);
}
static void sph_cvx_(v3_t s, float r, const cshape_t* B, float margin, pair_t* o) {
    int f;
    const float sep = cvx_sd_(B, s, &f) - r;
    v3_t n;
    if (!(sep < margin)) return;
    n = cvx_normal_(B, f);
    ppush_(o, sub3(s, mul3(n, r)), n, sep);
}

/* a capsule's axis segment against a box or hull Y (mg_collide.h
 * capsule_segment_convex): clipped by Y's planes pushed out by radius + margin,
 * at most one candidate, moved to the capsule's surface */
static void capsule_segment_convex_(const cshape_t* C, const cshape_t* Y, float margin, pair_t* o) {
    const float r = C->h.x, mr = margin + r;
    v3_t t;
    m3_t M;
    pair_t D;
    if (!(C->h.y > 0.0f)) return;
    t = mtv_(Y->R, sub3(C->c, Y->c));
    M.c0 = mtv_(Y->R, C->R.c0);
    M.c1 = mtv_(Y->R, C->R.c1);
    M.c2 = mtv_(Y->R, C->R.c2);
    D.n = 0;
    cvx_edge_one_(Y, mr, 0, t, M, cvx_radius_(Y) + mr, V(-C->h.y, 0.0f, 0.0f), V(C->h.y, 0.0f, 0.0f), &D, margin);
    if (D.n > 0) ppush_(o, sub3(D.p[0], mul3(D.nrm[0], r)), D.nrm[0], D.sep[0] - r);
}
static v3_t seg_closest_(v3_t a, v3_t b, v3_t p) {
    const v3_t ab = sub3(b, a);
    const float l2 = dot3(ab, ab);
    const float t = l2 > 0.0f ? fminf(fmaxf(dot3(sub3(p, a), ab) / l2, 0.0f), 1.0f) : 0.0f;
    return add3(a, mul3(ab, t));
}
static void seg_seg_closest_(v3_t a0, v3_t a1, v3_t b0, v3_t b1, v3_t* pa, v3_t* pb) {
    const v3_t d1 = sub3(a1, a0), d2 = sub3(b1, b0), r = sub3(a0, b0);
    const float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    const float c = dot3(d1, r), b = dot3(d1, d2);
    const float den = a * e - b * b;
    float s = 0.0f, t;
    if (a > 0.0f && den > 1e-12f * a * e) s = fminf(fmaxf((b * f - c * e) / den, 0.0f), 1.0f);
    t = e > 0.0f ? (b * s + f) / e : 0.0f;
    if (t < 0.0f || t > 1.0f) {
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        s = a > 0.0f ? fminf(fmaxf((b * t - c) / a, 0.0f), 1.0f) : 0.0f;
    }
    *pa = add3(a0, mul3(d1, s));
    *pb = add3(b0, mul3(d2, t));
}

static void collide_(const cshape_t* A, const cshape_t* B, float margin, pair_t* o) {
    v3_t ca[2], cb[2], pa, pb;
    float ra, rb;
    int na, nbs, k;
    if (A->type == MG_SHAPE_BOX && B->type == MG_SHAPE_BOX) { box_box_(A, B, margin, o); return; }
    na = A->type == MG_SHAPE_CAPSULE ? 2 : 1;
    nbs = B->type == MG_SHAPE_CAPSULE ? 2 : 1;
    ra = A->h.x; rb = B->h.x;
    ca[0] = A->type == MG_SHAPE_CAPSULE ? sub3(A->c, mul3(A->R.c0, A->h.y)) : A->c;
    ca[1] = add3(A->c, mul3(A->R.c0, A->h.y));
    cb[0] = B->type == MG_SHAPE_CAPSULE ? sub3(B->c, mul3(B->R.c0, B->h.y)) : B->c;
    cb[1] = add3(B->c, mul3(B->R.c0, B->h.y));
    if (A->type == MG_SHAPE_CONVEX || B->type == MG_SHAPE_CONVEX) {
        const int pa_ = A->type == MG_SHAPE_BOX || A->type == MG_SHAPE_CONVEX;
        const int pb_ = B->type == MG_SHAPE_BOX || B->type == MG_SHAPE_CONVEX;
        pair_t t;
        if (pa_ && pb_) { convex_convex_(A, B, margin, o); return; }
        if (pb_) {
            for (k = 0; k < na; ++k) sph_cvx_(ca[k], ra, B, margin, o);
            if (A->type == MG_SHAPE_CAPSULE) capsule_segment_convex_(A, B, margin, o);
            return;
        }
        t.n = 0;
        for (k = 0; k < nbs; ++k) sph_cvx_(cb[k], rb, A, margin, &t);
        if (B->type == MG_SHAPE_CAPSULE) capsule_segment_convex_(B, A, margin, &t);
        for (k = 0; k < t.n; ++k) ppush_(o, add3(t.p[k], mul3(t.nrm[k], t.sep[k])), mul3(t.nrm[k], -1.0f), t.sep[k]);
        return;
    }
    if (B->type == MG_SHAPE_BOX) {
        for (k = 0; k < na; ++k) sph_box_(ca[k], ra, B, margin, o);
        if (A->type == MG_SHAPE_CAPSULE) capsule_segment_convex_(A, B, margin, o);
        return;
    }
    if (A->type == MG_SHAPE_BOX) {
        pair_t t;
        t.n = 0;
        for (k = 0; k < nbs; ++k) sph_box_(cb[k], rb, A, margin, &t);
        if (B->type == MG_SHAPE_CAPSULE) capsule_segment_convex_(B, A, margin, &t);
        for (k = 0; k < t.n; ++k) ppush_(o, add3(t.p[k], mul3(t.nrm[k], t.sep[k])), mul3(t.nrm[k], -1.0f), t.sep[k]);
        return;
    }
    /* spheres and capsules: closest points of the axis segments, one contact */
    pa = A->c;
    pb = B->c;
    if (A->type == MG_SHAPE_CAPSULE && B->type == MG_SHAPE_CAPSULE) seg_seg_closest_(ca[0], ca[1], cb[0], cb[1], &pa, &pb);
    else if (A->type == MG_SHAPE_CAPSULE) pa = seg_closest_(ca[0], ca[1], B->c);
    else if (B->type == MG_SHAPE_CAPSULE) pb = seg_closest_(cb[0], cb[1], A->c);
    sph_sph_(pa, ra, pb, rb, margin, o);
}

/* pair screen (mg_env.hip pair_near): part of the narrow phase's definition */
static float bound_radius_(const float* sh) {
    const int t = (int)sh[0];
    if (t == MG_SHAPE_BOX) return sqrtf(sh[1] * sh[1] + sh[2] * sh[2] + sh[3] * sh[3]);
    if (t == MG_SHAPE_CAPSULE) return sh[1] + sh[2];
    return sh[1];
}
static int sphere_near_box_(v3_t c, float r, const float* shb, v3_t xb, q4_t qb, float off) {
    const v3_t cb = add3(xb, qrot_(qb, V(shb[4], shb[5], shb[6])));
    const m3_t Rb = qmat_(qmul_(qb, Q(shb[7], shb[8], shb[9], shb[10])));
    const v3_t loc = mtv_(Rb, sub3(c, cb));
    const v3_t e = V(loc.x - fminf(fmaxf(loc.x, -shb[1]), shb[1]), loc.y - fminf(fmaxf(loc.y, -shb[2]), shb[2]),
                     loc.z - fminf(fmaxf(loc.z, -shb[3]), shb[3]));
    const float rr = r + off;
    return dot3(e, e) < rr * rr * 1.0001f + 1e-6f;
}
/* shape-frame box of a box / hull (migym_capi.cpp shape_obb): o[0..2] centre, o[3..5] half extents */
static void shape_obb_(const float* sh, const float* hulls, float* o) {
    int k, i, c;
    for (k = 0; k < 6; ++k) o[k] = 0.0f;
    if ((int)sh[0] == MG_SHAPE_CONVEX) {
        const float* hv = hulls + (int)sh[2];
        const int nv = (int)hv[0];
        float lo[3], hi[3];
        for (c = 0; c < 3; ++c) { lo[c] = hv[MG_HULL_HEADER + c]; hi[c] = lo[c]; }
        for (i = 1; i < nv; ++i)
            for (c = 0; c < 3; ++c) {
                const float v = hv[MG_HULL_HEADER + 3 * i + c];
                lo[c] = v < lo[c] ? v : lo[c];
                hi[c] = hi[c] < v ? v : hi[c];
            }
        for (c = 0; c < 3; ++c) { o[c] = 0.5f * (lo[c] + hi[c]); o[3 + c] = 0.5f * (hi[c] - lo[c]); }
    } else {   /* box (the screen's only other participant) */
        o[3] = sh[1]; o[4] = sh[2]; o[5] = sh[3];
    }
}
/* mg_env.hip obb_apart: the two shape-frame boxes separated along one of their
 * six face axes by more than the contact offset plus a rounding slack */
static int obb_apart_boxes_(const float* sha, v3_t xa, q4_t qa, const float* oa, const float* shb, v3_t xb, q4_t qb,
                            const float* ob, float off) {
    float C[3][3], slack, rb, ra;
    const m3_t Ra = qmat_(qmul_(qa, Q(sha[7], sha[8], sha[9], sha[10])));
    const m3_t Rb = qmat_(qmul_(qb, Q(shb[7], shb[8], shb[9], shb[10])));
    v3_t ca, cb, d, A3[3], B3[3];
    float eA[3], eB[3];
    int i, j, apart = 0;
    ca = add3(add3(xa, qrot_(qa, V(sha[4], sha[5], sha[6]))), mv_(Ra, V(oa[0], oa[1], oa[2])));
    cb = add3(add3(xb, qrot_(qb, V(shb[4], shb[5], shb[6]))), mv_(Rb, V(ob[0], ob[1], ob[2])));
    for (i = 0; i < 3; ++i) { eA[i] = oa[3 + i]; eB[i] = ob[3 + i]; }
    d = sub3(cb, ca);
    slack = off + 1e-5f * (1.0f + (eA[0] + eA[1] + eA[2]) + (eB[0] + eB[1] + eB[2]) +
                           (fabsf(d.x) + fabsf(d.y) + fabsf(d.z)));
    A3[0] = Ra.c0; A3[1] = Ra.c1; A3[2] = Ra.c2;
    B3[0] = Rb.c0; B3[1] = Rb.c1; B3[2] = Rb.c2;
    for (i = 0; i < 3; ++i)
        for (j = 0; j < 3; ++j) C[i][j] = fabsf(dot3(A3[i], B3[j]));
    for (i = 0; i < 3; ++i) {
        rb = eB[0] * C[i][0] + eB[1] * C[i][1] + eB[2] * C[i][2];
        apart = apart || fabsf(dot3(d, A3[i])) > eA[i] + rb + slack;
    }
    for (j = 0; j < 3; ++j) {
        ra = eA[0] * C[0][j] + eA[1] * C[1][j] + eA[2] * C[2][j];
        apart = apart || fabsf(dot3(d, B3[j])) > eB[j] + ra + slack;
    }
    return apart;
}
static int obb_apart_(const float* sha, v3_t xa, q4_t qa, const float* shb, v3_t xb, q4_t qb, const float* hulls,
                      float off) {
    float oa[6], ob[6];
    shape_obb_(sha, hulls, oa);
    shape_obb_(shb, hulls, ob);
    return obb_apart_boxes_(sha, xa, qa, oa, shb, xb, qb, ob, off);
}
static int cvx_pair_(int ta, int tb) {
    const int pa = ta == MG_SHAPE_BOX || ta == MG_SHAPE_CONVEX, pb = tb == MG_SHAPE_BOX || tb == MG_SHAPE_CONVEX;
    return pa && pb && (ta == MG_SHAPE_CONVEX || tb == MG_SHAPE_CONVEX);
}
static int pair_near_(const step_t* P, const float* sha, v3_t xa, q4_t qa, const float* shb, v3_t xb, q4_t qb,
                      int ground, const float* hulls) {
    const v3_t cA = add3(xa, qrot_(qa, V(sha[4], sha[5], sha[6])));
    const float rA = bound_radius_(sha);
    v3_t cB, d;
    float rB, rr;
    if (ground) return dot3(P->n, cA) + P->pd - rA < P->co;
    cB = add3(xb, qrot_(qb, V(shb[4], shb[5], shb[6])));
    rB = bound_radius_(shb);
    d = sub3(cB, cA);
    rr = rA + rB + P->co;
    if (!(dot3(d, d) < rr * rr * 1.0001f + 1e-6f)) return 0;
    if ((int)shb[0] == MG_SHAPE_BOX && !sphere_near_box_(cA, rA, shb, xb, qb, P->co)) return 0;
    if ((int)sha[0] == MG_SHAPE_BOX && !sphere_near_box_(cB, rB, sha, xa, qa, P->co)) return 0;
    if (cvx_pair_((int)sha[0], (int)shb[0]) && obb_apart_(sha, xa, qa, shb, xb, qb, hulls, P->co)) return 0;
    return 1;
}

static void tangents_(v3_t n, v3_t* t1, v3_t* t2) {
    v3_t a = V(1.0f, 0.0f, 0.0f), t;
    float inv;
    if (!(fabsf(n.x) < 0.9f)) a = V(0.0f, 1.0f, 0.0f);
    t = cross3(n, a);
    inv = 1.0f / sqrtf(dot3(t, t));
    t = mul3(t, inv);
    *t1 = t;
    *t2 = cross3(n, t);
}

/* Friction patch of one shape pair (mg_env.hip patch_update):
 * PhysX patch friction — up to two anchors fixed on both bodies, kept while
 * the normal holds (cos >= OE_FP_COS) and the anchor's two copies stay within
 * the correlation distance, grown from the contacts in emitted order (the
 * first within the friction offset threshold, then the first farther than the
 * correlation distance from anchor 0). */
typedef struct { int cnt; v3_t nA, aA[2], aB[2]; } patch_t;
static v3_t qrot_inv_(q4_t q, v3_t v) { return qrot_(Q(-q.x, -q.y, -q.z, q.w), v); }
static void patch_load_(patch_t* R, const float* r) {
    int k;
    R->cnt = (int)r[0];
    R->nA = V(r[1], r[2], r[3]);
    for (k = 0; k < 2; ++k) {
        R->aA[k] = V(r[4 + 6 * k], r[5 + 6 * k], r[6 + 6 * k]);
        R->aB[k] = V(r[7 + 6 * k], r[8 + 6 * k], r[9 + 6 * k]);
    }
}
static void patch_store_(const patch_t* R, float* r) {
    int k;
    r[0] = (float)R->cnt;
    r[1] = R->nA.x; r[2] = R->nA.y; r[3] = R->nA.z;
    for (k = 0; k < 2; ++k) {
        r[4 + 6 * k] = R->aA[k].x; r[5 + 6 * k] = R->aA[k].y; r[6 + 6 * k] = R->aA[k].z;
        r[7 + 6 * k] = R->aB[k].x; r[8 + 6 * k] = R->aB[k].y; r[9 + 6 * k] = R->aB[k].z;
    }
}
static void patch_update_(patch_t* R, v3_t xa, q4_t qa, v3_t xb, q4_t qb, const pair_t* o, float fot, float corr) {
    const v3_t n0 = o->nrm[0];
    const float c2 = corr * corr;
    int cnt = R->cnt, k, j, kept;
    patch_t N;
    if (cnt > 0 && dot3(qrot_(qa, R->nA), n0) < OE_FP_COS) cnt = 0;
    N.cnt = 0;
    N.aA[0] = N.aA[1] = N.aB[0] = N.aB[1] = V(0.0f, 0.0f, 0.0f);
    for (k = 0; k < cnt && k < 2; ++k) {
        const v3_t d = sub3(add3(xa, qrot_(qa, R->aA[k])), add3(xb, qrot_(qb, R->aB[k])));
        if (dot3(d, d) <= c2) { N.aA[N.cnt] = R->aA[k]; N.aB[N.cnt] = R->aB[k]; N.cnt++; }
    }
    kept = N.cnt;   /* anchors kept from the last substep */
    /* growth (PhysX growPatches, as mg_env.hip patch_update) */
    {
        const int grow = N.cnt < 2;
        v3_t w0 = N.cnt > 0 ? add3(xa, qrot_(qa, N.aA[0])) : V(0.0f, 0.0f, 0.0f), w1 = V(0.0f, 0.0f, 0.0f);
        float dd = 0.0f;
        for (j = 0; j < o->n; ++j) {
            if (grow && o->sep[j] <= fot) {
                const v3_t pj = o->p[j];
                int put = -1;
                if (N.cnt == 0) {
                    put = 0;
                } else if (N.cnt == 1) {
                    const v3_t d = sub3(pj, w0);
                    const float d2 = dot3(d, d);
                    if (d2 > c2) { put = 1; dd = d2; }
                } else {
                    const v3_t e0 = sub3(pj, w0), e1 = sub3(pj, w1);
                    const float d0 = dot3(e0, e0), d1 = dot3(e1, e1);
                    if (d0 > d1) {
                        if (d0 > dd) { put = 1; dd = d0; }
                    } else if (d1 > dd) {
                        put = 0;
                        dd = d1;
                    }
                }
                if (put >= 0) {
                    const v3_t la = qrot_inv_(qa, sub3(pj, xa)), lb = qrot_inv_(qb, sub3(pj, xb));
                    if (put == 0) { N.aA[0] = la; N.aB[0] = lb; w0 = pj; }
                    else { N.aA[1] = la; N.aB[1] = lb; w1 = pj; }
                    if (N.cnt <= put) N.cnt = put + 1;
                }
            }
        }
    }
    N.nA = kept > 0 ? R->nA : qrot_inv_(qa, n0);   /* the creation normal while an anchor is kept */
    *R = N;
}

static cshape_t place_(const float* sh, v3_t x, q4_t q, const float* hulls) {
    cshape_t c;
    c.type = (int)sh[0];
    c.c = add3(x, qrot_(q, V(sh[4], sh[5], sh[6])));
    c.R = qmat_(qmul_(q, Q(sh[7], sh[8], sh[9], sh[10])));
    c.h = V(sh[1], sh[2], sh[3]);
    c.hv = c.type == MG_SHAPE_CONVEX ? hulls + (int)sh[2] : NULL;
    return c;
}

static void ground_pair_(const step_t* P, const cshape_t* s, pair_t* o) {
    const v3_t n = P->n;
    const float off = P->co;
    int k;
    if (s->type == MG_SHAPE_CONVEX) {
        pair_t D;
        const int nv = cvx_nv_(s);
        D.n = 0;
        for (k = 0; k < nv; ++k) {
            const v3_t p = cvx_vertex_(s, k);
            const float sep = dot3(n, p) + P->pd;
            if (sep < off) deep4_add_(&D, sep, p, n);
        }
        deep4_emit_(&D, o);
    } else if (s->type == MG_SHAPE_BOX) {
        const float d0 = dot3(n, s->R.c0), d1 = dot3(n, s->R.c1), d2 = dot3(n, s->R.c2);
        const float ad0 = fabsf(d0), ad1 = fabsf(d1), ad2 = fabsf(d2);
        int ia = 0;
        float best = ad0;
        v3_t a0, a1, a2, ai, e1, e2, cu;
        float di;
        if (ad1 > best) { ia = 1; best = ad1; }
        if (ad2 > best) ia = 2;
        a0 = mul3(s->R.c0, s->h.x); a1 = mul3(s->R.c1, s->h.y); a2 = mul3(s->R.c2, s->h.z);
        di = ia == 0 ? d0 : (ia == 1 ? d1 : d2);
        ai = ia == 0 ? a0 : (ia == 1 ? a1 : a2);
        e1 = ia == 0 ? a1 : a0;
        e2 = ia == 2 ? a1 : a2;
        cu = add3(s->c, mul3(ai, di > 0.0f ? -1.0f : 1.0f));
        for (k = 0; k < 4; ++k) {
            const float sx = (k & 1) ? 1.0f : -1.0f, sy = (k & 2) ? 1.0f : -1.0f;
            const v3_t p = add3(add3(cu, mul3(e1, sx)), mul3(e2, sy));
            const float sep = dot3(n, p) + P->pd;
            if (sep < off) ppush_(o, p, n, sep);
        }
    } else {
        const int ne = s->type == MG_SHAPE_CAPSULE ? 2 : 1;
        for (k = 0; k < ne; ++k) {
            v3_t c = s->c;
            float sep;
            if (s->type == MG_SHAPE_CAPSULE) c = k ? add3(s->c, mul3(s->R.c0, s->h.y)) : sub3(s->c, mul3(s->R.c0, s->h.y));
            sep = dot3(n, c) + P->pd - s->h.x;
            if (sep < off) ppush_(o, mad3(c, n, -s->h.x), n, sep);
        }
    }
}

/* env description, as the library's env_i row but with global body ids */
#define OP_MAXB 64   /* free bodies of a pile env (mg_internal.h MG_PILE_MAXB; migym_oracle_pile.c) */
typedef struct {
    int art_body, art_dof, art_tmpl, nf, free_b[OE_MAXF], ns, stat_b[OE_MAXS], mask;
    int env;   /* model env index (friction patch cache row) */
    /* a pile env (more than OE_MAXF free bodies, no articulation): its free
     * bodies pb and their actors pact, the static bodies' actors sact */
    int pile, np, pb[OP_MAXB], pact[OP_MAXB], sact[OE_MAXS];
} oenv_t;

#define OE_GM 64      /* lanes of a wide env (mg_env.hip: G = 16, or 64 above 16 links / slots) */
#define OE_SLOTS 32   /* velocity slots of a wide env (MG_ENV_SLOTS_WIDE) */
#define OE_ST0 80
#define OE_LIM0 128

/* sum of 16 slots in the device's DPP order (mg_env.hip red16): row_ror 8,
 * row_ror 4, quad xor 2, quad xor 1; every lane ends with this value */
static float red16_(const float* v) {
    float s[16], t[16], u0, u1;
    int i;
    for (i = 0; i < 16; ++i) s[i] = v[i] + v[(i + 8) & 15];
    for (i = 0; i < 4; ++i) t[i] = s[i] + s[(i + 4) & 15];
    u0 = t[0] + t[2];
    u1 = t[1] + t[3];
    return u0 + u1;
}
/* the same over G = 16 or 64 lanes: G = 64 adds the four rows' sums as
 * (r0 + r1) + (r2 + r3) (mg_env.hip redg) */
static float red_(const float* v, int G) {
    if (G == 64) return (red16_(v) + red16_(v + 16)) + (red16_(v + 32) + red16_(v + 48));
    return red16_(v);
}
static float redp_(const float* a, const float* b, int G) {
    float v[OE_GM];
    int i;
    for (i = 0; i < G; ++i) v[i] = a[i] * b[i];
    return red_(v, G);
}

typedef struct { int a, sa, b, sb; } epair_t;

/* candidate shape pairs of an env, in the device's order (migym_capi.cpp upload) */
static int env_pairs_(const mg_model* m, const oenv_t* ev, int ground, int L, int fb, epair_t* out, int cap) {
    static const int pb[4][4] = {{-1, 0, 1, 2}, {-1, -1, 3, 4}, {-1, -1, -1, 5}, {-1, -1, -1, -1}};
    int n = 0, k, j, t, l, sa, sb;
    const int* LIp = ev->art_tmpl >= 0
        ? m->tmpl_link_i + (size_t)m->artic_tmpl_i[(size_t)ev->art_tmpl * MG_ATMPL_I_N + 0] * MG_LINK_I_N : NULL;
#define OE_PUSH(A_, SA_, B_, SB_) do { if (n < cap) { out[n].a = (A_); out[n].sa = (SA_); out[n].b = (B_); out[n].sb = (SB_); } n++; } while (0)
#define OE_SHP(B_, S0_, NS_) do { const int* t_ = m->tmpl_body_i + (size_t)m->body_tmpl[B_] * MG_TBODY_I_N; S0_ = t_[0]; NS_ = t_[1]; } while (0)
    for (k = 0; k < ev->nf; ++k) {
        int sa0, nsa;
        OE_SHP(ev->free_b[k], sa0, nsa);
        for (sa = sa0; sa < sa0 + nsa; ++sa) {
            if (ground) OE_PUSH(OE_F0 + k, sa, -1, -1);
            for (t = 0; t < ev->ns; ++t) {
                int sb0, nsb;
                if (!((ev->mask >> (14 + 4 * k + t)) & 1)) continue;
                OE_SHP(ev->stat_b[t], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OE_PUSH(OE_F0 + k, sa, OE_ST0 + t, sb);
            }
            for (j = k + 1; j < ev->nf; ++j) {
                int sb0, nsb;
                if (!((ev->mask >> (8 + pb[k][j])) & 1)) continue;
                OE_SHP(ev->free_b[j], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OE_PUSH(OE_F0 + k, sa, OE_F0 + j, sb);
            }
            if (ev->art_body >= 0 && !fb && ((ev->mask >> k) & 1)) {   /* the fixed base (static) */
                int sb0, nsb;
                OE_SHP(ev->art_body, sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OE_PUSH(OE_F0 + k, sa, 0, sb);
            }
        }
    }
    for (l = fb ? 0 : 1; l < L; ++l) {     /* moving links (a floating base moves) */
        int sa0, nsa;
        const int bl = LIp[l * MG_LINK_I_N + 3];   /* the link's body; virtual links: none */
        if (bl < 0) continue;
        OE_SHP(ev->art_body + bl, sa0, nsa);
        for (sa = sa0; sa < sa0 + nsa; ++sa) {
            if (ground) OE_PUSH(l, sa, -1, -1);
            for (t = 0; t < ev->ns; ++t) {
                int sb0, nsb;
                if (!((ev->mask >> (4 + t)) & 1)) continue;
                OE_SHP(ev->stat_b[t], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OE_PUSH(l, sa, OE_ST0 + t, sb);
            }
            for (k = 0; k < ev->nf; ++k) {
                int sb0, nsb;
                if (!((ev->mask >> k) & 1)) continue;
                OE_SHP(ev->free_b[k], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OE_PUSH(l, sa, OE_F0 + k, sb);
            }
        }
    }
#undef OE_PUSH
#undef OE_SHP
    return n;
}

static const float* shp_(const mg_model* m, int s) { return m->shapes + (size_t)s * MG_SHAPE_STRIDE; }


#define OE_MAXPAIRS 512

static float dot6_(const float* a, const float* b) {   /* fused chain, as mg_world.h dot6 */
    return fmaf(a[5], b[5], fmaf(a[4], b[4], fmaf(a[3], b[3], fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])))));
}
static sv_t sv6_(const float* a) { return SVc(V(a[0], a[1], a[2]), V(a[3], a[4], a[5])); }
static void put6_(float* a, sv_t s) { a[0] = s.w.x; a[1] = s.w.y; a[2] = s.w.z; a[3] = s.v.x; a[4] = s.v.y; a[5] = s.v.z; }

/* link l's mass row; a virtual link (ball joint: tmpl_link_i body -1) has none —
 * zero mass and inertia, identity principal frame (mg_env.hip k_artic_lanes) */
static const float* link_mass_(const mg_model* m, const int* LI, int b0, int l) {
    static const float zero[MG_MASS_N] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    const int bl = LI[l * MG_LINK_I_N + 3];
    return bl < 0 ? zero : m->body_mass + (size_t)(b0 + bl) * MG_MASS_N;
}

/* world-frame spatial inertia about O (mg_env.hip world_inertia) */
static void world_inertia_(const float* M, q4_t ql, v3_t xl, v3_t O, float* I) {
    const float m = M[11];
    const v3_t com = V(M[8], M[9], M[10]);
    const q4_t iq = Q(M[4], M[5], M[6], M[7]);
    const v3_t Id = V(M[1] > 0.0f ? 1.0f / M[1] : 0.0f, M[2] > 0.0f ? 1.0f / M[2] : 0.0f, M[3] > 0.0f ? 1.0f / M[3] : 0.0f);
    const s3_t Ic = sym_rdrt_(qmat_(qmul_(ql, iq)), Id);
    const v3_t c = sub3(add3(xl, qrot_(ql, com)), O);
    const float cc2 = dot3(c, c);
    const float ic[9] = {Ic.xx, Ic.xy, Ic.xz, Ic.xy, Ic.yy, Ic.yz, Ic.xz, Ic.yz, Ic.zz};
    const float cv[3] = {c.x, c.y, c.z};
    const v3_t mc = mul3(c, m);
    const float sk[9] = {0.0f, -mc.z, mc.y, mc.z, 0.0f, -mc.x, -mc.y, mc.x, 0.0f};
    int i, k;
    for (i = 0; i < 3; ++i)
        for (k = 0; k < 3; ++k) {
            const float dg = i == k ? m * cc2 : 0.0f;
            I[i * 6 + k] = ic[i * 3 + k] + (dg - cv[i] * (cv[k] * m));
            I[i * 6 + 3 + k] = sk[i * 3 + k];
            I[(3 + i) * 6 + k] = sk[k * 3 + i];
            I[(3 + i) * 6 + 3 + k] = i == k ? m : 0.0f;
        }
}

/* x = M^-1 b for a symmetric positive definite 6x6 M (row-major): left-looking
 * Cholesky, forward and backward substitution (mg_env.hip spd6_solve) */
static void spd6_solve_(const float* M, const float* b, float* x) {
    float Lm[36], y[6];
    int i, j, k;
    for (j = 0; j < 6; ++j) {
        float sj = M[j * 6 + j], dj, inv;
        for (k = 0; k < j; ++k) sj = sj - Lm[j * 6 + k] * Lm[j * 6 + k];
        dj = sqrtf(sj);
        inv = 1.0f / dj;
        Lm[j * 6 + j] = dj;
        for (i = j + 1; i < 6; ++i) {
            float t = M[i * 6 + j];
            for (k = 0; k < j; ++k) t = t - Lm[i * 6 + k] * Lm[j * 6 + k];
            Lm[i * 6 + j] = t * inv;
        }
    }
    for (i = 0; i < 6; ++i) {
        float t = b[i];
        for (k = 0; k < i; ++k) t = t - Lm[i * 6 + k] * y[k];
        y[i] = t / Lm[i * 6 + i];
    }
    for (i = 5; i >= 0; --i) {
        float t = y[i];
        for (k = i + 1; k < 6; ++k) t = t - Lm[k * 6 + i] * x[k];
        x[i] = t / Lm[i * 6 + i];
    }
}

/* World-frame articulated-body algorithm about the base origin x0 (RBDA ch. 7,
 * every quantity in one frame; mg_env.hip aba_world, mg_artic.hip
 * k_artic_world): unconstrained joint accelerations qdd with implicit drives
 * and the effort-limit re-solve. Sets W (kinematics, motion axes, inertias),
 * mdiag (armature + implicit drive term), tau0d / impd (drive force, implicit
 * coefficient) for the final attempt. Shared by env_step_ and artic_step.
 * Floating base (fb): the root's spatial velocity (w, v at x0) is u[D..D+5];
 * the inward pass also folds into link 0, a0 = -IA_0^-1 pA_0 (relative to
 * gravity) starts the outward pass, and qdd[D..D+5] = (w', a0.v + g + w x v).
 * ext (AoS [6] per body, world force / torque at the COM) or NULL. */
typedef struct {
    q4_t ql[OR_MAXL], qrl[OR_MAXL];
    v3_t xl[OR_MAXL], zl[OR_MAXL], rrl[OR_MAXL];
    float Iw[OR_MAXL][36], xi[OR_MAXL][6], va[OR_MAXL][6], ccv[OR_MAXL][6], pav[OR_MAXL][6], Ua[OR_MAXL][6];
    float Dd[OR_MAXL], uu[OR_MAXL];
    float ru[6];              /* floating root: (w, v_O) after the unconstrained update */
} aba_ws_t;

static void aba_world_(const step_t* P, const mg_model* m, const float* LF, const int* LI, int L, int D, int b0,
                       int d0, const float* q, const float* u, const float* props, const float* tgt, v3_t x0, q4_t q0,
                       v3_t gw, aba_ws_t* W, float* qdd, float* mdiag, float* tau0d, float* impd, int fb,
                       const float* ext, int G) {
    const float h = P->h;
    q4_t* ql = W->ql; q4_t* qrl = W->qrl;
    v3_t* xl = W->xl; v3_t* zl = W->zl; v3_t* rrl = W->rrl;
    float (*Iw)[36] = W->Iw;
    float (*xi)[6] = W->xi; float (*va)[6] = W->va; float (*ccv)[6] = W->ccv; float (*pav)[6] = W->pav;
    float (*Ua)[6] = W->Ua;
    float* Dd = W->Dd; float* uu = W->uu;
    int l, i, d;
    if (L > 0) {
        unsigned xmask = 0u, xpos = 0u;
        int att;
        for (att = 0; att < 2; ++att) {
            unsigned nm;
            for (l = 1; l < L; ++l) {
                const float* lf = LF + l * MG_LINK_F_N;
                const int jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
                const v3_t po = V(lf[0], lf[1], lf[2]), ax = V(lf[7], lf[8], lf[9]);
                const q4_t qo = Q(lf[3], lf[4], lf[5], lf[6]);
                const float qj = dj >= 0 ? q[dj] : 0.0f;
                const int ball = (int)lf[10];       /* a ball joint's link (mg_spatial.h link_joint) */
                qrl[l] = qo; rrl[l] = po;
                if (ball == 1) qrl[l] = qmul_(qo, qexp_(V(q[dj], q[dj + 1], q[dj + 2])));
                else if (ball > 1) qrl[l] = qo;
                else if (jt == MG_JOINT_REVOLUTE) qrl[l] = qmul_(qo, qaxang_(ax, qj));
                else if (jt == MG_JOINT_PRISMATIC) rrl[l] = add3(po, qrot_(qo, mul3(ax, qj)));
            }
            for (l = 0; l < L; ++l) {
                const int p = LI[l * MG_LINK_I_N + 0];
                if (p < 0) { ql[l] = q0; xl[l] = x0; zl[l] = V(0.0f, 0.0f, 0.0f); }
                else {
                    const float* lf = LF + l * MG_LINK_F_N;
                    ql[l] = qnorm_(qmul_(ql[p], qrl[l]));
                    xl[l] = add3(xl[p], qrot_(ql[p], rrl[l]));
                    zl[l] = qrot_(ql[l], V(lf[7], lf[8], lf[9]));
                }
            }
            for (l = 0; l < L; ++l) {
                const int jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
                sv_t x = sv0();
                if (l > 0 && dj >= 0) {
                    if (jt == MG_JOINT_REVOLUTE) x = SVc(zl[l], cross3(sub3(xl[l], x0), zl[l]));
                    else x = SVc(V(0.0f, 0.0f, 0.0f), zl[l]);
                }
                put6_(xi[l], x);
                world_inertia_(link_mass_(m, LI, b0, l), ql[l], xl[l], x0, Iw[l]);
            }
            for (i = 0; i < 6; ++i) va[0][i] = fb ? u[D + i] : 0.0f;
            for (l = 1; l < L; ++l) {
                const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
                const float qd = dj >= 0 ? u[dj] : 0.0f;
                for (i = 0; i < 6; ++i) va[l][i] = va[p][i] + xi[l][i] * qd;
            }
            for (l = 0; l < L; ++l) {
                const int dj = LI[l * MG_LINK_I_N + 2];
                const float qd = dj >= 0 ? u[dj] : 0.0f;
                const sv_t v = sv6_(va[l]);
                const sv_t vJ = svmul_(sv6_(xi[l]), qd);
                const int ball = (int)LF[l * MG_LINK_F_N + 10];   /* ball joint: v_parent x vJ (mg_env.hip aba_vp) */
                sv_t vb = v;
                float Iv[6];
                if (ball >= 2) {
                    int pb = LI[l * MG_LINK_I_N + 0];
                    pb = LI[pb * MG_LINK_I_N + 0];
                    if (ball == 3) pb = LI[pb * MG_LINK_I_N + 0];
                    vb = sv6_(va[pb]);
                }
                for (i = 0; i < 6; ++i) Iv[i] = dot6_(&Iw[l][i * 6], va[l]);
                put6_(ccv[l], crm_(vb, vJ));
                {
                    sv_t pb = crf_(v, sv6_(Iv));
                    if (ext && LI[l * MG_LINK_I_N + 3] >= 0) {
                        const float* x = ext + (size_t)(b0 + LI[l * MG_LINK_I_N + 3]) * 6;
                        const float* M = link_mass_(m, LI, b0, l);
                        const v3_t f = V(x[0], x[1], x[2]), t = V(x[3], x[4], x[5]);
                        const v3_t c = sub3(add3(xl[l], qrot_(ql[l], V(M[8], M[9], M[10]))), x0);
                        pb = SVc(sub3(pb.w, add3(t, cross3(c, f))), sub3(pb.v, f));
                    }
                    put6_(pav[l], pb);
                }
            }
            for (l = L - 1; l >= 1; --l) {
                const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
                float uinvD = 0.0f;
                if (dj >= 0) {
                    const float* pr = props + (size_t)(d0 + dj) * MG_DOFPROP_N;
                    const float* tg = tgt + (size_t)(d0 + dj) * 3;
                    const int mode = (int)pr[0];
                    const float kp = pr[1], kd = pr[2], eff = pr[3], arm = pr[8];
                    const float qv = q[dj], uv = u[dj];
                    float tau = 0.0f, imp = 0.0f, Dv, uvv, invD;
                    for (i = 0; i < 6; ++i) Ua[l][i] = dot6_(&Iw[l][i * 6], xi[l]);
                    if (mode == MG_DOF_MODE_POS) {
                        tau = kp * (tg[0] - qv - h * uv) + kd * (tg[1] - uv);
                        imp = h * kd + h * h * kp;
                    } else if (mode == MG_DOF_MODE_VEL) {
                        tau = kd * (tg[1] - uv);
                        imp = h * kd;
                    } else if (mode == MG_DOF_MODE_EFFORT) {
                        tau = tg[2];
                    }
                    if (eff > 0.0f) {
                        if ((xmask >> dj) & 1u) {
                            tau = ((xpos >> dj) & 1u) ? eff : -eff;
                            imp = 0.0f;
                        } else if (imp == 0.0f) {
                            tau = fminf(fmaxf(tau, -eff), eff);
                        }
                    }
                    Dv = dot6_(xi[l], Ua[l]) + arm + imp;
                    uvv = tau - dot6_(xi[l], pav[l]);
                    invD = 1.0f / Dv;
                    uinvD = uvv * invD;
                    for (i = 0; i < 36; ++i) Iw[l][i] = Iw[l][i] - Ua[l][i / 6] * (Ua[l][i % 6] * invD);
                    Dd[l] = Dv;
                    uu[l] = uvv;
                    mdiag[dj] = arm + imp;
                    tau0d[dj] = tau;
                    impd[dj] = imp;
                }
                if (p > 0 || (fb && p == 0)) {
                    for (i = 0; i < 6; ++i) {
                        float pv = pav[l][i] + dot6_(&Iw[l][i * 6], ccv[l]);
                        if (dj >= 0) pv = pv + Ua[l][i] * uinvD;
                        pav[p][i] = pav[p][i] + pv;
                    }
                    for (i = 0; i < 36; ++i) Iw[p][i] = Iw[p][i] + Iw[l][i];
                }
            }
            if (fb) {
                float nb6[6], a0[6];
                v3_t w, vo, av;
                for (i = 0; i < 6; ++i) nb6[i] = -pav[0][i];
                spd6_solve_(Iw[0], nb6, a0);
                for (i = 0; i < 6; ++i) va[0][i] = a0[i];
                w = V(u[D + 0], u[D + 1], u[D + 2]);
                vo = V(u[D + 3], u[D + 4], u[D + 5]);
                av = add3(add3(V(a0[3], a0[4], a0[5]), gw), cross3(w, vo));
                qdd[D + 0] = a0[0]; qdd[D + 1] = a0[1]; qdd[D + 2] = a0[2];
                qdd[D + 3] = av.x; qdd[D + 4] = av.y; qdd[D + 5] = av.z;
                {   /* the root link's damping and speed limits (as a free body's) */
                    const float* tf = m->tmpl_body_f + (size_t)m->body_tmpl[b0] * MG_TBODY_F_N;
                    const float lkeep = 1.0f - fminf(tf[0] * h, 1.0f), akeep = 1.0f - fminf(tf[1] * h, 1.0f);
                    v3_t wn = mul3(mad3(w, V(a0[0], a0[1], a0[2]), h), akeep);
                    v3_t vn = mul3(mad3(vo, av, h), lkeep);
                    const float w2 = dot3(wn, wn), mw2 = tf[3] * tf[3];
                    const float v2 = dot3(vn, vn), mv2 = tf[2] * tf[2];
                    if (w2 > mw2) wn = mul3(wn, sqrtf(mw2 / w2));
                    if (v2 > mv2) vn = mul3(vn, sqrtf(mv2 / v2));
                    W->ru[0] = wn.x; W->ru[1] = wn.y; W->ru[2] = wn.z;
                    W->ru[3] = vn.x; W->ru[4] = vn.y; W->ru[5] = vn.z;
                }
            } else {
                va[0][0] = 0.0f; va[0][1] = 0.0f; va[0][2] = 0.0f;
                va[0][3] = -gw.x; va[0][4] = -gw.y; va[0][5] = -gw.z;
            }
            for (l = 1; l < L; ++l) {
                const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
                float a6[6];
                for (i = 0; i < 6; ++i) a6[i] = va[p][i] + ccv[l][i];
                if (dj >= 0) {
                    float t16[OE_GM], acc;
                    for (i = 0; i < OE_GM; ++i) t16[i] = i < 6 ? Ua[l][i] * a6[i] : 0.0f;
                    acc = (uu[l] - red_(t16, G)) / Dd[l];
                    for (i = 0; i < 6; ++i) a6[i] = a6[i] + xi[l][i] * acc;
                    qdd[dj] = acc;
                }
                for (i = 0; i < 6; ++i) va[l][i] = a6[i];
            }
            nm = xmask;
            for (d = 0; d < D; ++d) {
                const float eff = props[(size_t)(d0 + d) * MG_DOFPROP_N + 3];
                if (eff > 0.0f && impd[d] != 0.0f) {
                    const float actf = tau0d[d] - impd[d] * qdd[d];
                    if (actf > eff) { nm |= 1u << d; xpos |= 1u << d; }
                    else if (actf < -eff) nm |= 1u << d;
                }
            }
            if (nm == xmask) break;
            xmask = nm;
        }
    }
}

/* the TGS normal rows of one sweep, in contact order (mg_env.hip normal_pass) */
static void normal_pass_(const step_t* P, int nct, const float* cs0, const float* ce, const float* cvn0,
                         float (*ck)[3], float (*clam)[3], float (*Jr)[OE_GM], float (*Wr)[OE_GM], float* u,
                         const float* dp, int G, int pos) {
    int c, ln;
    for (c = 0; c < nct; ++c) {
        const float s = cs0[c] + redp_(Jr[c * 3], dp, G);
        float tg, lam, dl, nl;
        if (pos) {
            tg = -s * P->inv_sub;
            if (s < 0.0f) tg = fminf(tg, P->maxdep);
        } else {
            tg = s > 0.0f ? -s * P->inv_h : 0.0f;
            if (ce[c] > 0.0f && cvn0[c] < -P->bounce) tg = fmaxf(tg, -ce[c] * cvn0[c]);
        }
        lam = clam[c][0];
        dl = ck[c][0] * (tg - redp_(Jr[c * 3], u, G));
        nl = fmaxf(lam + dl, 0.0f);
        dl = nl - lam;
        for (ln = 0; ln < G; ++ln) u[ln] = u[ln] + Wr[c * 3][ln] * dl;
        clam[c][0] = nl;
    }
}

static int env_step_(const step_t* P, const mg_model* m, const oenv_t* ev, float* state, float* dof, const float* tgt,
                     const float* props, const float* ext, float* cforce, float* fcache) {
    const int b0 = ev->art_body, d0 = ev->art_dof, nfr = ev->nf;
    const int* ti = ev->art_tmpl >= 0 ? m->artic_tmpl_i + (size_t)ev->art_tmpl * MG_ATMPL_I_N : NULL;
    const int L = ti ? ti[1] : 0, D = ti ? ti[2] : 0;
    const int fb = (ti && !ti[3]) ? 1 : 0;     /* floating base: root slots D..D+5 */
    const int NS = D + 6 * fb;                  /* articulation slots; free bodies follow */
    const float* LF = ti ? m->tmpl_link_f + (size_t)ti[0] * MG_LINK_F_N : NULL;
    const int* LI = ti ? m->tmpl_link_i + (size_t)ti[0] * MG_LINK_I_N : NULL;
    const float h = P->h;
    const v3_t gvec = V(P->g[0], P->g[1], P->g[2]);
    static __thread epair_t pairs[OE_MAXPAIRS];   /* per thread: oracle_step_mt */
    int npair;
    v3_t x0 = V(0.0f, 0.0f, 0.0f), gw = V(0.0f, 0.0f, 0.0f);
    q4_t q0 = Q(0.0f, 0.0f, 0.0f, 1.0f);
    /* slots */
    float q[OE_GM], u[OE_GM], dp[OE_GM], qdd[OE_GM], mdiag[OE_GM], tau0d[OE_GM], impd[OE_GM];
    /* links */
    static __thread aba_ws_t W;   /* per thread: oracle_step_mt */
    v3_t* xl = W.xl; v3_t* zl = W.zl; q4_t* ql = W.ql;
    v3_t lsum[OR_MAXL];
    sv_t vl[OR_MAXL];
    float (*Iw)[36] = W.Iw;
    float (*xi)[6] = W.xi;
    unsigned amask[OR_MAXL];
    int dlink[OE_GM], drev[OE_GM];
    static __thread float Lc[OE_SLOTS][OE_SLOTS], Mi[OE_SLOTS][OE_SLOTS];
    float invd[OE_SLOTS];
    /* free bodies */
    v3_t fx[OE_MAXF], fxc[OE_MAXF], fcom[OE_MAXF], finvI[OE_MAXF], fext[OE_MAXF], text[OE_MAXF], fsum[OE_MAXF];
    q4_t fq[OE_MAXF], fiq[OE_MAXF];
    float finvm[OE_MAXF], lkeep[OE_MAXF], akeep[OE_MAXF], mlv2[OE_MAXF], mav2[OE_MAXF], gon[OE_MAXF];
    s3_t fIw[OE_MAXF];
    /* contacts and rows */
    int ca[OE_MAXCT], cb[OE_MAXCT];
    v3_t cp[OE_MAXCT], cd[OE_MAXCT][3];
    float cs0[OE_MAXCT], ce[OE_MAXCT], cvn0[OE_MAXCT], ck[OE_MAXCT][3], clam[OE_MAXCT][3];
    /* friction anchors (mg_env.hip EnvLds apt ...): row k's point, tangents in cd[k][1..2] */
    v3_t apt[OE_MAXCT];
    float ae[OE_MAXCT][2], amu[OE_MAXCT], psum[OE_MAXCT];
    int aa[OE_MAXCT], ab[OE_MAXCT], alast[OE_MAXCT], apair[OE_MAXCT], apart[OE_MAXCT], pstart[OE_MAXCT];
    int aclamp[OE_MAXCT][2];
    char held[OE_FPP];
    float* fcr = fcache ? fcache + (size_t)ev->env * OE_FC_N : NULL;
    static __thread float Jr[OE_MAXCT * 3][OE_GM], Wr[OE_MAXCT * 3][OE_GM];
    int d, l, k, c, i, j, st_, it;
    /* lanes: 16, or 64 for an env of more than 16 links / velocity slots (migym_capi.cpp groups) */
    const int G = (L > 16 || NS + 6 * nfr > 16) ? 64 : 16;
    const int MAXCT = G == 64 ? 48 : 16;
    if (L > OR_MAXL || NS + 6 * nfr > OE_SLOTS || nfr > OE_MAXF) return -1;
    npair = env_pairs_(m, ev, P->ground, L, fb, pairs, OE_MAXPAIRS);
    if (npair > OE_MAXPAIRS) return -1;
    for (i = 0; i < OE_GM; ++i) { q[i] = 0.0f; u[i] = 0.0f; dp[i] = 0.0f; }
    if (L > 0) {
        const float* s0 = state + (size_t)b0 * MG_STATE_N;
        const float grav_on = m->tmpl_body_f[(size_t)m->body_tmpl[b0] * MG_TBODY_F_N + 4];
        x0 = V(s0[0], s0[1], s0[2]);
        q0 = qnorm_(Q(s0[3], s0[4], s0[5], s0[6]));
        gw = grav_on != 0.0f ? gvec : V(0.0f, 0.0f, 0.0f);
    }
    for (l = 0; l < L; ++l) {
        const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
        amask[l] = (p >= 0 ? amask[p] : 0u) | (dj >= 0 ? (1u << dj) : 0u);
        if (dj >= 0) { dlink[dj] = l; drev[dj] = LI[l * MG_LINK_I_N + 1] == MG_JOINT_REVOLUTE ? 1 : 0; }
        lsum[l] = V(0.0f, 0.0f, 0.0f);
    }
    for (d = 0; d < D; ++d) { q[d] = dof[(d0 + d) * 2 + 0]; u[d] = dof[(d0 + d) * 2 + 1]; }
    if (fb) {   /* root slots: w and the velocity of the base origin v_O = v_com - w x (R c) */
        const float* s0 = state + (size_t)b0 * MG_STATE_N;
        const float* M0 = m->body_mass + (size_t)b0 * MG_MASS_N;
        const v3_t w = V(s0[10], s0[11], s0[12]), vc = V(s0[7], s0[8], s0[9]);
        const v3_t vo = sub3(vc, cross3(w, qrot_(q0, V(M0[8], M0[9], M0[10]))));
        u[D + 0] = w.x; u[D + 1] = w.y; u[D + 2] = w.z;
        u[D + 3] = vo.x; u[D + 4] = vo.y; u[D + 5] = vo.z;
    }
    for (k = 0; k < nfr; ++k) {
        const int b = ev->free_b[k];
        const float* s = state + (size_t)b * MG_STATE_N;
        const float* M = m->body_mass + (size_t)b * MG_MASS_N;
        const float* tf = m->tmpl_body_f + (size_t)m->body_tmpl[b] * MG_TBODY_F_N;
        fx[k] = V(s[0], s[1], s[2]);
        fq[k] = qnorm_(Q(s[3], s[4], s[5], s[6]));
        for (i = 0; i < 6; ++i) u[NS + 6 * k + i] = s[7 + i];
        finvm[k] = M[0];
        finvI[k] = V(M[1], M[2], M[3]);
        fiq[k] = Q(M[4], M[5], M[6], M[7]);
        fcom[k] = V(M[8], M[9], M[10]);
        lkeep[k] = 1.0f - fminf(tf[0] * h, 1.0f);
        akeep[k] = 1.0f - fminf(tf[1] * h, 1.0f);
        mlv2[k] = tf[2] * tf[2];
        mav2[k] = tf[3] * tf[3];
        gon[k] = tf[4];
        fext[k] = V(0.0f, 0.0f, 0.0f); text[k] = V(0.0f, 0.0f, 0.0f);
        if (ext) {
            const float* x = ext + (size_t)b * 6;
            fext[k] = V(x[0], x[1], x[2]);
            text[k] = V(x[3], x[4], x[5]);
        }
        fsum[k] = V(0.0f, 0.0f, 0.0f);
    }

    for (st_ = 0; st_ < P->substeps; ++st_) {
        int nct = 0, link_rows = 0, nanc = 0, npatch = 0;
        int ppair[OE_MAXCT], pslot[OE_MAXCT], pnum[OE_MAXCT];
        float pmu[OE_MAXCT];
        /* the pairs that held a patch at the end of the last substep */
        for (i = 0; i < OE_FPP; ++i) {
            held[i] = fcr ? fcr[(size_t)i * (OE_FP_N + 1) + OE_FP_N] != 0.0f : 0;
            if (fcr) fcr[(size_t)i * (OE_FP_N + 1) + OE_FP_N] = 0.0f;
        }
        for (c = 0; c < OE_MAXCT; ++c) pstart[c] = 0;
        /* ---- 1. unconstrained motion: world-frame ABA about x0 (mg_env.hip aba_world) */
        if (L > 0) aba_world_(P, m, LF, LI, L, D, b0, d0, q, u, props, tgt, x0, q0, gw, &W, qdd, mdiag, tau0d, impd, fb,
                              ext, G);
        for (k = 0; k < nfr; ++k) {
            const int s0 = NS + 6 * k;
            const s3_t Iw = sym_rdrt_(qmat_(qmul_(fq[k], fiq[k])), finvI[k]);
            v3_t v = V(u[s0 + 0], u[s0 + 1], u[s0 + 2]), w = V(u[s0 + 3], u[s0 + 4], u[s0 + 5]);
            float v2, w2;
            fIw[k] = Iw;
            fxc[k] = add3(fx[k], qrot_(fq[k], fcom[k]));
            if (gon[k] != 0.0f) v = mad3(v, gvec, h);
            v = mad3(v, fext[k], finvm[k] * h);
            w = mad3(w, symmul_(Iw, text[k]), h);
            v = mul3(v, lkeep[k]);
            w = mul3(w, akeep[k]);
            v2 = dot3(v, v);
            if (v2 > mlv2[k]) v = mul3(v, sqrtf(mlv2[k] / v2));
            w2 = dot3(w, w);
            if (w2 > mav2[k]) w = mul3(w, sqrtf(mav2[k] / w2));
            u[s0 + 0] = v.x; u[s0 + 1] = v.y; u[s0 + 2] = v.z;
            u[s0 + 3] = w.x; u[s0 + 4] = w.y; u[s0 + 5] = w.z;
        }
        for (d = 0; d < D; ++d) {
            const float maxv = props[(size_t)(d0 + d) * MG_DOFPROP_N + 4];
            float w = u[d] + h * qdd[d];
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            u[d] = w;
        }
        for (d = D; d < NS; ++d) u[d] = W.ru[d - D];
        for (i = 0; i < OE_GM; ++i) dp[i] = 0.0f;

        /* ---- 2. narrow phase, pair order */
        for (i = 0; i < npair; ++i) {
            const epair_t* pp = &pairs[i];
            const float* sha = shp_(m, pp->sa);
            v3_t xa, xb;
            q4_t qa, qb;
            cshape_t sA, sB;
            pair_t o;
            float mu, rest;
            if (pp->a >= OE_F0) { xa = fx[pp->a - OE_F0]; qa = fq[pp->a - OE_F0]; }
            else { xa = xl[pp->a]; qa = ql[pp->a]; }
            sA = place_(sha, xa, qa, m->hulls);
            o.n = 0;
            if (pp->b < 0) {
                if (!pair_near_(P, sha, xa, qa, sha, xa, qa, 1, m->hulls)) continue;
                ground_pair_(P, &sA, &o);
                mu = 0.5f * (sha[11] + P->mu_g);
                rest = 0.5f * (sha[12] + P->e_g);
            } else {
                const float* shb = shp_(m, pp->sb);
                if (pp->b >= OE_ST0) {
                    const float* ss = state + (size_t)ev->stat_b[pp->b - OE_ST0] * MG_STATE_N;
                    xb = V(ss[0], ss[1], ss[2]);
                    qb = qnorm_(Q(ss[3], ss[4], ss[5], ss[6]));
                } else if (pp->b >= OE_F0) {
                    xb = fx[pp->b - OE_F0];
                    qb = fq[pp->b - OE_F0];
                } else {
                    xb = xl[pp->b];
                    qb = ql[pp->b];
                }
                if (!pair_near_(P, sha, xa, qa, shb, xb, qb, 0, m->hulls)) continue;
                sB = place_(shb, xb, qb, m->hulls);
                collide_(&sA, &sB, P->co, &o);
                mu = 0.5f * (sha[11] + shb[11]);
                rest = 0.5f * (sha[12] + shb[12]);
            }
            {
                const int slot0 = nct;
                for (j = 0; j < o.n; ++j) {
                    if (nct < MAXCT) {
                        ca[nct] = pp->a;
                        cb[nct] = pp->b;
                        cp[nct] = o.p[j];
                        cd[nct][0] = o.nrm[j];
                        cs0[nct] = o.sep[j] - P->ro;
                        ce[nct] = rest;
                        if (pp->a < OE_F0) link_rows = 1;
                        nct++;
                    }
                }
                /* the pair's friction patch (mg_env.hip: its first contact placed), in pair order */
                if (o.n > 0 && slot0 < MAXCT) {
                    ppair[npatch] = i;
                    pslot[npatch] = slot0;
                    pnum[npatch] = o.n < MAXCT - slot0 ? o.n : MAXCT - slot0;
                    pmu[npatch] = mu;
                    npatch++;
                }
            }
        }
        /* friction patches (mg_env.hip: the pass after the narrow phase, one per lane) */
        for (k = 0; k < npatch; ++k) {
            const int slot0 = pslot[k], pn = pnum[k], ip = ppair[k];
            const int a = ca[slot0], b = cb[slot0];
            patch_t R;
            pair_t o;
            v3_t pxa, pxb = V(0.0f, 0.0f, 0.0f), t1, t2;
            q4_t pqa, pqb = Q(0.0f, 0.0f, 0.0f, 1.0f);
            o.n = pn;
            for (j = 0; j < pn; ++j) { o.p[j] = cp[slot0 + j]; o.nrm[j] = cd[slot0 + j][0]; o.sep[j] = cs0[slot0 + j]; }
            if (a >= OE_F0) { pxa = fx[a - OE_F0]; pqa = fq[a - OE_F0]; }
            else { pxa = xl[a]; pqa = ql[a]; }
            if (b >= OE_ST0) {
                const float* ss = state + (size_t)ev->stat_b[b - OE_ST0] * MG_STATE_N;
                pxb = V(ss[0], ss[1], ss[2]);
                pqb = qnorm_(Q(ss[3], ss[4], ss[5], ss[6]));
            } else if (b >= OE_F0) {
                pxb = fx[b - OE_F0];
                pqb = fq[b - OE_F0];
            } else if (b >= 0) {
                pxb = xl[b];
                pqb = ql[b];
            }
            R.cnt = 0;
            if (ip < OE_FPP && held[ip]) patch_load_(&R, fcr + (size_t)ip * (OE_FP_N + 1));
            patch_update_(&R, pxa, pqa, pxb, pqb, &o, P->fot, P->corr);
            if (ip < OE_FPP && fcr) {
                patch_store_(&R, fcr + (size_t)ip * (OE_FP_N + 1));
                fcr[(size_t)ip * (OE_FP_N + 1) + OE_FP_N] = 1.0f;
            }
            pstart[slot0] = 1;
            tangents_(o.nrm[0], &t1, &t2);
            for (j = 0; j < R.cnt; ++j) {
                if (nanc < MAXCT) {
                    const v3_t wA = add3(pxa, qrot_(pqa, R.aA[j])), wB = add3(pxb, qrot_(pqb, R.aB[j]));
                    const v3_t dr = sub3(wA, wB);
                    const float kd = 0.8f * P->inv_h;   /* position sweeps: close 80 % of the substep-start drift */
                    apt[nanc] = wA;
                    cd[nanc][1] = t1;
                    cd[nanc][2] = t2;
                    ae[nanc][0] = fminf(fmaxf(-dot3(dr, t1) * kd, -P->maxdep), P->maxdep);
                    ae[nanc][1] = fminf(fmaxf(-dot3(dr, t2) * kd, -P->maxdep), P->maxdep);
                    amu[nanc] = pmu[k];
                    /* the patch's other anchor, when it has a row: 1 next, 2 previous */
                    apart[nanc] = R.cnt == 2 ? (j == 0 ? (nanc + 1 < MAXCT ? 1 : 0) : 2) : 0;
                    aa[nanc] = a;
                    ab[nanc] = b;
                    alast[nanc] = slot0 + pn - 1;
                    apair[nanc] = ip;
                }
                nanc++;
            }
        }
        if (nanc > MAXCT) nanc = MAXCT;

        /* joint-limit rows (mg_env.hip): DOF order, after the contacts */
        for (d = 0; d < D; ++d) {
            const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
            if (pr[7] != 0.0f) {
                const float lo = pr[5], hi = pr[6];
                const float q1 = q[d] + h * u[d];
                const float mg = 0.05f * (hi - lo);
                if (q1 - lo < mg || hi - q1 < mg) {
                    const int sgn = (q1 - lo) < (hi - q1) ? 1 : -1;
                    if (nct < MAXCT) {
                        ca[nct] = OE_LIM0 + d;
                        cb[nct] = sgn;
                        cp[nct] = V(0.0f, 0.0f, 0.0f);
                        cd[nct][0] = V(0.0f, 0.0f, 0.0f);
                        cs0[nct] = sgn > 0 ? q[d] - lo : hi - q[d];
                        ce[nct] = 0.0f;
                        link_rows = 1;
                        nct++;
                    }
                }
            }
        }
        /* ---- 3. rows */
        if (link_rows) {
            for (l = 0; l < L; ++l) world_inertia_(link_mass_(m, LI, b0, l), ql[l], xl[l], x0, Iw[l]);
            for (l = L - 1; l >= 1; --l) {
                const int p = LI[l * MG_LINK_I_N + 0];
                if (p > 0 || (fb && p == 0))
                    for (i = 0; i < 36; ++i) Iw[p][i] = Iw[p][i] + Iw[l][i];
            }
            for (i = 0; i < NS; ++i)
                for (j = 0; j < NS; ++j) Lc[i][j] = 0.0f;
            for (i = 0; i < 6 * fb; ++i)           /* root block: IC_0 */
                for (j = 0; j < 6; ++j) Lc[D + i][D + j] = Iw[0][i * 6 + j];
            for (i = 0; i < D; ++i) {
                const int li_ = dlink[i];
                float F[6];
                int r6, jl;
                for (r6 = 0; r6 < 6; ++r6) F[r6] = dot6_(&Iw[li_][r6 * 6], xi[li_]);
                Lc[i][i] = dot6_(xi[li_], F) + mdiag[i];
                jl = LI[li_ * MG_LINK_I_N + 0];
                while (jl > 0) {
                    const int dj = LI[jl * MG_LINK_I_N + 2];
                    if (dj >= 0) {
                        const float hv = dot6_(xi[jl], F);
                        Lc[i][dj] = hv;
                        Lc[dj][i] = hv;
                    }
                    jl = LI[jl * MG_LINK_I_N + 0];
                }
                for (r6 = 0; r6 < 6 * fb; ++r6) {   /* root columns: (IC_l xi_l)[r] */
                    Lc[i][D + r6] = F[r6];
                    Lc[D + r6][i] = F[r6];
                }
            }
            for (j = 0; j < NS; ++j) {
                float s = Lc[j][j], djv;
                for (k = 0; k < j; ++k) s = s - Lc[j][k] * Lc[j][k];
                djv = sqrtf(s);
                invd[j] = 1.0f / djv;
                Lc[j][j] = djv;
                for (i = j + 1; i < NS; ++i) {
                    float t = Lc[i][j];
                    for (k = 0; k < j; ++k) t = t - Lc[i][k] * Lc[j][k];
                    Lc[i][j] = t * invd[j];
                }
            }
            for (j = 0; j < NS; ++j) {       /* column j of M_eff^-1 (device lane j) */
                for (i = 0; i < NS; ++i) {
                    float t = i == j ? 1.0f : 0.0f;
                    for (k = 0; k < i; ++k) t = t - Lc[i][k] * Mi[k][j];
                    Mi[i][j] = t * invd[i];
                }
                for (i = NS - 1; i >= 0; --i) {
                    float t = Mi[i][j];
                    for (k = i + 1; k < NS; ++k) t = t - Lc[k][i] * Mi[k][j];
                    Mi[i][j] = t * invd[i];
                }
            }
        }
        /* row 0 of slot c: contact c's normal; rows 1, 2: anchor c's friction rows */
        for (c = 0; c < (nct > nanc ? nct : nanc); ++c) {
            int rw;
            for (rw = 0; rw < 3; ++rw) {
                const int a = rw == 0 ? ca[c] : aa[c], b = rw == 0 ? cb[c] : ab[c];
                const v3_t p = rw == 0 ? cp[c] : apt[c];
                const v3_t dir = cd[c][rw];
                float* J = Jr[c * 3 + rw];
                float* W = Wr[c * 3 + rw];
                int ln;
                if (rw == 0 ? c >= nct : c >= nanc) continue;
                for (ln = 0; ln < G; ++ln) {
                    float Jv = 0.0f, Wv = 0.0f;
                    if (a >= OE_LIM0) {
                        if (rw == 0 && ln == a - OE_LIM0) Jv = (float)b;
                    } else if (ln < D) {
                        if (a < OE_F0 && ln < 32 && ((amask[a] >> ln) & 1u)) {
                            const int jl = dlink[ln];
                            Jv = drev[ln] ? dot3(cross3(zl[jl], sub3(p, xl[jl])), dir) : dot3(zl[jl], dir);
                        }
                    } else if (ln < NS) {           /* floating root: unit spatial axes at x0 */
                        if (a < OE_F0) Jv = ln - D < 3 ? vc_(cross3(sub3(p, x0), dir), ln - D) : vc_(dir, ln - D - 3);
                    } else if ((ln - NS) / 6 < nfr) {
                        const int fk = (ln - NS) / 6, fc = (ln - NS) % 6;
                        const float sg = a == OE_F0 + fk ? 1.0f : (b == OE_F0 + fk ? -1.0f : 0.0f);
                        if (sg != 0.0f) {
                            const v3_t rd = cross3(sub3(p, fxc[fk]), dir);
                            if (fc < 3) {
                                const float dc = fc == 0 ? dir.x : (fc == 1 ? dir.y : dir.z);
                                Jv = sg * dc;
                                Wv = sg * (finvm[fk] * dc);
                            } else {
                                const v3_t iw = symmul_(fIw[fk], rd);
                                Jv = sg * (fc == 3 ? rd.x : (fc == 4 ? rd.y : rd.z));
                                Wv = sg * (fc == 3 ? iw.x : (fc == 4 ? iw.y : iw.z));
                            }
                        }
                    }
                    J[ln] = Jv;
                    W[ln] = Wv;
                }
                if (link_rows) {
                    for (ln = 0; ln < NS; ++ln) {
                        float w = 0.0f;
                        /* column ln of M_eff^-1 (the solve lane ln ran), entry k */
                        for (k = 0; k < NS; ++k) w = w + Mi[k][ln] * J[k];
                        W[ln] = w;
                    }
                }
                {
                    const float den = redp_(J, W, G);
                    ck[c][rw] = den > 0.0f ? 1.0f / den : 0.0f;
                }
                clam[c][rw] = 0.0f;
            }
            if (c < nct) cvn0[c] = redp_(Jr[c * 3], u, G);
        }

        /* ---- 4. TGS */
        for (it = 0; it < P->npos + P->nvel; ++it) {
            const int pos = it < P->npos;
            int ln;
            normal_pass_(P, nct, cs0, ce, cvn0, ck, clam, Jr, Wr, u, dp, G, pos);
            {   /* running sums restarting at a patch's first contact */
                float run = 0.0f;
                for (c = 0; c < nct; ++c) {
                    run = pstart[c] ? clam[c][0] : run + clam[c][0];
                    psum[c] = run;
                }
            }
            for (c = 0; c < nanc; ++c) {   /* anchors: close the drift, share mu N of the patch */
                const float mun = amu[c] * psum[alast[c]];
                int rw;
                for (rw = 1; rw < 3; ++rw) {
                    /* half the patch's budget mu N per direction for each of two anchors */
                    const float lim = (apart[c] ? 0.5f : 1.0f) * mun;
                    const float lam = clam[c][rw];
                    const float tg = pos ? ae[c][rw - 1] : 0.0f;
                    float raw, nl, dl;
                    raw = lam + ck[c][rw] * (tg - redp_(Jr[c * 3 + rw], u, G));
                    nl = fminf(fmaxf(raw, -lim), lim);
                    if (it == P->npos + P->nvel - 1) aclamp[c][rw - 1] = raw > lim || raw < -lim;
                    dl = nl - lam;
                    for (ln = 0; ln < G; ++ln) u[ln] = u[ln] + Wr[c * 3 + rw][ln] * dl;
                    clam[c][rw] = nl;
                }
            }
            /* slipping in the last iteration: every anchor of the patch clamped
             * along one direction; the patch lets go of its anchors */
            if (it == P->npos + P->nvel - 1) {
                for (c = 0; c < nanc; ++c) {
                    const int o = apart[c] == 1 ? c + 1 : (apart[c] == 2 ? c - 1 : c);
                    if (((aclamp[c][0] && aclamp[o][0]) || (aclamp[c][1] && aclamp[o][1])) && apair[c] < OE_FPP && fcr)
                        fcr[(size_t)apair[c] * (OE_FP_N + 1)] = 0.0f;
                }
            }
            /* the last position sweep and the velocity sweeps end with the normal rows again (mg_env.hip) */
            if (it >= P->npos - 1) normal_pass_(P, nct, cs0, ce, cvn0, ck, clam, Jr, Wr, u, dp, G, pos);
            if (pos)
                for (ln = 0; ln < G; ++ln) dp[ln] = dp[ln] + u[ln] * P->sub;
        }

        /* ---- 5. integrate */
        {
            float qn[OE_GM];
            for (d = 0; d < D; ++d) {
                const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
                const float maxv = pr[4];
                float w = u[d], x;
                if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
                x = q[d] + dp[d];
                if (pr[7] != 0.0f) {
                    const float lo = pr[5], hi = pr[6];
                    if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                    if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
                }
                qn[d] = x; u[d] = w;
            }
            for (d = 0; d < D; ++d) {   /* ball joints: th <- log(exp(th) exp(dpos)) */
                const int bk = dof_ball_(LF, LI, L, d);
                if (bk > 0) {
                    const int f = d - (bk - 1);
                    const v3_t tn = ball_step_(V(q[f], q[f + 1], q[f + 2]), V(dp[f], dp[f + 1], dp[f + 2]));
                    qn[d] = bk == 1 ? tn.x : (bk == 2 ? tn.y : tn.z);
                }
            }
            for (d = 0; d < D; ++d) q[d] = qn[d];
        }
        /* contact impulse sums: normal impulses in contact order, then the anchors' friction */
        for (c = 0; c < nct + nanc; ++c) {
            const int fr_ = c >= nct, kk = fr_ ? c - nct : c;
            const int a = fr_ ? aa[kk] : ca[kk], b = fr_ ? ab[kk] : cb[kk];
            v3_t imp;
            if (a >= OE_LIM0) continue;
            if (fr_) imp = mad3(mul3(cd[kk][1], clam[kk][1]), cd[kk][2], clam[kk][2]);
            else imp = mul3(cd[kk][0], clam[kk][0]);
            if (a >= OE_F0) fsum[a - OE_F0] = add3(fsum[a - OE_F0], imp);
            else lsum[a] = add3(lsum[a], imp);
            if (b >= OE_F0 && b < OE_ST0) fsum[b - OE_F0] = sub3(fsum[b - OE_F0], imp);
        }
        if (fb) {   /* floating root: the origin moves by dpos_v, the orientation turns by dpos_w */
            x0 = add3(x0, V(dp[D + 3], dp[D + 4], dp[D + 5]));
            q0 = qint_(q0, V(dp[D + 0], dp[D + 1], dp[D + 2]));
        }
        for (k = 0; k < nfr; ++k) {
            const int s0 = NS + 6 * k;
            const v3_t dx = V(dp[s0 + 0], dp[s0 + 1], dp[s0 + 2]);
            const v3_t dth = V(dp[s0 + 3], dp[s0 + 4], dp[s0 + 5]);
            const v3_t xc1 = add3(fxc[k], dx);
            fq[k] = qint_(fq[k], dth);
            fx[k] = sub3(xc1, qrot_(fq[k], fcom[k]));
        }
    }

    for (k = 0; k < nfr; ++k) {
        const int b = ev->free_b[k];
        float* s = state + (size_t)b * MG_STATE_N;
        s[0] = fx[k].x; s[1] = fx[k].y; s[2] = fx[k].z;
        s[3] = fq[k].x; s[4] = fq[k].y; s[5] = fq[k].z; s[6] = fq[k].w;
        for (i = 0; i < 6; ++i) s[7 + i] = u[NS + 6 * k + i];
        cforce[(size_t)b * 3 + 0] = fsum[k].x * P->inv_dt;
        cforce[(size_t)b * 3 + 1] = fsum[k].y * P->inv_dt;
        cforce[(size_t)b * 3 + 2] = fsum[k].z * P->inv_dt;
    }
    if (L == 0) return 0;
    for (d = 0; d < D; ++d) { dof[(d0 + d) * 2 + 0] = q[d]; dof[(d0 + d) * 2 + 1] = u[d]; }
    for (l = 0; l < L; ++l) {
        const int p = LI[l * MG_LINK_I_N + 0], jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
        const int bl = LI[l * MG_LINK_I_N + 3];      /* -1: virtual link (no body) */
        const float* M = link_mass_(m, LI, b0, l);
        float* so = bl >= 0 ? state + (size_t)(b0 + bl) * MG_STATE_N : NULL;
        v3_t ww, vw, com = V(M[8], M[9], M[10]);
        if (p < 0) {
            const q4_t qc = Q(-q0.x, -q0.y, -q0.z, q0.w);
            const v3_t w = fb ? V(u[D + 0], u[D + 1], u[D + 2]) : V(0.0f, 0.0f, 0.0f);
            const v3_t vo = fb ? V(u[D + 3], u[D + 4], u[D + 5]) : V(0.0f, 0.0f, 0.0f);
            ql[l] = q0; xl[l] = x0; vl[l] = SVc(qrot_(qc, w), qrot_(qc, vo));
        } else {
            q4_t qrel; v3_t rr; sv_t sj;
            const float qdj = dj >= 0 ? u[dj] : 0.0f;
            joint_(LF + l * MG_LINK_F_N, jt, q, dj, &qrel, &rr, &sj);
            ql[l] = qnorm_(qmul_(ql[p], qrel));
            xl[l] = add3(xl[p], qrot_(ql[p], rr));
            vl[l] = svadd_(xmot_(mt_(qmat_(qrel)), rr, vl[p]), svmul_(sj, qdj));
        }
        if (!so) continue;
        ww = qrot_(ql[l], vl[l].w);
        vw = qrot_(ql[l], add3(vl[l].v, cross3(vl[l].w, com)));
        so[0] = xl[l].x; so[1] = xl[l].y; so[2] = xl[l].z;
        so[3] = ql[l].x; so[4] = ql[l].y; so[5] = ql[l].z; so[6] = ql[l].w;
        so[7] = vw.x; so[8] = vw.y; so[9] = vw.z;
        so[10] = ww.x; so[11] = ww.y; so[12] = ww.z;
        cforce[(size_t)(b0 + bl) * 3 + 0] = lsum[l].x * P->inv_dt;
        cforce[(size_t)(b0 + bl) * 3 + 1] = lsum[l].y * P->inv_dt;
        cforce[(size_t)(b0 + bl) * 3 + 2] = lsum[l].z * P->inv_dt;
    }
    return 0;
}

/* Coupled-env classification (include/migym.h, actor_coll). Fills envs[] and
 * marks the root bodies the per-env step owns. Returns the env count, or -1. */
static int oe_collide_(const mg_model* m, int a, int b) {
    const int* ca = m->actor_coll + (size_t)a * MG_ACOLL_N;
    const int* cb = m->actor_coll + (size_t)b * MG_ACOLL_N;
    return (ca[1] == cb[1] || ca[1] == -1 || cb[1] == -1) && (ca[2] & cb[2]) == 0;
}

static int classify_envs_(const mg_model* m, oenv_t* envs, char* owned) {
    const int na = m->num_actors, nenv = m->num_envs;
    int e, a, n = 0, *start, *list;
    if (!m->actor_coll) return 0;
    /* actors bucketed by env, in actor order (counting sort) */
    start = (int*)calloc((size_t)nenv + 1, sizeof(int));
    list = (int*)malloc((size_t)(na > 0 ? na : 1) * sizeof(int));
    if (!start || !list) { free(start); free(list); return -1; }
    for (a = 0; a < na; ++a) {
        const int ea = m->actor_coll[(size_t)a * MG_ACOLL_N];
        if (ea < 0 || ea >= nenv) { free(start); free(list); return -1; }
        start[ea + 1]++;
    }
    for (e = 0; e < nenv; ++e) start[e + 1] += start[e];
    {
        int* fill = (int*)calloc((size_t)(nenv > 0 ? nenv : 1), sizeof(int));
        if (!fill) { free(start); free(list); return -1; }
        for (a = 0; a < na; ++a) {
            const int ea = m->actor_coll[(size_t)a * MG_ACOLL_N];
            list[start[ea] + fill[ea]++] = a;
        }
        free(fill);
    }
    for (e = 0; e < nenv; ++e) {
        int art[2], fr[OP_MAXB + 1], stc[OE_MAXS + 1], nart = 0, nf = 0, ns = 0, i, j, coupled = 0, mask = 0;
        int nart_all = 0, nf_all = 0, ns_all = 0, x;
        oenv_t* ev = &envs[n];
        for (x = start[e]; x < start[e + 1]; ++x) {
            const int r0 = m->actor_root_body[list[x]];
            const int kind = m->body_kind[r0];
            a = list[x];
            if (kind == MG_BODY_LINK) { if (nart < 2) art[nart++] = a; nart_all++; }
            else if (kind == MG_BODY_FREE) { if (nf <= OP_MAXB) fr[nf++] = a; nf_all++; }
            else { if (ns <= OE_MAXS) stc[ns++] = a; ns_all++; }
        }
        for (i = 0; i < nf; ++i) {
            for (j = 0; j < ns; ++j) coupled |= oe_collide_(m, fr[i], stc[j]);
            for (j = i + 1; j < nf; ++j) coupled |= oe_collide_(m, fr[i], fr[j]);
        }
        for (i = 0; i < nart; ++i) {
            const int r0 = m->actor_root_body[art[i]];
            for (j = 0; j < ns; ++j) coupled |= oe_collide_(m, art[i], stc[j]);
            for (j = 0; j < nf; ++j) coupled |= oe_collide_(m, art[i], fr[j]);
            for (j = 0; j < m->num_artics; ++j) {   /* a floating base always steps here */
                const int* ai = m->artic_i + (size_t)j * MG_ARTIC_I_N;
                if (ai[0] == r0 && !m->artic_tmpl_i[(size_t)ai[2] * MG_ATMPL_I_N + 3]) coupled = 1;
            }
        }
        if (!coupled) continue;
        ev->art_body = -1; ev->art_dof = 0; ev->art_tmpl = -1;
        ev->env = e;
        ev->pile = 0;
        if (nart_all == 0 && nf_all > OE_MAXF) {   /* a pile env (migym_oracle_pile.c) */
            if (nf_all > OP_MAXB || ns_all > OE_MAXS) { n = -1; break; }
            ev->pile = 1;
            ev->np = nf;
            for (i = 0; i < nf; ++i) {
                ev->pact[i] = fr[i];
                ev->pb[i] = m->actor_root_body[fr[i]];
                owned[ev->pb[i]] = 1;
            }
            ev->nf = 0;
            ev->free_b[0] = ev->pb[0];
            ev->ns = ns;
            for (i = 0; i < ns; ++i) { ev->sact[i] = stc[i]; ev->stat_b[i] = m->actor_root_body[stc[i]]; }
            ev->mask = 0;
            n++;
            continue;
        }
        if (nart_all > 1 || nf_all > OE_MAXF || ns_all > OE_MAXS) { n = -1; break; }
        if (nart == 1) {
            const int r0 = m->actor_root_body[art[0]];
            for (i = 0; i < m->num_artics; ++i) {
                const int* ai = m->artic_i + (size_t)i * MG_ARTIC_I_N;
                if (ai[0] == r0) { ev->art_body = r0; ev->art_dof = ai[1]; ev->art_tmpl = ai[2]; }
            }
            if (ev->art_body < 0) { n = -1; break; }
            owned[r0] = 1;
        }
        ev->nf = nf;
        for (i = 0; i < nf; ++i) { ev->free_b[i] = m->actor_root_body[fr[i]]; owned[ev->free_b[i]] = 1; }
        ev->ns = ns;
        for (i = 0; i < ns; ++i) ev->stat_b[i] = m->actor_root_body[stc[i]];
        for (i = 0; i < nf; ++i) {
            static const int pb[4][4] = {{-1, 0, 1, 2}, {-1, -1, 3, 4}, {-1, -1, -1, 5}, {-1, -1, -1, -1}};
            if (nart == 1 && oe_collide_(m, art[0], fr[i])) mask |= 1 << i;
            for (j = i + 1; j < nf; ++j)
                if (oe_collide_(m, fr[i], fr[j])) mask |= 1 << (8 + pb[i][j]);
            for (j = 0; j < ns; ++j)
                if (oe_collide_(m, fr[i], stc[j])) mask |= 1 << (14 + 4 * i + j);
        }
        for (j = 0; j < ns; ++j)
            if (nart == 1 && oe_collide_(m, art[0], stc[j])) mask |= 1 << (4 + j);
        ev->mask = mask;
        n++;
    }
    free(start);
    free(list);
    return n;
}

/* The OBB pair screen as a test entry point (shapes as oracle_collide2's, hull
 * records ha / hb): 1 when mg_env.hip's obb_apart rejects the pair. */
int oracle_obb_apart(const float* a, const float* ha, const float* b, const float* hb, float off) {
    float sa[MG_SHAPE_STRIDE] = {0}, sb[MG_SHAPE_STRIDE] = {0}, oa[6], ob[6];
    sa[0] = a[0]; sa[1] = a[8]; sa[2] = 0.0f; sa[3] = a[10]; sa[10] = 1.0f;
    sb[0] = b[0]; sb[1] = b[8]; sb[2] = 0.0f; sb[3] = b[10]; sb[10] = 1.0f;
    if ((int)a[0] == MG_SHAPE_BOX) sa[2] = a[9];
    if ((int)b[0] == MG_SHAPE_BOX) sb[2] = b[9];
    shape_obb_(sa, ha, oa);
    shape_obb_(sb, hb, ob);
    return obb_apart_boxes_(sa, V(a[1], a[2], a[3]), Q(a[4], a[5], a[6], a[7]), oa,
                            sb, V(b[1], b[2], b[3]), Q(b[4], b[5], b[6], b[7]), ob, off);
}

/* Narrow phase as a test entry point: shapes given as [type, c.xyz, q.xyzw,
 * h.xyz] (11 floats); out[4][7] = point.xyz, normal.xyz, separation. Returns
 * the contact count. */
int oracle_collide2(const float* a, const float* ha, const float* b, const float* hb, float margin, float* out) {
    cshape_t A, B;
    pair_t o;
    int k;
    A.type = (int)a[0]; A.c = V(a[1], a[2], a[3]); A.R = qmat_(Q(a[4], a[5], a[6], a[7])); A.h = V(a[8], a[9], a[10]);
    B.type = (int)b[0]; B.c = V(b[1], b[2], b[3]); B.R = qmat_(Q(b[4], b[5], b[6], b[7])); B.h = V(b[8], b[9], b[10]);
    A.hv = ha;
    B.hv = hb;
    o.n = 0;
    collide_(&A, &B, margin, &o);
    for (k = 0; k < o.n; ++k) {
        out[k * 7 + 0] = o.p[k].x; out[k * 7 + 1] = o.p[k].y; out[k * 7 + 2] = o.p[k].z;
        out[k * 7 + 3] = o.nrm[k].x; out[k * 7 + 4] = o.nrm[k].y; out[k * 7 + 5] = o.nrm[k].z;
        out[k * 7 + 6] = o.sep[k];
    }
    return o.n;
}

/* test entry: shapes as [type, c.xyz, q.xyzw, h.xyz]; hull records (convex) or NULL */
int oracle_collide(const float* a, const float* b, float margin, float* out) {
    return oracle_collide2(a, NULL, b, NULL, margin, out);
}
