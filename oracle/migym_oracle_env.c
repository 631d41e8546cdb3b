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

#define OE_MAXF 4
#define OE_MAXS 4
#define OE_MAXCT 20
#define OE_F0 16
#define OE_PMAX 4

typedef struct { int type; v3_t c; m3_t R; v3_t h; } cshape_t;
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
        sa = fminf(fmaxf(sa, -ha[ei]), ha[ei]);
        sb = fminf(fmaxf(sb, -hb[ej]), hb[ej]);
        ca = add3(pa, mul3(ua, sa));
        cb = add3(pb, mul3(ub, sb));
        ppush_(o, mul3(add3(ca, cb), 0.5f), mul3(ax, -1.0f), best_edge);
        return;
    }
    {
        const int refA = face < 3;
        const cshape_t* Rf = refA ? A : B;
        const cshape_t* In = refA ? B : A;
        const int fa = refA ? face : face - 3;
        const float hr[3] = {Rf->h.x, Rf->h.y, Rf->h.z}, hi[3] = {In->h.x, In->h.y, In->h.z};
        v3_t nref = mcol_(Rf->R, fa), iax, ifc, eu, ev, U, W, rc, inrm;
        int ik = 0, iu, iv, ru, rv, np = 4, side, m, used[8];
        float bestd = 1e30f, px[8], py[8], dep[8], den;
        v3_t pts[8];
        if (dot3(sub3(In->c, Rf->c), nref) < 0.0f) nref = mul3(nref, -1.0f);
        for (k = 0; k < 3; ++k) {
            const float dk = -fabsf(dot3(nref, mcol_(In->R, k)));
            if (dk < bestd) { bestd = dk; ik = k; }
        }
        iax = mcol_(In->R, ik);
        ifc = add3(In->c, mul3(iax, dot3(nref, iax) > 0.0f ? -hi[ik] : hi[ik]));
        iu = ik == 0 ? 1 : 0; iv = ik == 2 ? 1 : 2;
        eu = mul3(mcol_(In->R, iu), hi[iu]); ev = mul3(mcol_(In->R, iv), hi[iv]);
        ru = fa == 0 ? 1 : 0; rv = fa == 2 ? 1 : 2;
        U = mcol_(Rf->R, ru); W = mcol_(Rf->R, rv);
        rc = add3(Rf->c, mul3(nref, hr[fa]));
        {
            const v3_t q0 = sub3(sub3(ifc, eu), ev), q1 = sub3(add3(ifc, eu), ev);
            const v3_t q2 = add3(add3(ifc, eu), ev), q3 = add3(sub3(ifc, eu), ev);
            px[0] = dot3(sub3(q0, rc), U); py[0] = dot3(sub3(q0, rc), W);
            px[1] = dot3(sub3(q1, rc), U); py[1] = dot3(sub3(q1, rc), W);
            px[2] = dot3(sub3(q2, rc), U); py[2] = dot3(sub3(q2, rc), W);
            px[3] = dot3(sub3(q3, rc), U); py[3] = dot3(sub3(q3, rc), W);
        }
        for (side = 0; side < 4; ++side) {
            const float lim = side < 2 ? hr[ru] : hr[rv];
            const float sg = (side & 1) ? -1.0f : 1.0f;
            float ox[8], oy[8];
            int no = 0;
            for (k = 0; k < np; ++k) {
                const int k2 = k + 1 == np ? 0 : k + 1;
                const float a0 = sg * (side < 2 ? px[k] : py[k]) - lim;
                const float a1 = sg * (side < 2 ? px[k2] : py[k2]) - lim;
                if (a0 <= 0.0f && no < 8) { ox[no] = px[k]; oy[no] = py[k]; no = no + 1; }
                if ((a0 <= 0.0f) != (a1 <= 0.0f) && no < 8) {
                    const float tt = a0 / (a0 - a1);
                    ox[no] = px[k] + (px[k2] - px[k]) * tt;
                    oy[no] = py[k] + (py[k2] - py[k]) * tt;
                    no = no + 1;
                }
            }
            np = no;
            for (k = 0; k < np; ++k) { px[k] = ox[k]; py[k] = oy[k]; }
            if (np == 0) return;
        }
        inrm = mul3(iax, dot3(nref, iax) > 0.0f ? -1.0f : 1.0f);
        den = dot3(inrm, nref);
        for (k = 0; k < np; ++k) {
            const v3_t qq = add3(add3(rc, mul3(U, px[k])), mul3(W, py[k]));
            float tt = 0.0f;
            if (fabsf(den) > 1e-6f) tt = dot3(sub3(ifc, qq), inrm) / den;
            pts[k] = add3(qq, mul3(nref, tt));
            dep[k] = tt;
        }
        for (k = 0; k < 8; ++k) used[k] = 0;
        for (m = 0; m < OE_PMAX; ++m) {
            int bk = -1;
            float bd = margin;
            for (k = 0; k < np; ++k)
                if (!used[k] && dep[k] < bd) { bd = dep[k]; bk = k; }
            if (bk < 0) break;
            used[bk] = 1;
            {
                const v3_t n = refA ? mul3(nref, -1.0f) : nref;
                const v3_t pA = refA ? sub3(pts[bk], mul3(nref, dep[bk])) : pts[bk];
                ppush_(o, pA, n, dep[bk]);
            }
        }
    }
}

static void collide_(const cshape_t* A, const cshape_t* B, float margin, pair_t* o) {
    v3_t ca[2], cb[2];
    float ra, rb;
    int na, nbs, k, m;
    if (A->type == MG_SHAPE_BOX && B->type == MG_SHAPE_BOX) { box_box_(A, B, margin, o); return; }
    na = A->type == MG_SHAPE_CAPSULE ? 2 : 1;
    nbs = B->type == MG_SHAPE_CAPSULE ? 2 : 1;
    ra = A->h.x; rb = B->h.x;
    ca[0] = A->type == MG_SHAPE_CAPSULE ? sub3(A->c, mul3(A->R.c0, A->h.y)) : A->c;
    ca[1] = add3(A->c, mul3(A->R.c0, A->h.y));
    cb[0] = B->type == MG_SHAPE_CAPSULE ? sub3(B->c, mul3(B->R.c0, B->h.y)) : B->c;
    cb[1] = add3(B->c, mul3(B->R.c0, B->h.y));
    if (B->type == MG_SHAPE_BOX) {
        for (k = 0; k < na; ++k) sph_box_(ca[k], ra, B, margin, o);
        return;
    }
    if (A->type == MG_SHAPE_BOX) {
        pair_t t;
        t.n = 0;
        for (k = 0; k < nbs; ++k) sph_box_(cb[k], rb, A, margin, &t);
        for (k = 0; k < t.n; ++k) ppush_(o, add3(t.p[k], mul3(t.nrm[k], t.sep[k])), mul3(t.nrm[k], -1.0f), t.sep[k]);
        return;
    }
    for (k = 0; k < na; ++k)
        for (m = 0; m < nbs; ++m) sph_sph_(ca[k], ra, cb[m], rb, margin, o);
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

static cshape_t place_(const float* sh, v3_t x, q4_t q) {
    cshape_t c;
    c.type = (int)sh[0];
    c.c = add3(x, qrot_(q, V(sh[4], sh[5], sh[6])));
    c.R = qmat_(qmul_(q, Q(sh[7], sh[8], sh[9], sh[10])));
    c.h = V(sh[1], sh[2], sh[3]);
    return c;
}

static void ground_pair_(const step_t* P, const cshape_t* s, pair_t* o) {
    const v3_t n = P->n;
    const float off = P->co;
    int k;
    if (s->type == MG_SHAPE_BOX) {
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

typedef struct {
    int a, b;
    v3_t d[3], ra, rb;
    float s0, mu, e, vn0, k[3], lam[3];
} ect_t;

/* env description, as the library's env_i row but with global body ids */
typedef struct {
    int art_body, art_dof, art_tmpl, nf, free_b[OE_MAXF], ns, stat_b[OE_MAXS], mask;
} oenv_t;

typedef struct {
    const step_t* P;
    const mg_model* m;
    const float* props;
    const float* tgt;
    float* state;
    int L, D;
    const int* LI;
    int nct;
    ect_t ct[OE_MAXCT];
    float Jr[OE_MAXCT * 3][OR_MAXL], Wr[OE_MAXCT * 3][OR_MAXL];
    float q[OR_MAXL], qd[OR_MAXL], dq[OR_MAXL];
    v3_t fv[OE_MAXF], fw[OE_MAXF], fdx[OE_MAXF], fdth[OE_MAXF], fxc[OE_MAXF];
    float finvm[OE_MAXF];
    s3_t fIw[OE_MAXF];
} ectx_t;

static void eadd_(ectx_t* X, int a, int b, const pair_t* o, float mu, float rest) {
    int j;
    for (j = 0; j < o->n; ++j) {
        ect_t* c;
        if (X->nct >= OE_MAXCT) return;
        c = &X->ct[X->nct];
        c->a = a; c->b = b;
        c->d[0] = o->nrm[j];
        tangents_(o->nrm[j], &c->d[1], &c->d[2]);
        c->ra = a >= OE_F0 ? sub3(o->p[j], X->fxc[a - OE_F0]) : o->p[j];
        c->rb = b >= OE_F0 ? sub3(o->p[j], X->fxc[b - OE_F0]) : V(0.0f, 0.0f, 0.0f);
        c->s0 = o->sep[j] - X->P->ro;
        c->mu = mu; c->e = rest;
        X->nct = X->nct + 1;
    }
}

static float erel_(const ectx_t* X, const ect_t* C, int c, int rw, int motion) {
    const v3_t dir = C->d[rw];
    float va = 0.0f, vb = 0.0f;
    int d;
    if (C->a >= OE_F0) {
        const int k = C->a - OE_F0;
        va = motion ? dot3(dir, X->fdx[k]) + dot3(X->fdth[k], cross3(C->ra, dir))
                    : dot3(dir, X->fv[k]) + dot3(X->fw[k], cross3(C->ra, dir));
    } else {
        const float* J = X->Jr[c * 3 + rw];
        for (d = 0; d < X->D; ++d) va = va + J[d] * (motion ? X->dq[d] : X->qd[d]);
    }
    if (C->b >= OE_F0) {
        const int k = C->b - OE_F0;
        vb = motion ? dot3(dir, X->fdx[k]) + dot3(X->fdth[k], cross3(C->rb, dir))
                    : dot3(dir, X->fv[k]) + dot3(X->fw[k], cross3(C->rb, dir));
    }
    return va - vb;
}

static void eapply_(ectx_t* X, const ect_t* C, int c, int rw, float dl) {
    const v3_t dir = C->d[rw];
    int d;
    if (C->a >= OE_F0) {
        const int k = C->a - OE_F0;
        X->fv[k] = mad3(X->fv[k], dir, dl * X->finvm[k]);
        X->fw[k] = mad3(X->fw[k], symmul_(X->fIw[k], cross3(C->ra, dir)), dl);
    } else {
        const float* W = X->Wr[c * 3 + rw];
        for (d = 0; d < X->D; ++d) X->qd[d] = X->qd[d] + W[d] * dl;
    }
    if (C->b >= OE_F0) {
        const int k = C->b - OE_F0;
        X->fv[k] = mad3(X->fv[k], dir, -(dl * X->finvm[k]));
        X->fw[k] = mad3(X->fw[k], symmul_(X->fIw[k], cross3(C->rb, dir)), -dl);
    }
}

static void enormal_(ectx_t* X, int c, float tgt) {
    ect_t* C = &X->ct[c];
    float dl = C->k[0] * (tgt - erel_(X, C, c, 0, 0));
    const float nl = fmaxf(C->lam[0] + dl, 0.0f);
    dl = nl - C->lam[0];
    C->lam[0] = nl;
    eapply_(X, C, c, 0, dl);
}

static void efriction_(ectx_t* X, int c) {
    ect_t* C = &X->ct[c];
    const float lim = C->mu * C->lam[0];
    int rw;
    for (rw = 1; rw < 3; ++rw) {
        const float nl = fminf(fmaxf(C->lam[rw] - C->k[rw] * erel_(X, C, c, rw, 0), -lim), lim);
        const float dl = nl - C->lam[rw];
        C->lam[rw] = nl;
        eapply_(X, C, c, rw, dl);
    }
}

static const float* shp_(const mg_model* m, int s) { return m->shapes + (size_t)s * MG_SHAPE_STRIDE; }

static si_t link_inertia_(const float* M) {
    const float mass = M[11];
    const v3_t com = V(M[8], M[9], M[10]);
    const q4_t iq = Q(M[4], M[5], M[6], M[7]);
    const v3_t Id = V(M[1] > 0.0f ? 1.0f / M[1] : 0.0f, M[2] > 0.0f ? 1.0f / M[2] : 0.0f, M[3] > 0.0f ? 1.0f / M[3] : 0.0f);
    const m3_t Rq = qmat_(iq);
    return sirigid_(mass, com, mmul_(mmul_(Rq, M3c(V(Id.x, 0.0f, 0.0f), V(0.0f, Id.y, 0.0f), V(0.0f, 0.0f, Id.z))), mt_(Rq)));
}

static int env_step_(const step_t* P, const mg_model* m, const oenv_t* ev, float* state, float* dof, const float* tgt,
                     const float* props, const float* ext, float* cforce) {
    static ectx_t X;   /* large scratch; the oracle is single-threaded */
    const int b0 = ev->art_body, d0 = ev->art_dof, nfr = ev->nf, nst = ev->ns, cmask = ev->mask;
    const int* ti = ev->art_tmpl >= 0 ? m->artic_tmpl_i + (size_t)ev->art_tmpl * MG_ATMPL_I_N : NULL;
    const int L = ti ? ti[1] : 0, D = ti ? ti[2] : 0;
    const float* LF = ti ? m->tmpl_link_f + (size_t)ti[0] * MG_LINK_F_N : NULL;
    const int* LI = ti ? m->tmpl_link_i + (size_t)ti[0] * MG_LINK_I_N : NULL;
    const float h = P->h;
    const v3_t gvec = V(P->g[0], P->g[1], P->g[2]);
    v3_t x0 = V(0.0f, 0.0f, 0.0f), gb = V(0.0f, 0.0f, 0.0f);
    q4_t q0 = Q(0.0f, 0.0f, 0.0f, 1.0f);
    float mdiag[OR_MAXL], qdd[OR_MAXL], tau0d[OR_MAXL], impd[OR_MAXL];
    v3_t lsum[OR_MAXL];
    v3_t fx[OE_MAXF], fcom[OE_MAXF], finvI[OE_MAXF], fsum[OE_MAXF], fext[OE_MAXF], text[OE_MAXF];
    q4_t fq[OE_MAXF], fiq[OE_MAXF];
    float lkeep[OE_MAXF], akeep[OE_MAXF], mlv2[OE_MAXF], mav2[OE_MAXF], gon[OE_MAXF];
    m3_t E[OR_MAXL];
    v3_t r[OR_MAXL], xl[OR_MAXL], zl[OR_MAXL];
    sv_t Sj[OR_MAXL], vl[OR_MAXL], cl[OR_MAXL], pA[OR_MAXL], U[OR_MAXL], al[OR_MAXL];
    si_t IA[OR_MAXL];
    float Dl[OR_MAXL], ul[OR_MAXL], Mf[OR_MAXL][OR_MAXL], invd[OR_MAXL];
    q4_t ql[OR_MAXL];
    int d, l, k, c, st_, it;
    if (L > OR_MAXL || (ti && !ti[3])) return -1;
    X.P = P; X.m = m; X.props = props; X.tgt = tgt; X.state = state; X.L = L; X.D = D; X.LI = LI;
    if (L > 0) {
        const float* s0 = state + (size_t)b0 * MG_STATE_N;
        const float grav_on = m->tmpl_body_f[(size_t)m->body_tmpl[b0] * MG_TBODY_F_N + 4];
        x0 = V(s0[0], s0[1], s0[2]);
        q0 = qnorm_(Q(s0[3], s0[4], s0[5], s0[6]));
        gb = qrot_(Q(-q0.x, -q0.y, -q0.z, q0.w), grav_on != 0.0f ? gvec : V(0.0f, 0.0f, 0.0f));
    }
    for (d = 0; d < D; ++d) { X.q[d] = dof[(d0 + d) * 2 + 0]; X.qd[d] = dof[(d0 + d) * 2 + 1]; }
    for (l = 0; l < L; ++l) lsum[l] = V(0.0f, 0.0f, 0.0f);
    for (k = 0; k < nfr; ++k) {
        const int b = ev->free_b[k];
        const float* s = state + (size_t)b * MG_STATE_N;
        const float* M = m->body_mass + (size_t)b * MG_MASS_N;
        const float* tf = m->tmpl_body_f + (size_t)m->body_tmpl[b] * MG_TBODY_F_N;
        fx[k] = V(s[0], s[1], s[2]);
        fq[k] = qnorm_(Q(s[3], s[4], s[5], s[6]));
        X.fv[k] = V(s[7], s[8], s[9]);
        X.fw[k] = V(s[10], s[11], s[12]);
        X.finvm[k] = M[0];
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
        int first_link_row;
        if (L > 0) {
          unsigned xmask = 0u, xpos = 0u;
          int att;
          for (att = 0; att < 2; ++att) {
            unsigned nm;
            for (l = 0; l < L; ++l) {
                const int p = LI[l * MG_LINK_I_N + 0], jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
                if (p < 0) {
                    E[l] = M3c(V(1.0f, 0.0f, 0.0f), V(0.0f, 1.0f, 0.0f), V(0.0f, 0.0f, 1.0f));
                    r[l] = V(0.0f, 0.0f, 0.0f);
                    Sj[l] = sv0(); vl[l] = sv0(); cl[l] = sv0();
                    ql[l] = q0; xl[l] = x0; zl[l] = V(0.0f, 0.0f, 0.0f);
                } else {
                    q4_t qrel; v3_t rr; sv_t s, vJ;
                    const float* lf = LF + l * MG_LINK_F_N;
                    const float qj = dj >= 0 ? X.q[dj] : 0.0f, qdj = dj >= 0 ? X.qd[dj] : 0.0f;
                    joint_(lf, jt, qj, &qrel, &rr, &s);
                    E[l] = mt_(qmat_(qrel));
                    r[l] = rr;
                    Sj[l] = s;
                    vJ = svmul_(s, qdj);
                    vl[l] = svadd_(xmot_(E[l], rr, vl[p]), vJ);
                    cl[l] = crm_(vl[l], vJ);
                    ql[l] = qnorm_(qmul_(ql[p], qrel));
                    xl[l] = add3(xl[p], qrot_(ql[p], rr));
                    zl[l] = qrot_(ql[l], V(lf[7], lf[8], lf[9]));
                }
                IA[l] = link_inertia_(m->body_mass + (size_t)(b0 + l) * MG_MASS_N);
                pA[l] = crf_(vl[l], simul_(IA[l], vl[l]));
            }
            for (l = L - 1; l >= 1; --l) {
                const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
                si_t Ia = IA[l];
                sv_t pa;
                if (dj >= 0) {
                    const float* pr = props + (size_t)(d0 + dj) * MG_DOFPROP_N;
                    const float* tg = tgt + (size_t)(d0 + dj) * 3;
                    const int mode = (int)pr[0];
                    const float kp = pr[1], kd = pr[2], eff = pr[3], arm = pr[8];
                    float tau = 0.0f, imp = 0.0f, invD;
                    if (mode == MG_DOF_MODE_POS) {
                        tau = kp * (tg[0] - X.q[dj] - h * X.qd[dj]) + kd * (tg[1] - X.qd[dj]);
                        imp = h * kd + h * h * kp;
                    } else if (mode == MG_DOF_MODE_VEL) {
                        tau = kd * (tg[1] - X.qd[dj]);
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
                    tau0d[dj] = tau;
                    impd[dj] = imp;
                    mdiag[dj] = arm + imp;
                    U[l] = simul_(Ia, Sj[l]);
                    Dl[l] = svdot_(Sj[l], U[l]) + arm + imp;
                    ul[l] = tau - svdot_(Sj[l], pA[l]);
                    invD = 1.0f / Dl[l];
                    Ia.A = msub_(Ia.A, mouter_(U[l].w, U[l].w, invD));
                    Ia.B = msub_(Ia.B, mouter_(U[l].w, U[l].v, invD));
                    Ia.C = msub_(Ia.C, mouter_(U[l].v, U[l].v, invD));
                    pa = svadd_(svadd_(pA[l], simul_(Ia, cl[l])), svmul_(U[l], ul[l] * invD));
                } else {
                    pa = svadd_(pA[l], simul_(Ia, cl[l]));
                }
                if (p > 0) {
                    IA[p] = siadd_(IA[p], xin_t_(E[l], r[l], Ia));
                    pA[p] = svadd_(pA[p], xfrc_t_(E[l], r[l], pa));
                }
            }
            al[0] = SVc(V(0.0f, 0.0f, 0.0f), mul3(gb, -1.0f));
            for (l = 1; l < L; ++l) {
                const int p = LI[l * MG_LINK_I_N + 0], dj = LI[l * MG_LINK_I_N + 2];
                sv_t ap = svadd_(xmot_(E[l], r[l], al[p]), cl[l]);
                if (dj >= 0) {
                    const float acc = (ul[l] - svdot_(U[l], ap)) / Dl[l];
                    qdd[dj] = acc;
                    ap = svadd_(ap, svmul_(Sj[l], acc));
                }
                al[l] = ap;
            }
            nm = xmask;
            for (d = 0; d < D; ++d) {
                const float eff = props[(size_t)(d0 + d) * MG_DOFPROP_N + 3];
                if (eff > 0.0f && impd[d] != 0.0f) {
                    const float act = tau0d[d] - impd[d] * qdd[d];
                    if (act > eff) { nm |= 1u << d; xpos |= 1u << d; }
                    else if (act < -eff) nm |= 1u << d;
                }
            }
            if (nm == xmask) break;
            xmask = nm;
          }
            for (d = 0; d < D; ++d) {
                const float maxv = props[(size_t)(d0 + d) * MG_DOFPROP_N + 4];
                float w = X.qd[d] + h * qdd[d];
                if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
                X.qd[d] = w;
                X.dq[d] = 0.0f;
            }
        }
        for (k = 0; k < nfr; ++k) {
            v3_t v = X.fv[k], w = X.fw[k];
            float v2, w2;
            X.fIw[k] = sym_rdrt_(qmat_(qmul_(fq[k], fiq[k])), finvI[k]);
            X.fxc[k] = add3(fx[k], qrot_(fq[k], fcom[k]));
            if (gon[k] != 0.0f) v = mad3(v, gvec, h);
            v = mad3(v, fext[k], X.finvm[k] * h);
            w = mad3(w, symmul_(X.fIw[k], text[k]), h);
            v = mul3(v, lkeep[k]);
            w = mul3(w, akeep[k]);
            v2 = dot3(v, v);
            if (v2 > mlv2[k]) v = mul3(v, sqrtf(mlv2[k] / v2));
            w2 = dot3(w, w);
            if (w2 > mav2[k]) w = mul3(w, sqrtf(mav2[k] / w2));
            X.fv[k] = v; X.fw[k] = w;
            X.fdx[k] = V(0.0f, 0.0f, 0.0f); X.fdth[k] = V(0.0f, 0.0f, 0.0f);
        }

        /* contacts, in the device's pair order */
        X.nct = 0;
        for (k = 0; k < nfr; ++k) {
            const int bk = ev->free_b[k];
            const int* tk = m->tmpl_body_i + (size_t)m->body_tmpl[bk] * MG_TBODY_I_N;
            int sa, s, j, sb;
            for (sa = tk[0]; sa < tk[0] + tk[1]; ++sa) {
                const float* sha = shp_(m, sa);
                const cshape_t ca = place_(sha, fx[k], fq[k]);
                pair_t o;
                if (P->ground) {
                    o.n = 0;
                    ground_pair_(P, &ca, &o);
                    eadd_(&X, OE_F0 + k, -1, &o, 0.5f * (sha[11] + P->mu_g), 0.5f * (sha[12] + P->e_g));
                }
                for (s = 0; s < nst; ++s) {
                    const int bs = ev->stat_b[s];
                    const float* ss = state + (size_t)bs * MG_STATE_N;
                    const int* ts = m->tmpl_body_i + (size_t)m->body_tmpl[bs] * MG_TBODY_I_N;
                    const v3_t xs = V(ss[0], ss[1], ss[2]);
                    const q4_t qs = qnorm_(Q(ss[3], ss[4], ss[5], ss[6]));
                    if (!((cmask >> (14 + k * 4 + s)) & 1)) continue;
                    for (sb = ts[0]; sb < ts[0] + ts[1]; ++sb) {
                        const float* shb = shp_(m, sb);
                        const cshape_t cb = place_(shb, xs, qs);
                        o.n = 0;
                        collide_(&ca, &cb, P->co, &o);
                        eadd_(&X, OE_F0 + k, -1, &o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                for (j = k + 1; j < nfr; ++j) {
                    const int bit = k == 0 ? j - 1 : (k == 1 ? j + 1 : 5);
                    const int bj = ev->free_b[j];
                    const int* tj = m->tmpl_body_i + (size_t)m->body_tmpl[bj] * MG_TBODY_I_N;
                    if (!((cmask >> (8 + bit)) & 1)) continue;
                    for (sb = tj[0]; sb < tj[0] + tj[1]; ++sb) {
                        const float* shb = shp_(m, sb);
                        const cshape_t cb = place_(shb, fx[j], fq[j]);
                        o.n = 0;
                        collide_(&ca, &cb, P->co, &o);
                        eadd_(&X, OE_F0 + k, OE_F0 + j, &o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                if (L > 0 && ((cmask >> k) & 1)) {
                    const int* t0 = m->tmpl_body_i + (size_t)m->body_tmpl[b0] * MG_TBODY_I_N;
                    for (sb = t0[0]; sb < t0[0] + t0[1]; ++sb) {
                        const float* shb = shp_(m, sb);
                        const cshape_t cb = place_(shb, xl[0], ql[0]);
                        o.n = 0;
                        collide_(&ca, &cb, P->co, &o);
                        eadd_(&X, OE_F0 + k, -1, &o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
            }
        }
        first_link_row = X.nct;
        for (l = 1; l < L; ++l) {
            const int* tl = m->tmpl_body_i + (size_t)m->body_tmpl[b0 + l] * MG_TBODY_I_N;
            int sa, s, sb;
            for (sa = tl[0]; sa < tl[0] + tl[1]; ++sa) {
                const float* sha = shp_(m, sa);
                const cshape_t ca = place_(sha, xl[l], ql[l]);
                pair_t o;
                if (P->ground) {
                    o.n = 0;
                    ground_pair_(P, &ca, &o);
                    eadd_(&X, l, -1, &o, 0.5f * (sha[11] + P->mu_g), 0.5f * (sha[12] + P->e_g));
                }
                for (s = 0; s < nst; ++s) {
                    const int bs = ev->stat_b[s];
                    const float* ss = state + (size_t)bs * MG_STATE_N;
                    const int* ts = m->tmpl_body_i + (size_t)m->body_tmpl[bs] * MG_TBODY_I_N;
                    const v3_t xs = V(ss[0], ss[1], ss[2]);
                    const q4_t qs = qnorm_(Q(ss[3], ss[4], ss[5], ss[6]));
                    if (!((cmask >> (4 + s)) & 1)) continue;
                    for (sb = ts[0]; sb < ts[0] + ts[1]; ++sb) {
                        const float* shb = shp_(m, sb);
                        const cshape_t cb = place_(shb, xs, qs);
                        o.n = 0;
                        collide_(&ca, &cb, P->co, &o);
                        eadd_(&X, l, -1, &o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
                for (k = 0; k < nfr; ++k) {
                    const int bk = ev->free_b[k];
                    const int* tk = m->tmpl_body_i + (size_t)m->body_tmpl[bk] * MG_TBODY_I_N;
                    if (!((cmask >> k) & 1)) continue;
                    for (sb = tk[0]; sb < tk[0] + tk[1]; ++sb) {
                        const float* shb = shp_(m, sb);
                        const cshape_t cb = place_(shb, fx[k], fq[k]);
                        o.n = 0;
                        collide_(&ca, &cb, P->co, &o);
                        eadd_(&X, l, OE_F0 + k, &o, 0.5f * (sha[11] + shb[11]), 0.5f * (sha[12] + shb[12]));
                    }
                }
            }
        }

        /* rows */
        if (X.nct > first_link_row) {
            int i, j;
            for (l = 0; l < L; ++l) IA[l] = link_inertia_(m->body_mass + (size_t)(b0 + l) * MG_MASS_N);
            for (i = 0; i < D; ++i)
                for (j = 0; j < D; ++j) Mf[i][j] = 0.0f;
            for (l = L - 1; l >= 1; --l) {
                const int p = LI[l * MG_LINK_I_N + 0];
                if (p > 0) IA[p] = siadd_(IA[p], xin_t_(E[l], r[l], IA[l]));
            }
            for (l = 1; l < L; ++l) {
                const int di = LI[l * MG_LINK_I_N + 2];
                sv_t Fv;
                if (di < 0) continue;
                Fv = simul_(IA[l], Sj[l]);
                Mf[di][di] = svdot_(Sj[l], Fv) + mdiag[di];
                j = l;
                while (LI[j * MG_LINK_I_N + 0] > 0) {
                    int dj;
                    Fv = xfrc_t_(E[j], r[j], Fv);
                    j = LI[j * MG_LINK_I_N + 0];
                    dj = LI[j * MG_LINK_I_N + 2];
                    if (dj >= 0) {
                        const float hv = svdot_(Fv, Sj[j]);
                        Mf[di][dj] = hv;
                        Mf[dj][di] = hv;
                    }
                }
            }
            for (j = 0; j < D; ++j) {
                float s = Mf[j][j], dj;
                for (k = 0; k < j; ++k) s = s - Mf[j][k] * Mf[j][k];
                dj = sqrtf(s);
                invd[j] = 1.0f / dj;
                Mf[j][j] = dj;
                for (i = j + 1; i < D; ++i) {
                    float t = Mf[i][j];
                    for (k = 0; k < j; ++k) t = t - Mf[i][k] * Mf[j][k];
                    Mf[i][j] = t * invd[j];
                }
            }
        }
        for (c = 0; c < X.nct; ++c) {
            ect_t* C = &X.ct[c];
            const v3_t pw = C->a < OE_F0 ? C->ra : add3(C->ra, X.fxc[C->a - OE_F0]);
            int rw;
            for (rw = 0; rw < 3; ++rw) {
                const v3_t dir = C->d[rw];
                float wa = 0.0f, wb = 0.0f;
                if (C->a >= OE_F0) {
                    const int kk = C->a - OE_F0;
                    const v3_t rd = cross3(C->ra, dir);
                    wa = X.finvm[kk] + dot3(rd, symmul_(X.fIw[kk], rd));
                } else {
                    float* J = X.Jr[c * 3 + rw];
                    float* W = X.Wr[c * 3 + rw];
                    int j = C->a, i;
                    for (d = 0; d < D; ++d) J[d] = 0.0f;
                    while (j > 0) {
                        const int dof_ = LI[j * MG_LINK_I_N + 2];
                        if (dof_ >= 0) {
                            if (LI[j * MG_LINK_I_N + 1] == MG_JOINT_REVOLUTE) J[dof_] = dot3(cross3(zl[j], sub3(pw, xl[j])), dir);
                            else J[dof_] = dot3(zl[j], dir);
                        }
                        j = LI[j * MG_LINK_I_N + 0];
                    }
                    for (i = 0; i < D; ++i) {
                        float t = J[i];
                        for (k = 0; k < i; ++k) t = t - Mf[i][k] * W[k];
                        W[i] = t * invd[i];
                    }
                    for (i = D - 1; i >= 0; --i) {
                        float t = W[i];
                        for (k = i + 1; k < D; ++k) t = t - Mf[k][i] * W[k];
                        W[i] = t * invd[i];
                    }
                    for (d = 0; d < D; ++d) wa = wa + J[d] * W[d];
                }
                if (C->b >= OE_F0) {
                    const int kk = C->b - OE_F0;
                    const v3_t rd = cross3(C->rb, dir);
                    wb = X.finvm[kk] + dot3(rd, symmul_(X.fIw[kk], rd));
                }
                C->k[rw] = 1.0f / (wa + wb);
                C->lam[rw] = 0.0f;
            }
        }
        for (c = 0; c < X.nct; ++c) X.ct[c].vn0 = erel_(&X, &X.ct[c], c, 0, 0);

        for (it = 0; it < P->npos; ++it) {
            for (c = 0; c < X.nct; ++c) {
                const float s = X.ct[c].s0 + erel_(&X, &X.ct[c], c, 0, 1);
                float tg = -s * P->inv_sub;
                if (s < 0.0f) tg = fminf(tg, P->maxdep);
                enormal_(&X, c, tg);
            }
            for (c = 0; c < X.nct; ++c) efriction_(&X, c);
            for (d = 0; d < D; ++d) X.dq[d] = X.dq[d] + X.qd[d] * P->sub;
            for (k = 0; k < nfr; ++k) {
                X.fdx[k] = mad3(X.fdx[k], X.fv[k], P->sub);
                X.fdth[k] = mad3(X.fdth[k], X.fw[k], P->sub);
            }
        }
        for (it = 0; it < P->nvel; ++it) {
            for (c = 0; c < X.nct; ++c) {
                const float s = X.ct[c].s0 + erel_(&X, &X.ct[c], c, 0, 1);
                float tg = s > 0.0f ? -s * P->inv_h : 0.0f;
                if (X.ct[c].e > 0.0f && X.ct[c].vn0 < -P->bounce) tg = fmaxf(tg, -X.ct[c].e * X.ct[c].vn0);
                enormal_(&X, c, tg);
            }
            for (c = 0; c < X.nct; ++c) efriction_(&X, c);
        }
        for (c = 0; c < X.nct; ++c) {
            const ect_t* C = &X.ct[c];
            v3_t imp = mul3(C->d[0], C->lam[0]);
            imp = mad3(imp, C->d[1], C->lam[1]);
            imp = mad3(imp, C->d[2], C->lam[2]);
            if (C->a >= OE_F0) fsum[C->a - OE_F0] = add3(fsum[C->a - OE_F0], imp);
            else if (C->a >= 0) lsum[C->a] = add3(lsum[C->a], imp);
            if (C->b >= OE_F0) fsum[C->b - OE_F0] = sub3(fsum[C->b - OE_F0], imp);
        }
        for (d = 0; d < D; ++d) {
            const float* pr = props + (size_t)(d0 + d) * MG_DOFPROP_N;
            const float maxv = pr[4];
            float w = X.qd[d], x;
            if (maxv > 0.0f) w = fminf(fmaxf(w, -maxv), maxv);
            x = X.q[d] + X.dq[d];
            if (pr[7] != 0.0f) {
                const float lo = pr[5], hi = pr[6];
                if (x < lo) { x = lo; if (w < 0.0f) w = 0.0f; }
                if (x > hi) { x = hi; if (w > 0.0f) w = 0.0f; }
            }
            X.q[d] = x; X.qd[d] = w;
        }
        for (k = 0; k < nfr; ++k) {
            const v3_t xc1 = add3(X.fxc[k], X.fdx[k]);
            fq[k] = qint_(fq[k], X.fdth[k]);
            fx[k] = sub3(xc1, qrot_(fq[k], fcom[k]));
        }
    }

    for (k = 0; k < nfr; ++k) {
        const int b = ev->free_b[k];
        float* s = state + (size_t)b * MG_STATE_N;
        s[0] = fx[k].x; s[1] = fx[k].y; s[2] = fx[k].z;
        s[3] = fq[k].x; s[4] = fq[k].y; s[5] = fq[k].z; s[6] = fq[k].w;
        s[7] = X.fv[k].x; s[8] = X.fv[k].y; s[9] = X.fv[k].z;
        s[10] = X.fw[k].x; s[11] = X.fw[k].y; s[12] = X.fw[k].z;
        cforce[(size_t)b * 3 + 0] = fsum[k].x * P->inv_dt;
        cforce[(size_t)b * 3 + 1] = fsum[k].y * P->inv_dt;
        cforce[(size_t)b * 3 + 2] = fsum[k].z * P->inv_dt;
    }
    if (L == 0) return 0;
    for (d = 0; d < D; ++d) { dof[(d0 + d) * 2 + 0] = X.q[d]; dof[(d0 + d) * 2 + 1] = X.qd[d]; }
    for (l = 0; l < L; ++l) {
        const int p = LI[l * MG_LINK_I_N + 0], jt = LI[l * MG_LINK_I_N + 1], dj = LI[l * MG_LINK_I_N + 2];
        const float* M = m->body_mass + (size_t)(b0 + l) * MG_MASS_N;
        float* so = state + (size_t)(b0 + l) * MG_STATE_N;
        v3_t ww, vw, com = V(M[8], M[9], M[10]);
        if (p < 0) {
            ql[l] = q0; xl[l] = x0; vl[l] = sv0();
        } else {
            q4_t qrel; v3_t rr; sv_t s;
            const float qj = dj >= 0 ? X.q[dj] : 0.0f, qdj = dj >= 0 ? X.qd[dj] : 0.0f;
            joint_(LF + l * MG_LINK_F_N, jt, qj, &qrel, &rr, &s);
            ql[l] = qnorm_(qmul_(ql[p], qrel));
            xl[l] = add3(xl[p], qrot_(ql[p], rr));
            vl[l] = svadd_(xmot_(mt_(qmat_(qrel)), rr, vl[p]), svmul_(s, qdj));
        }
        ww = qrot_(ql[l], vl[l].w);
        vw = qrot_(ql[l], add3(vl[l].v, cross3(vl[l].w, com)));
        so[0] = xl[l].x; so[1] = xl[l].y; so[2] = xl[l].z;
        so[3] = ql[l].x; so[4] = ql[l].y; so[5] = ql[l].z; so[6] = ql[l].w;
        so[7] = vw.x; so[8] = vw.y; so[9] = vw.z;
        so[10] = ww.x; so[11] = ww.y; so[12] = ww.z;
        cforce[(size_t)(b0 + l) * 3 + 0] = lsum[l].x * P->inv_dt;
        cforce[(size_t)(b0 + l) * 3 + 1] = lsum[l].y * P->inv_dt;
        cforce[(size_t)(b0 + l) * 3 + 2] = lsum[l].z * P->inv_dt;
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
        int art[2], fr[OE_MAXF + 1], stc[OE_MAXS + 1], nart = 0, nf = 0, ns = 0, i, j, coupled = 0, mask = 0;
        int nart_all = 0, nf_all = 0, ns_all = 0, x;
        oenv_t* ev = &envs[n];
        for (x = start[e]; x < start[e + 1]; ++x) {
            const int r0 = m->actor_root_body[list[x]];
            const int kind = m->body_kind[r0];
            a = list[x];
            if (kind == MG_BODY_LINK) { if (nart < 2) art[nart++] = a; nart_all++; }
            else if (kind == MG_BODY_FREE) { if (nf <= OE_MAXF) fr[nf++] = a; nf_all++; }
            else { if (ns <= OE_MAXS) stc[ns++] = a; ns_all++; }
        }
        for (i = 0; i < nf; ++i) {
            for (j = 0; j < ns; ++j) coupled |= oe_collide_(m, fr[i], stc[j]);
            for (j = i + 1; j < nf; ++j) coupled |= oe_collide_(m, fr[i], fr[j]);
        }
        for (i = 0; i < nart; ++i) {
            for (j = 0; j < ns; ++j) coupled |= oe_collide_(m, art[i], stc[j]);
            for (j = 0; j < nf; ++j) coupled |= oe_collide_(m, art[i], fr[j]);
        }
        if (!coupled) continue;
        if (nart_all > 1 || nf_all > OE_MAXF || ns_all > OE_MAXS) { n = -1; break; }
        ev->art_body = -1; ev->art_dof = 0; ev->art_tmpl = -1;
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

/* Narrow phase as a test entry point: shapes given as [type, c.xyz, q.xyzw,
 * h.xyz] (11 floats); out[4][7] = point.xyz, normal.xyz, separation. Returns
 * the contact count. */
int oracle_collide(const float* a, const float* b, float margin, float* out) {
    cshape_t A, B;
    pair_t o;
    int k;
    A.type = (int)a[0]; A.c = V(a[1], a[2], a[3]); A.R = qmat_(Q(a[4], a[5], a[6], a[7])); A.h = V(a[8], a[9], a[10]);
    B.type = (int)b[0]; B.c = V(b[1], b[2], b[3]); B.R = qmat_(Q(b[4], b[5], b[6], b[7])); B.h = V(b[8], b[9], b[10]);
    o.n = 0;
    collide_(&A, &B, margin, &o);
    for (k = 0; k < o.n; ++k) {
        out[k * 7 + 0] = o.p[k].x; out[k * 7 + 1] = o.p[k].y; out[k * 7 + 2] = o.p[k].z;
        out[k * 7 + 3] = o.nrm[k].x; out[k * 7 + 4] = o.nrm[k].y; out[k * 7 + 5] = o.nrm[k].z;
        out[k * 7 + 6] = o.sep[k];
    }
    return o.n;
}
