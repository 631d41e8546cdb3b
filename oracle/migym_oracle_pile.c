/*
 * migym_oracle_pile.c — TEST INFRASTRUCTURE ONLY (included by migym_oracle.c
 * after migym_oracle_env.c, whose narrow phase it calls). CPU restatement of
 * the free-body pile step, test_isaacgym_amd/csrc/mg_pile.hip k_pile_step
 * (DESIGN.md §3.10): a coupled env with more than two free bodies and no
 * articulation — the pyramid of 30 balls per env of
 * examples/1080_balls_of_solitude.py:96-136 (ball.urdf, group i, filter 0), or
 * boxes, capsules and hulls heaped on the ground and on up to four static bodies.
 *
 * Per substep: free flight as a free body (migym_oracle.c rigid_body_step);
 * the narrow phase of every candidate shape pair in pair order (the coupled
 * step's screen and contacts, migym_oracle_env.c pair_near_ / collide_ /
 * ground_pair_); the pairs with contacts ("active pairs") coloured greedily in
 * pair order so that no two pairs of one colour share a free body (PhysX's GPU
 * constraint partitioning); then the TGS sweeps visit the active pairs colour by
 * colour — a pair's friction rows (two tangents per point, the pyramid clamp at
 * mu times the point's normal impulse), then its normal rows (op_solve_pair_). The device solves
 * a colour's pairs on parallel lanes; they touch disjoint bodies, so its result
 * equals this sequential visit bit for bit. PHYSICS PARITY WITH PHYSX IS
 * UNPINNED (see migym_oracle.c); the colouring and per-point friction are this
 * build's conventions.
 */

#define OP_ST0 64         /* participant id of static body s (MG_PILE_ST0) */
#define OP_MAXAP 128      /* active pairs per substep (MG_PILE_MAXAP) */
#define OP_MAXPT 256      /* contact points per substep (MG_PILE_MAXPT) */
#define OP_MAXPAIRS 8192  /* candidate shape pairs per env (MG_PILE_MAXPAIRS) */

typedef struct { int a, b, pt0, pn, color; float mu, e; } pap_t;
typedef struct { v3_t n, ra, rb, t1, t2; float s0, kn, kt1, kt2, vn0, ln, lt1, lt2; } ppt_t;

/* candidate shape pairs of a pile env, in the device's order (migym_capi.cpp
 * upload): per free body k and shape of k: the ground, the static bodies it may
 * touch, then the later free bodies it may touch (oe_collide_) */
static int pile_pairs_(const mg_model* m, const oenv_t* ev, int ground, epair_t* out, int cap) {
    int n = 0, k, j, t, sa, sb;
#define OP_PUSH(A_, SA_, B_, SB_) do { if (n < cap) { out[n].a = (A_); out[n].sa = (SA_); out[n].b = (B_); out[n].sb = (SB_); } n++; } while (0)
#define OP_SHP(B_, S0_, NS_) do { const int* t_ = m->tmpl_body_i + (size_t)m->body_tmpl[B_] * MG_TBODY_I_N; S0_ = t_[0]; NS_ = t_[1]; } while (0)
    for (k = 0; k < ev->np; ++k) {
        int sa0, nsa;
        OP_SHP(ev->pb[k], sa0, nsa);
        for (sa = sa0; sa < sa0 + nsa; ++sa) {
            if (ground) OP_PUSH(k, sa, -1, -1);
            for (t = 0; t < ev->ns; ++t) {
                int sb0, nsb;
                if (!oe_collide_(m, ev->pact[k], ev->sact[t])) continue;
                OP_SHP(ev->stat_b[t], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OP_PUSH(k, sa, OP_ST0 + t, sb);
            }
            for (j = k + 1; j < ev->np; ++j) {
                int sb0, nsb;
                if (!oe_collide_(m, ev->pact[k], ev->pact[j])) continue;
                OP_SHP(ev->pb[j], sb0, nsb);
                for (sb = sb0; sb < sb0 + nsb; ++sb) OP_PUSH(k, sa, j, sb);
            }
        }
    }
#undef OP_PUSH
#undef OP_SHP
    return n;
}

/* relative velocity of A over B along d at lever arms ra, rb (mg_pile.hip
 * pair_constants); B static or the ground (dynb 0): A's terms only */
static float op_rel_(int dynb, v3_t d, v3_t ra, v3_t rb, v3_t va, v3_t wa, v3_t vb, v3_t wb) {
    const float ua = dot3(d, va) + dot3(cross3(ra, d), wa);
    return dynb ? ua - (dot3(d, vb) + dot3(cross3(rb, d), wb)) : ua;
}
/* 1 / effective mass of a row along d (mg_pile.hip row_k) */
static float op_k_(int dynb, v3_t d, v3_t ra, v3_t rb, float ima, float imb, const s3_t* Ia, const s3_t* Ib) {
    const v3_t ca = cross3(ra, d);
    const float ka = ima + dot3(ca, symmul_(*Ia, ca));
    if (!dynb) return 1.0f / ka;
    {
        const v3_t cb = cross3(rb, d);
        return 1.0f / ((ka + imb) + dot3(cb, symmul_(*Ib, cb)));
    }
}

typedef struct {
    v3_t x[OP_MAXB], xc[OP_MAXB], v[OP_MAXB], w[OP_MAXB], dx[OP_MAXB], dth[OP_MAXB], fsum[OP_MAXB];
    q4_t q[OP_MAXB];
    s3_t Iw[OP_MAXB];
    float invm[OP_MAXB];
} pbody_t;

/* the velocities a pair's rows act on: A's, and B's when B is a free body
 * (dynb); against a static body or the ground a row has A's terms only */
typedef struct { int dynb; float ima, imb; s3_t Ia, Ib; v3_t dxa, dta, dxb, dtb, va, wa, vb, wb; } prow_t;

/* A's (and B's) part of a row along d at lever arms ra, rb: the relative
 * velocity (mg_pile.hip rel_v) and the relative motion over the substep */
static float op_relv_(const prow_t* R, v3_t d, v3_t ca, v3_t cb) {
    const float ua = dot3(d, R->va) + dot3(ca, R->wa);
    return R->dynb ? ua - (dot3(d, R->vb) + dot3(cb, R->wb)) : ua;
}
static float op_reld_(const prow_t* R, v3_t d, v3_t ca, v3_t cb) {
    const float ua = dot3(d, R->dxa) + dot3(ca, R->dta);
    return R->dynb ? ua - (dot3(d, R->dxb) + dot3(cb, R->dtb)) : ua;
}
/* apply impulse dl along d: A gets +dl, B -dl */
static void op_apply_(prow_t* R, v3_t d, v3_t ca, v3_t cb, float dl) {
    R->va = fmad3_(R->va, d, dl * R->ima);
    R->wa = fmad3_(R->wa, symmul_(R->Ia, ca), dl);
    if (R->dynb) {
        R->vb = fmad3_(R->vb, d, -(dl * R->imb));
        R->wb = fmad3_(R->wb, symmul_(R->Ib, cb), -dl);
    }
}

/* the pair's normal rows, point order (mg_pile.hip normal_rows) */
static void op_normal_rows_(const step_t* P, const pap_t* pr, ppt_t* pt, prow_t* R, int pos) {
    int j;
    for (j = 0; j < pr->pn; ++j) {
        ppt_t* c = &pt[pr->pt0 + j];
        const v3_t ca = cross3(c->ra, c->n), cb = cross3(c->rb, c->n);
        const float s = c->s0 + op_reld_(R, c->n, ca, cb);
        const float tgt = pos ? pos_target_(P, s) : vel_target_(P, s, pr->e, c->vn0);
        const float vn = op_relv_(R, c->n, ca, cb);
        const float nl = fmaxf(fmaf(c->kn, tgt - vn, c->ln), 0.0f);
        const float dl = nl - c->ln;
        c->ln = nl;
        op_apply_(R, c->n, ca, cb, dl);
    }
}

/* the pair's friction rows, point order, t1 then t2 (mg_pile.hip
 * friction_rows): the pyramid clamp at mu times the point's normal impulse; a
 * position sweep also closes the tangential drift of the point's two copies
 * over the substep so far, as a normal row closes its separation */
static void op_friction_rows_(const step_t* P, const pap_t* pr, ppt_t* pt, prow_t* R, int pos) {
    int j, r;
    for (j = 0; j < pr->pn; ++j) {
        ppt_t* c = &pt[pr->pt0 + j];
        const float lim = pr->mu * c->ln;
        for (r = 0; r < 2; ++r) {
            const v3_t t = r == 0 ? c->t1 : c->t2;
            const float kt = r == 0 ? c->kt1 : c->kt2, lt = r == 0 ? c->lt1 : c->lt2;
            const v3_t ca = cross3(c->ra, t), cb = cross3(c->rb, t);
            const float vt = op_relv_(R, t, ca, cb);
            const float ft = pos ? -op_reld_(R, t, ca, cb) * P->inv_sub : 0.0f;
            const float nl = clamp_sym_(fmaf(kt, ft - vt, lt), lim);
            const float d = nl - lt;
            if (r == 0) c->lt1 = nl; else c->lt2 = nl;
            op_apply_(R, t, ca, cb, d);
        }
    }
}

/* one active pair in one sweep (mg_pile.hip solve_pair). Sweep order, as the
 * free bodies' ground patch (migym_oracle.c rigid_body_step, DESIGN.md
 * §3.2.1): a position sweep solves the friction rows, then the normal rows, so
 * the velocity it integrates is the one non-penetration had the last word on —
 * only the first one opens with the normal rows too (the friction budget needs
 * a normal impulse); a velocity sweep is normal, friction, normal rows */
static void op_solve_pair_(const step_t* P, const pap_t* pr, ppt_t* pt, pbody_t* B, int pos, int first) {
    const int a = pr->a, b = pr->b, dynb = b >= 0 && b < OP_ST0;
    const v3_t z = V(0.0f, 0.0f, 0.0f);
    prow_t R;
    R.dynb = dynb;
    R.ima = B->invm[a]; R.Ia = B->Iw[a];
    R.dxa = B->dx[a]; R.dta = B->dth[a]; R.va = B->v[a]; R.wa = B->w[a];
    if (dynb) {
        R.imb = B->invm[b]; R.Ib = B->Iw[b];
        R.dxb = B->dx[b]; R.dtb = B->dth[b]; R.vb = B->v[b]; R.wb = B->w[b];
    } else {
        const s3_t Z = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        R.imb = 0.0f; R.Ib = Z;
        R.dxb = z; R.dtb = z; R.vb = z; R.wb = z;
    }
    if (!pos || first) op_normal_rows_(P, pr, pt, &R, pos);
    op_friction_rows_(P, pr, pt, &R, pos);
    op_normal_rows_(P, pr, pt, &R, pos);
    B->v[a] = R.va; B->w[a] = R.wa;
    if (dynb) { B->v[b] = R.vb; B->w[b] = R.wb; }
}

static int pile_step_(const step_t* P, const mg_model* m, const oenv_t* ev, float* state, const float* ext,
                      float* cforce) {
    static __thread struct {
        epair_t pairs[OP_MAXPAIRS];
        pap_t ap[OP_MAXAP];
        ppt_t pt[OP_MAXPT];
        int ord[OP_MAXAP];
        pbody_t B;
    } W;
    pbody_t* B = &W.B;
    const int nb = ev->np, ns = ev->ns;
    const int npair = pile_pairs_(m, ev, P->ground, W.pairs, OP_MAXPAIRS);
    v3_t sx[OE_MAXS];
    q4_t sq[OE_MAXS];
    int k, i, j, it, st_;
    if (nb > OP_MAXB || npair > OP_MAXPAIRS) return -1;
    for (k = 0; k < ns; ++k) {
        const float* ss = state + (size_t)ev->stat_b[k] * MG_STATE_N;
        sx[k] = V(ss[0], ss[1], ss[2]);
        sq[k] = qnorm_(Q(ss[3], ss[4], ss[5], ss[6]));
    }
    for (k = 0; k < nb; ++k) {
        const float* st = state + (size_t)ev->pb[k] * MG_STATE_N;
        B->x[k] = V(st[0], st[1], st[2]);
        B->q[k] = qnorm_(Q(st[3], st[4], st[5], st[6]));
        B->v[k] = V(st[7], st[8], st[9]);
        B->w[k] = V(st[10], st[11], st[12]);
        B->fsum[k] = V(0.0f, 0.0f, 0.0f);
    }
    for (st_ = 0; st_ < P->substeps; ++st_) {
        int nap = 0, npt = 0, ncol = 0, no = 0;
        unsigned long long used[OP_MAXB];
        /* ---- 1. free flight (rigid_body_step's order) */
        for (k = 0; k < nb; ++k) {
            const int b = ev->pb[k];
            const float* M = m->body_mass + (size_t)b * MG_MASS_N;
            const float* tf = m->tmpl_body_f + (size_t)m->body_tmpl[b] * MG_TBODY_F_N;
            const float invm = M[0], h = P->h;
            const v3_t invI = V(M[1], M[2], M[3]), com = V(M[8], M[9], M[10]);
            const q4_t iq = Q(M[4], M[5], M[6], M[7]);
            const float lin_keep = 1.0f - fminf(tf[0] * h, 1.0f), ang_keep = 1.0f - fminf(tf[1] * h, 1.0f);
            const float max_lv2 = tf[2] * tf[2], max_av2 = tf[3] * tf[3];
            v3_t v = B->v[k], w = B->w[k];
            float v2, w2;
            B->Iw[k] = sym_rdrt_(qmat_(inertia_frame_(B->q[k], iq)), invI);
            B->xc[k] = com_world_(B->x[k], B->q[k], com);
            B->invm[k] = invm;
            if (tf[4] != 0.0f) v = mad3(v, V(P->g[0], P->g[1], P->g[2]), h);
            if (ext) {
                const float* e = ext + (size_t)b * 6;
                v = mad3(v, V(e[0], e[1], e[2]), invm * h);
                w = mad3(w, symmul_(B->Iw[k], V(e[3], e[4], e[5])), h);
            }
            v = mul3(v, lin_keep);
            w = mul3(w, ang_keep);
            v2 = dot3(v, v);
            if (v2 > max_lv2) v = mul3(v, sqrtf(max_lv2 / v2));
            w2 = dot3(w, w);
            if (w2 > max_av2) w = mul3(w, sqrtf(max_av2 / w2));
            B->v[k] = v; B->w[k] = w;
            B->dx[k] = V(0.0f, 0.0f, 0.0f);
            B->dth[k] = V(0.0f, 0.0f, 0.0f);
            used[k] = 0ull;
        }
        /* ---- 2. narrow phase in pair order; pairs are kept until the first one
         * that would overflow the active-pair or point table (it and every later
         * one dropped for this substep) */
        for (i = 0; i < npair; ++i) {
            const epair_t* pp = &W.pairs[i];
            const float* sha = shp_(m, pp->sa);
            const int a = pp->a, b = pp->b, dynb = b >= 0 && b < OP_ST0;
            const v3_t xa = B->x[a];
            const q4_t qa = B->q[a];
            cshape_t sA, sB;
            pair_t o;
            float mu, e;
            o.n = 0;
            if (b < 0) {
                if (!pair_near_(P, sha, xa, qa, sha, xa, qa, 1, m->hulls)) continue;
                sA = place_(sha, xa, qa, m->hulls);
                ground_pair_(P, &sA, &o);
                mu = 0.5f * (sha[11] + P->mu_g);
                e = 0.5f * (sha[12] + P->e_g);
            } else {
                const float* shb = shp_(m, pp->sb);
                const v3_t xb = dynb ? B->x[b] : sx[b - OP_ST0];
                const q4_t qb = dynb ? B->q[b] : sq[b - OP_ST0];
                if (!pair_near_(P, sha, xa, qa, shb, xb, qb, 0, m->hulls)) continue;
                sA = place_(sha, xa, qa, m->hulls);
                sB = place_(shb, xb, qb, m->hulls);
                collide_(&sA, &sB, P->co, &o);
                mu = 0.5f * (sha[11] + shb[11]);
                e = 0.5f * (sha[12] + shb[12]);
            }
            if (o.n == 0) continue;
            if (nap >= OP_MAXAP || npt + o.n > OP_MAXPT) break;
            W.ap[nap].a = a; W.ap[nap].b = b; W.ap[nap].pt0 = npt; W.ap[nap].pn = o.n;
            W.ap[nap].mu = mu; W.ap[nap].e = e; W.ap[nap].color = -1;
            for (j = 0; j < o.n; ++j) {
                ppt_t* c = &W.pt[npt + j];
                c->n = o.nrm[j];
                c->s0 = o.sep[j] - P->ro;
                c->ra = sub3(o.p[j], B->xc[a]);
                c->rb = dynb ? sub3(o.p[j], B->xc[b]) : V(0.0f, 0.0f, 0.0f);
            }
            npt += o.n;
            nap++;
        }
        /* ---- 3. row constants */
        for (i = 0; i < nap; ++i) {
            const pap_t* pr = &W.ap[i];
            const int a = pr->a, b = pr->b, dynb = b >= 0 && b < OP_ST0;
            const s3_t Z = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            const v3_t z = V(0.0f, 0.0f, 0.0f);
            const float ima = B->invm[a], imb = dynb ? B->invm[b] : 0.0f;
            const s3_t Ia = B->Iw[a], Ib = dynb ? B->Iw[b] : Z;
            const v3_t va = B->v[a], wa = B->w[a], vb = dynb ? B->v[b] : z, wb = dynb ? B->w[b] : z;
            for (j = 0; j < pr->pn; ++j) {
                ppt_t* c = &W.pt[pr->pt0 + j];
                tangents_(c->n, &c->t1, &c->t2);
                c->kn = op_k_(dynb, c->n, c->ra, c->rb, ima, imb, &Ia, &Ib);
                c->kt1 = op_k_(dynb, c->t1, c->ra, c->rb, ima, imb, &Ia, &Ib);
                c->kt2 = op_k_(dynb, c->t2, c->ra, c->rb, ima, imb, &Ia, &Ib);
                c->vn0 = op_rel_(dynb, c->n, c->ra, c->rb, va, wa, vb, wb);
                c->ln = 0.0f; c->lt1 = 0.0f; c->lt2 = 0.0f;
            }
        }
        /* ---- 4. greedy colouring in pair order (the lowest colour free on both
         * bodies; statics and the ground take none); a pair with no colour left
         * among 64 is not solved */
        for (i = 0; i < nap; ++i) {
            const int a = W.ap[i].a, b = W.ap[i].b, dynb = b >= 0 && b < OP_ST0;
            const unsigned long long taken = used[a] | (dynb ? used[b] : 0ull);
            int c = -1;
            if (taken != ~0ull) {
                c = 0;
                while ((taken >> c) & 1ull) c++;
                used[a] |= 1ull << c;
                if (dynb) used[b] |= 1ull << c;
                if (c + 1 > ncol) ncol = c + 1;
            }
            W.ap[i].color = c;
        }
        for (k = 0; k < ncol; ++k)
            for (i = 0; i < nap; ++i)
                if (W.ap[i].color == k) W.ord[no++] = i;
        /* ---- 5. TGS: position sweeps (then the motion deltas), velocity sweeps */
        for (it = 0; it < P->npos; ++it) {
            for (i = 0; i < no; ++i) op_solve_pair_(P, &W.ap[W.ord[i]], W.pt, B, 1, it == 0);
            for (k = 0; k < nb; ++k) {
                B->dx[k] = fmad3_(B->dx[k], B->v[k], P->sub);
                B->dth[k] = fmad3_(B->dth[k], B->w[k], P->sub);
            }
        }
        for (it = 0; it < P->nvel; ++it)
            for (i = 0; i < no; ++i) op_solve_pair_(P, &W.ap[W.ord[i]], W.pt, B, 0, 0);
        /* ---- 6. pose; the contact impulses per body, in pair order */
        for (k = 0; k < nb; ++k) {
            const float* M = m->body_mass + (size_t)ev->pb[k] * MG_MASS_N;
            const v3_t com = V(M[8], M[9], M[10]);
            const v3_t xc1 = add3(B->xc[k], B->dx[k]);
            B->q[k] = qint_(B->q[k], B->dth[k]);
            B->x[k] = origin_from_com_(xc1, B->q[k], com);
        }
        for (i = 0; i < nap; ++i) {
            const pap_t* pr = &W.ap[i];
            const int dynb = pr->b >= 0 && pr->b < OP_ST0;
            for (j = 0; j < pr->pn; ++j) {
                const ppt_t* c = &W.pt[pr->pt0 + j];
                const v3_t f = add3(add3(mul3(c->n, c->ln), mul3(c->t1, c->lt1)), mul3(c->t2, c->lt2));
                B->fsum[pr->a] = add3(B->fsum[pr->a], f);
                if (dynb) B->fsum[pr->b] = sub3(B->fsum[pr->b], f);
            }
        }
    }
    for (k = 0; k < nb; ++k) {
        float* st = state + (size_t)ev->pb[k] * MG_STATE_N;
        float* cf = cforce + (size_t)ev->pb[k] * 3;
        st[0] = B->x[k].x; st[1] = B->x[k].y; st[2] = B->x[k].z;
        st[3] = B->q[k].x; st[4] = B->q[k].y; st[5] = B->q[k].z; st[6] = B->q[k].w;
        st[7] = B->v[k].x; st[8] = B->v[k].y; st[9] = B->v[k].z;
        st[10] = B->w[k].x; st[11] = B->w[k].y; st[12] = B->w[k].z;
        cf[0] = B->fsum[k].x * P->inv_dt; cf[1] = B->fsum[k].y * P->inv_dt; cf[2] = B->fsum[k].z * P->inv_dt;
    }
    return 0;
}
