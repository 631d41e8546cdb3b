/*
 * migym_oracle_render.c — TEST INFRASTRUCTURE ONLY (included by
 * migym_oracle.c). CPU restatement of the camera ray caster
 * (test_isaacgym_amd/csrc/mg_render.hip), one pixel at a time,
 * in the kernel's order of operations, without its culling (a culled shape
 * cannot be the nearest hit, so images agree bit for bit).
 *
 * What it is pinned to. Isaac Gym's renderer is closed; its outputs in the
 * reference tree are examples/interop_images/cam-<frame>-<env>.png (16 envs of
 * examples/interop_torch.py:56-120 at frames 0..50). tests/test_render.py
 * checks this restatement against the fixture extracted from them
 * (tests/golden/interop_fixture.json): the ball's silhouette per frame (camera
 * placement and projection, examples/interop_torch.py:111, default 90-degree
 * field of view, gravity and frame cadence), the 1 m ground checker and the
 * absence of neighbouring envs' balls. Shading values are not pinned.
 *
 * Camera frame: looks along local +x, image up = the sim's up axis; pixel
 * (c, r) -> ray fma(l, a, f + u b), a = (cx - c - 0.5)/fx, b = (cy - r - 0.5)/fy.
 */

typedef struct {
    int type, seg;
    float r, g, b;
    v3_t c;
    m3_t R;
    v3_t h;
    const float* hv;
} rws_t;

static const float R_INF = __builtin_inff();

/* explicit fused multiply-adds, as the kernel (fmaf is correctly rounded) */
static float fdot_(v3_t a, v3_t b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static v3_t fma3_(v3_t a, float s, v3_t c) { return V(fmaf(a.x, s, c.x), fmaf(a.y, s, c.y), fmaf(a.z, s, c.z)); }
static v3_t fmt_(m3_t R, v3_t v) { return V(fdot_(R.c0, v), fdot_(R.c1, v), fdot_(R.c2, v)); }

static float ray_sphere_(v3_t o, v3_t d, v3_t c, float r, float tmin) {
    v3_t oc = sub3(o, c);
    float bb = fdot_(oc, d);
    float cc = fmaf(-r, r, fdot_(oc, oc));
    float dd = fdot_(d, d);
    float disc = fmaf(-dd, cc, bb * bb);
    float t;
    if (!(disc >= 0.0f)) return R_INF;
    t = (-bb - sqrtf(disc)) / dd;
    return t >= tmin ? t : R_INF;
}

static void slab_(float o, float d, float h, float* tn, float* tf) {
    float inv = 1.0f / d;
    float t1 = (-h - o) * inv;
    float t2 = (h - o) * inv;
    *tn = fmaxf(*tn, fminf(t1, t2));
    *tf = fminf(*tf, fmaxf(t1, t2));
}

static float ray_box_(v3_t o, v3_t d, const rws_t* s, float tmin, float tmax) {
    v3_t ol = fmt_(s->R, sub3(o, s->c));
    v3_t dl = fmt_(s->R, d);
    float tn = -R_INF, tf = tmax;   /* entry point only: back faces are not drawn */
    slab_(ol.x, dl.x, s->h.x, &tn, &tf);
    slab_(ol.y, dl.y, s->h.y, &tn, &tf);
    slab_(ol.z, dl.z, s->h.z, &tn, &tf);
    return (tn <= tf && tn >= tmin) ? tn : R_INF;
}

static float ray_capsule_(v3_t o, v3_t d, const rws_t* s, float tmin) {
    float r = s->h.x, hl = s->h.y;
    v3_t ax = s->R.c0;
    v3_t pa = fma3_(ax, -hl, s->c);
    v3_t ba = mul3(ax, 2.0f * hl);
    v3_t oa = sub3(o, pa);
    float baba = fdot_(ba, ba), bard = fdot_(ba, d), baoa = fdot_(ba, oa);
    float rdoa = fdot_(d, oa), oaoa = fdot_(oa, oa), dd = fdot_(d, d);
    float a = fmaf(baba, dd, -(bard * bard));
    float b = fmaf(baba, rdoa, -(baoa * bard));
    float c = fmaf(baba, oaoa, -(baoa * baoa)) - r * r * baba;
    float hh = fmaf(b, b, -(a * c));
    float t = R_INF, t0, t1;
    if (!(hh >= 0.0f)) return R_INF;
    if (a > 0.0f) {
        float tb = (-b - sqrtf(hh)) / a;
        float y = fmaf(tb, bard, baoa);
        if (y > 0.0f && y < baba && tb >= tmin) t = tb;
    }
    t0 = ray_sphere_(o, d, pa, r, tmin);
    t1 = ray_sphere_(o, d, add3(pa, ba), r, tmin);
    t = t0 < t ? t0 : t;
    t = t1 < t ? t1 : t;
    return t;
}

static float ray_convex_(v3_t o, v3_t d, const rws_t* s, float tmin, float tmax) {
    const v3_t ol = fmt_(s->R, sub3(o, s->c));
    const v3_t dl = fmt_(s->R, d);
    const int nv = (int)s->hv[0], nf = (int)s->hv[1];
    const float* pl = s->hv + MG_HULL_HEADER + 3 * nv;
    float tn = -R_INF, tf = tmax;
    int f;
    for (f = 0; f < nf; ++f) {
        const v3_t n = V(pl[4 * f + 0], pl[4 * f + 1], pl[4 * f + 2]);
        const float dist = fdot_(n, ol) - pl[4 * f + 3];
        const float den = fdot_(n, dl);
        if (den < 0.0f) tn = fmaxf(tn, -dist / den);
        else if (den > 0.0f) tf = fminf(tf, -dist / den);
        else if (dist > 0.0f) return R_INF;
    }
    return (tn <= tf && tn >= tmin) ? tn : R_INF;
}

static float ray_shape_(v3_t o, v3_t d, const rws_t* s, float tmin, float tmax) {
    if (s->type == MG_SHAPE_CONVEX) return ray_convex_(o, d, s, tmin, tmax);
    if (s->type == MG_SHAPE_BOX) return ray_box_(o, d, s, tmin, tmax);
    if (s->type == MG_SHAPE_SPHERE) return ray_sphere_(o, d, s->c, s->h.x, tmin);
    return ray_capsule_(o, d, s, tmin);
}

static v3_t shape_normal_(const rws_t* s, v3_t p) {
    v3_t dp = sub3(p, s->c);
    float t;
    if (s->type == MG_SHAPE_SPHERE) return mul3(dp, 1.0f / s->h.x);
    if (s->type == MG_SHAPE_BOX) {
        v3_t pl = fmt_(s->R, dp), axis;
        float qx = fabsf(pl.x) / s->h.x, qy = fabsf(pl.y) / s->h.y, qz = fabsf(pl.z) / s->h.z;
        float best = qx, comp;
        int k = 0;
        if (qy > best) { k = 1; best = qy; }
        if (qz > best) k = 2;
        axis = k == 0 ? s->R.c0 : (k == 1 ? s->R.c1 : s->R.c2);
        comp = k == 0 ? pl.x : (k == 1 ? pl.y : pl.z);
        return mul3(axis, comp < 0.0f ? -1.0f : 1.0f);
    }
    if (s->type == MG_SHAPE_CONVEX) {
        const v3_t pl = fmt_(s->R, dp);
        const int nv = (int)s->hv[0], nf = (int)s->hv[1];
        const float* pp = s->hv + MG_HULL_HEADER + 3 * nv;
        float best = -R_INF;
        v3_t nl = V(0.0f, 0.0f, 1.0f);
        int f;
        for (f = 0; f < nf; ++f) {
            const v3_t n = V(pp[4 * f + 0], pp[4 * f + 1], pp[4 * f + 2]);
            const float dist = fdot_(n, pl) - pp[4 * f + 3];
            if (dist > best) { best = dist; nl = n; }
        }
        return fma3_(s->R.c2, nl.z, fma3_(s->R.c1, nl.y, mul3(s->R.c0, nl.x)));
    }
    t = fdot_(dp, s->R.c0);
    t = fminf(fmaxf(t, -s->h.y), s->h.y);
    return mul3(fma3_(s->R.c0, -t, dp), 1.0f / s->h.x);
}

static unsigned q8_(float x) { return (unsigned)(fminf(fmaxf(x, 0.0f), 1.0f) * 255.0f + 0.5f); }

/* One camera. state: AoS [nb][13] in global body order; body_tmpl [nb];
 * tbi [ntb][MG_TBODY_I_N]; shapes [ns][MG_SHAPE_STRIDE]; hulls (or NULL); env_body_first
 * [num_envs+1]; color [nb][3]; seg [nb]. Outputs may be NULL. */
int oracle_render(const mg_sim_params* p, const float* state, const int32_t* body_tmpl, const int32_t* tbi,
                  const float* shapes, const float* hulls, const int32_t* env_body_first, const float* color,
                  const int32_t* seg, const mg_camera* cam, uint8_t* rgba_out, float* depth_out, int32_t* seg_out,
                  const mg_light* light) {
    rws_t ws[MG_RENDER_MAX_SHAPES];
    int ns = 0, b, k, row, col;
    v3_t o, f, l, u, upv, leftv, fwdv, L, gn;
    q4_t q;
    float ifx, ify, lx = 0.3f, ly = 0.2f, lz = 1.0f, inv, h0, lcol[3], amb[3];
    int up_axis = p->up_axis == 0 ? 0 : 1;

    /* the env's shapes in the world frame */
    for (b = env_body_first[cam->env]; b < env_body_first[cam->env + 1]; ++b) {
        const float* st = state + (size_t)b * MG_STATE_N;
        v3_t pb = V(st[0], st[1], st[2]);
        q4_t qb = Q(st[3], st[4], st[5], st[6]);
        int t = body_tmpl[b];
        int sh0 = tbi[t * MG_TBODY_I_N + 0], nsh = tbi[t * MG_TBODY_I_N + 1];
        for (k = 0; k < nsh; ++k) {
            const float* sh = shapes + (size_t)(sh0 + k) * MG_SHAPE_STRIDE;
            rws_t* w;
            if (ns >= MG_RENDER_MAX_SHAPES) return -1;
            w = &ws[ns++];
            w->type = (int)sh[0];
            w->seg = seg[b];
            w->r = color[3 * b + 0]; w->g = color[3 * b + 1]; w->b = color[3 * b + 2];
            w->c = add3(pb, qrot_(qb, V(sh[4], sh[5], sh[6])));
            w->R = qmat_(qmul_(qb, Q(sh[7], sh[8], sh[9], sh[10])));
            if (w->type == MG_SHAPE_BOX) w->h = V(sh[1], sh[2], sh[3]);
            else if (w->type == MG_SHAPE_SPHERE || w->type == MG_SHAPE_CONVEX) w->h = V(sh[1], 0.0f, 0.0f);
            else w->h = V(sh[1], sh[2], 0.0f);
            w->hv = w->type == MG_SHAPE_CONVEX ? hulls + (int)sh[2] : NULL;
        }
    }

    /* camera pose and frame */
    o = V(cam->p[0], cam->p[1], cam->p[2]);
    q = Q(cam->q[0], cam->q[1], cam->q[2], cam->q[3]);
    if (cam->body >= 0) {
        const float* st = state + (size_t)cam->body * MG_STATE_N;
        v3_t pb = V(st[0], st[1], st[2]);
        q4_t qb = Q(st[3], st[4], st[5], st[6]);
        if (cam->follow == 1) {
            o = add3(pb, qrot_(qb, o));
            q = qmul_(qb, q);
        } else {
            o = add3(pb, o);
        }
    }
    if (up_axis == 1) {
        upv = V(0.0f, 0.0f, 1.0f);
        leftv = V(0.0f, 1.0f, 0.0f);
        fwdv = V(1.0f, 0.0f, 0.0f);
    } else {
        upv = V(0.0f, 1.0f, 0.0f);
        leftv = V(-1.0f, 0.0f, 0.0f);
        fwdv = V(0.0f, 0.0f, -1.0f);
        ly = 1.0f; lz = 0.2f;
    }
    for (k = 0; k < 3; ++k) { lcol[k] = 0.7f; amb[k] = 0.3f; }
    if (light) {   /* mg_set_light (migym_capi.cpp mg_render_cameras) */
        lx = light->dir[0]; ly = light->dir[1]; lz = light->dir[2];
        for (k = 0; k < 3; ++k) { lcol[k] = light->color[k]; amb[k] = light->ambient[k]; }
    }
    inv = 1.0f / sqrtf(lx * lx + ly * ly + lz * lz);
    L = V(lx * inv, ly * inv, lz * inv);
    f = qrot_(q, fwdv);
    l = qrot_(q, leftv);
    u = qrot_(q, upv);
    ifx = 1.0f / cam->fx;
    ify = 1.0f / cam->fy;
    gn = V(p->ground_normal[0], p->ground_normal[1], p->ground_normal[2]);

    h0 = fdot_(gn, o) + p->ground_distance;
    for (row = 0; row < cam->height; ++row) {
        v3_t rb = fma3_(u, (cam->cy - ((float)row + 0.5f)) * ify, f);
        for (col = 0; col < cam->width; ++col) {
            size_t px = (size_t)row * cam->width + col;
            float a = (cam->cx - ((float)col + 0.5f)) * ifx;
            v3_t d = fma3_(l, a, rb);
            float best = cam->far_plane, dd;
            int hit = -2, j, shadow = 0, sgv;
            unsigned rgba;
            v3_t pp, n, ps;
            if (p->has_ground) {
                float dn = fdot_(gn, d);
                if (dn < 0.0f) {
                    float t = -h0 / dn;
                    if (t >= cam->near_plane && t < best) { best = t; hit = -1; }
                }
            }
            dd = fdot_(d, d);
            (void)dd;
            for (j = 0; j < ns; ++j) {
                float t = ray_shape_(o, d, &ws[j], cam->near_plane, best);
                if (t < best) { best = t; hit = j; }
            }
            if (hit == -2) {
                if (rgba_out) memcpy(rgba_out + 4 * px, &(uint32_t){0xFF000000u}, 4);
                if (depth_out) depth_out[px] = -R_INF;
                if (seg_out) seg_out[px] = 0;
                continue;
            }
            pp = fma3_(d, best, o);
            n = hit >= 0 ? shape_normal_(&ws[hit], pp) : gn;
            ps = fma3_(n, 1e-3f, pp);
            for (j = 0; j < ns && !shadow; ++j) shadow = ray_shape_(ps, L, &ws[j], 0.0f, R_INF) < R_INF;
            if (hit >= 0) {
                float lam = fmaxf(fdot_(n, L), 0.0f);
                float kr = shadow ? amb[0] : fmaf(lcol[0], lam, amb[0]);
                float kg = shadow ? amb[1] : fmaf(lcol[1], lam, amb[1]);
                float kb = shadow ? amb[2] : fmaf(lcol[2], lam, amb[2]);
                rgba = q8_(ws[hit].r * kr) | (q8_(ws[hit].g * kg) << 8) | (q8_(ws[hit].b * kb) << 16) | 0xFF000000u;
                sgv = ws[hit].seg;
            } else {
                float uu = pp.x, vv = up_axis == 1 ? pp.y : pp.z;
                int par = ((int)floorf(uu) + (int)floorf(vv)) & 1;
                float kk = shadow ? 0.55f : 1.0f;
                float cr = (par ? 108.0f / 255.0f : 143.0f / 255.0f) * kk;
                float cb = (par ? 113.0f / 255.0f : 150.0f / 255.0f) * kk;
                rgba = q8_(cr) | (q8_(cr) << 8) | (q8_(cb) << 16) | 0xFF000000u;
                sgv = 0;
            }
            if (rgba_out) memcpy(rgba_out + 4 * px, &rgba, 4);
            if (depth_out) depth_out[px] = -best;
            if (seg_out) seg_out[px] = sgv;
        }
    }
    return 0;
}
