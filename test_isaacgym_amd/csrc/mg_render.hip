// mg_render.hip — camera sensors: gym.render_all_camera_sensors /
// get_camera_image[_gpu_tensor] (config 5, test11_servo_vecenv_camerazoom.py:
// 327-342,388,458-460; examples/interop_torch.py:105-120,173-174).
//
// Ray casting, not rasterisation: a camera sees one env's handful of convex
// shapes (boxes, spheres, capsules) and the ground plane, so every pixel is a
// loop over a short shape list held in LDS — no geometry pipeline, no depth
// buffer, no atomics. The work is dominated by writing the images (5.76 MB per
// 1600x900 RGBA camera), so the kernel is shaped as a streaming store:
//   - a camera's pixels are cut into linear row-major runs of 16384; one
//     workgroup (4 waves) owns one run and each lane shades 4 consecutive
//     pixels per pass, so a wave stores 1 KB of color (+1 KB depth, +1 KB
//     segmentation) contiguously with one 16-B store per lane per image;
//   - the env's shapes are transformed to the world frame once per workgroup
//     (one lane per shape) from the pose snapshot taken at
//     render_all_camera_sensors, and shapes whose bounding sphere cannot
//     project into the run's rows are culled for the primary rays (shadow rays
//     still test every shape);
//   - the camera record is read with uniform (scalar) loads.
// Shading: Lambert + ambient on bodies, a 1 m checker ground,
// hard shadows from one directional light, black sky; color quantised to RGBA8.
// The C restatement is oracle/migym_oracle_render.c (same order of operations,
// -ffp-contract=off on both sides: images agree bit for bit).
#include "mg_internal.h"
#include "mg_math.h"

namespace {

// world-frame shape of the camera's env, staged in LDS
struct WS {
    int   type, seg;
    float r, g, b;
    V3    c;        // centre
    M3    R;        // columns: shape axes in the world
    V3    h;        // box half extents; sphere (radius, 0, 0); capsule (radius, half length, 0)
    float brad;     // bounding radius
    float brad2;    // (padded bounding radius)^2 of the per-ray rejection tests
    const float* hv;   // convex: hull record
};

// Per-pixel arithmetic uses explicit fused multiply-adds (fmaf: correctly
// rounded, so the C restatement's fmaf gives the same bits): dot products as
// fma chains, ray = fma(l, a, f + u b).
__device__ __forceinline__ float fdot(V3 a, V3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ V3 fma3(V3 a, float s, V3 c) {
    return v3(fmaf(a.x, s, c.x), fmaf(a.y, s, c.y), fmaf(a.z, s, c.z));
}
__device__ __forceinline__ V3 fmt(const M3& R, V3 v) { return v3(fdot(R.c0, v), fdot(R.c1, v), fdot(R.c2, v)); }

// Conservative per-ray rejection by the bounding sphere (cheap, no division):
// true only if the half-line o + t d (t >= 0) cannot reach the shape. The
// slack (padded radius, 1e-5 relative) exceeds the rounding of the test, so a
// rejected shape is one the exact intersection would have missed as well and
// the images stay bit-identical to the unculled restatement.
__device__ __forceinline__ bool ray_misses_bound(V3 o, V3 d, float dd, const WS& s) {
    const V3 oc = vsub(s.c, o);
    const float sp = fdot(oc, d);
    const float oc2 = fdot(oc, oc);
    if (!(oc2 > s.brad2)) return false;
    return sp < 0.0f || fmaf(oc2, dd, -(sp * sp)) > fmaf(1e-5f, oc2, s.brad2) * dd;
}

__device__ __forceinline__ float ray_sphere(V3 o, V3 d, V3 c, float r, float tmin) {
    const V3 oc = vsub(o, c);
    const float bb = fdot(oc, d);
    const float cc = fmaf(-r, r, fdot(oc, oc));
    const float dd = fdot(d, d);
    const float disc = fmaf(-dd, cc, bb * bb);
    if (!(disc >= 0.0f)) return __builtin_inff();
    const float t = (-bb - sqrtf(disc)) / dd;
    return t >= tmin ? t : __builtin_inff();
}

__device__ __forceinline__ void slab(float o, float d, float h, float& tn, float& tf) {
    const float inv = 1.0f / d;
    const float t1 = (-h - o) * inv;
    const float t2 = (h - o) * inv;
    tn = fmaxf(tn, fminf(t1, t2));
    tf = fminf(tf, fmaxf(t1, t2));
}

__device__ __forceinline__ float ray_box(V3 o, V3 d, const WS& s, float tmin, float tmax) {
    const V3 ol = fmt(s.R, vsub(o, s.c));
    const V3 dl = fmt(s.R, d);
    // entry point only: a ray that starts inside the box (a camera mounted in
    // its body's collision box) sees through it, as back faces are not drawn
    float tn = -__builtin_inff(), tf = tmax;
    slab(ol.x, dl.x, s.h.x, tn, tf);
    slab(ol.y, dl.y, s.h.y, tn, tf);
    slab(ol.z, dl.z, s.h.z, tn, tf);
    return (tn <= tf && tn >= tmin) ? tn : __builtin_inff();
}

__device__ __forceinline__ float ray_capsule(V3 o, V3 d, const WS& s, float tmin) {
    const float r = s.h.x, hl = s.h.y;
    const V3 ax = s.R.c0;
    const V3 pa = fma3(ax, -hl, s.c);
    const V3 ba = vscale(ax, 2.0f * hl);
    const V3 oa = vsub(o, pa);
    const float baba = fdot(ba, ba), bard = fdot(ba, d), baoa = fdot(ba, oa);
    const float rdoa = fdot(d, oa), oaoa = fdot(oa, oa), dd = fdot(d, d);
    const float a = fmaf(baba, dd, -(bard * bard));
    const float b = fmaf(baba, rdoa, -(baoa * bard));
    const float c = fmaf(baba, oaoa, -(baoa * baoa)) - r * r * baba;
    const float hh = fmaf(b, b, -(a * c));
    if (!(hh >= 0.0f)) return __builtin_inff();   // the infinite cylinder is missed
    float t = __builtin_inff();
    if (a > 0.0f) {
        const float tb = (-b - sqrtf(hh)) / a;
        const float y = fmaf(tb, bard, baoa);
        if (y > 0.0f && y < baba && tb >= tmin) t = tb;
    }
    const float t0 = ray_sphere(o, d, pa, r, tmin);
    const float t1 = ray_sphere(o, d, vadd(pa, ba), r, tmin);
    t = t0 < t ? t0 : t;
    t = t1 < t ? t1 : t;
    return t;
}

// convex hull: clip the ray by the face planes in the hull frame (entry point only)
__device__ __forceinline__ float ray_convex(V3 o, V3 d, const WS& s, float tmin, float tmax) {
    const V3 ol = fmt(s.R, vsub(o, s.c));
    const V3 dl = fmt(s.R, d);
    const int nv = (int)s.hv[0], nf = (int)s.hv[1];
    const float* pl = s.hv + MG_HULL_HEADER + 3 * nv;
    float tn = -__builtin_inff(), tf = tmax;
    for (int f = 0; f < nf; ++f) {
        const V3 n = v3(pl[4 * f + 0], pl[4 * f + 1], pl[4 * f + 2]);
        const float dist = fdot(n, ol) - pl[4 * f + 3];
        const float den = fdot(n, dl);
        if (den < 0.0f) tn = fmaxf(tn, -dist / den);
        else if (den > 0.0f) tf = fminf(tf, -dist / den);
        else if (dist > 0.0f) return __builtin_inff();
    }
    return (tn <= tf && tn >= tmin) ? tn : __builtin_inff();
}

__device__ __forceinline__ float ray_shape(V3 o, V3 d, const WS& s, float tmin, float tmax) {
    if (s.type == MG_SHAPE_CONVEX) return ray_convex(o, d, s, tmin, tmax);
    if (s.type == MG_SHAPE_BOX) return ray_box(o, d, s, tmin, tmax);
    if (s.type == MG_SHAPE_SPHERE) return ray_sphere(o, d, s.c, s.h.x, tmin);
    return ray_capsule(o, d, s, tmin);
}

__device__ __forceinline__ V3 shape_normal(const WS& s, V3 p) {
    const V3 dp = vsub(p, s.c);
    if (s.type == MG_SHAPE_SPHERE) return vscale(dp, 1.0f / s.h.x);
    if (s.type == MG_SHAPE_BOX) {
        const V3 pl = fmt(s.R, dp);
        const float qx = fabsf(pl.x) / s.h.x, qy = fabsf(pl.y) / s.h.y, qz = fabsf(pl.z) / s.h.z;
        int k = 0;
        float best = qx;
        if (qy > best) { k = 1; best = qy; }
        if (qz > best) k = 2;
        const V3 axis = k == 0 ? s.R.c0 : (k == 1 ? s.R.c1 : s.R.c2);
        const float sg = (k == 0 ? pl.x : (k == 1 ? pl.y : pl.z)) < 0.0f ? -1.0f : 1.0f;
        return vscale(axis, sg);
    }
    if (s.type == MG_SHAPE_CONVEX) {            // the face plane the point is farthest out of
        const V3 pl = fmt(s.R, dp);
        const int nv = (int)s.hv[0], nf = (int)s.hv[1];
        const float* pp = s.hv + MG_HULL_HEADER + 3 * nv;
        float best = -__builtin_inff();
        V3 nl = v3(0.0f, 0.0f, 1.0f);
        for (int f = 0; f < nf; ++f) {
            const V3 n = v3(pp[4 * f + 0], pp[4 * f + 1], pp[4 * f + 2]);
            const float dist = fdot(n, pl) - pp[4 * f + 3];
            if (dist > best) { best = dist; nl = n; }
        }
        return fma3(s.R.c2, nl.z, fma3(s.R.c1, nl.y, vscale(s.R.c0, nl.x)));
    }
    float t = fdot(dp, s.R.c0);
    t = fminf(fmaxf(t, -s.h.y), s.h.y);
    return vscale(fma3(s.R.c0, -t, dp), 1.0f / s.h.x);
}

__device__ __forceinline__ unsigned q8(float x) {
    return (unsigned)(fminf(fmaxf(x, 0.0f), 1.0f) * 255.0f + 0.5f);
}

// packed RGBA of the ground: index par | shadow << 1
__device__ __forceinline__ unsigned ground_rgba(int i) {
    const int par = i & 1;
    const float k = (i & 2) ? 0.55f : 1.0f;
    const float cr = (par ? 108.0f / 255.0f : 143.0f / 255.0f) * k;
    const float cb = (par ? 113.0f / 255.0f : 150.0f / 255.0f) * k;
    return q8(cr) | (q8(cr) << 8) | (q8(cb) << 16) | 0xFF000000u;
}

struct Cam {
    V3 o, f, l, u;
    float cx, cy, ifx, ify, near_plane, far_plane;
    float h0;            // dot(gn, o) + gpd: the camera's height over the ground
};

// one pixel: nearest hit among ground + the culled shape list, shadow ray
// against every shape (ground pixels: the shapes whose shadow footprint can
// fall in the run), shading. rb = f + u b of the pixel's row.
__device__ __forceinline__ void shade(const MgRenderArgs& A, const Cam& C, const WS* sws, const int* act, int nact,
                                      int nall, const int* gsh, int ngsh, const unsigned* glut, V3 rb, int col,
                                      unsigned& rgba, float& depth, int& seg) {
    const float a = (C.cx - ((float)col + 0.5f)) * C.ifx;
    const V3 d = fma3(C.l, a, rb);
    const V3 gn = v3(A.gn[0], A.gn[1], A.gn[2]);
    float best = C.far_plane;
    int hit = -2;
    if (A.has_ground) {
        const float dn = fdot(gn, d);
        if (dn < 0.0f) {
            const float t = -C.h0 / dn;
            if (t >= C.near_plane && t < best) { best = t; hit = -1; }
        }
    }
    const float dd = fdot(d, d);
    for (int j = 0; j < nact; ++j) {
        const int s = act[j];
        if (ray_misses_bound(C.o, d, dd, sws[s])) continue;
        const float t = ray_shape(C.o, d, sws[s], C.near_plane, best);
        if (t < best) { best = t; hit = s; }
    }
    if (hit == -2) {
        rgba = 0xFF000000u;
        depth = -__builtin_inff();
        seg = 0;
        return;
    }
    const V3 p = fma3(d, best, C.o);
    const V3 n = hit >= 0 ? shape_normal(sws[hit], p) : gn;
    const V3 L = v3(A.light[0], A.light[1], A.light[2]);
    const V3 ps = fma3(n, 1e-3f, p);
    bool shadow = false;
    if (hit >= 0) {
        for (int j = 0; j < nall && !shadow; ++j)
            shadow = !ray_misses_bound(ps, L, 1.0f, sws[j]) &&
                     ray_shape(ps, L, sws[j], 0.0f, __builtin_inff()) < __builtin_inff();
    } else {
        for (int j = 0; j < ngsh && !shadow; ++j) {
            const int s = gsh[j];
            shadow = !ray_misses_bound(ps, L, 1.0f, sws[s]) &&
                     ray_shape(ps, L, sws[s], 0.0f, __builtin_inff()) < __builtin_inff();
        }
    }
    if (hit >= 0) {
        const float lam = fmaxf(fdot(n, L), 0.0f);
        const float kr = shadow ? A.lamb[0] : fmaf(A.lcol[0], lam, A.lamb[0]);
        const float kg = shadow ? A.lamb[1] : fmaf(A.lcol[1], lam, A.lamb[1]);
        const float kb = shadow ? A.lamb[2] : fmaf(A.lcol[2], lam, A.lamb[2]);
        rgba = q8(sws[hit].r * kr) | (q8(sws[hit].g * kg) << 8) | (q8(sws[hit].b * kb) << 16) | 0xFF000000u;
        seg = sws[hit].seg;
    } else {
        const float uu = p.x, vv = A.up_axis == 1 ? p.y : p.z;
        const int par = ((int)floorf(uu) + (int)floorf(vv)) & 1;
        rgba = glut[par | (shadow ? 2 : 0)];
        seg = 0;
    }
    depth = -best;
}

__global__ void __launch_bounds__(256) k_render(MgRenderArgs A) {
    __shared__ WS sws[MG_RENDER_MAX_SHAPES];
    __shared__ int act[MG_RENDER_MAX_SHAPES];    // primary rays: shapes that can appear in the run
    __shared__ int gsh[MG_RENDER_MAX_SHAPES];    // ground shadow rays: shapes whose footprint can
    __shared__ int s_nact, s_ngsh;               //   fall in the run

    // camera of this workgroup (uniform binary search over the prefix blk0)
    const int blk = blockIdx.x;
    int lo = 0, hi = A.ncam - 1;
    if (A.uniform_nblk > 0) {
        lo = blk / A.uniform_nblk;       // equal-size cameras: no search (each probe is a dependent load)
    } else {
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (A.cams[mid].blk0 <= blk) lo = mid; else hi = mid - 1;
        }
    }
    const MgRenderCam& K = A.cams[lo];
    const int W = K.w, H = K.h;
    const int npx = W * H;
    const int px_begin = (blk - K.blk0) * MG_RENDER_RUN;
    const int px_end = min(px_begin + MG_RENDER_RUN, npx);
    const int nb = A.nb;
    const float* S = A.state;

    // camera pose (FOLLOW_TRANSFORM / FOLLOW_POSITION / fixed)
    Cam C;
    {
        V3 o = v3(K.p[0], K.p[1], K.p[2]);
        Q4 q = q4(K.q[0], K.q[1], K.q[2], K.q[3]);
        if (K.slot >= 0) {
            const int i = K.slot;
            const V3 pb = v3(S[0 * nb + i], S[1 * nb + i], S[2 * nb + i]);
            const Q4 qb = q4(S[3 * nb + i], S[4 * nb + i], S[5 * nb + i], S[6 * nb + i]);
            if (K.follow == 1) {
                o = vadd(pb, qrot(qb, o));
                q = qmul(qb, q);
            } else {
                o = vadd(pb, o);
            }
        }
        C.o = o;
        C.f = qrot(q, v3(A.fwd[0], A.fwd[1], A.fwd[2]));
        C.l = qrot(q, v3(A.left[0], A.left[1], A.left[2]));
        C.u = qrot(q, v3(A.up[0], A.up[1], A.up[2]));
        C.cx = K.cx; C.cy = K.cy; C.ifx = K.ifx; C.ify = K.ify;
        C.near_plane = K.near_plane; C.far_plane = K.far_plane;
        C.h0 = fdot(v3(A.gn[0], A.gn[1], A.gn[2]), o) + A.gpd;
    }
    unsigned glut[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) glut[i] = ground_rgba(i);

    // the env's shapes in the world frame, one lane per shape
    const int s0 = A.env_shape_first[K.env];
    const int ns = A.env_shape_first[K.env + 1] - s0;
    const int t = threadIdx.x;
    const int row0 = px_begin / W, row1 = (px_end - 1) / W;
    // can a sphere (c, R) project into rows row0..row1? (conservative)
    auto in_rows = [&](V3 c, float R) -> bool {
        const V3 dv = vsub(c, C.o);
        const float z = vdot(dv, C.f), yu = vdot(dv, C.u);
        if (z + R < C.near_plane) return false;
        if (z - R <= 0.5f * C.near_plane) return true;
        const float b_hi = fmaxf((yu + R) / (z - R), (yu + R) / (z + R));
        const float b_lo = fminf((yu - R) / (z - R), (yu - R) / (z + R));
        const float fy = 1.0f / C.ify;
        const float r_top = C.cy - b_hi * fy - 2.0f;
        const float r_bot = C.cy - b_lo * fy + 2.0f;
        return !(r_bot < (float)row0 || r_top > (float)(row1 + 1));
    };
    if (t < 64) {
        bool keep = false, gkeep = false;
        if (t < ns) {
            const MgRShape rs = A.rshapes[s0 + t];
            const int i = rs.slot;
            const V3 pb = v3(S[0 * nb + i], S[1 * nb + i], S[2 * nb + i]);
            const Q4 qb = q4(S[3 * nb + i], S[4 * nb + i], S[5 * nb + i], S[6 * nb + i]);
            const float* sh = A.shapes + (size_t)rs.shape * MG_SHAPE_STRIDE;
            WS w;
            w.type = (int)sh[0];
            w.seg = rs.seg;
            w.r = rs.r; w.g = rs.g; w.b = rs.b;
            w.c = vadd(pb, qrot(qb, v3(sh[4], sh[5], sh[6])));
            w.R = qmat(qmul(qb, q4(sh[7], sh[8], sh[9], sh[10])));
            if (w.type == MG_SHAPE_BOX) {
                w.h = v3(sh[1], sh[2], sh[3]);
                w.brad = sqrtf(vdot(w.h, w.h));
            } else if (w.type == MG_SHAPE_SPHERE) {
                w.h = v3(sh[1], 0.0f, 0.0f);
                w.brad = sh[1];
            } else if (w.type == MG_SHAPE_CONVEX) {
                w.h = v3(sh[1], 0.0f, 0.0f);
                w.brad = sh[1];
            } else {
                w.h = v3(sh[1], sh[2], 0.0f);
                w.brad = sh[1] + sh[2];
            }
            w.hv = w.type == MG_SHAPE_CONVEX ? A.hulls + (int)sh[2] : nullptr;
            {
                const float rp = w.brad * 1.01f + 1e-3f;
                w.brad2 = rp * rp;
            }
            sws[t] = w;
            // primary-ray culling: rows the bounding sphere can project to. A
            // camera strictly inside a box or sphere sees none of it (only entry
            // points are hits and they all lie behind the near plane).
            const V3 ol = fmt(w.R, vsub(C.o, w.c));      // as in ray_box / ray_sphere
            const V3 os = vsub(C.o, w.c);
            bool in_hull = w.type == MG_SHAPE_CONVEX;
            if (in_hull) {                      // strictly inside every face plane (as ray_convex)
                const int nv = (int)w.hv[0], nf = (int)w.hv[1];
                const float* pp = w.hv + MG_HULL_HEADER + 3 * nv;
                for (int f = 0; f < nf; ++f)
                    in_hull = in_hull && fdot(v3(pp[4 * f], pp[4 * f + 1], pp[4 * f + 2]), ol) - pp[4 * f + 3] < 0.0f;
            }
            const bool inside =
                C.near_plane > 0.0f &&
                ((w.type == MG_SHAPE_BOX && fabsf(ol.x) < w.h.x && fabsf(ol.y) < w.h.y && fabsf(ol.z) < w.h.z) ||
                 (w.type == MG_SHAPE_SPHERE && fmaf(-w.h.x, w.h.x, fdot(os, os)) < 0.0f) || in_hull);
            keep = !inside && in_rows(w.c, w.brad * 1.001f + 1e-4f);
            // ground shadow culling: the ground points whose shadow ray (from 1e-3
            // above the plane, towards L) passes within the bounding radius of
            // the centre lie in a disk of radius (R + 1e-3) / (L . n) around the
            // centre's projection along L onto the plane; the shape can shadow
            // this run only if that disk can project into its rows
            if (A.has_ground) {
                const V3 gn = v3(A.gn[0], A.gn[1], A.gn[2]);
                const V3 L = v3(A.light[0], A.light[1], A.light[2]);
                const float ln = vdot(L, gn);
                if (!(ln > 0.05f)) {
                    gkeep = true;
                } else {
                    const float hc = vdot(gn, w.c) + A.gpd;
                    const V3 cg = vmad(w.c, L, -hc / ln);
                    gkeep = in_rows(cg, (w.brad * 1.01f + 3e-3f) / ln * 1.01f + 1e-3f);
                }
            }
        }
        const unsigned long long m = __ballot(keep);
        if (keep) act[__popcll(m & ((1ull << t) - 1ull))] = t;
        const unsigned long long gm = __ballot(gkeep);
        if (gkeep) gsh[__popcll(gm & ((1ull << t) - 1ull))] = t;
        if (t == 0) {
            s_nact = __popcll(m);
            s_ngsh = __popcll(gm);
        }
    }
    __syncthreads();
    const int nact = s_nact;
    const int ngsh = s_ngsh;
    const int nall = ns;

    const int wave = t >> 6, lane = t & 63;
#pragma unroll 1
    for (int pass = 0; pass < MG_RENDER_PASSES; ++pass) {
        const int px0 = px_begin + ((pass * MG_RENDER_WAVES + wave) * 64 + lane) * MG_RENDER_LANE_PX;
        if (px0 >= px_end) continue;
        int row = px0 / W;
        int col = px0 - row * W;
        V3 rb = fma3(C.u, (C.cy - ((float)row + 0.5f)) * C.ify, C.f);
        unsigned rgba[MG_RENDER_LANE_PX];
        float dep[MG_RENDER_LANE_PX];
        int sg[MG_RENDER_LANE_PX];
#pragma unroll
        for (int k = 0; k < MG_RENDER_LANE_PX; ++k) {
            rgba[k] = 0u; dep[k] = 0.0f; sg[k] = 0;
            if (px0 + k < px_end)
                shade(A, C, sws, act, nact, nall, gsh, ngsh, glut, rb, col, rgba[k], dep[k], sg[k]);
            if (++col == W) {
                col = 0;
                ++row;
                rb = fma3(C.u, (C.cy - ((float)row + 0.5f)) * C.ify, C.f);
            }
        }
        if (K.vec && px0 + MG_RENDER_LANE_PX <= px_end) {
            if (K.color) *(uint4*)(K.color + (size_t)px0 * 4) = make_uint4(rgba[0], rgba[1], rgba[2], rgba[3]);
            if (K.depth) *(float4*)(K.depth + px0) = make_float4(dep[0], dep[1], dep[2], dep[3]);
            if (K.seg) *(int4*)(K.seg + px0) = make_int4(sg[0], sg[1], sg[2], sg[3]);
        } else {
#pragma unroll
            for (int k = 0; k < MG_RENDER_LANE_PX; ++k) {
                if (px0 + k >= px_end) break;
                if (K.color) *(unsigned*)(K.color + (size_t)(px0 + k) * 4) = rgba[k];
                if (K.depth) K.depth[px0 + k] = dep[k];
                if (K.seg) K.seg[px0 + k] = sg[k];
            }
        }
    }
}

}  // namespace

hipError_t mg_launch_render(const MgRenderArgs& A, int nblocks, hipStream_t s) {
    if (nblocks <= 0 || A.ncam <= 0) return hipSuccess;
    MG_LAUNCH(k_render, dim3(nblocks), dim3(256), 0, s, A);
    return hipGetLastError();
}
