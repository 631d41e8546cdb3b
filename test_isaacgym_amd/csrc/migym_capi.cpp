// migym_capi.cpp — host side of libmigym.so: the C ABI declared in
// include/migym.h. Owns the engine state in HBM (SoA, env index as the
// coalesced axis), launches the step kernels and the tensor-API copy kernels on
// the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdarg>
#include <cstring>
#include <string>
#include <map>
#include <vector>

#include "mg_internal.h"
#include "mg_chainlink.h"

thread_local MgKernelTimer* mg_timer = nullptr;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(MG_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <class T>
hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void**)p, n * sizeof(T));
}

// host AoS [n][ncol] -> device SoA [ncol][n]
template <class T>
std::vector<T> to_soa(const T* aos, int n, int ncol) {
    std::vector<T> soa((size_t)n * ncol);
    for (int i = 0; i < n; ++i)
        for (int f = 0; f < ncol; ++f) soa[(size_t)f * n + i] = aos[(size_t)i * ncol + f];
    return soa;
}

struct ArticGroup {
    int chain;                     // serial chain with one DOF per moving link (MgArticArgs.chain)
    // k_artic_chain's shared constants (mg_chainlink.h): the stepped instances'
    // global first body / first DOF, whether their link mass rows and gravity
    // flags agree (set at upload), whether their DOF properties agree (upload
    // and mg_set_dof_props), the constants themselves
    std::vector<int> step_body0, step_dof0;
    bool uni_mass = false, uni_dof = false;
    float uni[MG_CHAIN_UNI_N] = {};
    int tmpl, first_link, nl, ndof, fixed_base;
    int nbody;                     // bodies per instance (nl minus the virtual links of ball joints)
    int offset, count;             // into the template-sorted instance list (all instances)
    int step_offset, step_count;   // into the list stepped by k_artic_chain / k_artic_lanes (uncoupled envs)
    // the stepped instances' rows are affine in the instance (MgArticArgs::aff),
    // and so are their fused-refresh rows (out_aff: rigid-body row og0 + a nl +
    // l, actor row or0 + a)
    int aff = 0, aff_b0 = 0, aff_d0 = 0, aff_ds = 0;
    int out_aff = 0, out_g0 = 0, out_r0 = 0;
};

// coupled envs (mg_env.hip) of one articulation template (tmpl -1: none)
struct EnvGroup {
    int tmpl, first_link, nl, ndof, floating;
    int wide;            // 64 lanes per env (mg_env.hip k_env_step<32, 64>), else 16
    int max_free;        // most free bodies of one env of the group (velocity slots)
    int offset, count;   // rows of d_env
};

}  // namespace

struct mg_sim {
    int device = 0;
    mg_sim_params params{};
    bool uploaded = false;

    int nenv = 0, na = 0, nb = 0, nd = 0, ntb = 0, ns = 0, nf = 0, nartic = 0, ntl = 0;
    int max_actor_dofs = 0;
    int nf1 = 0;   // single-shape free bodies (storage slots 0..nf1-1)
    int nf_rigid = 0;   // free bodies of uncoupled envs (slots 0..nf_rigid-1), free-body kernel

    float* d_state = nullptr;     // [13][nb]
    float* d_mass = nullptr;      // [12][nb]
    // Bodies are stored in an internal order (free bodies first, by launch group
    // and template; then each articulation's links contiguously; then the rest)
    // so every kernel's lanes touch contiguous SoA slots. Tensors stay in the
    // global (Isaac Gym) order: the gather / scatter index maps fold in `perm`.
    int* d_body_tmpl = nullptr;   // [nb] internal order
    int* d_free_global = nullptr; // [nf] global ids of the free bodies (internal 0..nf-1)
    int* d_perm = nullptr;        // [nb] global body -> internal slot
    float* d_tbf = nullptr;
    float* d_trec = nullptr;      // [ntb][MG_TREC_N] compact template records (k_rigid_step1)
    int* d_tbi = nullptr;
    float* d_shapes = nullptr;
    float* d_hulls = nullptr;     // convex hull records (MG_SHAPE_CONVEX)
    float* d_shape_obb = nullptr; // [ns][MG_OBB_N] shape-frame boxes (coupled step's pair screen)
    int* d_actor_root = nullptr;  // [na] internal slot of each actor's root body
    int* d_body_actor = nullptr;  // [nb] global body -> the actor it is the root of, or -1
    // Step fusion (mg_set_fusion): a device-resident, non-indexed root-state set
    // of a sim whose actor roots are all single-shape free bodies is read by the
    // next simulate's free-body kernel (d_root_row: internal slot -> actor row,
    // -1 for non-roots) instead of a scatter launch; any earlier reader of the
    // state flushes it as the scatter. A root refresh into the bound root tensor
    // also gathers the bound rigid-body tensor (one launch), and the rigid-body
    // refresh that follows is served by it while the state is unchanged.
    int* d_root_row = nullptr;
    bool roots_free = false;
    int fusion = 0;   // opt-in (mg_set_fusion): Isaac Gym copies at set time and refreshes exactly what is asked
    const float* pend_root = nullptr;
    const float* pend_tgt[3] = {nullptr, nullptr, nullptr};   // fused DOF target sets (pos, vel, force)
    // stream-capture id (0: eager) at which each deferred set / the paired
    // refresh happened: fused work is only combined within one capture (or
    // eagerly), so a graph never relies on work it did not record
    unsigned long long pend_root_cap = 0, pend_tgt_cap[3] = {0, 0, 0}, rb_cap = 0;
    float* bind_root = nullptr;
    float* bind_rb = nullptr;
    float* bind_dof = nullptr;    // the persistent DOF-state tensor (mg_bind_dof_refresh_target)
    long long state_gen = 0, rb_gen = -1, out_gen = -1;   // out_gen: bound tensors written by the step
    unsigned long long out_cap = 0;
    // DOF state generation (simulate, mg_set_dof_state) and the one the step
    // wrote into the bound DOF tensor (MG_FUSE_STEP_OUT)
    long long dof_sgen = 0, dof_gen = -1;
    unsigned long long dof_cap = 0;
    // MG_FUSE_STEP_OUT covers the sim: every body is stepped by a kernel that
    // writes its rows (single-shape free bodies in k_rigid_step1, links of
    // uncoupled serial chains in k_artic_chain), so the refreshes after a
    // simulate can be served by the step itself
    bool step_out_ok = false;
    int* d_slot_global = nullptr; // [nb] internal slot -> global body (rigid-body tensor row)
    int* d_slot_actor = nullptr;  // [nb] internal slot -> actor row it is the root of, or -1
    int last_set_deferred = 0;    // the last mg_set_* left its source to be read by the next simulate
    int* d_actor_dof = nullptr;   // [na+1]
    float* d_cforce = nullptr;    // [3][nb]
    float* d_ext = nullptr;       // [6][nb]
    bool ext_pending = false;

    float* d_dof = nullptr;       // [2][nd]: pos, vel
    float* d_dof_tgt = nullptr;   // [3][nd]: target pos, target vel, actuation force
    float* d_dof_props = nullptr; // [12][nd]
    int* d_artic = nullptr;       // [nartic][4] sorted by template
    float* d_link_f = nullptr;
    int* d_link_i = nullptr;
    std::vector<ArticGroup> groups;
    int* d_artic_step = nullptr;  // [..][4] instances stepped by k_artic_chain / k_artic_lanes
    int* d_env = nullptr;         // [n_coupled][MG_ENV_I_N] coupled envs, by group
    int* d_pairs = nullptr;       // [..][4] candidate shape pairs of the coupled envs
    float* d_fpatch = nullptr;    // [pairs][MG_FP_N] friction patch records (coupled step, persistent)
    float* d_gpatch = nullptr;    // [MG_FP_N][nf1] ground patches of the single-shape free bodies (persistent)
    float* d_chain_uni = nullptr; // [groups][MG_CHAIN_UNI_N] shared constants of chain groups (ArticGroup.uni)
    unsigned* d_fp_mask = nullptr;   // [n_coupled][MG_FP_W] pairs holding a patch
    float* d_env_carry = nullptr;    // [n_coupled][mg_env_carry_floats] coupled step state between substep launches
    int nhull_floats = 0;            // floats of the hull table (k_env_np stages it in LDS when small)
    float* d_env_ctab = nullptr;     // [n_coupled][mg_env_ctab_floats] contacts of one substep (k_env_np -> k_env_step)
    int n_coupled = 0;
    std::vector<EnvGroup> env_groups;
    // free-body piles (mg_pile.hip): coupled envs of more than MG_ENV_MAXF free
    // bodies and no articulation, one wavefront each
    int n_pile = 0;
    int* d_pile_i = nullptr;      // [n_pile][MG_PILE_I_N]
    int* d_pile_body = nullptr;   // their free bodies' internal slots
    unsigned* d_pile_pairs = nullptr;  // packed candidate pairs (local shape slots, mg_internal.h)
    int* d_pile_slots = nullptr;  // [..][2] local shape slots: participant, shape

    float* d_stage = nullptr;     // host-transfer staging (floats)
    size_t stage_n = 0;
    // CPU pipeline (host state tensors): a full host root set is read by the next
    // step kernel (no scatter launch; h_root_in below); and from the
    // first mg_fetch_host_state on, the step kernels that write their own rows
    // (step_out_ok) write root / rigid-body / DOF rows into d_host_out, laid out as
    // the host stage, so the fetch copies them without gathering (ho_*_gen: the
    // state generation they hold)
    // host sources are copied at the set call into this page-locked buffer (then
    // sent in stream order), so the caller may overwrite its tensor right away —
    // Isaac Gym's copy-at-set — even though the transfer itself is asynchronous;
    // pin_ev: the last transfer out of it (waited on before it is refilled)
    char* h_pin = nullptr;
    size_t h_pin_n = 0;
    hipEvent_t pin_ev = nullptr;
    bool pin_ev_pending = false;
    float* d_host_out = nullptr;
    size_t host_out_n = 0;
    // zero-copy variants (mg_host_stage): the host stage itself, page-locked and
    // mapped into the device's address space — the step kernels write their rows
    // into it over PCIe and the fetch's remaining gathers do too (no copy); and
    // a mapped input buffer the step kernel reads a host root set from
    // (root_ev: its last reader, waited on before it is refilled)
    bool has_light = false;           // mg_set_light (else the default light)
    mg_light light{};
    float* h_stage = nullptr;
    float* d_stage_alias = nullptr;
    size_t h_stage_n = 0;
    float* h_root_in = nullptr;
    float* d_root_in_alias = nullptr;
    hipEvent_t root_ev = nullptr;
    bool root_ev_pending = false;
    bool ho_alias = false;            // the last fetch staged into h_stage: the step writes there
    const float* ho_written = nullptr;   // the stage the last simulate wrote (ho_*_gen refer to it)
    long long ho_root_gen = -1, ho_rb_gen = -1, ho_dof_gen = -1;
    int* d_stage_idx = nullptr;
    size_t stage_idx_n = 0;

    // host copies kept for the camera renderer's shape lists
    std::vector<int> h_perm, h_body_tmpl, h_tbi;
    // camera render (mg_render.hip)
    float* d_rstate = nullptr;    // [13][nb] pose snapshot of render_all_camera_sensors
    bool rstate_valid = false;
    MgRShape* d_rshapes = nullptr;
    int* d_env_shape_first = nullptr;
    int n_rshapes = 0;
    bool render_ready = false;
    MgRenderCam* d_cams = nullptr;
    int cam_cap = 0;
    std::vector<mg_camera> cam_host;      // last uploaded table (as given)
    std::vector<MgRenderCam> cam_dev;     // its device form
    int cam_blocks = 0;
    hipEvent_t rev_b = nullptr, rev_e = nullptr;
    bool rendered = false;

    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    bool timing = false;          // mg_set_kernel_timing: events around eager launches
    bool timed_step = false;      // the last simulate recorded ev_begin / ev_end
    hipStream_t last_stream = nullptr;
    bool stepped = false;
    bool capturing = false;       // the last simulate was recorded into a graph
    // ring of per-simulate event pairs for live kernel timing (bench.py roofline)
    static constexpr int kRing = 256;
    static constexpr int kKern = 8;   // kernels timed per simulate (dispatch timestamps)
    hipEvent_t ring_b[kRing] = {}, ring_e[kRing] = {};
    hipEvent_t kern_b[kRing][kKern] = {}, kern_e[kRing][kKern] = {};
    int kern_n[kRing] = {};
    int kern_miss[kRing] = {};    // launches of that simulate past kKern (untimed)
    long long ring_n = 0;
    // coupled env k (env order) -> its row of d_env and the float offset /
    // length of its contact-table record (mg_debug_copy_env_ctab)
    std::vector<long long> cenv_ctab_off;
    std::vector<int> cenv_ctab_n;
};

namespace {

MgStep make_step(const mg_sim_params& p) {
    MgStep P{};
    const int ss = p.substeps > 0 ? p.substeps : 1;
    const int np = p.num_position_iterations > 0 ? p.num_position_iterations : 1;
    P.substeps = ss;
    P.npos = np;
    P.nvel = p.num_velocity_iterations > 0 ? p.num_velocity_iterations : 0;
    P.h = p.dt / (float)ss;
    P.sub = P.h / (float)np;
    P.inv_sub = 1.0f / P.sub;
    P.inv_h = 1.0f / P.h;
    P.inv_dt = 1.0f / p.dt;
    for (int k = 0; k < 3; ++k) P.g[k] = p.gravity[k];
    P.contact_offset = p.contact_offset;
    P.rest_offset = p.rest_offset;
    P.max_depen = p.max_depenetration_velocity;
    P.bounce_thresh = p.bounce_threshold_velocity;
    P.fric_offset = p.friction_offset_threshold;
    P.fric_corr = p.friction_correlation_distance;
    P.has_ground = p.has_ground;
    const float nx = p.ground_normal[0], ny = p.ground_normal[1], nz = p.ground_normal[2];
    P.n[0] = nx; P.n[1] = ny; P.n[2] = nz;
    P.pd = p.ground_distance;
    // tangent basis: t1 = normalize(n x a), t2 = n x t1
    float ax = 1.0f, ay = 0.0f, az = 0.0f;
    if (!(std::fabs(nx) < 0.9f)) { ax = 0.0f; ay = 1.0f; }
    float t1x = ny * az - nz * ay, t1y = nz * ax - nx * az, t1z = nx * ay - ny * ax;
    const float inv = 1.0f / std::sqrt(t1x * t1x + t1y * t1y + t1z * t1z);
    t1x = t1x * inv; t1y = t1y * inv; t1z = t1z * inv;
    P.t1[0] = t1x; P.t1[1] = t1y; P.t1[2] = t1z;
    P.t2[0] = ny * t1z - nz * t1y;
    P.t2[1] = nz * t1x - nx * t1z;
    P.t2[2] = nx * t1y - ny * t1x;
    P.mu_ground = p.ground_dynamic_friction;
    P.e_ground = p.ground_restitution;
    return P;
}

int ensure_stage(mg_sim* s, size_t nfloat, size_t nidx) {
    if (nfloat > s->stage_n) {
        if (s->d_stage) (void)hipFree(s->d_stage);
        s->d_stage = nullptr;
        HIP_TRY(dalloc(&s->d_stage, nfloat));
        s->stage_n = nfloat;
    }
    if (nidx > s->stage_idx_n) {
        if (s->d_stage_idx) (void)hipFree(s->d_stage_idx);
        s->d_stage_idx = nullptr;
        HIP_TRY(dalloc(&s->d_stage_idx, nidx));
        s->stage_idx_n = nidx;
    }
    return MG_OK;
}

// gather `n` rows of `ncol` SoA fields into dst (host or device)
int refresh_rows(mg_sim* s, const float* soa, int stride, int ncol, const int* ids, int n, float* dst,
                 int dst_host, hipStream_t st) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!dst && n > 0) return fail(MG_ERR_ARG, "null destination");
    HIP_TRY(hipSetDevice(s->device));
    if (n == 0) return MG_OK;
    if (!dst_host) {
        HIP_TRY(mg_launch_gather_rows(soa, stride, ncol, ids, n, dst, st));
        return MG_OK;
    }
    int rc = ensure_stage(s, (size_t)n * ncol, 0);
    if (rc) return rc;
    HIP_TRY(mg_launch_gather_rows(soa, stride, ncol, ids, n, s->d_stage, st));
    HIP_TRY(hipMemcpyAsync(dst, s->d_stage, (size_t)n * ncol * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MG_OK;
}

// copy host data into the sim's page-locked buffer now and send it to the device
// in stream order: n parts (src[k], bytes[k]) to dst[k]
int pin_h2d(mg_sim* s, int n, const void* const* src, const size_t* bytes, void* const* dst, hipStream_t st) {
    size_t total = 0;
    for (int k = 0; k < n; ++k) total += (bytes[k] + 255) & ~(size_t)255;
    if (total > s->h_pin_n) {
        if (s->pin_ev_pending) HIP_TRY(hipEventSynchronize(s->pin_ev));
        if (s->h_pin) (void)hipHostFree(s->h_pin);
        s->h_pin = nullptr;
        s->h_pin_n = 0;
        HIP_TRY(hipHostMalloc((void**)&s->h_pin, total, hipHostMallocDefault));
        s->h_pin_n = total;
    }
    if (!s->pin_ev) HIP_TRY(hipEventCreateWithFlags(&s->pin_ev, hipEventDisableTiming));
    if (s->pin_ev_pending) HIP_TRY(hipEventSynchronize(s->pin_ev));   // the previous transfer left it
    size_t at = 0;
    for (int k = 0; k < n; ++k) {
        std::memcpy(s->h_pin + at, src[k], bytes[k]);
        HIP_TRY(hipMemcpyAsync(dst[k], s->h_pin + at, bytes[k], hipMemcpyHostToDevice, st));
        at += (bytes[k] + 255) & ~(size_t)255;
    }
    HIP_TRY(hipEventRecord(s->pin_ev, st));
    s->pin_ev_pending = true;
    return MG_OK;
}

// stage a host source (and optional index list) to the device
int stage_src(mg_sim* s, const float* src, int src_host, size_t nfloat, const int* idx, int n_idx,
              hipStream_t st, const float** dsrc, const int** didx) {
    *dsrc = src;
    *didx = idx;
    if (!src_host) return MG_OK;
    int rc = ensure_stage(s, nfloat, idx ? (size_t)n_idx : 0);
    if (rc) return rc;
    const void* srcs[2] = {src, idx};
    const size_t bytes[2] = {nfloat * sizeof(float), idx && n_idx > 0 ? (size_t)n_idx * sizeof(int) : 0};
    void* dsts[2] = {s->d_stage, s->d_stage_idx};
    if ((rc = pin_h2d(s, bytes[1] ? 2 : 1, srcs, bytes, dsts, st))) return rc;
    *dsrc = s->d_stage;
    if (idx && n_idx > 0) *didx = s->d_stage_idx;
    return MG_OK;
}

// id of the stream capture in progress on st + 1, or 0 when st is not capturing
unsigned long long capture_id(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(st, &cs, &id) != hipSuccess || cs != hipStreamCaptureStatusActive) return 0;
    return id + 1;
}
// may this call defer / combine work? always eagerly; inside a stream capture
// only when the caller opted in (MG_FUSE_IN_CAPTURE): a deferred set left at
// the end of a captured region would never be applied by its replays
bool fuse_here(const mg_sim* s, unsigned long long cid) { return cid == 0 || (s->fusion & MG_FUSE_IN_CAPTURE); }

// apply a deferred root-state set as the ordinary scatter (a reader of the
// state comes before the next simulate)
int flush_root(mg_sim* s, hipStream_t st) {
    if (!s->pend_root) return MG_OK;
    const float* src = s->pend_root;
    s->pend_root = nullptr;
    HIP_TRY(mg_launch_scatter_rows(src, MG_STATE_N, s->d_actor_root, nullptr, s->na, s->na, s->d_state, s->nb, st));
    if (src == s->d_root_in_alias) {   // the mapped input buffer's reader
        HIP_TRY(hipEventRecord(s->root_ev, st));
        s->root_ev_pending = true;
    }
    return MG_OK;
}

// apply a deferred DOF target column (0 pos, 1 vel, 2 force) as a copy
int flush_tgt(mg_sim* s, int k, hipStream_t st) {
    if (!s->pend_tgt[k]) return MG_OK;
    const float* src = s->pend_tgt[k];
    s->pend_tgt[k] = nullptr;
    HIP_TRY(hipMemcpyAsync(s->d_dof_tgt + (size_t)k * s->nd, src, (size_t)s->nd * sizeof(float),
                           hipMemcpyDeviceToDevice, st));
    return MG_OK;
}

int set_dof_columns(mg_sim* s, const float* src, int src_host, int ncol, float* dst0, float* dst1,
                    const int* idx, int n_idx, hipStream_t st) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (s->nd == 0) return MG_OK;
    if (!src) return fail(MG_ERR_ARG, "null source tensor");
    if (idx && n_idx < 0) return fail(MG_ERR_ARG, "negative index count");
    HIP_TRY(hipSetDevice(s->device));
    const float* dsrc;
    const int* didx;
    int rc = stage_src(s, src, src_host, (size_t)s->nd * ncol, idx, n_idx, st, &dsrc, &didx);
    if (rc) return rc;
    float* dst[2] = {dst0, dst1};
    if (idx)
        HIP_TRY(mg_launch_scatter_dofs(dsrc, ncol, s->d_actor_dof, didx, n_idx, s->na, s->max_actor_dofs, dst, st));
    else
        HIP_TRY(mg_launch_scatter_dofs(dsrc, ncol, nullptr, nullptr, s->nd, 0, 1, dst, st));
    return MG_OK;
}

// Shape-frame box of a shape (the coupled step's pair screen, mg_env.hip
// obb_apart; oracle: shape_obb_): centre and half extents; a hull's from the
// min / max of its vertices
void shape_obb(const float* sh, const float* hulls, float* o) {
    const int t = (int)sh[0];
    for (int k = 0; k < MG_OBB_N; ++k) o[k] = 0.0f;
    if (t == MG_SHAPE_CONVEX && hulls) {
        const float* hv = hulls + (int)sh[2];
        const int nv = (int)hv[0];
        float lo[3], hi[3];
        for (int c = 0; c < 3; ++c) { lo[c] = hv[MG_HULL_HEADER + c]; hi[c] = lo[c]; }
        for (int i = 1; i < nv; ++i)
            for (int c = 0; c < 3; ++c) {
                const float v = hv[MG_HULL_HEADER + 3 * i + c];
                lo[c] = std::min(lo[c], v);
                hi[c] = std::max(hi[c], v);
            }
        for (int c = 0; c < 3; ++c) {
            o[c] = 0.5f * (lo[c] + hi[c]);
            o[3 + c] = 0.5f * (hi[c] - lo[c]);
        }
    } else if (t == MG_SHAPE_BOX) {
        o[3] = sh[1]; o[4] = sh[2]; o[5] = sh[3];
    } else if (t == MG_SHAPE_CAPSULE) {
        o[3] = sh[1] + sh[2]; o[4] = sh[1]; o[5] = sh[1];
    } else {
        o[3] = sh[1]; o[4] = sh[1]; o[5] = sh[1];
    }
}

void free_all(mg_sim* s) {
    void* ptrs[] = {s->d_state, s->d_mass, s->d_body_tmpl, s->d_free_global, s->d_perm, s->d_tbf, s->d_trec, s->d_tbi, s->d_shapes, s->d_hulls, s->d_shape_obb,
                    s->d_actor_root, s->d_root_row, s->d_slot_global, s->d_slot_actor, s->d_body_actor, s->d_actor_dof, s->d_cforce, s->d_ext, s->d_dof, s->d_dof_tgt,
                    s->d_dof_props, s->d_artic, s->d_artic_step, s->d_env, s->d_pairs, s->d_fpatch, s->d_gpatch, s->d_chain_uni, s->d_fp_mask, s->d_env_carry, s->d_env_ctab, s->d_link_f, s->d_link_i, s->d_stage, s->d_stage_idx, s->d_host_out,
                    s->d_pile_i, s->d_pile_body, s->d_pile_pairs, s->d_pile_slots, s->d_rstate, s->d_rshapes, s->d_env_shape_first, s->d_cams};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
}

}  // namespace

extern "C" {

int32_t mg_abi_version(void) { return MG_ABI_VERSION; }
const char* mg_last_error(void) { return g_err.c_str(); }

int32_t mg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

mg_sim* mg_create_sim(int32_t device, const mg_sim_params* params) {
    if (!params) { fail(MG_ERR_ARG, "null params"); return nullptr; }
    int n = mg_device_count();
    if (n <= 0) { fail(MG_ERR_DEVICE, "no HIP device available (libmigym needs an MI355X)"); return nullptr; }
    if (device < 0 || device >= n) { fail(MG_ERR_DEVICE, "device %d out of range (%d visible)", device, n); return nullptr; }
    if (hipSetDevice(device) != hipSuccess) { fail(MG_ERR_DEVICE, "hipSetDevice(%d) failed", device); return nullptr; }
    mg_sim* s = new mg_sim();
    s->device = device;
    s->params = *params;
    for (int k = 0; k < mg_sim::kRing; ++k) {
        bool ok = hipEventCreate(&s->ring_b[k]) == hipSuccess && hipEventCreate(&s->ring_e[k]) == hipSuccess;
        for (int j = 0; j < mg_sim::kKern && ok; ++j)
            ok = hipEventCreate(&s->kern_b[k][j]) == hipSuccess && hipEventCreate(&s->kern_e[k][j]) == hipSuccess;
        if (!ok) {
            fail(MG_ERR_DEVICE, "hipEventCreate failed");
            mg_destroy_sim(s);
            return nullptr;
        }
    }
    return s;
}

void mg_destroy_sim(mg_sim* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipDeviceSynchronize();
    free_all(s);
    for (int k = 0; k < mg_sim::kRing; ++k) {
        if (s->ring_b[k]) (void)hipEventDestroy(s->ring_b[k]);
        if (s->ring_e[k]) (void)hipEventDestroy(s->ring_e[k]);
        for (int j = 0; j < mg_sim::kKern; ++j) {
            if (s->kern_b[k][j]) (void)hipEventDestroy(s->kern_b[k][j]);
            if (s->kern_e[k][j]) (void)hipEventDestroy(s->kern_e[k][j]);
        }
    }
    if (s->rev_b) (void)hipEventDestroy(s->rev_b);
    if (s->rev_e) (void)hipEventDestroy(s->rev_e);
    if (s->pin_ev) (void)hipEventDestroy(s->pin_ev);
    if (s->h_pin) (void)hipHostFree(s->h_pin);
    if (s->root_ev) (void)hipEventDestroy(s->root_ev);
    if (s->h_root_in) (void)hipHostFree(s->h_root_in);
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    delete s;
}

int32_t mg_set_sim_params(mg_sim* s, const mg_sim_params* p) {
    if (!s || !p) return fail(MG_ERR_ARG, "null argument");
    s->params = *p;
    return MG_OK;
}

// k_artic_chain's shared constants (mg_chainlink.h). Link mass constants and
// the gravity flag: from the stepped instances' global rows, when they all
// agree (set once: mass properties are fixed after upload).
static void chain_uni_mass(const mg_model* m, ArticGroup& g) {
    const int b0 = g.step_body0[0];
    bool ok = true;
    const float grav = m->tmpl_body_f[(size_t)m->body_tmpl[b0] * MG_TBODY_F_N + 4];
    for (size_t i = 1; i < g.step_body0.size() && ok; ++i) {
        const int bi = g.step_body0[i];
        ok = m->tmpl_body_f[(size_t)m->body_tmpl[bi] * MG_TBODY_F_N + 4] == grav;
        for (int l = 1; l < g.nl && ok; ++l)
            ok = std::memcmp(m->body_mass + (size_t)(bi + l) * MG_MASS_N, m->body_mass + (size_t)(b0 + l) * MG_MASS_N,
                             MG_MASS_N * sizeof(float)) == 0;
    }
    g.uni_mass = ok;
    if (!ok) return;
    for (int l = 1; l < g.nl; ++l) {
        const float* r = m->body_mass + (size_t)(b0 + l) * MG_MASS_N;
        const ChainLink k = chain_link_make(r[11], v3(r[8], r[9], r[10]), r[1], r[2], r[3], q4(r[4], r[5], r[6], r[7]));
        float* u = g.uni + MG_CHAIN_UNI_LINK + 10 * (l - 1);
        u[0] = k.m;
        u[1] = k.com.x; u[2] = k.com.y; u[3] = k.com.z;
        for (int j = 0; j < 6; ++j) u[4 + j] = k.ib[j];
    }
    g.uni[MG_CHAIN_UNI_GRAV] = grav;
}
// DOF properties (global DOF order, MG_DOFPROP_N per DOF): fields 0..8 of each
// DOF of the chain, when every stepped instance has the same
static void chain_uni_dof(const float* props, ArticGroup& g) {
    const int d0 = g.step_dof0[0];
    bool ok = true;
    for (size_t i = 1; i < g.step_dof0.size() && ok; ++i)
        for (int d = 0; d < g.ndof && ok; ++d)
            ok = std::memcmp(props + (size_t)(g.step_dof0[i] + d) * MG_DOFPROP_N, props + (size_t)(d0 + d) * MG_DOFPROP_N,
                             9 * sizeof(float)) == 0;
    g.uni_dof = ok;
    g.uni[MG_CHAIN_UNI_DOFOK] = ok ? 1.0f : 0.0f;   // read by the kernel (graph replays see changes)
    if (!ok) return;
    for (int d = 0; d < g.ndof; ++d)
        for (int j = 0; j < 9; ++j) g.uni[MG_CHAIN_UNI_DOF + 9 * d + j] = props[(size_t)(d0 + d) * MG_DOFPROP_N + j];
}
static hipError_t chain_uni_upload(mg_sim* s) {
    if (!s->d_chain_uni) return hipSuccess;
    std::vector<float> u(s->groups.size() * MG_CHAIN_UNI_N, 0.0f);
    for (size_t i = 0; i < s->groups.size(); ++i)
        std::memcpy(&u[i * MG_CHAIN_UNI_N], s->groups[i].uni, MG_CHAIN_UNI_N * sizeof(float));
    return hipMemcpy(s->d_chain_uni, u.data(), u.size() * sizeof(float), hipMemcpyHostToDevice);
}

int32_t mg_upload_model(mg_sim* s, const mg_model* m) {
    if (!s || !m) return fail(MG_ERR_ARG, "null argument");
    if (s->uploaded) return fail(MG_ERR_STATE, "model already uploaded");
    if (m->num_bodies < 0 || m->num_actors < 0 || m->num_dofs < 0) return fail(MG_ERR_ARG, "negative sizes");
    HIP_TRY(hipSetDevice(s->device));
    const int nb = m->num_bodies, na = m->num_actors, nd = m->num_dofs;
    s->nenv = m->num_envs; s->na = na; s->nb = nb; s->nd = nd;
    s->ntb = m->num_tmpl_bodies; s->ns = m->num_shapes;
    s->nartic = m->num_artics; s->ntl = m->num_tmpl_links;

    // validate indices on the host before anything reaches a kernel
    for (int b = 0; b < nb; ++b) {
        const int t = m->body_tmpl[b];
        if (t < 0 || t >= s->ntb) return fail(MG_ERR_ARG, "body %d: template %d out of range", b, t);
        const int s0 = m->tmpl_body_i[t * MG_TBODY_I_N + 0], sc = m->tmpl_body_i[t * MG_TBODY_I_N + 1];
        if (s0 < 0 || sc < 0 || s0 + sc > s->ns) return fail(MG_ERR_ARG, "template body %d: bad shape range", t);
    }
    for (int k = 0; k < s->ns; ++k) {
        const float* sh = m->shapes + (size_t)k * MG_SHAPE_STRIDE;
        const int t = (int)sh[0];
        if (t < MG_SHAPE_SPHERE || t > MG_SHAPE_CONVEX) return fail(MG_ERR_ARG, "shape %d: unknown type %d", k, t);
        if (t != MG_SHAPE_CONVEX) continue;
        const long off = (long)sh[2], nh = m->hulls ? m->num_hull_floats : 0;
        if (off < 0 || off + MG_HULL_HEADER > nh) return fail(MG_ERR_ARG, "shape %d: hull offset %ld out of range", k, off);
        const int nv = (int)m->hulls[off], nfc = (int)m->hulls[off + 1], ned = (int)m->hulls[off + 2];
        if (nv < 4 || nv > MG_HULL_MAX_VERTS || nfc < 4 || nfc > MG_HULL_MAX_FACES || ned < 0 ||
            ned > 3 * MG_HULL_MAX_VERTS || off + MG_HULL_HEADER + 3L * nv + 4L * nfc + 2L * ned > nh)
            return fail(MG_ERR_ARG, "shape %d: bad hull record (%d vertices, %d faces, %d edges)", k, nv, nfc, ned);
        for (int e = 0; e < 2 * ned; ++e) {
            const float vi = m->hulls[off + MG_HULL_HEADER + 3L * nv + 4L * nfc + e];
            if (!(vi >= 0.0f && vi < (float)nv)) return fail(MG_ERR_ARG, "shape %d: hull edge vertex out of range", k);
        }
    }
    for (int a = 0; a < na; ++a) {
        if (m->actor_root_body[a] < 0 || m->actor_root_body[a] >= nb) return fail(MG_ERR_ARG, "actor %d: bad root", a);
        if (m->actor_dof[a] > m->actor_dof[a + 1]) return fail(MG_ERR_ARG, "actor_dof not monotone");
        s->max_actor_dofs = std::max(s->max_actor_dofs, m->actor_dof[a + 1] - m->actor_dof[a]);
    }
    if (na > 0 && (m->actor_dof[0] != 0 || m->actor_dof[na] != nd)) return fail(MG_ERR_ARG, "actor_dof must span [0, num_dofs]");

    // ---- coupled envs: envs where two bodies may touch (actor_coll rule, see
    // migym.h) step in the per-env kernel; everything else in the free-body /
    // articulation kernels
    std::vector<char> coupled_body(nb, 0);           // free roots / articulation roots of coupled envs
    std::vector<std::array<int, MG_ENV_I_N>> env_rows;   // global body ids, converted below
    std::vector<int> env_tmpl;
    std::vector<int> pairs;                              // [..][4] shape pairs of the coupled envs
    // pile envs (mg_pile.hip): rows with global body ids (converted below),
    // the free bodies, their candidate pairs
    std::vector<std::array<int, MG_PILE_I_N>> pile_rows;
    std::vector<int> pile_body, pile_slots;
    std::vector<unsigned> pile_pairs;
    // envs built alike (the same shapes, filters and order) share one slot table
    // and pair list: 4096 pyramids read one 2 KB list through L2
    std::map<std::pair<std::vector<int>, std::vector<unsigned>>, std::pair<int, int>> pile_list_at;
    if (m->actor_coll && na > 0) {
        for (int a = 0; a + 1 < na; ++a)
            if (m->actor_root_body[a + 1] <= m->actor_root_body[a])
                return fail(MG_ERR_ARG, "actor_coll needs actors in body order");
        std::vector<int> artic_of_root(nb, -1);
        for (int k = 0; k < m->num_artics; ++k) {
            const int r0 = m->artic_i[(size_t)k * MG_ARTIC_I_N + 0];
            if (r0 < 0 || r0 >= nb) return fail(MG_ERR_ARG, "articulation %d: bad first body", k);
            artic_of_root[r0] = k;
        }
        const int ne = m->num_envs;
        std::vector<std::vector<int>> env_actors(ne > 0 ? ne : 0);
        for (int a = 0; a < na; ++a) {
            const int e = m->actor_coll[(size_t)a * MG_ACOLL_N + 0];
            if (e < 0 || e >= ne) return fail(MG_ERR_ARG, "actor %d: env %d out of range", a, e);
            env_actors[e].push_back(a);
        }
        auto collide = [m](int a, int b) {
            const int ga = m->actor_coll[(size_t)a * MG_ACOLL_N + 1], gb = m->actor_coll[(size_t)b * MG_ACOLL_N + 1];
            const int fa = m->actor_coll[(size_t)a * MG_ACOLL_N + 2], fb = m->actor_coll[(size_t)b * MG_ACOLL_N + 2];
            return (ga == gb || ga == -1 || gb == -1) && (fa & fb) == 0;
        };
        for (int e = 0; e < ne; ++e) {
            std::vector<int> art, fr, stc;
            for (int a : env_actors[e]) {
                const int r0 = m->actor_root_body[a];
                const int kind = m->body_kind[r0];
                if (kind == MG_BODY_LINK) art.push_back(a);
                else if (kind == MG_BODY_FREE) fr.push_back(a);
                else stc.push_back(a);
            }
            bool coupled = false;
            for (size_t i = 0; i < fr.size(); ++i) {
                for (int t : stc) coupled = coupled || collide(fr[i], t);
                for (size_t j = i + 1; j < fr.size(); ++j) coupled = coupled || collide(fr[i], fr[j]);
            }
            for (int a : art) {
                for (int t : stc) coupled = coupled || collide(a, t);
                for (int f : fr) coupled = coupled || collide(a, f);
                // a floating-base articulation always steps here (ground contacts,
                // the root's own dynamics)
                const int k = artic_of_root[m->actor_root_body[a]];
                if (k >= 0 && !m->artic_tmpl_i[m->artic_i[(size_t)k * MG_ARTIC_I_N + 2] * MG_ATMPL_I_N + 3])
                    coupled = true;
            }
            if (!coupled) continue;
            if (art.empty() && fr.size() > MG_ENV_MAXF) {
                // a pile (mg_pile.hip): lane k = free body k; pairs
                // per free body k and shape of k: the ground, the static bodies it
                // may touch, the later free bodies it may touch
                if (fr.size() > MG_PILE_MAXB || stc.size() > MG_ENV_MAXS)
                    return fail(MG_ERR_UNSUPPORTED,
                                "env %d: %zu free / %zu static bodies in contact range; a pile env supports %d / %d",
                                e, fr.size(), stc.size(), MG_PILE_MAXB, MG_ENV_MAXS);
                std::array<int, MG_PILE_I_N> row;
                row.fill(0);
                row[0] = (int)pile_body.size();
                row[1] = (int)fr.size();
                row[4] = (int)stc.size();
                for (size_t t = 0; t < stc.size(); ++t) row[5 + t] = m->actor_root_body[stc[t]];
                for (int f : fr) {
                    pile_body.push_back(m->actor_root_body[f]);
                    coupled_body[m->actor_root_body[f]] = 1;
                }
                const bool ground = s->params.has_ground != 0;
                auto shp = [m](int b, int* s0, int* ns) {
                    const int* t = m->tmpl_body_i + (size_t)m->body_tmpl[b] * MG_TBODY_I_N;
                    *s0 = t[0];
                    *ns = t[1];
                };
                // local shape slots: the free bodies' shapes in body order, then the statics'
                std::vector<int> slots;
                std::vector<int> first_slot(fr.size() + stc.size());
                for (size_t k = 0; k < fr.size() + stc.size(); ++k) {
                    const bool st = k >= fr.size();
                    int sb0, nsb;
                    shp(m->actor_root_body[st ? stc[k - fr.size()] : fr[k]], &sb0, &nsb);
                    first_slot[k] = (int)slots.size() / 2;
                    for (int sb = sb0; sb < sb0 + nsb; ++sb) {
                        slots.push_back(st ? MG_PILE_ST0 + (int)(k - fr.size()) : (int)k);
                        slots.push_back(sb);
                    }
                }
                if ((int)slots.size() / 2 > MG_PILE_MAXSH)
                    return fail(MG_ERR_UNSUPPORTED, "env %d: %zu collision shapes; a pile env supports %d", e,
                                slots.size() / 2, MG_PILE_MAXSH);
                std::vector<unsigned> plist;
                for (int k = 0; k < (int)fr.size(); ++k) {
                    int sa0, nsa;
                    shp(m->actor_root_body[fr[k]], &sa0, &nsa);
                    for (int sa = sa0; sa < sa0 + nsa; ++sa) {
                        const unsigned la = (unsigned)(first_slot[k] + (sa - sa0));
                        auto push = [&](int owner, int sb, int sb0) {
                            plist.push_back(la | (unsigned)(first_slot[owner] + (sb - sb0)) << 8);
                        };
                        if (ground) plist.push_back(la | (unsigned)MG_PILE_GROUND << 8);
                        for (int t = 0; t < (int)stc.size(); ++t) {
                            if (!collide(fr[k], stc[t])) continue;
                            int sb0, nsb;
                            shp(m->actor_root_body[stc[t]], &sb0, &nsb);
                            for (int sb = sb0; sb < sb0 + nsb; ++sb) push((int)fr.size() + t, sb, sb0);
                        }
                        for (int j = k + 1; j < (int)fr.size(); ++j) {
                            if (!collide(fr[k], fr[j])) continue;
                            int sb0, nsb;
                            shp(m->actor_root_body[fr[j]], &sb0, &nsb);
                            for (int sb = sb0; sb < sb0 + nsb; ++sb) push(j, sb, sb0);
                        }
                    }
                }
                row[3] = (int)plist.size();
                row[10] = (int)slots.size() / 2;
                if (row[3] > MG_PILE_MAXPAIRS)
                    return fail(MG_ERR_UNSUPPORTED, "env %d: %d candidate shape pairs; a pile env supports %d", e,
                                row[3], MG_PILE_MAXPAIRS);
                auto key = std::make_pair(slots, plist);
                auto it = pile_list_at.find(key);
                if (it != pile_list_at.end()) {
                    row[2] = it->second.first;
                    row[9] = it->second.second;
                } else {
                    row[2] = (int)pile_pairs.size();
                    row[9] = (int)pile_slots.size() / 2;
                    pile_list_at.emplace(std::move(key), std::make_pair(row[2], row[9]));
                    pile_pairs.insert(pile_pairs.end(), plist.begin(), plist.end());
                    pile_slots.insert(pile_slots.end(), slots.begin(), slots.end());
                }
                pile_rows.push_back(row);
                continue;
            }
            if (art.size() > 1 || fr.size() > MG_ENV_MAXF || stc.size() > MG_ENV_MAXS)
                return fail(MG_ERR_UNSUPPORTED,
                            "env %d: %zu articulations / %zu free / %zu static bodies in contact range; the "
                            "coupled step supports 1 / %d / %d", e, art.size(), fr.size(), stc.size(),
                            MG_ENV_MAXF, MG_ENV_MAXS);
            int art_nl = 0, art_nd = 0, art_fb = 0, art_fl = 0;
            if (!art.empty()) {
                const int k = artic_of_root[m->actor_root_body[art[0]]];
                const int t = k >= 0 ? m->artic_i[(size_t)k * MG_ARTIC_I_N + 2] : -1;
                if (t < 0 || t >= m->num_artic_tmpls) return fail(MG_ERR_ARG, "env %d: bad articulation", e);
                art_nl = m->artic_tmpl_i[t * MG_ATMPL_I_N + 1];
                art_nd = m->artic_tmpl_i[t * MG_ATMPL_I_N + 2];
                art_fb = m->artic_tmpl_i[t * MG_ATMPL_I_N + 3] ? 0 : 1;
                const int fl = m->artic_tmpl_i[t * MG_ATMPL_I_N + 0];
                if (fl < 0 || art_nl < 1 || fl + art_nl > m->num_tmpl_links)
                    return fail(MG_ERR_ARG, "env %d: bad articulation template %d", e, t);
                art_fl = fl;
            }
            if (art_nd + 6 * art_fb + 6 * (int)fr.size() > MG_ENV_SLOTS_WIDE || art_nl > MG_MAX_LINKS)
                return fail(MG_ERR_UNSUPPORTED, "env %d: %d links, %d DOFs%s + %zu free bodies exceed the %d links / %d "
                            "velocity slots of the coupled step", e, art_nl, art_nd, art_fb ? " + a floating base" : "",
                            fr.size(), MG_MAX_LINKS, MG_ENV_SLOTS_WIDE);
            std::array<int, MG_ENV_I_N> row;
            row.fill(0);
            row[0] = -1;
            int tmpl = -1;
            if (!art.empty()) {
                const int r0 = m->actor_root_body[art[0]];
                const int k = artic_of_root[r0];
                if (k < 0) return fail(MG_ERR_ARG, "env %d: articulated actor without articulation record", e);
                row[0] = r0;
                row[1] = m->artic_i[(size_t)k * MG_ARTIC_I_N + 1];
                tmpl = m->artic_i[(size_t)k * MG_ARTIC_I_N + 2];
                coupled_body[r0] = 1;
            }
            row[2] = (int)fr.size();
            for (size_t i = 0; i < fr.size(); ++i) {
                row[3 + i] = m->actor_root_body[fr[i]];
                coupled_body[row[3 + i]] = 1;
            }
            row[7] = (int)stc.size();
            for (size_t i = 0; i < stc.size(); ++i) row[8 + i] = m->actor_root_body[stc[i]];
            int mask = 0;
            static const int pair_bit[4][4] = {{-1, 0, 1, 2}, {-1, -1, 3, 4}, {-1, -1, -1, 5}, {-1, -1, -1, -1}};
            for (size_t i = 0; i < fr.size(); ++i) {
                if (!art.empty() && collide(art[0], fr[i])) mask |= 1 << i;
                for (size_t j = i + 1; j < fr.size(); ++j)
                    if (collide(fr[i], fr[j])) mask |= 1 << (8 + pair_bit[i][j]);
                for (size_t t = 0; t < stc.size(); ++t)
                    if (collide(fr[i], stc[t])) mask |= 1 << (14 + 4 * i + t);
            }
            for (size_t t = 0; t < stc.size(); ++t)
                if (!art.empty() && collide(art[0], stc[t])) mask |= 1 << (4 + t);
            row[12] = mask;
            row[13] = tmpl;
            // candidate shape pairs, in the order the step solves them
            auto shp = [m](int b, int* s0, int* ns) {
                const int* t = m->tmpl_body_i + (size_t)m->body_tmpl[b] * MG_TBODY_I_N;
                *s0 = t[0];
                *ns = t[1];
            };
            auto push = [&pairs](int a, int sa, int b, int sb) {
                pairs.push_back(a); pairs.push_back(sa); pairs.push_back(b); pairs.push_back(sb);
            };
            static const int pbit[4][4] = {{-1, 0, 1, 2}, {-1, -1, 3, 4}, {-1, -1, -1, 5}, {-1, -1, -1, -1}};
            const bool ground = s->params.has_ground != 0;
            row[14] = (int)(pairs.size() / 4);
            for (int k = 0; k < (int)fr.size(); ++k) {
                int sa0, nsa;
                shp(row[3 + k], &sa0, &nsa);
                for (int sa = sa0; sa < sa0 + nsa; ++sa) {
                    if (ground) push(MG_ENV_FREE0 + k, sa, -1, -1);
                    for (int t = 0; t < (int)stc.size(); ++t) {
                        if (!((mask >> (14 + 4 * k + t)) & 1)) continue;
                        int sb0, nsb;
                        shp(row[8 + t], &sb0, &nsb);
                        for (int sb = sb0; sb < sb0 + nsb; ++sb) push(MG_ENV_FREE0 + k, sa, MG_ENV_STATIC0 + t, sb);
                    }
                    for (int j = k + 1; j < (int)fr.size(); ++j) {
                        if (!((mask >> (8 + pbit[k][j])) & 1)) continue;
                        int sb0, nsb;
                        shp(row[3 + j], &sb0, &nsb);
                        for (int sb = sb0; sb < sb0 + nsb; ++sb) push(MG_ENV_FREE0 + k, sa, MG_ENV_FREE0 + j, sb);
                    }
                    if (row[0] >= 0 && !art_fb && ((mask >> k) & 1)) {   // the fixed base (static)
                        int sb0, nsb;
                        shp(row[0], &sb0, &nsb);
                        for (int sb = sb0; sb < sb0 + nsb; ++sb) push(MG_ENV_FREE0 + k, sa, 0, sb);
                    }
                }
            }
            for (int l = art_fb ? 0 : 1; l < art_nl; ++l) {     // moving links (a floating base moves)
                // the link's body (virtual links of ball / multi-axis joints: none)
                const int bl = m->tmpl_link_i[(size_t)(art_fl + l) * MG_LINK_I_N + 3];
                if (bl < 0) continue;
                int sa0, nsa;
                shp(row[0] + bl, &sa0, &nsa);
                for (int sa = sa0; sa < sa0 + nsa; ++sa) {
                    if (ground) push(l, sa, -1, -1);
                    for (int t = 0; t < (int)stc.size(); ++t) {
                        if (!((mask >> (4 + t)) & 1)) continue;
                        int sb0, nsb;
                        shp(row[8 + t], &sb0, &nsb);
                        for (int sb = sb0; sb < sb0 + nsb; ++sb) push(l, sa, MG_ENV_STATIC0 + t, sb);
                    }
                    for (int k = 0; k < (int)fr.size(); ++k) {
                        if (!((mask >> k) & 1)) continue;
                        int sb0, nsb;
                        shp(row[3 + k], &sb0, &nsb);
                        for (int sb = sb0; sb < sb0 + nsb; ++sb) push(l, sa, MG_ENV_FREE0 + k, sb);
                    }
                }
            }
            row[15] = (int)(pairs.size() / 4) - row[14];
            env_rows.push_back(row);
            env_tmpl.push_back(tmpl);
        }
    }

    // free bodies ordered by template body (stable): bodies of one kind share
    // waves, so e.g. the servo scene's airborne UAVs and grounded vehicles do
    // not interleave lane by lane (results do not depend on the order).
    // Templates whose instances start farthest from the ground plane come
    // first: a launch larger than one resident round dispatches the array back
    // to front (mg_launch_rigid_step), i.e. the likely-in-contact (long) waves
    // first and the airborne (short) ones last, filling the last round's tail.
    // Free bodies of coupled envs come last (the per-env kernel reads them).
    std::vector<int> free_ids, free_cpl;
    for (int b = 0; b < nb; ++b)
        if (m->body_kind[b] == MG_BODY_FREE) (coupled_body[b] ? free_cpl : free_ids).push_back(b);
    auto nshapes = [m](int b) { return m->tmpl_body_i[m->body_tmpl[b] * MG_TBODY_I_N + 1]; };
    std::vector<double> clear_sum(m->num_tmpl_bodies, 0.0);
    std::vector<int> clear_n(m->num_tmpl_bodies, 0);
    {
        const mg_sim_params& p = s->params;
        float gn[3] = {0.0f, 0.0f, 0.0f};
        float gd = 0.0f;
        if (p.has_ground) {
            for (int k = 0; k < 3; ++k) gn[k] = p.ground_normal[k];
            gd = p.ground_distance;
        } else {
            gn[p.up_axis == 0 ? 1 : 2] = 1.0f;
        }
        for (int b : free_ids) {
            const float* x = m->body_state0 + (size_t)b * MG_STATE_N;
            clear_sum[m->body_tmpl[b]] += (double)gn[0] * x[0] + (double)gn[1] * x[1] + (double)gn[2] * x[2] + gd;
            clear_n[m->body_tmpl[b]] += 1;
        }
    }
    auto clearance = [&](int t) { return clear_n[t] ? clear_sum[t] / clear_n[t] : 0.0; };
    std::stable_sort(free_ids.begin(), free_ids.end(), [&](int a, int b) {
        const bool ma = nshapes(a) > 1, mb = nshapes(b) > 1;   // single-shape bodies first
        if (ma != mb) return !ma;
        const int ta = m->body_tmpl[a], tb = m->body_tmpl[b];
        if (ta == tb) return false;
        const double ca = clearance(ta), cb = clearance(tb);
        if (ca != cb) return ca > cb;
        return ta < tb;
    });
    s->nf1 = 0;
    for (int b : free_ids) s->nf1 += nshapes(b) <= 1 ? 1 : 0;
    s->nf_rigid = (int)free_ids.size();
    free_ids.insert(free_ids.end(), free_cpl.begin(), free_cpl.end());
    s->nf = (int)free_ids.size();

    // internal storage order: free bodies (as above), articulation links
    // (instance by instance, template by template), everything else
    std::vector<int> order(free_ids), perm(nb, -1);
    std::vector<char> placed(nb, 0);
    for (int b : free_ids) placed[b] = 1;

    // articulation instances grouped by template
    s->groups.clear();
    std::vector<int> artic_sorted, artic_step;
    for (int t = 0; t < m->num_artic_tmpls; ++t) {
        ArticGroup g;
        g.tmpl = t;
        g.first_link = m->artic_tmpl_i[t * MG_ATMPL_I_N + 0];
        g.nl = m->artic_tmpl_i[t * MG_ATMPL_I_N + 1];
        g.ndof = m->artic_tmpl_i[t * MG_ATMPL_I_N + 2];
        g.fixed_base = m->artic_tmpl_i[t * MG_ATMPL_I_N + 3];
        if (g.nl < 1 || g.nl > MG_MAX_LINKS || g.ndof > g.nl || g.ndof > MG_MAX_DOFS || g.first_link < 0 ||
            g.first_link + g.nl > s->ntl)
            return fail(MG_ERR_UNSUPPORTED, "articulation template %d: %d links / %d dofs unsupported", t, g.nl, g.ndof);
        g.nbody = 0;
        for (int l = 0; l < g.nl; ++l) {
            const int* li = m->tmpl_link_i + (size_t)(g.first_link + l) * MG_LINK_I_N;
            if (li[0] >= l || (l > 0 && li[0] < 0) || (l == 0 && li[0] != -1))
                return fail(MG_ERR_ARG, "articulation template %d: links not in topological order", t);
            if (li[2] >= g.ndof) return fail(MG_ERR_ARG, "articulation template %d: bad dof index", t);
            // real links carry bodies 0, 1, 2, ... in link order; virtual links
            // (the first two of a ball joint) are revolute with a DOF and no body
            if (li[3] >= 0) {
                if (li[3] != g.nbody) return fail(MG_ERR_ARG, "articulation template %d: link bodies out of order", t);
                g.nbody++;
            } else if (l == 0 || li[1] != MG_JOINT_REVOLUTE || li[2] < 0) {
                return fail(MG_ERR_ARG, "articulation template %d: bad virtual link %d", t, l);
            }
        }
        g.chain = g.fixed_base && g.ndof == g.nl - 1 && g.nbody == g.nl;
        for (int l = 1; l < g.nl && g.chain; ++l) {
            const int* li = m->tmpl_link_i + (size_t)(g.first_link + l) * MG_LINK_I_N;
            g.chain = li[0] == l - 1 && li[2] == l - 1 && (li[1] == MG_JOINT_REVOLUTE || li[1] == MG_JOINT_PRISMATIC);
        }
        g.offset = (int)artic_sorted.size() / MG_ARTIC_I_N;
        g.count = 0;
        g.step_offset = (int)artic_step.size() / MG_ARTIC_I_N;
        g.step_count = 0;
        // Link stride (row field 3): link l of an instance is body first + l * stride.
        // Instances that step in k_artic_chain (one lane per articulation) are laid
        // out link-major in blocks of 64, the kernel's wavefront: link l of the
        // block's instances are 64 consecutive slots, so every per-link load and
        // store of a wave is one contiguous 256-B access (link-contiguous storage
        // strides the lanes nl * 4 B apart). Everything else: stride 1.
        const bool blocked = g.chain && g.nl >= 2 && g.nl <= 4;
        std::vector<int> blk_k, blk_sorted, blk_step;
        for (int k = 0; k < m->num_artics; ++k) {
            const int* ai = m->artic_i + (size_t)k * MG_ARTIC_I_N;
            if (ai[2] != t) continue;
            if (ai[0] < 0 || ai[0] + g.nbody > nb || ai[1] < 0 || ai[1] + g.ndof > nd)
                return fail(MG_ERR_ARG, "articulation %d out of range", k);
            const bool cpl = coupled_body[ai[0]] != 0;
            const bool blk = blocked && !cpl;
            if (blk) {
                blk_k.push_back(k);
                blk_sorted.push_back((int)artic_sorted.size());
                blk_step.push_back((int)artic_step.size());
            }
            for (int j = 0; j < MG_ARTIC_I_N; ++j) artic_sorted.push_back(j == 3 ? 1 : ai[j]);
            if (!cpl) {
                for (int j = 0; j < MG_ARTIC_I_N; ++j) artic_step.push_back(j == 3 ? 1 : ai[j]);
                g.step_count++;
                g.step_body0.push_back(ai[0]);
                g.step_dof0.push_back(ai[1]);
            }
            for (int l = 0; l < g.nbody; ++l) {
                if (placed[ai[0] + l]) return fail(MG_ERR_ARG, "articulation %d overlaps another body", k);
                placed[ai[0] + l] = 1;
                if (!blk) order.push_back(ai[0] + l);
            }
            g.count++;
        }
        for (size_t i0 = 0; i0 < blk_k.size(); i0 += 64) {
            const int cnt = (int)std::min<size_t>(64, blk_k.size() - i0);
            for (int l = 0; l < g.nbody; ++l)
                for (int j = 0; j < cnt; ++j) order.push_back(m->artic_i[(size_t)blk_k[i0 + j] * MG_ARTIC_I_N] + l);
            for (int j = 0; j < cnt; ++j) {
                artic_sorted[blk_sorted[i0 + j] + 3] = cnt;
                artic_step[blk_step[i0 + j] + 3] = cnt;
            }
        }
        if (!g.fixed_base && g.step_count > 0)
            return fail(MG_ERR_UNSUPPORTED, "articulation template %d: a floating base steps in the coupled "
                        "per-env kernel, which needs actor_coll", t);
        if (blocked && g.step_count > 0) chain_uni_mass(m, g);
        s->groups.push_back(g);
    }

    for (int b = 0; b < nb; ++b)
        if (!placed[b]) order.push_back(b);
    for (int i = 0; i < nb; ++i) perm[order[i]] = i;
    for (size_t k = 0; k < artic_sorted.size(); k += MG_ARTIC_I_N) artic_sorted[k] = perm[artic_sorted[k]];
    for (size_t k = 0; k < artic_step.size(); k += MG_ARTIC_I_N) artic_step[k] = perm[artic_step[k]];
    // chain groups whose stepped rows follow the blocked layout from one base
    // slot and one DOF stride: the kernel computes them (MgArticArgs::aff)
    for (ArticGroup& g : s->groups) {
        g.aff = 0;
        if (!(g.chain && g.nl >= 2 && g.nl <= 4) || g.step_count == 0) continue;
        const int* r0 = artic_step.data() + (size_t)g.step_offset * MG_ARTIC_I_N;
        const int B = r0[0], D = r0[1];
        const int DS = g.step_count > 1 ? r0[MG_ARTIC_I_N + 1] - D : 0;
        bool ok = true;
        for (int k = 0; k < g.step_count && ok; ++k) {
            const int* r = r0 + (size_t)k * MG_ARTIC_I_N;
            const int blk = k / 64, j = k % 64, cnt = std::min(64, g.step_count - blk * 64);
            ok = r[0] == B + blk * 64 * g.nbody + j && r[3] == cnt && r[1] == D + k * DS;
        }
        if (ok) { g.aff = 1; g.aff_b0 = B; g.aff_d0 = D; g.aff_ds = DS; }
    }
    // coupled env rows: internal slots, grouped by articulation template (-1 first)
    std::vector<int> env_flat;
    s->env_groups.clear();
    s->cenv_ctab_off.assign(env_rows.size(), -1);
    s->cenv_ctab_n.assign(env_rows.size(), 0);
    // (and by lane width: an env of more than 16 links or velocity slots runs
    // 64 lanes wide, mg_env.hip; the oracle decides per env the same way)
    for (int t = -1; t < m->num_artic_tmpls; ++t)
    for (int wide = 0; wide < 2; ++wide) {
        EnvGroup g{};
        g.tmpl = t;
        g.wide = wide;
        if (t >= 0) {
            g.first_link = m->artic_tmpl_i[t * MG_ATMPL_I_N + 0];
            g.nl = m->artic_tmpl_i[t * MG_ATMPL_I_N + 1];
            g.ndof = m->artic_tmpl_i[t * MG_ATMPL_I_N + 2];
            g.floating = m->artic_tmpl_i[t * MG_ATMPL_I_N + 3] ? 0 : 1;
        }
        g.offset = (int)env_flat.size() / MG_ENV_I_N;
        for (size_t r = 0; r < env_rows.size(); ++r) {
            if (env_tmpl[r] != t) continue;
            const int slots = (t >= 0 ? g.ndof + 6 * g.floating : 0) + 6 * env_rows[r][2];
            if ((g.nl > 16 || slots > 16) != (wide != 0)) continue;
            std::array<int, MG_ENV_I_N> row = env_rows[r];
            g.max_free = std::max(g.max_free, row[2]);
            if (row[0] >= 0) row[0] = perm[row[0]];
            for (int i = 0; i < row[2]; ++i) row[3 + i] = perm[row[3 + i]];
            for (int i = 0; i < row[7]; ++i) row[8 + i] = perm[row[8 + i]];
            env_flat.insert(env_flat.end(), row.begin(), row.end());
            // k_env_np writes env j of the group at the group's base + j records
            s->cenv_ctab_off[r] = (long long)g.offset * mg_env_ctab_floats() +
                                  (long long)g.count * mg_env_ctab_record_floats(wide);
            s->cenv_ctab_n[r] = mg_env_ctab_record_floats(wide);
            g.count++;
        }
        if (g.count > 0) s->env_groups.push_back(g);
    }
    s->n_coupled = (int)env_rows.size();
    s->n_pile = (int)pile_rows.size();
    for (auto& r : pile_rows)
        for (int t = 0; t < r[4]; ++t) r[5 + t] = perm[r[5 + t]];
    for (int& b : pile_body) b = perm[b];
    std::vector<int> root_int(na), tmpl_int(nb);
    for (int a = 0; a < na; ++a) root_int[a] = perm[m->actor_root_body[a]];
    for (int i = 0; i < nb; ++i) tmpl_int[i] = m->body_tmpl[order[i]];
    std::vector<float> st0((size_t)nb * MG_STATE_N), ms0((size_t)nb * MG_MASS_N);
    for (int i = 0; i < nb; ++i) {
        std::memcpy(&st0[(size_t)i * MG_STATE_N], m->body_state0 + (size_t)order[i] * MG_STATE_N, MG_STATE_N * sizeof(float));
        std::memcpy(&ms0[(size_t)i * MG_MASS_N], m->body_mass + (size_t)order[i] * MG_MASS_N, MG_MASS_N * sizeof(float));
    }

    // device buffers
    HIP_TRY(dalloc(&s->d_state, (size_t)nb * MG_STATE_N));
    HIP_TRY(dalloc(&s->d_mass, (size_t)nb * MG_MASS_N));
    HIP_TRY(dalloc(&s->d_body_tmpl, nb));
    HIP_TRY(dalloc(&s->d_free_global, s->nf));
    HIP_TRY(dalloc(&s->d_perm, nb));
    HIP_TRY(dalloc(&s->d_tbf, (size_t)s->ntb * MG_TBODY_F_N));
    HIP_TRY(dalloc(&s->d_tbi, (size_t)s->ntb * MG_TBODY_I_N));
    HIP_TRY(dalloc(&s->d_trec, (size_t)s->ntb * MG_TREC_N));
    HIP_TRY(dalloc(&s->d_shapes, (size_t)s->ns * MG_SHAPE_STRIDE));
    HIP_TRY(dalloc(&s->d_hulls, (size_t)(m->hulls ? m->num_hull_floats : 0)));
    s->nhull_floats = m->hulls ? m->num_hull_floats : 0;
    HIP_TRY(dalloc(&s->d_actor_root, na));
    HIP_TRY(dalloc(&s->d_actor_dof, na + 1));
    HIP_TRY(dalloc(&s->d_cforce, (size_t)nb * 3));
    HIP_TRY(dalloc(&s->d_ext, (size_t)nb * 6));
    HIP_TRY(dalloc(&s->d_dof, (size_t)nd * 2));
    HIP_TRY(dalloc(&s->d_dof_tgt, (size_t)nd * 3));
    HIP_TRY(dalloc(&s->d_dof_props, (size_t)nd * MG_DOFPROP_N));
    HIP_TRY(dalloc(&s->d_artic, artic_sorted.size()));
    HIP_TRY(dalloc(&s->d_artic_step, artic_step.size()));
    HIP_TRY(dalloc(&s->d_env, env_flat.size()));
    HIP_TRY(dalloc(&s->d_pairs, pairs.size()));
    HIP_TRY(dalloc(&s->d_link_f, (size_t)s->ntl * MG_LINK_F_N));
    HIP_TRY(dalloc(&s->d_link_i, (size_t)s->ntl * MG_LINK_I_N));

    auto h2d = [](void* d, const void* h, size_t bytes) -> hipError_t {
        if (bytes == 0 || !h) return hipSuccess;
        return hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    };
    std::vector<float> st = to_soa(st0.data(), nb, MG_STATE_N);
    std::vector<float> ms = to_soa(ms0.data(), nb, MG_MASS_N);
    HIP_TRY(h2d(s->d_state, st.data(), st.size() * sizeof(float)));
    HIP_TRY(h2d(s->d_mass, ms.data(), ms.size() * sizeof(float)));
    HIP_TRY(h2d(s->d_body_tmpl, tmpl_int.data(), (size_t)nb * sizeof(int)));
    HIP_TRY(h2d(s->d_free_global, free_ids.data(), free_ids.size() * sizeof(int)));
    HIP_TRY(h2d(s->d_perm, perm.data(), (size_t)nb * sizeof(int)));
    HIP_TRY(h2d(s->d_tbf, m->tmpl_body_f, (size_t)s->ntb * MG_TBODY_F_N * sizeof(float)));
    HIP_TRY(h2d(s->d_tbi, m->tmpl_body_i, (size_t)s->ntb * MG_TBODY_I_N * sizeof(int)));
    {
        // compact template records of the single-shape kernel: template floats,
        // then the first shape record (type -1: no shape)
        std::vector<float> trec((size_t)s->ntb * MG_TREC_N, 0.0f);
        for (int t = 0; t < s->ntb; ++t) {
            float* r = &trec[(size_t)t * MG_TREC_N];
            std::memcpy(r, m->tmpl_body_f + (size_t)t * MG_TBODY_F_N, MG_TBODY_F_N * sizeof(float));
            const int s0 = m->tmpl_body_i[t * MG_TBODY_I_N + 0], sc = m->tmpl_body_i[t * MG_TBODY_I_N + 1];
            if (sc > 0) {
                const float* sr = m->shapes + (size_t)s0 * MG_SHAPE_STRIDE;
                std::memcpy(r + MG_TBODY_F_N, sr, MG_SHAPE_STRIDE * sizeof(float));
                // pad[0] of the copy: bounding radius of the shape about the body
                // origin (k_rigid_step1 skips the candidates of a wave whose bodies
                // all clear the ground by more than it); -1: unknown, never skipped
                double ext = -1.0;
                switch ((int)sr[0]) {
                    case MG_SHAPE_SPHERE: ext = sr[1]; break;
                    case MG_SHAPE_BOX: ext = std::sqrt((double)sr[1] * sr[1] + (double)sr[2] * sr[2] + (double)sr[3] * sr[3]); break;
                    case MG_SHAPE_CAPSULE: ext = (double)sr[1] + sr[2]; break;
                    case MG_SHAPE_CONVEX: ext = sr[1]; break;
                    default: break;
                }
                const double po = std::sqrt((double)sr[4] * sr[4] + (double)sr[5] * sr[5] + (double)sr[6] * sr[6]);
                r[MG_TBODY_F_N + 13] = (ext >= 0.0 && std::isfinite(ext + po)) ? (float)((ext + po) * (1.0 + 1e-6)) : -1.0f;
            } else {
                r[MG_TBODY_F_N] = -1.0f;
            }
        }
        // one mass row per template when all its free bodies share it (the kernel
        // then reads it from the record instead of 44 B per body)
        std::vector<int> seen(s->ntb, 0), uniform(s->ntb, 1);
        for (int b = 0; b < nb; ++b) {
            if (m->body_kind[b] != MG_BODY_FREE) continue;
            const int t = m->body_tmpl[b];
            const float* mr = m->body_mass + (size_t)b * MG_MASS_N;
            float* r = &trec[(size_t)t * MG_TREC_N];
            if (!seen[t]) {
                std::memcpy(r + MG_TREC_MASS, mr, MG_MASS_N * sizeof(float));
                seen[t] = 1;
            } else if (std::memcmp(r + MG_TREC_MASS, mr, MG_MASS_N * sizeof(float)) != 0) {
                uniform[t] = 0;
            }
        }
        for (int t = 0; t < s->ntb; ++t) trec[(size_t)t * MG_TREC_N + 5] = seen[t] && uniform[t] ? 1.0f : 0.0f;
        HIP_TRY(h2d(s->d_trec, trec.data(), trec.size() * sizeof(float)));
    }
    HIP_TRY(h2d(s->d_shapes, m->shapes, (size_t)s->ns * MG_SHAPE_STRIDE * sizeof(float)));
    if (m->hulls) HIP_TRY(h2d(s->d_hulls, m->hulls, (size_t)m->num_hull_floats * sizeof(float)));
    {
        std::vector<float> obb((size_t)std::max(s->ns, 1) * MG_OBB_N, 0.0f);
        for (int k = 0; k < s->ns; ++k) shape_obb(m->shapes + (size_t)k * MG_SHAPE_STRIDE, m->hulls, &obb[(size_t)k * MG_OBB_N]);
        HIP_TRY(dalloc(&s->d_shape_obb, obb.size()));
        HIP_TRY(h2d(s->d_shape_obb, obb.data(), obb.size() * sizeof(float)));
    }
    HIP_TRY(h2d(s->d_actor_root, root_int.data(), (size_t)na * sizeof(int)));
    {
        std::vector<int> body_actor(nb, -1);
        for (int a = 0; a < na; ++a) body_actor[m->actor_root_body[a]] = a;
        HIP_TRY(dalloc(&s->d_body_actor, (size_t)std::max(nb, 1)));
        HIP_TRY(h2d(s->d_body_actor, body_actor.data(), (size_t)nb * sizeof(int)));
    }
    {
        // fusable root sets: every actor root is a single-shape free body of the
        // free-body kernel (internal slots 0..nf1-1), and that kernel steps all
        // free bodies (no multi-shape ones, no articulations, no coupled envs)
        std::vector<int> row(nb, -1);
        bool ok = s->nf1 == s->nf_rigid && s->nf_rigid == s->nf && s->nartic == 0 && s->n_coupled == 0 &&
                  s->n_pile == 0 && na > 0;
        for (int a = 0; a < na && ok; ++a) {
            const int slot = root_int[a];
            ok = slot >= 0 && slot < s->nf1 && row[slot] < 0;
            if (ok) row[slot] = a;
        }
        s->roots_free = ok;
        HIP_TRY(dalloc(&s->d_root_row, (size_t)std::max(nb, 1)));
        HIP_TRY(h2d(s->d_root_row, row.data(), (size_t)nb * sizeof(int)));
    }
    {
        // rows the step kernels write with the refresh fused into them
        // (MG_FUSE_STEP_OUT): internal slot -> rigid-body row / actor row
        std::vector<int> slot_actor(nb, -1);
        for (int a = 0; a < na; ++a) slot_actor[root_int[a]] = a;
        HIP_TRY(dalloc(&s->d_slot_global, (size_t)std::max(nb, 1)));
        HIP_TRY(h2d(s->d_slot_global, order.data(), (size_t)nb * sizeof(int)));
        HIP_TRY(dalloc(&s->d_slot_actor, (size_t)std::max(nb, 1)));
        HIP_TRY(h2d(s->d_slot_actor, slot_actor.data(), (size_t)nb * sizeof(int)));
        // chain groups whose fused-refresh rows are affine in the instance
        for (ArticGroup& g : s->groups) {
            g.out_aff = 0;
            if (!g.aff) continue;
            const int* r0 = artic_step.data() + (size_t)g.step_offset * MG_ARTIC_I_N;
            const int G0 = order[r0[0]], A0 = slot_actor[r0[0]];
            bool ok = A0 >= 0;
            for (int k = 0; k < g.step_count && ok; ++k) {
                const int* r = r0 + (size_t)k * MG_ARTIC_I_N;
                ok = slot_actor[r[0]] == A0 + k;
                for (int l = 0; l < g.nl && ok; ++l) ok = order[r[0] + l * r[3]] == G0 + k * g.nl + l;
            }
            if (ok) { g.out_aff = 1; g.out_g0 = G0; g.out_r0 = A0; }
        }
        long long covered = s->nf1 == s->nf_rigid && s->nf_rigid == s->nf ? s->nf1 : -1;
        for (const ArticGroup& g : s->groups) {
            if (covered < 0) break;
            if (g.count == 0) continue;
            if (!(g.chain && g.nl >= 2 && g.nl <= 4) || g.step_count != g.count) covered = -1;
            else covered += (long long)g.step_count * g.nbody;
        }
        s->step_out_ok = s->n_coupled == 0 && s->n_pile == 0 && nb > 0 && covered == nb;
    }
    HIP_TRY(h2d(s->d_actor_dof, m->actor_dof, (size_t)(na + 1) * sizeof(int)));
    HIP_TRY(hipMemset(s->d_cforce, 0, (size_t)nb * 3 * sizeof(float)));
    HIP_TRY(hipMemset(s->d_ext, 0, (size_t)nb * 6 * sizeof(float)));
    if (nd > 0) {
        std::vector<float> ds = to_soa(m->dof_state0, nd, 2);
        HIP_TRY(h2d(s->d_dof, ds.data(), ds.size() * sizeof(float)));
        HIP_TRY(hipMemset(s->d_dof_tgt, 0, (size_t)nd * 3 * sizeof(float)));
        std::vector<float> dp = to_soa(m->dof_props, nd, MG_DOFPROP_N);
        HIP_TRY(h2d(s->d_dof_props, dp.data(), dp.size() * sizeof(float)));
    }
    for (ArticGroup& g : s->groups)
        if (g.uni_mass) chain_uni_dof(m->dof_props, g);
    HIP_TRY(dalloc(&s->d_chain_uni, std::max<size_t>(s->groups.size(), 1) * MG_CHAIN_UNI_N));
    HIP_TRY(chain_uni_upload(s));
    HIP_TRY(h2d(s->d_artic, artic_sorted.data(), artic_sorted.size() * sizeof(int)));
    HIP_TRY(h2d(s->d_artic_step, artic_step.data(), artic_step.size() * sizeof(int)));
    HIP_TRY(h2d(s->d_env, env_flat.data(), env_flat.size() * sizeof(int)));
    HIP_TRY(h2d(s->d_pairs, pairs.data(), pairs.size() * sizeof(int)));
    if (s->n_pile > 0) {
        std::vector<int> flat;
        for (const auto& r : pile_rows) flat.insert(flat.end(), r.begin(), r.end());
        HIP_TRY(dalloc(&s->d_pile_i, flat.size()));
        HIP_TRY(h2d(s->d_pile_i, flat.data(), flat.size() * sizeof(int)));
        HIP_TRY(dalloc(&s->d_pile_body, pile_body.size()));
        HIP_TRY(h2d(s->d_pile_body, pile_body.data(), pile_body.size() * sizeof(int)));
        HIP_TRY(dalloc(&s->d_pile_pairs, std::max<size_t>(pile_pairs.size(), 1)));
        if (!pile_pairs.empty())
            HIP_TRY(h2d(s->d_pile_pairs, pile_pairs.data(), pile_pairs.size() * sizeof(unsigned)));
        HIP_TRY(dalloc(&s->d_pile_slots, std::max<size_t>(pile_slots.size(), 2)));
        if (!pile_slots.empty()) HIP_TRY(h2d(s->d_pile_slots, pile_slots.data(), pile_slots.size() * sizeof(int)));
    }
    {   // no friction patch yet: every pair starts without anchors
        const size_t np = std::max<size_t>(pairs.size() / 4, 1), nm = (size_t)std::max(s->n_coupled, 1) * MG_FP_W;
        HIP_TRY(dalloc(&s->d_fpatch, np * MG_FP_N));
        HIP_TRY(dalloc(&s->d_fp_mask, nm));
        HIP_TRY(hipMemset(s->d_fpatch, 0, np * MG_FP_N * sizeof(float)));
        HIP_TRY(hipMemset(s->d_fp_mask, 0, nm * sizeof(unsigned)));
        // the coupled step's per-env records between its launches (mg_env.hip)
        const size_t nc = (size_t)std::max(s->n_coupled, 1);
        HIP_TRY(dalloc(&s->d_env_carry, nc * mg_env_carry_floats()));
        HIP_TRY(dalloc(&s->d_env_ctab, nc * mg_env_ctab_floats()));
        const size_t ng = (size_t)std::max(s->nf1, 1) * MG_FP_N;   // no ground patch yet
        HIP_TRY(dalloc(&s->d_gpatch, ng));
        HIP_TRY(hipMemset(s->d_gpatch, 0, ng * sizeof(float)));
    }
    HIP_TRY(h2d(s->d_link_f, m->tmpl_link_f, (size_t)s->ntl * MG_LINK_F_N * sizeof(float)));
    HIP_TRY(h2d(s->d_link_i, m->tmpl_link_i, (size_t)s->ntl * MG_LINK_I_N * sizeof(int)));
    HIP_TRY(hipDeviceSynchronize());
    s->h_perm = perm;
    s->h_body_tmpl.assign(m->body_tmpl, m->body_tmpl + nb);
    s->h_tbi.assign(m->tmpl_body_i, m->tmpl_body_i + (size_t)s->ntb * MG_TBODY_I_N);
    s->uploaded = true;
    return MG_OK;
}

// the pending DOF target columns as the kernels' inputs, with write-through
static void fused_targets(mg_sim* s, const float*& tp, const float*& tv, const float*& tf, float*& wp, float*& wv,
                          float*& wf) {
    const float** in[3] = {&tp, &tv, &tf};
    float** out[3] = {&wp, &wv, &wf};
    for (int k = 0; k < 3; ++k) {
        *out[k] = nullptr;
        if (s->pend_tgt[k]) {
            *in[k] = s->pend_tgt[k];
            *out[k] = s->d_dof_tgt + (size_t)k * s->nd;
        }
    }
}

int32_t mg_simulate(mg_sim* s, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "simulate before the model was uploaded");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const MgStep P = make_step(s->params);
    {   // deferred sets of another capture (or of the eager stream while capturing):
        // applied here as ordinary launches, not read by this step's kernels
        const unsigned long long cid = capture_id(st);
        if (s->pend_root && s->pend_root_cap != cid)
            if (int rc_ = flush_root(s, st)) return rc_;
        for (int k = 0; k < 3; ++k)
            if (s->pend_tgt[k] && s->pend_tgt_cap[k] != cid)
                if (int rc_ = flush_tgt(s, k, st)) return rc_;
    }
    // Under HIP stream capture (a hipGraph of the tensor-API step) the launches
    // are recorded as graph nodes; the timing events are left out (they would
    // become fixed nodes of the graph) and fetch_results does not block.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(st, &cap));
    s->capturing = cap != hipStreamCaptureStatusNone;
    MgKernelTimer timer{};
    struct TimerScope {
        ~TimerScope() { mg_timer = nullptr; }
    } timer_scope;
    int slot = 0;
    const bool timed = s->timing && !s->capturing;
    if (timed) {
        slot = (int)(s->ring_n % mg_sim::kRing);
        s->ev_begin = s->ring_b[slot];
        s->ev_end = s->ring_e[slot];
        HIP_TRY(hipEventRecord(s->ev_begin, st));
        timer.start = s->kern_b[slot];
        timer.stop = s->kern_e[slot];
        timer.cap = mg_sim::kKern;
        mg_timer = &timer;
    }
    // the refresh fused into the step (MG_FUSE_STEP_OUT): every body's rows are
    // written by the kernel that steps it (s->step_out_ok), into the bound
    // tensors (each one optional)
    const unsigned long long step_cid = capture_id(st);
    const bool step_out = (s->fusion & MG_FUSE_STEP_OUT) && fuse_here(s, step_cid) && s->step_out_ok &&
                          (s->bind_root || s->bind_rb || s->bind_dof);
    // the CPU pipeline's output stage (mg_fetch_host_state): the same kernels
    // write into the library's own buffer, so no caller-visible tensor changes
    float* ho_base = s->ho_alias ? s->d_stage_alias : s->d_host_out;
    const bool host_out = !step_out && ho_base && s->step_out_ok && step_cid == 0;
    float* ho_root = host_out ? ho_base : nullptr;
    float* ho_rb = host_out ? ho_base + (size_t)s->na * MG_STATE_N : nullptr;
    float* ho_dof = host_out && s->nd ? ho_base + (size_t)(s->na + s->nb) * MG_STATE_N : nullptr;
    for (size_t gi = 0; gi < s->groups.size(); ++gi) {
        const ArticGroup& g = s->groups[gi];
        if (g.step_count == 0) continue;
        MgArticArgs A{};
        // the DOF part's validity is a flag in the block (MG_CHAIN_UNI_DOFOK), not
        // a launch choice: a captured launch follows later set_dof_props
        A.uni = g.uni_mass ? s->d_chain_uni + gi * MG_CHAIN_UNI_N : nullptr;
        A.na = g.step_count; A.nb = s->nb; A.nd = s->nd;
        A.artic_i = s->d_artic_step + (size_t)g.step_offset * MG_ARTIC_I_N;
        A.aff = g.aff; A.ab0 = g.aff_b0; A.ad0 = g.aff_d0; A.ads = g.aff_ds;
        A.out_aff = g.out_aff; A.og0 = g.out_g0; A.or0 = g.out_r0;
        A.tmpl = g.tmpl; A.nl = g.nl; A.ndof = g.ndof; A.fixed_base = g.fixed_base; A.chain = g.chain; A.nbl = g.nbody;
        A.link_f = s->d_link_f + (size_t)g.first_link * MG_LINK_F_N;
        A.link_i = s->d_link_i + (size_t)g.first_link * MG_LINK_I_N;
        A.state = s->d_state; A.mass = s->d_mass; A.body_tmpl = s->d_body_tmpl; A.tbf = s->d_tbf;
        A.dof_pos = s->d_dof; A.dof_vel = s->d_dof + s->nd;
        A.dof_tpos = s->d_dof_tgt; A.dof_tvel = s->d_dof_tgt + s->nd; A.dof_force = s->d_dof_tgt + 2 * (size_t)s->nd;
        fused_targets(s, A.dof_tpos, A.dof_tvel, A.dof_force, A.tpos_w, A.tvel_w, A.force_w);
        A.dof_props = s->d_dof_props;
        A.ext = s->ext_pending ? s->d_ext : nullptr;
        A.cforce = s->d_cforce;
        if (step_out || host_out) {   // chain groups only (s->step_out_ok)
            A.out_rb = step_out ? s->bind_rb : ho_rb;
            A.out_root = step_out ? s->bind_root : ho_root;
            A.out_dof = step_out ? s->bind_dof : ho_dof;
            A.out_body = s->d_slot_global;
            A.out_root_row = s->d_slot_actor;
        }
        hipError_t e = mg_launch_artic_step(P, A, st);
        if (e != hipSuccess) return fail(MG_ERR_DEVICE, "articulation step launch: %s", hipGetErrorString(e));
    }
    for (const EnvGroup& g : s->env_groups) {
        MgEnvArgs A{};
        A.ne = g.count; A.nb = s->nb; A.nd = s->nd;
        A.env_i = s->d_env + (size_t)g.offset * MG_ENV_I_N;
        A.pairs = s->d_pairs;
        A.fpatch = s->d_fpatch;
        A.fp_mask = s->d_fp_mask + (size_t)g.offset * MG_FP_W;
        A.carry = s->d_env_carry + (size_t)g.offset * mg_env_carry_floats();
        A.ctab = s->d_env_ctab + (size_t)g.offset * mg_env_ctab_floats();
        A.nl = g.tmpl >= 0 ? g.nl : 0;
        A.ndof = g.tmpl >= 0 ? g.ndof : 0;
        A.floating = g.tmpl >= 0 ? g.floating : 0;
        A.max_free = g.max_free;
        A.link_f = s->d_link_f + (size_t)(g.tmpl >= 0 ? g.first_link : 0) * MG_LINK_F_N;
        A.link_i = s->d_link_i + (size_t)(g.tmpl >= 0 ? g.first_link : 0) * MG_LINK_I_N;
        A.state = s->d_state; A.mass = s->d_mass; A.body_tmpl = s->d_body_tmpl;
        A.tbf = s->d_tbf; A.tbi = s->d_tbi; A.shapes = s->d_shapes; A.hulls = s->d_hulls;
        A.shape_obb = s->d_shape_obb;
        A.nhull = s->nhull_floats;
        A.nshape = s->ns;
        A.dof_pos = s->d_dof; A.dof_vel = s->d_dof + s->nd;
        A.dof_tpos = s->d_dof_tgt; A.dof_tvel = s->d_dof_tgt + s->nd; A.dof_force = s->d_dof_tgt + 2 * (size_t)s->nd;
        fused_targets(s, A.dof_tpos, A.dof_tvel, A.dof_force, A.tpos_w, A.tvel_w, A.force_w);
        A.dof_props = s->d_dof_props;
        A.ext = s->ext_pending ? s->d_ext : nullptr;
        A.cforce = s->d_cforce;
        hipError_t e = mg_launch_env_step(P, A, st);
        if (e != hipSuccess) return fail(MG_ERR_DEVICE, "coupled env step launch: %s", hipGetErrorString(e));
    }
    if (s->n_pile > 0) {
        MgPileArgs A{};
        A.ne = s->n_pile; A.nb = s->nb;
        A.pile_i = s->d_pile_i; A.pile_body = s->d_pile_body; A.pairs = s->d_pile_pairs; A.slots = s->d_pile_slots;
        A.state = s->d_state; A.mass = s->d_mass; A.body_tmpl = s->d_body_tmpl; A.tbf = s->d_tbf;
        A.shapes = s->d_shapes; A.hulls = s->d_hulls; A.shape_obb = s->d_shape_obb;
        A.ext = s->ext_pending ? s->d_ext : nullptr;
        A.cforce = s->d_cforce;
        hipError_t e = mg_launch_pile_step(P, A, st);
        if (e != hipSuccess) return fail(MG_ERR_DEVICE, "pile step launch: %s", hipGetErrorString(e));
    }
    if (s->nf_rigid > 0) {
        MgRigidArgs A{};
        A.nf = s->nf_rigid; A.nf1 = s->nf1; A.nb = s->nb; A.free_ids = nullptr;   // internal slots 0..nf-1
        A.state = s->d_state; A.mass = s->d_mass; A.body_tmpl = s->d_body_tmpl;
        A.tbf = s->d_tbf; A.tbi = s->d_tbi; A.shapes = s->d_shapes; A.hulls = s->d_hulls;
        A.trec = s->d_trec; A.ntb = s->ntb;
        A.gpatch = s->d_gpatch;
        A.gstride = std::max(s->nf1, 1);
        A.ext = s->ext_pending ? s->d_ext : nullptr;
        A.cforce = s->d_cforce;
        bool reads_root_in = false;
        if (s->pend_root) {   // the deferred root set, read by the step kernel
            A.root_src = s->pend_root;
            A.root_row = s->d_root_row;
            reads_root_in = s->pend_root == s->d_root_in_alias;
            s->pend_root = nullptr;
        }
        if (step_out || host_out) {
            A.out_rb = step_out ? s->bind_rb : ho_rb;
            A.out_root = step_out ? s->bind_root : ho_root;
            A.out_body = s->d_slot_global;     // internal slot -> global body
            A.out_root_row = s->d_slot_actor;
        }
        HIP_TRY(mg_launch_rigid_step(P, A, st));
        if (reads_root_in) {
            HIP_TRY(hipEventRecord(s->root_ev, st));
            s->root_ev_pending = true;
        }
    }
    if (int rc_ = flush_root(s, st)) return rc_;   // a root set with no free-body launch
    if (s->groups.empty() && s->env_groups.empty())
        for (int k = 0; k < 3; ++k)
            if (int rc_ = flush_tgt(s, k, st)) return rc_;
    for (int k = 0; k < 3; ++k) s->pend_tgt[k] = nullptr;   // read (and written through) by the step
    s->state_gen++;
    s->dof_sgen++;
    if (host_out) {
        s->ho_written = ho_base;
        s->ho_root_gen = s->state_gen;
        s->ho_rb_gen = s->state_gen;
        s->ho_dof_gen = ho_dof ? s->dof_sgen : -1;
    }
    if (step_out) {
        if (s->bind_root) { s->out_gen = s->state_gen; s->out_cap = step_cid; }
        if (s->bind_rb) { s->rb_gen = s->state_gen; s->rb_cap = step_cid; }
        if (s->bind_dof) { s->dof_gen = s->dof_sgen; s->dof_cap = step_cid; }
    }
    if (s->ext_pending) {
        HIP_TRY(hipMemsetAsync(s->d_ext, 0, (size_t)s->nb * 6 * sizeof(float), st));
        s->ext_pending = false;
    }
    mg_timer = nullptr;
    if (!s->capturing) {
        if (timed) {
            HIP_TRY(hipEventRecord(s->ev_end, st));
            s->kern_n[slot] = timer.used;
            s->kern_miss[slot] = timer.missed;
            s->ring_n++;
        }
        s->timed_step = timed;
        s->last_stream = st;
        s->stepped = true;
    }
    return MG_OK;
}

int32_t mg_fetch_results(mg_sim* s, int32_t wait) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (wait && s->stepped && !s->capturing) {
        if (s->timed_step) HIP_TRY(hipEventSynchronize(s->ev_end));
        else HIP_TRY(hipStreamSynchronize(s->last_stream));
    }
    return MG_OK;
}

int32_t mg_fetch_host_state(mg_sim* s, float* dst, int32_t parts, void* stream) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (!s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!dst && parts) return fail(MG_ERR_ARG, "null destination");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(s->device));
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(st, &cap));
    if (cap != hipStreamCaptureStatusNone) return fail(MG_ERR_STATE, "mg_fetch_host_state while capturing");
    if (int rc_ = flush_root(s, st)) return rc_;
    // [na][13] roots, [nb][13] bodies, [nd][2] DOFs, [nb][3] contact forces; the
    // parts asked for are gathered and the span covering them copied at once
    const size_t off[5] = {0, (size_t)s->na * MG_STATE_N, (size_t)(s->na + s->nb) * MG_STATE_N,
                           (size_t)(s->na + s->nb) * MG_STATE_N + (size_t)s->nd * 2,
                           (size_t)(s->na + s->nb) * MG_STATE_N + (size_t)s->nd * 2 + (size_t)s->nb * 3};
    // zero-copy when dst is the sim's own mapped stage (mg_host_stage): the parts
    // the last simulate wrote are already there, the others are gathered into it
    const bool alias = s->h_stage && dst == s->h_stage && s->h_stage_n >= off[4];
    if (!alias && s->host_out_n < off[4]) {   // the output stage (simulate writes into it from now on)
        if (s->d_host_out) (void)hipFree(s->d_host_out);
        s->d_host_out = nullptr;
        HIP_TRY(dalloc(&s->d_host_out, std::max<size_t>(off[4], 1)));
        s->host_out_n = off[4];
        if (s->ho_written && !s->ho_alias) s->ho_written = nullptr;
    }
    s->ho_alias = alias;
    float* base = alias ? s->d_stage_alias : s->d_host_out;
    const bool fresh = s->ho_written == base;
    int lo = -1, hi = -1;
    for (int k = 0; k < 4; ++k) {
        if (!((parts >> k) & 1) || off[k + 1] == off[k]) continue;
        if (lo < 0) lo = k;
        hi = k;
        float* d = base + off[k];
        // parts the last simulate wrote there, with no state change since: no gather
        if (k == 0 && !(fresh && s->ho_root_gen == s->state_gen))
            HIP_TRY(mg_launch_gather_rows(s->d_state, s->nb, MG_STATE_N, s->d_actor_root, s->na, d, st));
        if (k == 1 && !(fresh && s->ho_rb_gen == s->state_gen))
            HIP_TRY(mg_launch_gather_rows(s->d_state, s->nb, MG_STATE_N, s->d_perm, s->nb, d, st));
        if (k == 2 && !(fresh && s->ho_dof_gen == s->dof_sgen))
            HIP_TRY(mg_launch_gather_rows(s->d_dof, s->nd, 2, nullptr, s->nd, d, st));
        if (k == 3) HIP_TRY(mg_launch_gather_rows(s->d_cforce, s->nb, 3, s->d_perm, s->nb, d, st));
    }
    if (lo >= 0 && !alias)
        HIP_TRY(hipMemcpyAsync(dst + off[lo], s->d_host_out + off[lo], (off[hi + 1] - off[lo]) * sizeof(float),
                               hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MG_OK;
}

int32_t mg_set_light(mg_sim* s, const mg_light* light) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (!light) {
        s->has_light = false;
        return MG_OK;
    }
    const float* d = light->dir;
    if (!(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] > 0.0f)) return fail(MG_ERR_ARG, "zero light direction");
    s->light = *light;
    s->has_light = true;
    return MG_OK;
}

float* mg_host_stage(mg_sim* s, int64_t nfloat) {
    if (!s || nfloat <= 0) { fail(MG_ERR_ARG, "null sim or empty stage"); return nullptr; }
    if (s->h_stage && s->h_stage_n >= (size_t)nfloat) return s->h_stage;
    if (hipSetDevice(s->device) != hipSuccess) { fail(MG_ERR_DEVICE, "hipSetDevice failed"); return nullptr; }
    if (s->h_stage) {
        (void)hipDeviceSynchronize();
        (void)hipHostFree(s->h_stage);
        s->h_stage = nullptr;
        s->d_stage_alias = nullptr;
        s->h_stage_n = 0;
        s->ho_alias = false;
        s->ho_written = nullptr;
    }
    float* h = nullptr;
    if (hipHostMalloc((void**)&h, (size_t)nfloat * sizeof(float), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess) {
        fail(MG_ERR_DEVICE, "hipHostMalloc of the host stage failed");
        return nullptr;
    }
    float* d = nullptr;
    if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess || !d) {
        (void)hipHostFree(h);
        fail(MG_ERR_DEVICE, "hipHostGetDevicePointer of the host stage failed");
        return nullptr;
    }
    std::memset(h, 0, (size_t)nfloat * sizeof(float));
    s->h_stage = h;
    s->d_stage_alias = d;
    s->h_stage_n = (size_t)nfloat;
    return h;
}

int32_t mg_set_fusion(mg_sim* s, int32_t flags) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    const int32_t prev = s->fusion;
    s->fusion = flags & (MG_FUSE_ROOT_SET | MG_FUSE_REFRESH | MG_FUSE_DOF_TARGETS | MG_FUSE_IN_CAPTURE | MG_FUSE_STEP_OUT);
    return prev;
}

int32_t mg_bind_refresh_targets(mg_sim* s, float* root_dst, float* rigid_body_dst) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    s->bind_root = root_dst;
    s->bind_rb = rigid_body_dst;
    s->rb_gen = -1;
    s->out_gen = -1;
    return MG_OK;
}

int32_t mg_bind_dof_refresh_target(mg_sim* s, float* dof_dst) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    s->bind_dof = dof_dst;
    s->dof_gen = -1;
    return MG_OK;
}

int32_t mg_discard_pending_sets(mg_sim* s) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    s->pend_root = nullptr;
    for (int k = 0; k < 3; ++k) s->pend_tgt[k] = nullptr;
    return MG_OK;
}

int32_t mg_step_out_supported(mg_sim* s) { return s && s->uploaded && s->step_out_ok ? 1 : 0; }

int32_t mg_last_set_deferred(mg_sim* s) { return s ? s->last_set_deferred : 0; }

int32_t mg_set_kernel_timing(mg_sim* s, int32_t on) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    const int32_t prev = s->timing ? 1 : 0;
    s->timing = on != 0;
    return prev;
}

float mg_last_step_ms(mg_sim* s) {
    if (!s || !s->stepped || !s->timed_step) return -1.0f;
    if (hipEventSynchronize(s->ev_end) != hipSuccess) return -1.0f;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, s->ev_begin, s->ev_end) != hipSuccess) return -1.0f;
    return ms;
}

int32_t mg_step_time_stats(mg_sim* s, int32_t n, float* avg_ms, float* min_ms, float* max_ms) {
    if (!s || n <= 0) return fail(MG_ERR_ARG, "bad arguments");
    if (s->ring_n == 0) return fail(MG_ERR_STATE, "no simulate() recorded");
    long long avail = s->ring_n < mg_sim::kRing ? s->ring_n : mg_sim::kRing;
    if (n > avail) n = (int32_t)avail;
    double sum = 0.0;
    float lo = 1e30f, hi = 0.0f;
    for (int32_t k = 0; k < n; ++k) {
        const int slot = (int)((s->ring_n - 1 - k) % mg_sim::kRing);
        HIP_TRY(hipEventSynchronize(s->ring_e[slot]));
        // sum of the step kernels' own durations (dispatch timestamps)
        float ms = 0.0f;
        for (int j = 0; j < s->kern_n[slot]; ++j) {
            float kms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&kms, s->kern_b[slot][j], s->kern_e[slot][j]));
            ms += kms;
        }
        sum += ms;
        lo = ms < lo ? ms : lo;
        hi = ms > hi ? ms : hi;
    }
    if (avg_ms) *avg_ms = (float)(sum / n);
    if (min_ms) *min_ms = lo;
    if (max_ms) *max_ms = hi;
    return n;
}

int32_t mg_step_untimed_launches(mg_sim* s, int32_t n) {
    if (!s || n <= 0) return fail(MG_ERR_ARG, "bad arguments");
    if (s->ring_n == 0) return fail(MG_ERR_STATE, "no simulate() recorded");
    const long long avail = s->ring_n < mg_sim::kRing ? s->ring_n : mg_sim::kRing;
    if (n > avail) n = (int32_t)avail;
    int32_t most = 0;
    for (int32_t k = 0; k < n; ++k) {
        const int slot = (int)((s->ring_n - 1 - k) % mg_sim::kRing);
        most = std::max(most, s->kern_miss[slot]);
    }
    return most;
}

// diagnostics (tests/test_franka_gpu.py, tools/diag_franka_env.py): coupled
// env k's contact table (k_env_np's output of the last substep run): the
// group's base and record size are the library's, so callers hard-code neither
int32_t mg_debug_copy_env_ctab(mg_sim* s, int32_t k, float* dst, int32_t cap) {
    if (!s || !s->uploaded || !s->d_env_ctab || !dst) return fail(MG_ERR_ARG, "bad arguments");
    if (k < 0 || k >= (int32_t)s->cenv_ctab_off.size()) return fail(MG_ERR_ARG, "no such coupled env");
    const int32_t n = s->cenv_ctab_n[k];
    if (cap < n) return fail(MG_ERR_ARG, "dst holds fewer floats than the env's contact table");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(dst, s->d_env_ctab + s->cenv_ctab_off[k], (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
    return n;
}

// diagnostics (tests/test_step_out_chain_gpu.py): per articulation group the
// facts that choose its chain-kernel form (mg_chain.hip mg_launch_artic_chain)
int32_t mg_debug_artic_groups(mg_sim* s, int32_t* out, int32_t cap) {
    if (!s || !s->uploaded || (!out && cap > 0)) return fail(MG_ERR_ARG, "bad arguments");
    const int32_t n = (int32_t)s->groups.size();
    for (int32_t i = 0; i < n && (i + 1) * MG_DEBUG_GROUP_N <= cap; ++i) {
        const ArticGroup& g = s->groups[i];
        int32_t* r = out + (size_t)i * MG_DEBUG_GROUP_N;
        r[0] = g.nl; r[1] = g.step_count; r[2] = g.chain; r[3] = g.uni_mass ? 1 : 0;
        r[4] = g.uni_dof ? 1 : 0; r[5] = g.aff; r[6] = g.out_aff; r[7] = s->step_out_ok ? 1 : 0;
    }
    return n;
}

// the S3 cube-pick controller (csrc/mg_ctrl.hip): independent of any sim, on
// the caller's stream (torch's current stream: ordered with the refreshes that
// filled its inputs and the sets that read its outputs)
int32_t mg_cube_pick_step(const mg_cube_pick_args* a, void* stream) {
    if (!a || a->n < 0) return fail(MG_ERR_ARG, "bad arguments");
    if (a->n == 0) return MG_OK;
    if (!a->rb || !a->box_row || !a->hand_row || !a->dof || !a->dof_row0 || !a->jac || (a->osc && !a->mm) ||
        !a->init_pos || !a->init_rot || !a->default_dof_pos || !a->hand_restart || !a->pos_action ||
        !a->effort_action)
        return fail(MG_ERR_ARG, "null tensor");
    HIP_TRY(mg_launch_cube_pick(*a, (hipStream_t)stream));
    return MG_OK;
}

int32_t mg_num_free_bodies(mg_sim* s) { return s ? s->nf : 0; }
int32_t mg_num_articulations(mg_sim* s) { return s ? s->nartic : 0; }
int32_t mg_num_coupled_envs(mg_sim* s) { return s ? s->n_coupled : 0; }
int32_t mg_num_pile_envs(mg_sim* s) { return s ? s->n_pile : 0; }

int32_t mg_refresh_actor_root_state(mg_sim* s, float* dst, int32_t dst_host, void* stream) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (!s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(s->device));
    if (int rc_ = flush_root(s, st)) return rc_;
    const unsigned long long cid = capture_id(st);
    if (!dst_host && dst && dst == s->bind_root && (s->fusion & MG_FUSE_STEP_OUT) && s->out_gen == s->state_gen &&
        s->out_cap == cid)
        return MG_OK;   // written by the step kernel (MG_FUSE_STEP_OUT)
    if (!dst_host && dst && dst == s->bind_root && s->bind_rb && (s->fusion & MG_FUSE_REFRESH) &&
        fuse_here(s, cid) && s->na > 0) {
        // the bound root and rigid-body tensors in one launch
        HIP_TRY(mg_launch_gather_rb_root(s->d_state, s->nb, MG_STATE_N, s->d_perm, s->nb, s->bind_rb, s->d_body_actor,
                                         dst, st));
        s->rb_gen = s->state_gen;
        s->rb_cap = cid;
        return MG_OK;
    }
    return refresh_rows(s, s->d_state, s->nb, MG_STATE_N, s->d_actor_root, s->na, dst, dst_host, st);
}
int32_t mg_refresh_rigid_body_state(mg_sim* s, float* dst, int32_t dst_host, void* stream) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (!s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(s->device));
    if (int rc_ = flush_root(s, st)) return rc_;
    const bool bound = !dst_host && dst && dst == s->bind_rb;
    if (bound && (s->fusion & (MG_FUSE_REFRESH | MG_FUSE_STEP_OUT)) && s->rb_gen == s->state_gen &&
        s->rb_cap == capture_id(st))
        return MG_OK;   // served by the paired gather / the step kernel of the same capture (or eagerly)
    const int rc = refresh_rows(s, s->d_state, s->nb, MG_STATE_N, s->d_perm, s->nb, dst, dst_host, st);
    if (rc == MG_OK && bound) {
        s->rb_gen = s->state_gen;
        s->rb_cap = capture_id(st);
    }
    return rc;
}
int32_t mg_refresh_dof_state(mg_sim* s, float* dst, int32_t dst_host, void* stream) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    if (!dst_host && dst && dst == s->bind_dof && (s->fusion & MG_FUSE_STEP_OUT) && s->dof_gen == s->dof_sgen &&
        s->dof_cap == capture_id((hipStream_t)stream))
        return MG_OK;   // written by the step kernel (MG_FUSE_STEP_OUT)
    return refresh_rows(s, s->d_dof, s->nd, 2, nullptr, s->nd, dst, dst_host, (hipStream_t)stream);
}
int32_t mg_refresh_net_contact_force(mg_sim* s, float* dst, int32_t dst_host, void* stream) {
    if (!s) return fail(MG_ERR_ARG, "null sim");
    return refresh_rows(s, s->d_cforce, s->nb, 3, s->d_perm, s->nb, dst, dst_host, (hipStream_t)stream);
}

int32_t mg_set_actor_root_state(mg_sim* s, const float* src, int32_t src_host, const int32_t* idx,
                                int32_t n_idx, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!src) return fail(MG_ERR_ARG, "null source tensor");
    if (idx && n_idx < 0) return fail(MG_ERR_ARG, "negative index count");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const float* dsrc;
    const int* didx;
    s->state_gen++;
    const unsigned long long cid = capture_id(st);
    s->last_set_deferred = 0;
    if (!src_host && !idx && s->roots_free && (s->fusion & MG_FUSE_ROOT_SET) && fuse_here(s, cid)) {
        if (s->pend_root && s->pend_root_cap != cid)
            if (int rc_ = flush_root(s, st)) return rc_;
        s->pend_root = src;   // read by the next simulate (a later full set replaces it)
        s->pend_root_cap = cid;
        s->last_set_deferred = 1;
        return MG_OK;
    }
    if (src_host && !idx && s->roots_free && cid == 0) {
        // CPU pipeline, full set: copied at the call into the library's own buffer
        // (Isaac Gym's copy-at-set), read by the next simulate's step kernel like
        // a fused device set — or by the scatter a reader of the state issues first
        const size_t bytes = (size_t)s->na * MG_STATE_N * sizeof(float);
        s->pend_root = nullptr;     // a later full set replaces an earlier deferred one
        if (!s->h_root_in) {        // page-locked and device-mapped: the step kernel reads it over PCIe
            HIP_TRY(hipHostMalloc((void**)&s->h_root_in, bytes, hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void**)&s->d_root_in_alias, s->h_root_in, 0));
            HIP_TRY(hipEventCreateWithFlags(&s->root_ev, hipEventDisableTiming));
        }
        if (s->root_ev_pending) HIP_TRY(hipEventSynchronize(s->root_ev));   // its last reader is done
        s->root_ev_pending = false;
        std::memcpy(s->h_root_in, src, bytes);
        s->pend_root = s->d_root_in_alias;
        s->pend_root_cap = 0;
        return MG_OK;
    }
    if (int rc_ = flush_root(s, st)) return rc_;
    int rc = stage_src(s, src, src_host, (size_t)s->na * MG_STATE_N, idx, n_idx, st, &dsrc, &didx);
    if (rc) return rc;
    HIP_TRY(mg_launch_scatter_rows(dsrc, MG_STATE_N, s->d_actor_root, didx, idx ? n_idx : s->na, s->na,
                                   s->d_state, s->nb, st));
    return MG_OK;
}

int32_t mg_set_rigid_body_state(mg_sim* s, const float* src, int32_t src_host, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!src) return fail(MG_ERR_ARG, "null source tensor");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const float* dsrc;
    const int* didx;
    if (int rc_ = flush_root(s, st)) return rc_;
    s->state_gen++;
    int rc = stage_src(s, src, src_host, (size_t)s->nb * MG_STATE_N, nullptr, 0, st, &dsrc, &didx);
    if (rc) return rc;
    // free bodies only: rows are selected through the free-body list
    HIP_TRY(mg_launch_scatter_rows(dsrc, MG_STATE_N, s->d_perm, s->d_free_global, s->nf, s->nb, s->d_state,
                                   s->nb, st));
    return MG_OK;
}

int32_t mg_set_dof_state(mg_sim* s, const float* src, int32_t src_host, const int32_t* idx, int32_t n_idx,
                         void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    s->dof_sgen++;
    s->last_set_deferred = 0;
    return set_dof_columns(s, src, src_host, 2, s->d_dof, s->d_dof + s->nd, idx, n_idx, (hipStream_t)stream);
}
// column k of the DOF targets; a device-resident full set is read by the next
// simulate's articulation kernels (MG_FUSE_DOF_TARGETS), else a scatter / copy
static int32_t set_dof_target(mg_sim* s, int k, const float* src, int32_t src_host, const int32_t* idx,
                              int32_t n_idx, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (s->nd == 0) return MG_OK;
    if (!src) return fail(MG_ERR_ARG, "null source tensor");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(s->device));
    const unsigned long long cid = capture_id(st);
    s->last_set_deferred = 0;
    if (!src_host && !idx && (s->fusion & MG_FUSE_DOF_TARGETS) && fuse_here(s, cid)) {
        if (s->pend_tgt[k] && s->pend_tgt_cap[k] != cid)
            if (int rc_ = flush_tgt(s, k, st)) return rc_;
        s->pend_tgt[k] = src;
        s->pend_tgt_cap[k] = cid;
        s->last_set_deferred = 1;
        return MG_OK;
    }
    if (int rc_ = flush_tgt(s, k, st)) return rc_;
    return set_dof_columns(s, src, src_host, 1, s->d_dof_tgt + (size_t)k * s->nd, nullptr, idx, n_idx, st);
}
int32_t mg_set_dof_position_target(mg_sim* s, const float* src, int32_t src_host, const int32_t* idx,
                                   int32_t n_idx, void* stream) {
    return set_dof_target(s, 0, src, src_host, idx, n_idx, stream);
}
int32_t mg_set_dof_velocity_target(mg_sim* s, const float* src, int32_t src_host, const int32_t* idx,
                                   int32_t n_idx, void* stream) {
    return set_dof_target(s, 1, src, src_host, idx, n_idx, stream);
}
int32_t mg_set_dof_actuation_force(mg_sim* s, const float* src, int32_t src_host, const int32_t* idx,
                                   int32_t n_idx, void* stream) {
    return set_dof_target(s, 2, src, src_host, idx, n_idx, stream);
}

int32_t mg_set_dof_props(mg_sim* s, const float* props_host) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (s->nd == 0) return MG_OK;
    if (!props_host) return fail(MG_ERR_ARG, "null props");
    HIP_TRY(hipSetDevice(s->device));
    std::vector<float> dp = to_soa(props_host, s->nd, MG_DOFPROP_N);
    HIP_TRY(hipMemcpy(s->d_dof_props, dp.data(), dp.size() * sizeof(float), hipMemcpyHostToDevice));
    for (ArticGroup& g : s->groups)
        if (g.uni_mass) chain_uni_dof(props_host, g);
    HIP_TRY(chain_uni_upload(s));
    return MG_OK;
}

int32_t mg_apply_rigid_body_force(mg_sim* s, const float* force, const float* torque, int32_t space,
                                  int32_t src_host, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (space != 0) return fail(MG_ERR_UNSUPPORTED, "only global-space forces are supported");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const float* parts[2] = {force, torque};
    for (int k = 0; k < 2; ++k) {
        if (!parts[k]) continue;
        const float* dsrc;
        const int* didx;
        int rc = stage_src(s, parts[k], src_host, (size_t)s->nb * 3, nullptr, 0, st, &dsrc, &didx);
        if (rc) return rc;
        HIP_TRY(mg_launch_scatter_rows(dsrc, 3, s->d_perm, nullptr, s->nb, s->nb, s->d_ext + (size_t)k * 3 * s->nb,
                                       s->nb, st));
        if (src_host) HIP_TRY(hipStreamSynchronize(st));  // staging buffer is reused by the next part
    }
    s->ext_pending = true;
    return MG_OK;
}

static int refresh_jac_mm(mg_sim* s, int32_t tmpl, float* jdst, float* mdst, int32_t dst_host, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!jdst && !mdst) return fail(MG_ERR_ARG, "null destination");
    const ArticGroup* g = nullptr;
    for (const ArticGroup& x : s->groups)
        if (x.tmpl == tmpl) g = &x;
    if (!g) return fail(MG_ERR_ARG, "no articulation template %d", tmpl);
    const int nc = g->ndof + (g->fixed_base ? 0 : 6);
    if (nc > 32) return fail(MG_ERR_UNSUPPORTED, "jacobian / mass matrix of more than 32 generalized velocities");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const size_t jper = (size_t)(g->nbody - (g->fixed_base ? 1 : 0)) * 6 * nc, mper = (size_t)nc * nc;
    const size_t jtot = jdst ? jper * g->count : 0, mtot = mdst ? mper * g->count : 0;
    float* jout = jdst;
    float* mout = mdst;
    if (dst_host) {
        int rc = ensure_stage(s, jtot + mtot, 0);
        if (rc) return rc;
        jout = jdst ? s->d_stage : nullptr;
        mout = mdst ? s->d_stage + jtot : nullptr;
    }
    MgArticArgs A{};
    A.na = g->count; A.nb = s->nb; A.nd = s->nd;
    A.artic_i = s->d_artic + (size_t)g->offset * MG_ARTIC_I_N;
    A.tmpl = g->tmpl; A.nl = g->nl; A.ndof = g->ndof; A.fixed_base = g->fixed_base; A.nbl = g->nbody;
    A.link_f = s->d_link_f + (size_t)g->first_link * MG_LINK_F_N;
    A.link_i = s->d_link_i + (size_t)g->first_link * MG_LINK_I_N;
    A.state = s->d_state; A.mass = s->d_mass;
    A.dof_pos = s->d_dof; A.dof_vel = s->d_dof + s->nd;
    if (mtot > 0) HIP_TRY(hipMemsetAsync(mout, 0, mtot * sizeof(float), st));
    HIP_TRY(mg_launch_jacobian(A, jout, mout, st));
    if (dst_host) {
        if (jtot) HIP_TRY(hipMemcpyAsync(jdst, jout, jtot * sizeof(float), hipMemcpyDeviceToHost, st));
        if (mtot) HIP_TRY(hipMemcpyAsync(mdst, mout, mtot * sizeof(float), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return MG_OK;
}

int32_t mg_refresh_jacobian(mg_sim* s, int32_t tmpl, float* dst, int32_t dst_host, void* stream) {
    if (!dst) return fail(MG_ERR_ARG, "null destination");
    return refresh_jac_mm(s, tmpl, dst, nullptr, dst_host, stream);
}
int32_t mg_refresh_mass_matrix(mg_sim* s, int32_t tmpl, float* dst, int32_t dst_host, void* stream) {
    if (!dst) return fail(MG_ERR_ARG, "null destination");
    return refresh_jac_mm(s, tmpl, nullptr, dst, dst_host, stream);
}
int32_t mg_refresh_jacobian_mass_matrix(mg_sim* s, int32_t tmpl, float* jac, float* mm, int32_t dst_host,
                                        void* stream) {
    return refresh_jac_mm(s, tmpl, jac, mm, dst_host, stream);
}


// ---- camera sensors ---------------------------------------------------------

int32_t mg_set_render_bodies(mg_sim* s, const int32_t* env_body_first, const float* color, const int32_t* seg) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!env_body_first || !color || !seg) return fail(MG_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(s->device));
    const int ne = s->nenv;
    if (env_body_first[0] != 0 || env_body_first[ne] != s->nb) return fail(MG_ERR_ARG, "env_body_first must span [0, num_bodies]");
    std::vector<MgRShape> rs;
    std::vector<int> first(ne + 1, 0);
    for (int e = 0; e < ne; ++e) {
        first[e] = (int)rs.size();
        if (env_body_first[e + 1] < env_body_first[e]) return fail(MG_ERR_ARG, "env_body_first not monotone");
        for (int b = env_body_first[e]; b < env_body_first[e + 1]; ++b) {
            const int t = s->h_body_tmpl[b];
            const int sh0 = s->h_tbi[(size_t)t * MG_TBODY_I_N + 0], nsh = s->h_tbi[(size_t)t * MG_TBODY_I_N + 1];
            for (int k = 0; k < nsh; ++k) {
                MgRShape r{};
                r.slot = s->h_perm[b];
                r.shape = sh0 + k;
                r.seg = seg[b];
                r.r = color[3 * (size_t)b + 0]; r.g = color[3 * (size_t)b + 1]; r.b = color[3 * (size_t)b + 2];
                rs.push_back(r);
            }
        }
        if ((int)rs.size() - first[e] > MG_RENDER_MAX_SHAPES)
            return fail(MG_ERR_UNSUPPORTED, "env %d has %d shapes; a camera's env may hold at most %d", e,
                        (int)rs.size() - first[e], MG_RENDER_MAX_SHAPES);
    }
    first[ne] = (int)rs.size();
    if (s->d_rshapes) (void)hipFree(s->d_rshapes);
    if (s->d_env_shape_first) (void)hipFree(s->d_env_shape_first);
    s->d_rshapes = nullptr; s->d_env_shape_first = nullptr;
    HIP_TRY(dalloc(&s->d_rshapes, rs.size()));
    HIP_TRY(dalloc(&s->d_env_shape_first, (size_t)ne + 1));
    if (!rs.empty()) HIP_TRY(hipMemcpy(s->d_rshapes, rs.data(), rs.size() * sizeof(MgRShape), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->d_env_shape_first, first.data(), first.size() * sizeof(int), hipMemcpyHostToDevice));
    s->n_rshapes = (int)rs.size();
    s->render_ready = true;
    return MG_OK;
}

int32_t mg_snapshot_render_state(mg_sim* s, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    HIP_TRY(hipSetDevice(s->device));
    if (!s->d_rstate) HIP_TRY(dalloc(&s->d_rstate, (size_t)s->nb * MG_STATE_N));
    if (int rc_ = flush_root(s, (hipStream_t)stream)) return rc_;
    HIP_TRY(hipMemcpyAsync(s->d_rstate, s->d_state, (size_t)s->nb * MG_STATE_N * sizeof(float),
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
    s->rstate_valid = true;
    return MG_OK;
}

int32_t mg_render_cameras(mg_sim* s, const mg_camera* cams, int32_t n, void* stream) {
    if (!s || !s->uploaded) return fail(MG_ERR_STATE, "sim has no uploaded model");
    if (!s->render_ready) return fail(MG_ERR_STATE, "mg_set_render_bodies was not called");
    if (!s->rstate_valid) return fail(MG_ERR_STATE, "no render snapshot (mg_snapshot_render_state)");
    if (n < 0 || (n > 0 && !cams)) return fail(MG_ERR_ARG, "bad camera list");
    if (n == 0) return MG_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    const bool same = (int)s->cam_host.size() == n &&
                      std::memcmp(s->cam_host.data(), cams, (size_t)n * sizeof(mg_camera)) == 0;
    if (!same) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(st, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return fail(MG_ERR_STATE, "camera table changed while the stream is being captured");
        std::vector<MgRenderCam> dev((size_t)n);
        long long blocks = 0;
        for (int i = 0; i < n; ++i) {
            const mg_camera& c = cams[i];
            if (c.env < 0 || c.env >= s->nenv) return fail(MG_ERR_ARG, "camera %d: env %d out of range", i, c.env);
            if (c.width <= 0 || c.height <= 0 || (long long)c.width * c.height > (1ll << 30))
                return fail(MG_ERR_ARG, "camera %d: bad size %dx%d", i, c.width, c.height);
            if (c.body >= s->nb) return fail(MG_ERR_ARG, "camera %d: body %d out of range", i, c.body);
            if (!(c.fx > 0.0f) || !(c.fy > 0.0f)) return fail(MG_ERR_ARG, "camera %d: bad focal length", i);
            MgRenderCam& d = dev[i];
            d.env = c.env; d.w = c.width; d.h = c.height;
            d.slot = c.body >= 0 ? s->h_perm[c.body] : -1;
            d.follow = c.follow;
            d.blk0 = (int)blocks;
            const long long npx = (long long)c.width * c.height;
            d.nblk = (int)((npx + MG_RENDER_RUN - 1) / MG_RENDER_RUN);
            blocks += d.nblk;
            const auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
            d.vec = (npx % MG_RENDER_LANE_PX == 0) && al16(c.color) && al16(c.depth) && al16(c.seg);
            d.fx = c.fx; d.fy = c.fy; d.cx = c.cx; d.cy = c.cy;
            d.ifx = 1.0f / c.fx; d.ify = 1.0f / c.fy;
            d.near_plane = c.near_plane; d.far_plane = c.far_plane;
            for (int k = 0; k < 3; ++k) d.p[k] = c.p[k];
            for (int k = 0; k < 4; ++k) d.q[k] = c.q[k];
            d.color = c.color; d.depth = c.depth; d.seg = c.seg;
        }
        if (blocks > (1ll << 31) - 1) return fail(MG_ERR_ARG, "too many pixels in one render call");
        if (n > s->cam_cap) {
            if (s->d_cams) (void)hipFree(s->d_cams);
            s->d_cams = nullptr;
            HIP_TRY(dalloc(&s->d_cams, (size_t)n));
            s->cam_cap = n;
        }
        HIP_TRY(hipMemcpy(s->d_cams, dev.data(), (size_t)n * sizeof(MgRenderCam), hipMemcpyHostToDevice));
        s->cam_host.assign(cams, cams + n);
        s->cam_dev = dev;
        s->cam_blocks = (int)blocks;
    }
    MgRenderArgs A{};
    A.ncam = n; A.nb = s->nb; A.cams = s->d_cams; A.state = s->d_rstate; A.shapes = s->d_shapes;
    A.hulls = s->d_hulls;
    A.uniform_nblk = s->cam_dev[0].nblk;
    for (int i = 1; i < n; ++i)
        if (s->cam_dev[i].nblk != A.uniform_nblk) { A.uniform_nblk = 0; break; }
    A.rshapes = s->d_rshapes; A.env_shape_first = s->d_env_shape_first;
    const mg_sim_params& p = s->params;
    A.has_ground = p.has_ground;
    for (int k = 0; k < 3; ++k) A.gn[k] = p.ground_normal[k];
    A.gpd = p.ground_distance;
    // camera frame (local axes): z-up sims look along +x with +z up (test11's
    // UAV camera, the controller's rot_coord3); y-up sims look along -z with +y
    // up (pinned by examples/graphics_images cam1, attached to a ball);
    // left = up x forward; light from above, a little off the up axis
    A.up_axis = p.up_axis == 0 ? 0 : 1;
    float lx = 0.3f, ly = 0.2f, lz = 1.0f;
    if (A.up_axis == 1) {
        A.fwd[0] = 1.0f; A.fwd[1] = 0.0f; A.fwd[2] = 0.0f;
        A.up[0] = 0.0f; A.up[1] = 0.0f; A.up[2] = 1.0f;
        A.left[0] = 0.0f; A.left[1] = 1.0f; A.left[2] = 0.0f;
    } else {
        A.fwd[0] = 0.0f; A.fwd[1] = 0.0f; A.fwd[2] = -1.0f;
        A.up[0] = 0.0f; A.up[1] = 1.0f; A.up[2] = 0.0f;
        A.left[0] = -1.0f; A.left[1] = 0.0f; A.left[2] = 0.0f;
        ly = 1.0f; lz = 0.2f;
    }
    for (int k = 0; k < 3; ++k) { A.lcol[k] = 0.7f; A.lamb[k] = 0.3f; }
    if (s->has_light) {
        lx = s->light.dir[0]; ly = s->light.dir[1]; lz = s->light.dir[2];
        for (int k = 0; k < 3; ++k) { A.lcol[k] = s->light.color[k]; A.lamb[k] = s->light.ambient[k]; }
    }
    const float inv = 1.0f / sqrtf(lx * lx + ly * ly + lz * lz);
    A.light[0] = lx * inv; A.light[1] = ly * inv; A.light[2] = lz * inv;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(st, &cap));
    const bool timed = s->timing && cap == hipStreamCaptureStatusNone;
    MgKernelTimer timer{};
    if (timed) {
        if (!s->rev_b) HIP_TRY(hipEventCreate(&s->rev_b));
        if (!s->rev_e) HIP_TRY(hipEventCreate(&s->rev_e));
        timer.start = &s->rev_b;
        timer.stop = &s->rev_e;
        timer.cap = 1;
        mg_timer = &timer;      // the launch carries the kernel's dispatch timestamps
    }
    const hipError_t e = mg_launch_render(A, s->cam_blocks, st);
    mg_timer = nullptr;
    HIP_TRY(e);
    s->rendered = timed;
    return MG_OK;
}

float mg_last_render_ms(mg_sim* s) {
    if (!s || !s->rendered) return -1.0f;
    if (hipEventSynchronize(s->rev_e) != hipSuccess) return -1.0f;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, s->rev_b, s->rev_e) != hipSuccess) return -1.0f;
    return ms;
}

}  // extern "C"
