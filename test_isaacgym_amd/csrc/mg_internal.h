// mg_internal.h — internal structures shared by the host side (migym_capi.cpp)
// and the HIP kernels (mg_rigid.hip, mg_artic.hip, mg_tensor.hip).
//
// Numerics contract: every kernel is compiled with -ffp-contract=off and uses no
// library transcendental in the step, so that the CPU restatement in
// oracle/migym_oracle.c (compiled the same way) reproduces it bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include "../../include/migym.h"

#define MG_MAX_CONTACTS 8     // contact slots per free body per substep
#define MG_MAX_LINKS    32    // articulation links (more than 16: the 64-lane kernels)
#define MG_MAX_DOFS     32

// Per-simulate constants derived on the host from mg_sim_params
// (one copy, passed by value as a kernel argument).
struct MgStep {
    float h;          // substep length dt / substeps
    float sub;        // TGS position sub-iteration length h / npos
    float inv_sub;    // 1 / sub
    float inv_h;      // 1 / h
    float inv_dt;     // 1 / dt (contact impulse -> force)
    float g[3];       // gravity
    int   substeps, npos, nvel;
    float contact_offset, rest_offset, max_depen, bounce_thresh;
    int   has_ground;
    float n[3];       // ground normal
    float pd;         // ground plane offset: dot(n, x) + pd = 0
    float t1[3], t2[3];   // ground tangent basis
    float mu_ground, e_ground;
    float fric_offset;   // friction_offset_threshold (coupled step: friction anchors)
    float fric_corr;     // friction_correlation_distance
};

// Compact per-template record of the single-shape free-body kernel (built at
// upload): the MG_TBODY_F_N template floats, then the template's first shape
// record (type -1 when it has none). Staged in LDS when the table fits.
// compact template record of k_rigid_step1: the template body floats (pad[0] =
// 1: all its free bodies share one mass row), the first shape record (pad[0] =
// bounding radius), then that shared mass row (MG_MASS_N floats)
#define MG_TREC_N        (MG_TBODY_F_N + MG_SHAPE_STRIDE + MG_MASS_N)
#define MG_TREC_MASS     (MG_TBODY_F_N + MG_SHAPE_STRIDE)
#ifndef MG_TREC_LDS_MAX
#define MG_TREC_LDS_MAX  (48 * 1024)
#endif

// Kernel argument block of the free-body step (SoA arrays, stride = nb).
struct MgRigidArgs {
    int          nf;          // number of free bodies
    int          nf1;         // of which single-shape (listed first in free_ids)
    int          nb;          // SoA stride (total bodies)
    const int*   free_ids;    // [nf] storage slots, or null: slot = lane index
    float*       state;       // [13][nb]
    const float* mass;        // [12][nb]
    const int*   body_tmpl;   // [nb]
    const float* tbf;         // [ntb][8]
    const int*   tbi;         // [ntb][4]
    const float* shapes;      // [ns][16]
    const float* hulls;       // convex hull records (MG_SHAPE_CONVEX)
    const float* ext;         // [6][nb] world force/torque at COM, or null
    float*       cforce;      // [3][nb] net contact force out
    const float* trec;        // [ntb][MG_TREC_N] compact template records
    int          ntb;         // template bodies
    const float* root_src;    // fused root-state set: [na][13] rows, or null
    const int*   root_row;    // [nb] internal slot -> actor row of root_src (-1: none)
    // refresh fused into the step (MG_FUSE_STEP_OUT): the bound rigid-body and
    // root tensors written by the step kernel itself, or null
    float*       out_rb;      // [nb][13] rigid-body tensor (global body order)
    float*       out_root;    // [na][13] actor root tensor
    const int*   out_body;    // [nb] internal slot -> global body (rigid-body row)
    const int*   out_root_row;// [nb] internal slot -> actor row (-1: not a root)
    // ground friction patches of the single-shape bodies (persistent, DESIGN.md
    // §3.2.1): SoA [MG_FP_N][gstride], slot b = internal slot b < nf1
    float*       gpatch;
    int          gstride;
};

// Articulation step arguments (lane = articulation instance).
struct MgArticArgs {
    int          na;          // articulation instances in this launch
    int          nb, nd;      // SoA strides
    const int*   artic_i;     // [na][4] first_body, first_dof, tmpl, pad
    // aff: instance a's row is computed, not loaded (migym_capi.cpp; the blocked
    // chain layout): first body ab0 + (a / 64) * 64 * nbl + a % 64, link stride
    // min(64, na - 64 (a / 64)), first DOF ad0 + a * ads
    int          aff, ab0, ad0, ads;
    // out_aff: instance a's fused-refresh rows too — link l's rigid-body row og0
    // + a nl + l, its actor-root row or0 + a (k_artic_chain<..., AFF>)
    int          out_aff, og0, or0;
    int          tmpl;        // template id handled by this launch
    int          nl, ndof;    // links / dofs of the template
    int          nbl;         // bodies of the template (nl minus virtual links; Jacobian rows)
    int          fixed_base;
    int          chain;       // fixed base, link l's parent l - 1 and DOF l - 1 (k_artic_chain)
    const float* link_f;      // [nl][16] template link constants
    const int*   link_i;      // [nl][4]
    float*       state;       // [13][nb]  link states (root = primary, others FK output)
    const float* mass;        // [12][nb]
    const int*   body_tmpl;
    const float* tbf;
    float*       dof_pos;     // [nd]
    float*       dof_vel;     // [nd]
    const float* dof_tpos;    // [nd]
    const float* dof_tvel;    // [nd]
    const float* dof_force;   // [nd]
    // fused DOF target sets (migym_capi.cpp): dof_* then point at the user's
    // tensors and each lane writes the value it read through to the sim's own
    // column (null: not fused)
    float*       tpos_w;
    float*       tvel_w;
    float*       force_w;
    const float* dof_props;   // [12][nd]
    const float* ext;         // [6][nb] or null
    float*       cforce;      // [3][nb]
    // k_artic_chain: the launch's shared constants (MG_CHAIN_UNI_N floats,
    // mg_chainlink.h) when every instance has the same DOF properties, link mass
    // rows and gravity flag, else null
    const float* uni;
    // refresh fused into the step (MG_FUSE_STEP_OUT, k_artic_chain): the bound
    // tensors the kernel writes itself, or null
    float*       out_rb;      // [nb][13] rigid-body tensor (global body order)
    float*       out_root;    // [na][13] actor root tensor
    float*       out_dof;     // [nd][2] DOF state tensor
    const int*   out_body;    // [nb] internal slot -> global body
    const int*   out_root_row;// [nb] internal slot -> actor row (-1: not a root)
};

// Coupled per-env step (mg_env.hip): MG_ENV_G lanes per env, one lane per
// generalized-velocity slot (articulation DOFs first, then, for a floating
// base, the root's spatial velocity (w, v at the base origin), then 6 per free
// body), so D + 6 fb + 6 nf <= MG_ENV_G. env_i rows (MG_ENV_I_N int32):
//   [0] first internal body of the env's articulation or -1, [1] its first DOF,
//   [2] free bodies nf <= MG_ENV_MAXF, [3..6] their internal slots,
//   [7] static bodies ns <= MG_ENV_MAXS, [8..11] their internal slots,
//   [12] collision mask: bit k art-free k, 4+s art-static s, 8+p free pair p
//        ((0,1),(0,2),(0,3),(1,2),(1,3),(2,3)), 14+4k+s free k-static s,
//   [13] articulation template or -1, [14] first pair, [15] pair count.
// Pairs ([4] int32): a, shape of a, b, shape of b (-1: ground). Participants:
// link l = l (link 0, the fixed base, only as b), free body k = MG_ENV_FREE0 + k,
// static body s = MG_ENV_STATIC0 + s, ground = -1.
#define MG_ENV_I_N    16
#define MG_ENV_G      16     // lanes per env (envs of more links / slots: 64, one per wavefront)
#define MG_ENV_SLOTS_WIDE 32 // velocity slots of a 64-lane env (its M_eff solve)
#define MG_ENV_MAXF    2
#define MG_ENV_MAXS    4
#define MG_ENV_MAXCT  16     // contacts per env per substep
#define MG_ENV_MAXCT_WIDE 48 // ... in a 64-lane env
#define MG_ENV_FREE0  64     // participant ids: links 0..MG_MAX_LINKS-1 below
#define MG_ENV_STATIC0 80
#define MG_ENV_LIMIT0 128     // joint-limit row of DOF d: a = MG_ENV_LIMIT0 + d, b = +1 lower / -1 upper

// Friction patches of the coupled step (mg_env.hip): one
// record per candidate shape pair (global pair index), MG_FP_N floats: anchor
// count, the patch normal in A's body frame, then per anchor its point in A's
// and in B's body frame; an env's pairs 0..MG_FP_MAXP-1 keep theirs across
// substeps and steps (bit set in the env's MG_FP_W-word mask), later pairs
// re-anchor every substep.
#define MG_FP_N 16
#define MG_FP_W 4
#define MG_FP_MAXP (32 * MG_FP_W)
#define MG_FP_NORMAL_COS 0.999f
#define MG_OBB_N 8   // shape_obb record: centre[3], half extents[3], pad[2]
struct MgEnvArgs {
    int          ne;          // envs in this launch
    int          nb, nd;
    const int*   env_i;       // [ne][MG_ENV_I_N]
    const int*   pairs;       // [..][4] candidate shape pairs (env_i[14], [15])
    int          nl, ndof;    // articulation template of this launch (0 links: none)
    int          floating;    // the template has a floating base: 6 root velocity slots after the DOFs
    int          max_free;    // most free bodies of one env in this launch (6 velocity slots each)
    const float* link_f;
    const int*   link_i;
    float*       state;
    const float* mass;
    const int*   body_tmpl;
    const float* tbf;
    const int*   tbi;
    const float* shapes;
    const float* hulls;       // convex hull records (MG_SHAPE_CONVEX)
    const float* shape_obb;   // [num_shapes][MG_OBB_N] shape-frame box: centre, half extents (pair screen)
    float*       fpatch;      // [num pairs][MG_FP_N] friction patch records (persistent)
    unsigned*    fp_mask;     // [ne][MG_FP_W] pairs whose record holds a patch (persistent)
    float*       dof_pos;
    float*       dof_vel;
    const float* dof_tpos;
    const float* dof_tvel;
    const float* dof_force;
    float*       tpos_w;      // fused DOF target sets: write-through (MgArticArgs)
    float*       tvel_w;
    float*       force_w;
    const float* dof_props;
    const float* ext;
    float*       cforce;
    // one substep per launch pair (mg_env.hip k_env_np + k_env_step)
    int          sub, last;   // this launch's substep; 1: the frame's last
    float*       carry;       // [ne][carry] the step's state between its substep launches
    int          nhull, nshape;   // floats of the hull table, shape records (k_env_np's LDS staging)
    float*       ctab;        // [ne][ctab] this substep's contacts and anchors (k_env_np -> k_env_step)
};

// Free-body pile step (mg_pile.hip): a coupled env with more
// than MG_ENV_MAXF free bodies and no articulation, one wavefront per env, lane
// k = free body k. pile_i rows (MG_PILE_I_N int32): [0] first entry of the env's
// free bodies in pile_body (internal slots), [1] their count nb <= MG_PILE_MAXB,
// [2] first candidate pair, [3] pair count, [4] static bodies ns <= MG_ENV_MAXS,
// [5..8] their internal slots, [9] first entry of its local shape slots in
// `slots`, [10] their count <= MG_PILE_MAXSH. A local shape slot ([2] int32):
// participant (free body k, or MG_PILE_ST0 + static body s), shape record —
// the free bodies' shapes in body order, then the static bodies'. A candidate
// pair (uint32): local slot of A | local slot of B << 8 (MG_PILE_GROUND: the
// ground plane), in the oracle's pair order. Envs built alike share their slot
// table and pair list.
#define MG_PILE_I_N      12
#define MG_PILE_MAXB     64
#define MG_PILE_ST0      64
#define MG_PILE_MAXAP    128     // active pairs (with contacts) per substep
#define MG_PILE_MAXPT    256     // contact points per substep
#define MG_PILE_MAXPAIRS 8192    // candidate shape pairs per env
#define MG_PILE_MAXSH    128     // local shape slots per env
#define MG_PILE_GROUND   255
struct MgPileArgs {
    int          ne;          // pile envs
    int          nb;          // SoA stride
    const int*   pile_i;      // [ne][MG_PILE_I_N]
    const int*   pile_body;   // free bodies' internal slots
    const unsigned* pairs;    // packed candidate pairs
    const int*   slots;       // [..][2] local shape slots
    float*       state;
    const float* mass;
    const int*   body_tmpl;
    const float* tbf;
    const float* shapes;
    const float* hulls;
    const float* shape_obb;   // [num_shapes][MG_OBB_N] (pair screen)
    const float* ext;         // [6][nb] or null
    float*       cforce;      // [3][nb]
};

// Camera render (mg_render.hip). One device record per camera; a camera's
// pixels are cut into linear runs of MG_RENDER_RUN pixels (row-major), one run
// per workgroup; blk0 = first workgroup of the camera (prefix over cameras).
#define MG_RENDER_LANE_PX 4                      // pixels per lane per pass (one 16-B store)
#define MG_RENDER_PASSES  16                     // passes per wave
#define MG_RENDER_WAVES   4                      // waves per workgroup
#define MG_RENDER_RUN (64 * MG_RENDER_LANE_PX * MG_RENDER_PASSES * MG_RENDER_WAVES)   // 16384 px
struct MgRenderCam {
    int   env, w, h, slot;         // slot: internal body slot followed, -1 fixed
    int   follow, blk0, nblk, vec; // vec: 16-B stores allowed (W*H % 4 == 0 and aligned images)
    float fx, fy, cx, cy, ifx, ify, near_plane, far_plane;
    float p[3], q[4];
    float pad;
    unsigned char* color;
    float* depth;
    int* seg;
};
// render shape reference: one per shape of every body, grouped by env
struct MgRShape {
    int   slot;                    // internal body slot
    int   shape;                   // shape record (MG_SHAPE_STRIDE floats)
    int   seg;
    float r, g, b;
    int   pad[2];
};
struct MgRenderArgs {
    int                 ncam, nb;
    int                 uniform_nblk;      // > 0: every camera has this many runs (camera = block / uniform_nblk)
    const MgRenderCam*  cams;
    const float*        state;     // snapshot [13][nb]
    const float*        shapes;
    const float*        hulls;
    const MgRShape*     rshapes;
    const int*          env_shape_first;   // [nenv + 1]
    int                 has_ground;
    float               gn[3], gpd;        // ground: dot(gn, x) + gpd = 0
    float               fwd[3], up[3], left[3];   // camera-frame view / up / left axes (local)
    int                 up_axis;           // 1: checker on (x, y); 0: on (x, z)
    float               light[3];          // unit direction towards the light
    float               lcol[3], lamb[3];  // light colour and ambient per channel (mg_set_light)
};

// Kernel timing by dispatch timestamps: while mg_timer is set (by mg_simulate,
// outside stream capture) every step kernel is launched with
// hipExtLaunchKernelGGL and a (start, stop) event pair from the timer, whose
// elapsed time is the kernel's own duration (the same begin / end the
// profiler reports), not the launch overhead around it.
struct MgKernelTimer {
    hipEvent_t* start;
    hipEvent_t* stop;
    int cap, used;
    int missed;   // launches past `cap`, run untimed (mg_step_untimed_launches)
};
extern thread_local MgKernelTimer* mg_timer;
#define MG_LAUNCH(kernel, grid, block, shmem, stream, ...)                                               \
    do {                                                                                                \
        MgKernelTimer* t_ = mg_timer;                                                                   \
        if (t_ && t_->used < t_->cap) {                                                                 \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, t_->start[t_->used],                \
                                  t_->stop[t_->used], 0, __VA_ARGS__);                                  \
            t_->used++;                                                                                 \
        } else {                                                                                        \
            if (t_) t_->missed++;                                                                       \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                        \
        }                                                                                               \
    } while (0)

// launchers (defined in the .hip files)
hipError_t mg_launch_render(const MgRenderArgs& A, int nblocks, hipStream_t s);
hipError_t mg_launch_cube_pick(const mg_cube_pick_args& A, hipStream_t s);
hipError_t mg_launch_env_step(const MgStep& P, const MgEnvArgs& A, hipStream_t s);
hipError_t mg_launch_pile_step(const MgStep& P, const MgPileArgs& A, hipStream_t s);
extern "C" int mg_env_carry_floats(void);   // per-env record sizes of the coupled step (mg_env.hip)
extern "C" int mg_env_ctab_floats(void);
int mg_env_ctab_record_floats(int wide);   // one env's contact table in a 16- / 64-lane group
hipError_t mg_launch_rigid_step(const MgStep& P, const MgRigidArgs& A, hipStream_t s);
hipError_t mg_launch_artic_step(const MgStep& P, const MgArticArgs& A, hipStream_t s);
hipError_t mg_launch_artic_lanes(const MgStep& P, const MgArticArgs& A, hipStream_t s);
hipError_t mg_launch_artic_chain(const MgStep& P, const MgArticArgs& A, hipStream_t s);
hipError_t mg_launch_gather_rows(const float* soa, int stride, int ncol, const int* ids, int n,
                                 float* aos, hipStream_t s);
hipError_t mg_launch_gather_rb_root(const float* soa, int stride, int ncol, const int* perm, int nb, float* rb,
                                    const int* body_actor, float* root, hipStream_t s);
hipError_t mg_launch_scatter_rows(const float* aos, int ncol, const int* ids, const int* sel,
                                  int n, int nrows, float* soa, int stride, hipStream_t s);
hipError_t mg_launch_scatter_dofs(const float* aos, int ncol, const int* actor_dof, const int* sel,
                                  int nsel, int nactors, int max_dofs, float* const* dst, hipStream_t s);
hipError_t mg_launch_jacobian(const MgArticArgs& A, float* jac, float* mm, hipStream_t s);
