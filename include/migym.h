/*
 * migym.h — C ABI of libmigym.so, the MI355X-native rigid-body engine that sits
 * behind the isaacgym.gymapi / gymtorch tensor API.
 *
 * This is the drop-in boundary of the hot path. The reference
 * binds these operations through Isaac Gym's closed pybind11 module; each entry
 * point below names the reference call site it replaces. The Python mirror
 * (test_isaacgym_amd/gymapi.py) binds them with ctypes; INTEGRATION.md shows the
 * binding stub.
 *
 * Conventions
 *   - plain pointers and sizes only; no torch types cross this boundary;
 *   - every function returns an int status (MG_OK == 0, negative on error) unless
 *     it returns a handle (NULL on failure), like Isaac Gym's creators returning
 *     None; mg_last_error() gives the message;
 *   - `stream` is a hipStream_t passed as void* (0 = the null stream); every
 *     device operation is enqueued on it, so it orders with the caller's torch
 *     work on the same stream;
 *   - `*_host` flags say whether a tensor pointer is host memory (CPU pipeline,
 *     use_gpu_pipeline=False) or device memory (GPU pipeline);
 *   - tensor layouts are those of Isaac Gym's tensor API:
 *       actor root state  (num_actors, 13)  [p.xyz, q.xyzw, v.xyz, w.xyz]
 *       rigid body state  (num_bodies, 13)  same columns
 *       dof state         (num_dofs, 2)     [pos, vel]
 *       net contact force (num_bodies, 3)
 *     rows are env-major, then actor creation order, then body/DOF tree order.
 */
#ifndef MIGYM_H
#define MIGYM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_ABI_VERSION 1

/* status codes */
#define MG_OK              0
#define MG_ERR_ARG        -1
#define MG_ERR_DEVICE     -2
#define MG_ERR_STATE      -3
#define MG_ERR_UNSUPPORTED -4

/* shape record types (mg_model.shapes[i*MG_SHAPE_STRIDE + 0]) */
#define MG_SHAPE_SPHERE   0
#define MG_SHAPE_BOX      1
#define MG_SHAPE_CAPSULE  2
#define MG_SHAPE_CONVEX   3   /* convex hull of a mesh: size[0] = bounding radius about the shape
                                 origin, size[1] = offset of its record in mg_model.hulls */

/* convex hull record (floats, shape-local frame): nv, nf, ne, 0, then nv vertices
 * (x, y, z), then nf face planes (n.x, n.y, n.z, d) with unit outward n and
 * n . x <= d inside, then ne edges (vertex index pairs; ne <= 3 MG_HULL_MAX_VERTS) */
#define MG_HULL_HEADER     4
/* the library's caps are PhysX's convex-mesh cooking limits (255 vertices, 255
 * polygons); the importer reduces a collision mesh to 32 vertices / 64 faces by
 * default (test_isaacgym_amd/_assets.py, MIGYM_HULL_CAPS raises that per mesh).
 * The per-env narrow phase walks a hull's vertices and edges in chunks (32
 * vertices / 96 edges on 16 lanes), so a hull past the importer's default costs
 * more chunks, not a rebuild. */
#define MG_HULL_MAX_VERTS 255
#define MG_HULL_MAX_FACES 255

/* body kinds (mg_model.body_kind) */
#define MG_BODY_FREE      0   /* single-body dynamic actor: free-body kernel */
#define MG_BODY_STATIC    1   /* fixed single-body actor: never integrated */
#define MG_BODY_LINK      2   /* link of an articulation: articulation kernel */

/* joint types (mg_model.tmpl_link_i[l*4 + 1]) — values of gymapi.JointType */
#define MG_JOINT_FIXED     0
#define MG_JOINT_REVOLUTE  1
#define MG_JOINT_PRISMATIC 2
#define MG_JOINT_BALL      3   /* never in tmpl_link_i: packed as three revolute links (tmpl_link_f[10]) */

/* DOF drive modes — values of gymapi.DofDriveMode */
#define MG_DOF_MODE_NONE   0
#define MG_DOF_MODE_POS    1
#define MG_DOF_MODE_VEL    2
#define MG_DOF_MODE_EFFORT 3

/* record strides (floats / int32 per record) */
#define MG_STATE_N        13  /* body/root state columns */
#define MG_MASS_N         12  /* inv_mass, inv_I[3] (principal), iq[4] (principal frame, xyzw), com[3], mass */
#define MG_TBODY_F_N       8  /* lin_damp, ang_damp, max_lin_vel, max_ang_vel, gravity_on, pad[3] */
#define MG_TBODY_I_N       4  /* shape_start, shape_count, pad, pad */
#define MG_SHAPE_STRIDE   16  /* type, size[3], p[3], q[4], friction, restitution, pad[3] */
#define MG_DOFPROP_N      12  /* mode, kp, kd, effort, max_vel, lower, upper, has_limits, armature, friction, pad[2] */
#define MG_LINK_F_N       16  /* joint origin p[3], q[4] (parent link frame), axis[3] (joint frame),
                                  ball place [1] (0: none, 1..3: a ball joint's links), pad[5] */
/* parent (local, -1 root), joint type, dof (local, -1 none), body (local body index of the
 * link, -1 for a virtual link). Kernel links drive at most one DOF each: a spherical
 * (JOINT_BALL) joint is packed as three revolute links about the joint frame's x, y, z
 * axes, the first two virtual (no body, no mass: test13_camera_spherical_joint.py's
 * dof_spherical_joint_test.urdf), marked by tmpl_link_f[10] = 1, 2, 3: its DOF
 * positions are the rotation vector of the joint (exponential coordinates, test13
 * quat2expcoord), the first link turning by exp of all three and the other two not at
 * all, so the three rates are the child frame's angular velocity; an MJCF body with
 * several hinges is likewise one virtual link per extra hinge. Real links carry body
 * indices 0, 1, 2, ... in link order. */
#define MG_LINK_I_N        4
#define MG_ARTIC_I_N       4  /* first_body, first_dof, tmpl, pad */
/* first_link (into tmpl_link_*), num_links, num_dofs, fixed_base. fixed_base 0: a
 * floating base (the root link moves freely, e.g. the MJCF ant of
 * examples/apply_forces.py:67); such an articulation steps in the coupled per-env
 * kernel (needs actor_coll) with num_dofs + 6 (+ 6 per free body of its env) <= 16
 * velocity slots; its Jacobian / mass-matrix tensors put the 6 root columns first. */
#define MG_ATMPL_I_N       4
#define MG_ACOLL_N         4  /* env, collision group, collision filter, pad */
#define MG_RENDER_MAX_SHAPES 64 /* shapes one camera's env may hold */

/* Simulation parameters: gymapi.SimParams + PhysXParams + the ground plane
 * (reference: test10_servo_vecenv.py:117-144 and :198-206). */
typedef struct mg_sim_params {
    float   dt;                         /* SimParams.dt */
    int32_t substeps;                   /* SimParams.substeps */
    float   gravity[3];                 /* SimParams.gravity */
    int32_t up_axis;                    /* 0 = Y, 1 = Z */
    int32_t num_position_iterations;    /* PhysXParams.num_position_iterations */
    int32_t num_velocity_iterations;    /* PhysXParams.num_velocity_iterations */
    float   contact_offset;             /* PhysXParams.contact_offset */
    float   rest_offset;                /* PhysXParams.rest_offset */
    float   bounce_threshold_velocity;  /* PhysXParams.bounce_threshold_velocity */
    float   max_depenetration_velocity; /* PhysXParams.max_depenetration_velocity */
    int32_t has_ground;                 /* gym.add_ground called */
    float   ground_normal[3];           /* PlaneParams.normal (normalised) */
    float   ground_distance;            /* plane: dot(n, x) + distance = 0 */
    float   ground_static_friction;
    float   ground_dynamic_friction;
    float   ground_restitution;
    float   friction_offset_threshold;      /* PhysXParams.friction_offset_threshold: contacts farther apart
                                               than this do not seed friction anchors */
    float   friction_correlation_distance;  /* PhysXParams.friction_correlation_distance: anchor spacing and
                                               the drift at which an anchor is dropped */
    int32_t reserved[6];
} mg_sim_params;

/* The packed scene, built by the host scene builder at prepare_sim / first
 * tensor access (reference: create_env/create_actor, test10_servo_vecenv.py:
 * 300-323; indexing semantics SURVEY.md §8a rows a2-a5). All pointers are host
 * memory; mg_upload_model copies them to HBM. */
typedef struct mg_model {
    int32_t num_envs, num_actors, num_bodies, num_dofs;
    int32_t num_tmpl_bodies, num_shapes;
    int32_t num_artics, num_artic_tmpls, num_tmpl_links;
    int32_t num_hull_floats;      /* length of `hulls` */
    int32_t reserved_i[6];

    const float*   body_state0;   /* [num_bodies][13] initial state, AoS */
    const float*   body_mass;     /* [num_bodies][MG_MASS_N] */
    const int32_t* body_kind;     /* [num_bodies] MG_BODY_* */
    const int32_t* body_tmpl;     /* [num_bodies] index into tmpl_body_* */
    const float*   tmpl_body_f;   /* [num_tmpl_bodies][MG_TBODY_F_N] */
    const int32_t* tmpl_body_i;   /* [num_tmpl_bodies][MG_TBODY_I_N] */
    const float*   shapes;        /* [num_shapes][MG_SHAPE_STRIDE] */
    const int32_t* actor_root_body; /* [num_actors] global body index of each actor's root */
    const int32_t* actor_dof;     /* [num_actors+1] first global DOF of each actor (CSR) */

    const float*   dof_state0;    /* [num_dofs][2] */
    const float*   dof_props;     /* [num_dofs][MG_DOFPROP_N] */
    const int32_t* artic_i;       /* [num_artics][MG_ARTIC_I_N] */
    const int32_t* artic_tmpl_i;  /* [num_artic_tmpls][MG_ATMPL_I_N] */
    const float*   tmpl_link_f;   /* [num_tmpl_links][MG_LINK_F_N] */
    const int32_t* tmpl_link_i;   /* [num_tmpl_links][MG_LINK_I_N] */
    /* [num_actors][MG_ACOLL_N]: env, collision group, collision filter, pad
     * (create_actor's group / filter, test10_servo_vecenv.py:317,323). Two actors
     * of an env collide when (group_a == group_b or either is -1) and
     * (filter_a & filter_b) == 0; the ground collides with everything. NULL: no
     * body-body contacts (every env steps in the uncoupled kernels). */
    const int32_t* actor_coll;
    /* convex hull records (MG_SHAPE_CONVEX shapes point into it), or NULL */
    const float*   hulls;
    const void*    reserved_p[1];
} mg_model;

typedef struct mg_sim mg_sim;

/* ---- library / device ---------------------------------------------------- */
int32_t     mg_abi_version(void);
const char* mg_last_error(void);
int32_t     mg_device_count(void);           /* HIP devices visible; 0 on a host without a GPU */

/* ---- sim lifetime ---------------------------------------------------------
 * gym.create_sim (test10_servo_vecenv.py:185) / gym.destroy_sim (:474).
 * Returns NULL when no HIP device is usable — the Python layer then returns
 * None, as Isaac Gym does (:187-189). */
mg_sim*     mg_create_sim(int32_t device, const mg_sim_params* params);
void        mg_destroy_sim(mg_sim* sim);
int32_t     mg_set_sim_params(mg_sim* sim, const mg_sim_params* params);
/* gym.prepare_sim (examples/franka_cube_ik_osc.py:288), or the lazy first
 * tensor access of test10 (which never calls prepare_sim). */
int32_t     mg_upload_model(mg_sim* sim, const mg_model* model);

/* ---- stepping --------------------------------------------------------------
 * gym.simulate(sim) (test10_servo_vecenv.py:380): one frame of dt as
 * `substeps` TGS substeps, one fused kernel per body class. Asynchronous. */
int32_t     mg_simulate(mg_sim* sim, void* stream);
/* gym.fetch_results(sim, wait) (:381): waits for the last simulate when wait. */
int32_t     mg_fetch_results(mg_sim* sim, int32_t wait);
/* gym.fetch_results(sim, True) in the CPU pipeline (test10_servo_vecenv.py:381,
 * host state tensors): waits for the last simulate and copies the current state
 * into one host buffer with a single synchronisation. Layout of dst (tensor row
 * orders): [na][13] actor roots, [nb][13] rigid bodies, [nd][2] DOF states,
 * [nb][3] net contact forces; `parts` bit k asks for part k (0 roots, 1 rigid
 * bodies, 2 DOFs, 3 contact forces; 0: wait only). The refresh_*_tensor calls
 * that follow (:394-396) are then host copies from it while no simulate or state
 * set intervenes (the Python layer tracks that), instead of a device round trip
 * each. Not while the stream is being captured. From the first call on, on a sim
 * whose bodies are all stepped by kernels that write their own rows (as
 * MG_FUSE_STEP_OUT), the step writes root / body / DOF rows into the sim's own
 * device copy of this layout, and a fetch after a simulate with no state set
 * since copies those parts without gathering them. */
int32_t     mg_fetch_host_state(mg_sim* sim, float* dst, int32_t parts, void* stream);
/* The sim's own host stage for mg_fetch_host_state: nfloat floats of page-locked
 * host memory mapped into the device's address space, owned by the sim (freed by
 * mg_destroy_sim; a larger request replaces it). Passed as mg_fetch_host_state's
 * dst, the fetch is zero-copy: the step kernels write their rows into it over
 * PCIe and the remaining parts are gathered straight into it — no device-to-host
 * copy. NULL on failure (mg_last_error). */
float*      mg_host_stage(mg_sim* sim, int64_t nfloat);

/* ---- tensor API: refresh (state -> user tensor) ----------------------------
 * gym.refresh_actor_root_state_tensor (:394), refresh_rigid_body_state_tensor
 * (:395), refresh_dof_state_tensor (:396), refresh_net_contact_force_tensor
 * (test12_add_joint.py.py:131). `dst` is the persistent tensor handed out by
 * acquire_*; a host dst is written synchronously. */
int32_t     mg_refresh_actor_root_state(mg_sim* sim, float* dst, int32_t dst_host, void* stream);
int32_t     mg_refresh_rigid_body_state(mg_sim* sim, float* dst, int32_t dst_host, void* stream);
int32_t     mg_refresh_dof_state(mg_sim* sim, float* dst, int32_t dst_host, void* stream);
int32_t     mg_refresh_net_contact_force(mg_sim* sim, float* dst, int32_t dst_host, void* stream);

/* ---- tensor API: set (user tensor -> state, applied at the next simulate) --
 * gym.set_actor_root_state_tensor (test10_servo_vecenv.py:456) and the
 * _indexed variant: `src` is (num_actors, 13); when `idx` is non-NULL only the
 * n_idx actor rows it lists are applied (idx is int32, host or device like src).
 * src is consumed in stream order, so the caller may reuse it right away
 * (Isaac Gym's copy-at-set contract, SURVEY.md §8b Ownership) — except for the
 * fused root set (mg_set_fusion, MG_FUSE_ROOT_SET, opt-in, off by default): a
 * device-resident, non-indexed set on a sim whose actor roots are
 * all single-shape free bodies is read by the next mg_simulate's free-body
 * kernel (the scatter fused into the step), or by the scatter that any earlier
 * call reading the state issues first (refresh_*, set_rigid_body_state, an
 * indexed or host set, the render snapshot). The caller keeps such a src alive
 * and unmodified until then (the gymapi layer holds the tensor). A host source
 * (src_host) is copied at the call into the sim's page-locked buffer, so it may
 * be overwritten at once; a full host set on such a sim is then read by the
 * next mg_simulate's step kernel too (no scatter launch). */
int32_t     mg_set_actor_root_state(mg_sim* sim, const float* src, int32_t src_host,
                                    const int32_t* idx, int32_t n_idx, void* stream);
/* gym.set_rigid_body_state_tensor (test/test05_isaacgym_vel_batch.py:367-385):
 * free bodies only (articulation links follow their joints). */
int32_t     mg_set_rigid_body_state(mg_sim* sim, const float* src, int32_t src_host, void* stream);
/* gym.set_dof_state_tensor[_indexed], set_dof_position_target_tensor,
 * set_dof_velocity_target_tensor, set_dof_actuation_force_tensor
 * (examples/franka_cube_ik_osc.py:409-410). idx lists actor indices. */
int32_t     mg_set_dof_state(mg_sim* sim, const float* src, int32_t src_host,
                             const int32_t* idx, int32_t n_idx, void* stream);
int32_t     mg_set_dof_position_target(mg_sim* sim, const float* src, int32_t src_host,
                                       const int32_t* idx, int32_t n_idx, void* stream);
int32_t     mg_set_dof_velocity_target(mg_sim* sim, const float* src, int32_t src_host,
                                       const int32_t* idx, int32_t n_idx, void* stream);
int32_t     mg_set_dof_actuation_force(mg_sim* sim, const float* src, int32_t src_host,
                                       const int32_t* idx, int32_t n_idx, void* stream);
/* DOF drive properties of every DOF, [num_dofs][MG_DOFPROP_N] host array
 * (gym.set_actor_dof_properties after prepare_sim). */
int32_t     mg_set_dof_props(mg_sim* sim, const float* props_host);
/* gym.apply_rigid_body_force_tensors(sim, forces, torques, space): (num_bodies,3)
 * each or NULL; space 0 = global (ENV_SPACE/GLOBAL), 1 = local (LOCAL_SPACE).
 * Applied at the body's centre of mass during the next simulate only. */
int32_t     mg_apply_rigid_body_force(mg_sim* sim, const float* force, const float* torque,
                                      int32_t space, int32_t src_host, void* stream);

/* ---- Jacobian / mass matrix (examples/franka_cube_ik_osc.py:305-316,345-346) */
/* For the articulation template `tmpl` (instances in actor order), fixed base:
 * Jacobian (instances, L-1, 6, D) — link 1..L-1, rows [linear velocity of the
 * link frame origin; angular velocity] in the world frame, one column per DOF;
 * mass matrix (instances, D, D) — joint-space inertia by the composite-rigid-
 * body algorithm, joint armature not included. Floating base (D + 6 <= 32):
 * six root columns first (linear velocity of the base-link origin, then
 * angular velocity, world axes), Jacobian (instances, L, 6, D + 6) over every
 * link, mass matrix (instances, D + 6, D + 6). At the current state. */
int32_t     mg_refresh_jacobian(mg_sim* sim, int32_t tmpl, float* dst, int32_t dst_host, void* stream);
int32_t     mg_refresh_mass_matrix(mg_sim* sim, int32_t tmpl, float* dst, int32_t dst_host, void* stream);
/* Both in one launch (one forward-kinematics pass): refresh_jacobian_tensors
 * followed by refresh_mass_matrix_tensors at the same state. Either pointer may
 * be NULL; both are device memory, or both host memory when dst_host. */
int32_t     mg_refresh_jacobian_mass_matrix(mg_sim* sim, int32_t tmpl, float* jac, float* mm, int32_t dst_host,
                                            void* stream);

/* ---- camera sensors (config 5: test11_servo_vecenv_camerazoom.py:327-342,388,
 * 458-460; examples/interop_torch.py:105-120,173-174) ------------------------
 * A camera sees its own env's bodies and the ground plane (what Isaac Gym's
 * camera sensors show: examples/interop_images/ holds no neighbouring env's ball,
 * DESIGN.md §3.8). Images are ray cast on the device:
 *   color (H, W, 4) RGBA8, depth (H, W) float32 = -(distance along the view
 *   axis), -inf where nothing is hit, segmentation (H, W) int32 = the body's
 *   segmentation id, 0 for ground and sky.
 * Camera frame: looks along its local +x with the sim's up axis (+z, or +y for
 * UP_AXIS_Y) as image up; pixel (c, r) is the ray f + a l + b u with
 * a = (cx - c - 0.5) / fx, b = (cy - r - 0.5) / fy. */
typedef struct mg_camera {
    int32_t  env;            /* env index: the scene is that env's bodies + ground */
    int32_t  width, height;
    int32_t  body;           /* global rigid-body index the camera is attached to, -1: fixed */
    int32_t  follow;         /* gymapi.CameraFollowMode: 0 FOLLOW_POSITION, 1 FOLLOW_TRANSFORM */
    float    fx, fy, cx, cy; /* pinhole intrinsics in pixels */
    float    near_plane, far_plane;
    float    p[3], q[4];     /* attached: pose in the body frame; fixed: world pose */
    int32_t  reserved;
    uint8_t* color;          /* device (H, W, 4) or NULL (not rendered) */
    float*   depth;          /* device (H, W) or NULL */
    int32_t* seg;            /* device (H, W) or NULL */
} mg_camera;

/* What the renderer draws per body: env_body_first [num_envs + 1] (global body
 * ranges of each env, CSR), color [num_bodies][3] in 0..1 (set_rigid_body_color),
 * seg [num_bodies] (segmentation ids). Host arrays; may be called again. */
int32_t     mg_set_render_bodies(mg_sim* sim, const int32_t* env_body_first, const float* color,
                                 const int32_t* seg);
/* gym.render_all_camera_sensors: freeze the body poses the cameras see (a device
 * copy of the state, in stream order); later renders use this snapshot. */
int32_t     mg_snapshot_render_state(mg_sim* sim, void* stream);
/* Render `n` cameras (host array) from the snapshot into their device images,
 * one launch. The camera table is uploaded when it changes (not allowed while
 * the stream is being captured into a graph). */
int32_t     mg_render_cameras(mg_sim* sim, const mg_camera* cams, int32_t n, void* stream);
/* Duration in ms of the last mg_render_cameras launch (HIP events), -1 if none. */
float       mg_last_render_ms(mg_sim* sim);
/* gym.set_light_parameters(sim, 0, intensity, ambient, direction)
 * (examples/domain_randomization.py:186): the directional light of later renders.
 * A body's colour c is drawn as c * (ambient + color * max(n . dir, 0)) per
 * channel (c * ambient in shadow); dir points towards the light (normalised
 * here). NULL restores the default: ambient 0.3, color 0.7, dir (0.3, 0.2, 1)
 * z-up / (0.3, 1, 0.2) y-up. The checker ground keeps its fixed colours. */
typedef struct mg_light {
    float dir[3];
    float color[3];
    float ambient[3];
} mg_light;
int32_t     mg_set_light(mg_sim* sim, const mg_light* light);

/* ---- step fusion ------------------------------------------------------------
 * MG_FUSE_ROOT_SET: the deferred root-state set described above.
 * MG_FUSE_DOF_TARGETS: a device-resident, non-indexed mg_set_dof_position_target /
 * _velocity_target / _actuation_force is read by the next mg_simulate's
 * articulation kernels (which write it through to the sim's own targets) instead
 * of a copy launch; the caller keeps src alive and unmodified until then (an
 * indexed or host set of the same column applies it first).
 * MG_FUSE_REFRESH: with targets bound by mg_bind_refresh_targets (the persistent
 * tensors acquire_actor_root_state_tensor / acquire_rigid_body_state_tensor hand
 * out), a root refresh into the bound root tensor also writes the bound
 * rigid-body tensor (one gather launch for test10_servo_vecenv.py:394-395), and
 * a rigid-body refresh into it is then served without a launch while no
 * simulate or set has changed the state. The bound rigid-body tensor is thus
 * refreshed no later than requested (possibly at the root refresh).
 * mg_set_fusion returns the previous flags. Every fusion is OFF by default:
 * with it on, a set source is read after the set call and a rigid-body tensor
 * may be refreshed early, which departs from Isaac Gym's tensor contract; the
 * gymapi layer (gym.set_step_fusion) checks the sources' torch version counters
 * and raises rather than read a source written after its set. The bound
 * pointers must stay valid for the sim's lifetime (NULL unbinds). */
#define MG_FUSE_ROOT_SET  1
#define MG_FUSE_REFRESH   2
#define MG_FUSE_DOF_TARGETS 4
/* MG_FUSE_IN_CAPTURE (opt-in): the fusions above also inside a stream capture
 * (hipGraph). Without it a captured set is an ordinary launch and a captured
 * rigid-body refresh is never skipped, so any captured region replays right; with
 * it the caller guarantees every captured set is consumed by a simulate in the
 * same capture (e.g. set -> simulate -> refresh per captured step, as bench.py). */
#define MG_FUSE_IN_CAPTURE  8
/* MG_FUSE_STEP_OUT: with targets bound by mg_bind_refresh_targets /
 * mg_bind_dof_refresh_target, on a sim whose bodies are all stepped by kernels
 * that write their own rows (mg_step_out_supported: single-shape free bodies —
 * the servo scene — and fixed-base serial chains of 2..4 links that touch
 * nothing — the S2 gimbal), mg_simulate's step kernels write the new state into
 * the bound root, rigid-body and DOF-state tensors themselves, and a refresh of
 * a bound tensor is then served without a launch while no set has changed the
 * state (the refresh fused into the step). The bound tensors thus hold the new
 * state from the simulate on, not from the refresh; the gymapi layer rebinds
 * (forcing a gather) when a bound tensor was written between the simulate and
 * its refresh. */
#define MG_FUSE_STEP_OUT    16
int32_t     mg_set_fusion(mg_sim* sim, int32_t flags);
/* replaces gym.acquire_actor_root_state_tensor / acquire_rigid_body_state_tensor's
 * persistent buffers as refresh targets (test10_servo_vecenv.py:372-374,394-395) */
int32_t     mg_bind_refresh_targets(mg_sim* sim, float* root_dst, float* rigid_body_dst);
/* the persistent DOF-state tensor of gym.acquire_dof_state_tensor
 * (test12_add_joint.py.py:129; test13_camera_spherical_joint.py:266-269) as the
 * target MG_FUSE_STEP_OUT writes; NULL unbinds */
int32_t     mg_bind_dof_refresh_target(mg_sim* sim, float* dof_dst);
/* 1 when every body of the uploaded model is stepped by a kernel that writes its
 * own refresh rows (MG_FUSE_STEP_OUT applies), else 0 */
int32_t     mg_step_out_supported(mg_sim* sim);
/* 1 when the last mg_set_actor_root_state / mg_set_dof_*_target /
 * mg_set_dof_actuation_force call deferred its read of the source to the next
 * mg_simulate (MG_FUSE_ROOT_SET / MG_FUSE_DOF_TARGETS), 0 when it copied it
 * during the call (Isaac Gym's copy-at-set) */
int32_t     mg_last_set_deferred(mg_sim* sim);
/* drop the deferred sets not yet read (the gymapi layer, when a deferred set's
 * source was written before the simulate that would read it: it raises, and the
 * set is not applied with data newer than the set call) */
int32_t     mg_discard_pending_sets(mg_sim* sim);

/* ---- introspection for tests and the bench ------------------------------- */
/* Kernel timing is opt-in (default off): while on, every eager simulate() and
 * render launches its kernels with dispatch-timestamp events (hipExtLaunch-
 * KernelGGL start / stop) and records begin / end events; while off, simulate
 * enqueues only its kernels and fetch_results(wait) synchronises the stream.
 * Stream capture never records events. Returns the previous setting. */
int32_t     mg_set_kernel_timing(mg_sim* sim, int32_t on);
/* Duration in ms of the last timed simulate()'s kernels (HIP events on `stream`),
 * -1 when unavailable. Synchronises on the step's end event. */
float       mg_last_step_ms(mg_sim* sim);
/* Average / min / max over the last n simulate() calls (at most 256; eager
 * calls only, not graph replays) of the summed duration in ms of that step's
 * kernels, each taken from its own dispatch timestamps (hipExtLaunchKernelGGL
 * start / stop events, the interval rocprofv3 reports for the kernel). Returns
 * the count used, or < 0. */
int32_t     mg_step_time_stats(mg_sim* sim, int32_t n, float* avg_ms, float* min_ms, float* max_ms);
/* Replaces no reference interface (diagnostics of this build): how many kernel
 * launches the most launch-heavy of the last n timed simulate() calls (at most
 * 256) made past the timer's slots — launches run untimed, whose durations
 * mg_step_time_stats' sums leave out (0: every kernel was timed). Or < 0. */
int32_t     mg_step_untimed_launches(mg_sim* sim, int32_t n);
/* Diagnostics: coupled env k's contact table (k = the k-th coupled env in env
 * order; in the Franka scene every env is coupled, so k is the env index) as
 * the narrow-phase launch k_env_np handed it to k_env_step in the last substep
 * run: 8 header floats ([0] contacts, [1] anchors, ints by bit pattern), MAXCT
 * contact records of 10 floats (participant a, b as int bits, point, normal,
 * separation, restitution), MAXCT anchor records of 14 floats, MAXCT 16 in a
 * 16-lane group and 48 in a 64-lane group. Copies into dst (cap floats at
 * least the record) and returns the record's length in floats, 8 + 24 MAXCT;
 * synchronises the device. < 0 on error. */
int32_t     mg_debug_copy_env_ctab(mg_sim* sim, int32_t k, float* dst, int32_t cap);
/* Diagnostics: per articulation group (up to cap / MG_DEBUG_GROUP_N groups)
 * the facts that pick its kernel form (mg_chain.hip): links, instances stepped
 * alone, serial chain, shared link masses (UNI), shared DOF properties, rows
 * affine in the instance (AFF), fused-refresh rows affine, refresh fusion
 * possible for the sim. Returns the number of groups, < 0 on error. */
#define MG_DEBUG_GROUP_N 8
int32_t     mg_debug_artic_groups(mg_sim* sim, int32_t* out, int32_t cap);
int         mg_env_ctab_floats(void);
int         mg_env_carry_floats(void);
/* Number of bodies advanced by the free-body kernel / articulations by the
 * articulation kernel in one simulate. */
int32_t     mg_num_free_bodies(mg_sim* sim);
int32_t     mg_num_articulations(mg_sim* sim);
/* Number of envs stepped by the coupled per-env kernel (envs whose bodies can
 * touch each other under the actor_coll rule, e.g. the Franka cube-pick scene,
 * and every env holding a floating-base articulation). */
int32_t     mg_num_coupled_envs(mg_sim* sim);
/* Number of those stepped as free-body piles (csrc/mg_pile.hip, DESIGN.md
 * §3.10): more than two free bodies, no articulation — the 30-ball pyramid per
 * env of examples/1080_balls_of_solitude.py:96-136. Replaces no reference entry
 * point of its own: gym.simulate (test10_servo_vecenv.py:380) steps them. */
int32_t     mg_num_pile_envs(mg_sim* sim);

/* ---- the S3 cube-pick controller on the device (csrc/mg_ctrl.hip) ----
 * Replaces the per-frame torch controller of examples/franka_cube_ik_osc.py
 * :348-410 (its grasp state machine, control_osc :59-79 / control_ik :51-56
 * and the gripper targets :403-407) for n envs, one launch, reading the sim's
 * own tensors in place: rigid-body rows (13 floats), DOF state rows (pos, vel),
 * the end-effector Jacobian block and the 7x7 mass-matrix block of each env at
 * element strides (a view such as jacobian[:, hand - 1, :, :7] needs no copy).
 * Writes the (n, 9) rows the script hands to set_dof_position_target_tensor /
 * set_dof_actuation_force_tensor: OSC sets effort[:, :7] and pos[:, 7:9], IK
 * pos[:, :9]; other entries are left as they are (the script's zeros). */
typedef struct mg_cube_pick_args {
    int32_t        n;              /* envs */
    int32_t        osc;            /* 1: operational-space control, 0: damped least-squares IK */
    const float*   rb;             /* rigid-body state rows (num_bodies, 13) */
    const int32_t* box_row;        /* (n) rows of the cubes */
    const int32_t* hand_row;       /* (n) rows of the hands */
    const float*   dof;            /* DOF state rows (num_dofs, 2) */
    const int32_t* dof_row0;       /* (n) first of the env's 9 DOF rows */
    const float*   jac;            /* env e's 6 x 7 block: jac[e jac_se + r jac_sr + c jac_sc] */
    int64_t        jac_se, jac_sr, jac_sc;
    const float*   mm;             /* env e's 7 x 7 block, likewise */
    int64_t        mm_se, mm_sr, mm_sc;
    const float*   init_pos;       /* (n, 3) the hands' start positions (:252-253) */
    const float*   init_rot;       /* (n, 4) and orientations */
    const float*   default_dof_pos;/* (9) null-space target (:187-191) */
    uint8_t*       hand_restart;   /* (n) the script's hand_restart flags (kept across frames) */
    float*         pos_action;     /* (n, 9) */
    float*         effort_action;  /* (n, 9) */
    float          kp, kd, kp_null, kd_null, damping, grasp_offset, box_size;
} mg_cube_pick_args;
int32_t     mg_cube_pick_step(const mg_cube_pick_args* args, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MIGYM_H */
