/*
 * leggedsim.h — C ABI of the MI355X-native vectorised legged-robot simulator.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json
 * (`LeggedRobot.step()`: PD -> rigid-body dynamics + contact x decimation ->
 * obs / reward / done / reset).  It replaces two reference interfaces:
 *
 *  (1) the IsaacGym tensor API the env calls:
 *        gym.create_sim / prepare_sim          legged_robot.py:240, base_task.py:56
 *        acquire_*_tensor + wrap_tensor        legged_robot.py:83-92,104-120, h1_env.py:37
 *        refresh_*_tensor                      legged_robot.py:639,678-679, h1_env.py:49
 *        set_dof_actuation_force_tensor        legged_robot.py:629
 *        simulate / fetch_results              legged_robot.py:630,637-638
 *        set_actor_root_state_tensor_indexed   legged_robot.py:553-555,592-594
 *        set_dof_state_tensor_indexed          legged_robot.py:570-572
 *        per-env shape friction / base mass    legged_robot.py:412-440,472-483
 *  (2) the whole control step `LeggedRobot.step` (legged_robot.py:615-647) with
 *      `post_physics_step` (:673-709) fused into ONE launch (lgs_step), so the
 *      Python side keeps the VecEnv contract but issues no per-op kernels and
 *      no device->host syncs (the reference's nonzero() calls at :511,:545,:697
 *      become in-kernel masks).
 *
 * Conventions
 *  - All state / env buffers are DEVICE pointers, fp32, env-major, contiguous:
 *      root_states [N,13] = pos(3) quat xyzw(4) lin vel of the root COM(3) ang vel(3)
 *      dof_state   [N*D,2] = (q, qd)
 *      net_contact_forces [N*B,3]   (from the last substep, like PhysX)
 *      rigid_body_states  [N*B,13]  (origin pos, quat, COM lin vel, ang vel)
 *    The caller owns these buffers and binds them once (lgs_bind_state);
 *    the simulator reads and writes them in place, so refresh_* is a no-op
 *    and a torch tensor view is always current.
 *  - Booleans (reset, time_out, last_contacts) are 1 byte (torch.bool).
 *  - Host-side descriptors (model, params) are copied at call time.
 *  - Every call returns LGS_OK (0) or a negative status; lgs_last_error()
 *    gives a thread-local message.  No call aborts the process.
 *  - Work is enqueued on the stream set with lgs_set_stream (default stream 0);
 *    nothing synchronises the host except lgs_synchronize.  Launches are
 *    hipGraph-capturable (no allocation or sync inside lgs_step/lgs_simulate).
 *  - One host thread per lgs_sim.
 */
#ifndef LEGGEDSIM_H
#define LEGGEDSIM_H

#include <stdint.h>

#ifdef __cplusplus
#define LGS_EXTERN extern "C"
#else
#define LGS_EXTERN
#endif
#define LGS_API LGS_EXTERN __attribute__((visibility("default")))

#define LGS_OK 0
#define LGS_ERR_ARG (-1)
#define LGS_ERR_HIP (-2)
#define LGS_ERR_STATE (-3)

#define LGS_MAX_BODIES 32
#define LGS_MAX_DOFS 26
#define LGS_MAX_DEPTH 10
#define LGS_MAX_FEET 4
#define LGS_MAX_CONTACT_BODIES 16
#define LGS_MAX_OBS 128
#define LGS_MAX_REWARDS 24
#define LGS_MAX_SELF_PROXIES 64
#define LGS_MAX_SELF_PAIRS 192

/* ---- articulated model (host pointers; see leggedsim/model.py) ---------- */
typedef struct lgs_model_desc {
    int32_t num_bodies;       /* B (after fixed-joint collapse)          */
    int32_t num_dofs;         /* D (revolute joints, DFS order)          */
    int32_t num_points;       /* P contact candidate points              */
    const int32_t* parent;    /* [B]  -1 for the floating root            */
    const int32_t* dof;       /* [B]  dof of the joint to the parent or -1 */
    const int32_t* subtree_end; /* [B] subtree(b) = [b, subtree_end[b])    */
    const int32_t* depth;     /* [B]                                     */
    const int32_t* chain;     /* [B][LGS_MAX_DEPTH] root..b, -1 padded    */
    const float* joint_rot;   /* [B][9] parent frame -> joint frame (row-major) */
    const float* joint_pos;   /* [B][3]                                  */
    const float* axis;        /* [B][3] joint axis in the child frame     */
    const float* mass;        /* [B]                                     */
    const float* com;         /* [B][3] body frame                        */
    const float* inertia;     /* [B][6] Ixx Iyy Izz Ixy Ixz Iyz about com  */
    const int32_t* dof_body;  /* [D]                                     */
    const float* dof_lower;   /* [D] URDF limits                          */
    const float* dof_upper;
    const float* dof_effort;
    const float* dof_velocity;
    const int32_t* pt_body;   /* [P]                                     */
    const float* pt_pos;      /* [P][3] body frame                        */
    const float* pt_radius;   /* [P]                                     */
    /* names, copied at lgs_create_sim (get_asset_rigid_body_names / get_asset_dof_names,
     * legged_robot.py:342-343); either may be NULL (the queries then return NULL / -1) */
    const char* const* body_names; /* [B] */
    const char* const* dof_names;  /* [D] */
} lgs_model_desc;

/* ---- simulation parameters: cfg.sim + cfg.sim.physx + cfg.asset
 *      (legged_robot_config.py:131-143, 225-242)                         */
typedef struct lgs_sim_params {
    float dt;                        /* sim.dt (0.005; H1_2 0.0025)        */
    float gravity[3];                /* (0,0,-9.81), z up                  */
    int32_t solver_iterations;       /* contact/limit PGS sweeps per substep */
    float contact_offset;            /* physx.contact_offset  (0.01 m)     */
    float rest_offset;               /* physx.rest_offset     (0.0)        */
    float max_depenetration_velocity;/* physx (1.0 m/s)                    */
    float baumgarte;                 /* penetration fraction corrected per substep */
    float ground_friction;           /* plane static/dynamic friction (1.0), averaged with shape friction */
    float armature;                  /* asset.armature (H1_2: 1e-3)        */
    int32_t clamp_joint_velocity;    /* clamp |qd| to the URDF velocity limit */
    int32_t max_contacts;            /* contact slots per env               */
    int32_t max_rows;                /* constraint rows per env (<= compiled capacity);
                                        joint-limit rows: max_rows - 3*max_contacts, plus the
                                        rows of the contact slots a substep leaves unused */
} lgs_sim_params;
/* Contact slots per substep (PhysX reports every touching shape; a fixed-capacity solver has
 * to choose).  In this order, while slots last:
 *   1. every body touching the ground gets ONE slot, for its first touching candidate point
 *      (candidate order; bodies in the order of those candidates),
 *   2. self contacts (pair order), at most max_self_contacts,
 *   3. the remaining touching ground candidates, in candidate order.
 * So planted feet cannot take the slots of a knee, hip or pelvis on the ground (its contact
 * force, the collision penalty and contact terminations depend on them).  Joint limits take
 * the limit rows in DOF order, then the rows of unused contact slots.  Whatever still does not
 * fit is counted: lgs_get_contact_stats. */

/* ---- self-collision (IsaacGym create_actor collision filter, legged_robot.py:373-374:
 *      cfg.asset.self_collisions == 0 lets the links of one actor collide; see
 *      leggedsim/selfcollision.py).  Every collision shape group is a capsule proxy in its
 *      body frame; the listed proxy pairs (never a body with itself or its parent) are
 *      tested every substep: closest points of the two segments, signed distance minus both
 *      radii and rest_offset, active below contact_offset.  A touching pair is one contact
 *      (normal from the second body to the first, a friction pair, the env's shape friction)
 *      in the slots after the ground contacts; up to max_self_contacts of them per substep,
 *      first in pair order, after one slot per touching ground body (the slot order above).
 *      The contact force joins both bodies' net contact force with opposite signs.      */
typedef struct lgs_self_collision_desc {
    int32_t num_proxies;          /* S <= LGS_MAX_SELF_PROXIES                          */
    const int32_t* proxy_body;    /* [S]                                                */
    const float* capsule;         /* [S][7] segment end points p0, p1 (body frame), radius */
    int32_t num_pairs;            /* Q <= LGS_MAX_SELF_PAIRS; 0 disables self-collision  */
    const int32_t* pair;          /* [Q][2] proxy indices                               */
    int32_t max_self_contacts;    /* contact slots self contacts may take per substep    */
} lgs_self_collision_desc;

/* ---- task (env) parameters: everything post_physics_step reads from cfg ---- */
enum lgs_obs_layout {
    LGS_OBS_QUADRUPED = 0,   /* legged_robot.py:800-807  [v*s, w*s, g, cmd*s, dq, qd*s, a]          */
    LGS_OBS_HUMANOID = 1     /* h1_env.py:68-95 / g1_env.py:108-141  obs=[w,g,cmd,dq,qd,a,sin,cos], priv=[v, obs] */
};

/* reward term ids; the task lists the active ones in alphabetical order
 * (class_to_dict uses dir(), legged_robot.py:822-836)                     */
enum lgs_reward_id {
    LGS_REW_ACTION_RATE = 0, LGS_REW_ALIVE, LGS_REW_ANG_VEL_XY, LGS_REW_BASE_HEIGHT,
    LGS_REW_COLLISION, LGS_REW_CONTACT, LGS_REW_CONTACT_NO_VEL, LGS_REW_DOF_ACC,
    LGS_REW_DOF_POS_LIMITS, LGS_REW_DOF_VEL, LGS_REW_DOF_VEL_LIMITS, LGS_REW_FEET_AIR_TIME,
    LGS_REW_FEET_CONTACT_FORCES, LGS_REW_FEET_STUMBLE, LGS_REW_FEET_SWING_HEIGHT,
    LGS_REW_HIP_POS, LGS_REW_LIN_VEL_Z, LGS_REW_ORIENTATION, LGS_REW_STAND_STILL,
    LGS_REW_TORQUE_LIMITS, LGS_REW_TORQUES, LGS_REW_TRACKING_ANG_VEL, LGS_REW_TRACKING_LIN_VEL,
    LGS_REW_COUNT
};

typedef struct lgs_task_params {
    int32_t obs_layout;            /* lgs_obs_layout                        */
    int32_t num_obs;               /* O                                     */
    int32_t num_privileged_obs;    /* P or 0                                */
    int32_t num_actions;           /* A (== D)                              */
    int32_t decimation;
    int32_t control_type;          /* 0 P, 1 V, 2 T (legged_robot.py:663-670) */
    float action_scale;
    float clip_actions, clip_observations;
    float control_dt;              /* decimation * sim.dt                   */
    float p_gains[LGS_MAX_DOFS], d_gains[LGS_MAX_DOFS];
    float default_dof_pos[LGS_MAX_DOFS];
    float torque_limits[LGS_MAX_DOFS];
    float soft_dof_pos_lower[LGS_MAX_DOFS], soft_dof_pos_upper[LGS_MAX_DOFS];
    float dof_vel_limits[LGS_MAX_DOFS];
    float obs_scale_lin_vel, obs_scale_ang_vel, obs_scale_dof_pos, obs_scale_dof_vel;
    float commands_scale[3];
    int32_t add_noise;
    float noise_vec[LGS_MAX_OBS];
    /* episode / commands / pushes */
    float max_episode_length;      /* ceil(episode_length_s / dt)            */
    float max_episode_length_s;
    int32_t resample_interval;     /* int(resampling_time / dt)              */
    int32_t heading_command;
    float cmd_lin_vel_x[2], cmd_lin_vel_y[2], cmd_ang_vel_yaw[2], cmd_heading[2];
    int32_t push_robots;
    int32_t push_interval;         /* int(ceil(push_interval_s / dt))        */
    float max_push_vel_xy;
    float base_init_state[13];
    /* bodies selected by name substring (legged_robot.py:346-407) */
    int32_t num_feet, feet_idx[LGS_MAX_FEET];
    int32_t num_penalised, penalised_idx[LGS_MAX_CONTACT_BODIES];
    int32_t num_termination, termination_idx[LGS_MAX_CONTACT_BODIES];
    int32_t num_hip, hip_dofs[8];
    /* rewards */
    int32_t num_rewards;
    int32_t reward_ids[LGS_MAX_REWARDS];
    float reward_scales[LGS_MAX_REWARDS];   /* already multiplied by dt      */
    int32_t has_termination_reward;
    float termination_scale;
    int32_t only_positive_rewards;
    float tracking_sigma, base_height_target, max_contact_force;
    float soft_dof_vel_limit, soft_torque_limit;
    /* humanoid gait phase (h1_env.py:55-65) */
    float phase_period, phase_offset, stance_threshold, swing_height_target;
    uint64_t seed;
    /* 1: refresh rigid_body_states [N,B,13] every control step (the humanoid envs
     * read it, h1_env.py:37,49); 0: leave it untouched (LeggedRobot never reads it) */
    int32_t write_body_states;
    /* 1: env origins are terrain tiles (legged_robot.py:582-585, custom_origins): reset_idx adds a
     * U[-1,1] xy offset to the root position (LGS_STREAM_RESET_ROOT draws 6, 7) */
    int32_t custom_origins;
    /* a task's reward terms written in Python (subclass _reward_* methods, legged_robot.py:817-840)
     * run between lgs_post_physics_rewards and lgs_post_physics_finish.  defer_reward_total = 1:
     * the kernel writes the raw sum of its own terms to rew (no only_positive_rewards clip, no
     * termination term; the caller adds its terms, clips and adds the termination term).
     * num_extra_sums: episode-sum rows after the native ones (and termination) that the caller
     * fills; they join the reset-time extras like the native sums. */
    int32_t defer_reward_total;
    int32_t num_extra_sums;
    /* with write_body_states: the bodies whose rigid_body_states rows each step refreshes (bit b =
     * body b; the humanoid tasks: their feet, the only rows h1_env.py:34-52 reads); 0 = every body.
     * lgs_forward_kinematics (refresh_rigid_body_state_tensor) always refreshes every body. */
    uint32_t body_state_mask;
} lgs_task_params;

/* ---- per-env buffers of the VecEnv (device pointers; torch owns them) ---- */
typedef struct lgs_env_buffers {
    float* actions;          /* [N,A] in: raw policy actions; out: clipped env.actions (0 on reset) */
    float* last_actions;     /* [N,A] */
    float* last_dof_vel;     /* [N,D] */
    float* last_root_vel;    /* [N,6] */
    float* torques;          /* [N,D] last substep's torques */
    float* commands;         /* [N,4] */
    float* feet_air_time;    /* [N,F] */
    uint8_t* last_contacts;  /* [N,F] bool */
    int64_t* episode_length; /* [N] */
    float* obs;              /* [N,O] */
    float* priv_obs;         /* [N,P] or NULL */
    float* rew;              /* [N]   */
    uint8_t* reset;          /* [N] bool */
    uint8_t* time_out;       /* [N] bool */
    float* episode_sums;     /* [num_rewards(+1 termination), N] */
    float* episode_acc;      /* [num_sums + 1]: sums over envs reset this step, then the count */
    float* base_lin_vel;     /* [N,3] */
    float* base_ang_vel;     /* [N,3] */
    float* projected_gravity;/* [N,3] */
    float* rpy;              /* [N,3] */
    float* env_origins;      /* [N,3] */
    float* phase;            /* [N]   humanoid, else NULL */
    float* leg_phase;        /* [N,2] humanoid, else NULL */
    float* rew_terms;        /* [num_rewards, N] per-term reward of this step (diagnostics) or NULL */
    int64_t* step_counter;   /* [1] device copy of common_step_counter, or NULL.  When set, lgs_step and
                                lgs_reset_all read the Philox step key from it instead of the by-value
                                argument, and lgs_step advances it by one after the step: a captured
                                hipGraph of K steps then draws fresh noise/commands on every replay. */
    /* extras (legged_robot.py:742-768), refreshed by lgs_step after the step when >= 1 env reset;
       each may be NULL.  lgs_step also zeroes episode_acc for the next step.                      */
    float* ep_means;         /* [num_sums] carried extras["episode"] values (rew_* / max_episode_length_s) */
    float* ep_snapshot;      /* [num_sums] this step's copy of ep_means (the step's extras["episode"]) */
    uint8_t* time_outs_carry;/* [N] extras["time_outs"]: time_out of the last step with a reset */
    /* optional [N,A] policy actions read by lgs_step in place of `actions` (which still
       receives the clipped copy, legged_robot.py:623-624): the caller's tensor is read
       directly, with no separate copy launch; NULL: the actions are already in `actions`. */
    const float* actions_in;
    /* optional [num_sums + 1]: the accumulator the NEXT control step adds into, when the caller
       alternates two episode_acc slots (lgs_step_deferred); the extras zero it with episode_acc */
    float* episode_acc_next;
} lgs_env_buffers;

typedef struct lgs_sim lgs_sim;

LGS_API const char* lgs_last_error(void);
LGS_API int lgs_version(void);

/* gym.create_sim + load_asset + create_env/actor x N (legged_robot.py:240,328,364-381) */
LGS_API int lgs_create_sim(const lgs_model_desc* model, const lgs_sim_params* params,
                           int32_t num_envs, int32_t device_id, lgs_sim** out);
LGS_API int lgs_destroy_sim(lgs_sim* sim);
LGS_API int lgs_set_stream(lgs_sim* sim, void* hip_stream);
LGS_API int lgs_synchronize(lgs_sim* sim);

/* _process_rigid_shape_props / _process_rigid_body_props (legged_robot.py:412-440, 472-483):
 * per-env shape friction and added root-body mass (host arrays [N]; NULL = unchanged) */
LGS_API int lgs_set_env_properties(lgs_sim* sim, const float* shape_friction, const float* added_base_mass);

/* bind the caller-owned state tensors (acquire_* + wrap_tensor) */
LGS_API int lgs_bind_state(lgs_sim* sim, float* root_states, float* dof_state,
                           float* net_contact_forces, float* rigid_body_states);

/* refresh_* : no-ops kept for API parity (the bound views are written in place) */
LGS_API int lgs_refresh(lgs_sim* sim);

/* set_dof_actuation_force_tensor: torques [N*D] used by the next lgs_simulate */
LGS_API int lgs_set_dof_actuation_force(lgs_sim* sim, const float* torques);
/* gym.simulate: ONE physics substep of every env (dynamics + contact + integrate) */
LGS_API int lgs_simulate(lgs_sim* sim);
/* forward kinematics only: rigid_body_states from root/dof state */
LGS_API int lgs_forward_kinematics(lgs_sim* sim);

/* set_*_tensor_indexed: copy rows `ids` (int32, device) from src into the bound state.
 * When src is the bound buffer itself this is a no-op. */
LGS_API int lgs_set_actor_root_state_indexed(lgs_sim* sim, const float* root_src, const int32_t* ids, int32_t n);
LGS_API int lgs_set_dof_state_indexed(lgs_sim* sim, const float* dof_src, const int32_t* ids, int32_t n);

/* task setup + the fused control step (LeggedRobot.step + post_physics_step) */
LGS_API int lgs_set_task(lgs_sim* sim, const lgs_task_params* task);
LGS_API int lgs_step(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* The two halves of lgs_step, for callers that act between them (a task's Python reward
 * terms) and for parity tests that check each half on its own.  lgs_step is bit-for-bit
 * lgs_step_physics followed by lgs_post_physics with the same step_counter.
 *  - lgs_step_physics: clip actions (legged_robot.py:623-624), decimation x (_compute_torques
 *    :649-671 + one substep :628-639), torques of the last substep, rigid_body_states for tasks
 *    that read them (h1_env.py:49).  No post-physics, no extras, no step-counter advance.
 *  - lgs_post_physics: post_physics_step (:673-709) + extras on the bound state, reading the
 *    clipped actions from env->actions, the last substep's torques from env->torques and the
 *    contact forces from the bound net_contact_forces; advances env->step_counter like lgs_step. */
LGS_API int lgs_step_physics(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
LGS_API int lgs_post_physics(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* lgs_post_physics in two parts around a caller's reward terms (compute_reward, :770-787):
 *  - _rewards: episode length, base-frame state, commands (:681-698), check_termination (:711-721)
 *    and the native reward terms (rew, per-term episode sums, reset/time_out); nothing is reset;
 *  - _finish: reset_idx of the envs whose reset byte is set, push, observations, bookkeeping,
 *    extras (:697-709), reading the base-frame state and commands the first part wrote.
 * lgs_post_physics == _rewards then _finish (without deferred rewards).                        */
LGS_API int lgs_post_physics_rewards(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
LGS_API int lgs_post_physics_finish(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* lgs_post_physics_rewards in two parts around a task's Python _post_physics_step_callback
 * (legged_robot.py:692; the reference's H1Robot / G1Robot override it, h1_env.py:55-65,
 * g1_env.py:56-105):
 *  - _prepare: episode length + 1, base-frame state (:681-690 into env->base_lin_vel,
 *    base_ang_vel, projected_gravity, rpy), the native callback (:488-517: command resampling,
 *    heading; the humanoid gait phase into env->phase / leg_phase);
 *  - _term_rewards: check_termination (:711-721) and the native reward terms on what the env
 *    buffers hold now (commands, phase, leg_phase, base-frame state, episode length).
 * _prepare then _term_rewards == _rewards, bit for bit, when the caller changes nothing.       */
LGS_API int lgs_post_physics_prepare(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
LGS_API int lgs_post_physics_term_rewards(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* reset_idx(all) as used by BaseTask.reset (base_task.py:82-86) */
LGS_API int lgs_reset_all(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* reset_idx(env_ids) (legged_robot.py:723-768) for an arbitrary subset: env_mask is a DEVICE
 * byte per env (nonzero = reset).  Resets dofs/root/commands/buffers of those envs, sets their
 * reset byte, and fills the extras like lgs_step (episode means over the reset envs, carried
 * time-outs); the step counter is not advanced. */
LGS_API int lgs_reset_idx(lgs_sim* sim, const lgs_env_buffers* env, const uint8_t* env_mask, int64_t step_counter);

/* lgs_step with its extras left to the step's consumer: the rollout's next policy launch
 * (include/ppo_mlp.h, pmlp_env_extras: pmlp_rollout_forward / pmlp_store_step_env), which does
 * k_step_extras' work on its own rows and once.  Until the consumer (or lgs_step_extras) has run,
 * env->ep_means / ep_snapshot / time_outs_carry hold the previous step's extras, episode_acc
 * holds this step's sums, last_root_vel[:, 0:2] every env's push draw, and the step counter is
 * not advanced.  The consumer zeroes episode_acc_next, not episode_acc (its other workgroups
 * still read that), so the caller alternates two slots: the next step's episode_acc is this
 * step's episode_acc_next.  lgs_step == lgs_step_deferred then lgs_step_extras, bit for bit.  */
LGS_API int lgs_step_deferred(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
LGS_API int lgs_step_extras(lgs_sim* sim, const lgs_env_buffers* env, int64_t step_counter);
/* the push bookkeeping a deferred step's consumer reads (device pointers owned by the sim):
 * vsim [N, 2] (the simulated xy base velocity before the all-env push draw) and pushed [3]
 * (the push flags of the two step-key parities, then the key of the last control step)      */
LGS_API int lgs_get_push_state(lgs_sim* sim, float** vsim, uint32_t** pushed);

/* gym.add_heightfield -- the rough-terrain ground of legged_gym (utils/terrain.py builds
 * height_field_raw; the reference's create_sim only ever adds the plane, legged_robot.py:240-257).
 * heights: HOST int16 [rows][cols]; sample (i, j) sits at world x = i*horizontal_scale - border_size,
 * y = j*horizontal_scale - border_size, z = heights[i][j]*vertical_scale.  Cell (i, j) is split into
 * two triangles along its (i,j)-(i+1,j+1) diagonal (terrain_utils.convert_heightfield_to_trimesh);
 * contact points are tested against the triangle under them (outside the map: its edge samples).
 * Replaces the z = 0 plane for every env; heights = NULL (or rows = 0) restores the plane. */
LGS_API int lgs_set_heightfield(lgs_sim* sim, const int16_t* heights, int32_t rows, int32_t cols,
                                float horizontal_scale, float vertical_scale, float border_size);

/* create_actor(..., self_collisions, 0) (legged_robot.py:373-374): the self-collision
 * proxies and pairs of every env (host descriptor, copied; NULL or num_pairs = 0: off) */
LGS_API int lgs_set_self_collision(lgs_sim* sim, const lgs_self_collision_desc* desc);

/* name/index queries (legged_robot.py:332-343, 388-407):
 *  lgs_get_counts     <- get_asset_dof_count / get_asset_rigid_body_count (:332-333)
 *  lgs_get_body_name  <- get_asset_rigid_body_names()[i] (:342); NULL when out of range or unnamed
 *  lgs_get_dof_name   <- get_asset_dof_names()[i] (:343); NULL likewise.  The strings are owned by
 *                        the sim and live until lgs_destroy_sim.
 *  lgs_find_body      <- find_actor_rigid_body_handle(env, actor, name) (:388-407): the body index
 *                        (bodies are env-major, so the index is the same in every env), -1 if absent
 *  lgs_find_dof       <- find_actor_dof_handle: the DOF index, -1 if absent                         */
LGS_API int lgs_get_counts(lgs_sim* sim, int32_t* num_envs, int32_t* num_bodies, int32_t* num_dofs);
LGS_API const char* lgs_get_body_name(lgs_sim* sim, int32_t index);
LGS_API const char* lgs_get_dof_name(lgs_sim* sim, int32_t index);
LGS_API int32_t lgs_find_body(lgs_sim* sim, const char* name);
LGS_API int32_t lgs_find_dof(lgs_sim* sim, const char* name);

/* capacity diagnostics (see the slot order above lgs_self_collision_desc): counts summed
 * over every env and substep of lgs_step / lgs_step_physics / lgs_simulate since the sim was
 * created or last reset:
 *   out[0] touching bodies that got no contact slot
 *   out[1] touching self-collision pairs without a slot
 *   out[2] violated joint limits without a constraint row
 * Synchronises the sim's stream; reset != 0 zeroes the counters afterwards. */
#define LGS_NUM_CONTACT_STATS 3
LGS_API int lgs_get_contact_stats(lgs_sim* sim, uint64_t* out, int32_t reset);

/* the compiled kernel shape the sim runs on: *dofs >= the model's DOFs, *bodies >= its bodies
 * (a robot without an instantiation of its own is padded to the smallest generic one that
 * fits -- inert DOFs and bodies, results bit-identical to the unpadded model), *rows the
 * constraint-row capacity.  Any pointer may be NULL. */
LGS_API int lgs_get_instantiation(lgs_sim* sim, int32_t* dofs, int32_t* bodies, int32_t* rows);

/* the factorisation order of that instantiation: 0 = the joint-space Cholesky eliminates
 * pivots in index order; CH > 0 = the model is D/CH equal chains of CH DOFs on the base and
 * the chain-structured kernel eliminates the chains' pivots level by level (every base-row
 * sum over the joint columns in level order; the CPU oracle takes it via
 * orc_set_factor_chain to reproduce the step bit for bit). */
LGS_API int lgs_get_factor_chain(lgs_sim* sim, int32_t* chain);

/* diagnostics: per-phase s_memtime cycle sums [N][24] of the last lgs_step
 * (only in a library built with -DLGS_PHASE_STAMPS; otherwise LGS_ERR_STATE) */
LGS_API int lgs_debug_set_phase_buffer(void* dev_ptr);

/* counter-based RNG used by every random draw of the step (Philox4x32-10);
 * exposed so tests and the oracle can reproduce the draws bit-exactly. */
LGS_API float lgs_uniform(uint64_t seed, uint32_t env, uint32_t step, uint32_t stream, uint32_t index);

/* random draw streams */
#define LGS_STREAM_NOISE 0u
#define LGS_STREAM_CMD 1u
#define LGS_STREAM_RESET_DOF 2u
#define LGS_STREAM_RESET_ROOT 3u
#define LGS_STREAM_RESET_CMD 4u
#define LGS_STREAM_PUSH 5u

#endif /* LEGGEDSIM_H */
