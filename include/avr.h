/* avr.h -- C-ABI of libavr.so, the MI355X-native replacement for the PyBullet calls on the
 * Assistive Gym step path.
 *
 * The reference reaches its physics through the PyBullet module API, one DIRECT client per env
 * (env.py:23).  One `env.step(a)` of FeedingJaco-v0 issues ~68 PyBullet calls:
 *   p.getJointStates            env.py:320-321, 393; feeding.py:126
 *   p.setJointMotorControlArray env.py:335-337
 *   p.stepSimulation  x5        env.py:342        (2 Bullet sub-steps each, feeding.py:289)
 *   p.getLinkState / multiplyTransforms / resetBasePositionAndOrientation
 *                               feeding.py:345-349 (update_targets), 124, 134
 *   p.getContactPoints          feeding.py:86-89, 111, 116
 *   p.getBasePositionAndOrientation / getBaseVelocity
 *                               feeding.py:59, 65, 100, 106, 125
 * avr_step() replaces that whole sequence for a batch of envs with one call; the task glue
 * (take_step env.py:274-351, get_total_force feeding.py:83-90, get_food_rewards :92-121,
 * _get_obs :123-142, reward :56-77, human_preferences env.py:412-448) is fused into the same
 * device launch.  The Python facade (assistive-vr-gym_amd/avr/env.py) keeps the gym
 * reset/step/observation/reward contract on top of this ABI.
 *
 * Conventions: every function returns 0 on success and a negative code on error; the message is
 * available from avr_last_error(sim).  A handle owns one HIP stream on one device and is not
 * thread-safe.  Host-pointer calls block until outputs are on the host; *_device calls take
 * device pointers and are asynchronous on avr_stream(sim).
 */
#ifndef AVR_H
#define AVR_H
#include <stddef.h>
#include <stdint.h>

#include "avr_model.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AVR_ABI_VERSION 6      /* 3: task-selected layouts (avr_model_desc.task), 5-kernel info, state getters;
                                  4: BedBathingPR2 (avr_model_desc bb_* fields, task 2);
                                  5: avr_graph_captures, per-handle device guard, t >= 0;
                                  6: avr_reset_ik self-contact screening (alt4), avr_robot_self_contact */
#define AVR_FLAGS_FAULT_MASK 0x1f  /* avr_get_flags bits 0-4; bit 5 (EPA budget) is informational */

typedef struct avr_config {
    int32_t n_envs;        /* envs owned by this handle (one GPU)                          */
    int32_t device;        /* HIP device ordinal                                           */
    int32_t env_offset;    /* global id of local env 0 (keys per-env RNG; sharding-stable)  */
    int32_t flags;         /* AVR_CFG_* bits, 0 = defaults                                  */
    uint64_t seed;         /* action RNG seed for avr_step_random (env.py:53 uses 1001)     */
} avr_config;

/* avr_config.flags: no flag is defined; avr_create rejects any set bit (bit 0 selected the
 * one-env-per-wavefront part-B kernel, removed in round 2: part B runs four envs per wavefront) */
#define AVR_CFG_RESERVED_MASK 0xffffffff

typedef struct avr_sim avr_sim;

/* Create a handle: copies the compiled scene to the device.  (replaces p.connect + the
 * loadURDF/createMultiBody/createConstraint scene build of world_creation.py:27-93)
 * model->task selects the task (AVR_TASK_FEEDING: FeedingJaco-v0, feeding.py; AVR_TASK_SCRATCH:
 * ScratchItchPR2-v0, scratch_itch.py) and with it the state layout (avr_model.h), the action and
 * observation sizes and the task glue. */
int avr_create(const avr_config *cfg, const avr_model_desc *model, avr_sim **out);
int avr_destroy(avr_sim *sim);

/* Per-env state blocks (n_envs x avr_task_state_words(task) floats, layout in avr_model.h).
 * (replaces resetJointState / resetBasePositionAndOrientation of the reset path) */
int avr_set_state(avr_sim *sim, const float *host_state);
int avr_get_state(avr_sim *sim, float *host_state);
/* Set the state of the envs whose mask byte is non-zero (auto-reset of finished episodes). */
int avr_set_state_masked(avr_sim *sim, const uint8_t *env_mask, const float *host_state);

/* n_frames x p.stepSimulation with the motors as they are, no task glue, then the reset
 * observation (feeding.py:319-320, 325).  obs may be NULL. */
int avr_settle(avr_sim *sim, int32_t n_frames, float *host_obs);

/* Episode reset of the envs whose mask byte is non-zero (mask NULL = all): their state rows
 * are taken from host_state[n_envs*STATE_WORDS] (the host reset path: scene randomisation and
 * IK, feeding.py:144-307), then n_frames x stepSimulation drop the food into the spoon
 * (feeding.py:318-320) and their reset observation goes to host_obs rows (feeding.py:325).
 * Unmasked envs and their host_obs rows are left untouched.  Replaces FeedingEnv.reset(). */
int avr_reset(avr_sim *sim, const uint8_t *env_mask, const float *host_state, int32_t n_frames, float *host_obs);

/* One gym step for every env: act[n_envs*act_dim] -> obs[n_envs*obs_dim], rew[n_envs],
 * done[n_envs] (TimeLimit 200), info[n_envs*2] = {total_force_on_human, task_success}
 * (FeedingJaco: act 7, obs 25, feeding.py:30-81; ScratchItchPR2: act 7, obs 30,
 * scratch_itch.py:30-82). */
int avr_step(avr_sim *sim, const float *act, float *obs, float *rew, uint8_t *done, float *info);
/* avr_step_device: the same with device buffers, asynchronous on avr_stream(sim).  The step's
 * launch sequence is replayed from a captured HIP graph keyed by (d_obs, d_rew, d_done, d_info,
 * mode); d_act is first copied (stream-ordered) into the handle's own action buffer, so a caller
 * may pass a fresh action buffer every step without a re-capture. */
int avr_step_device(avr_sim *sim, const float *d_act, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info);
/* Same, with synthetic actions a[e,t] ~ U(-1,1)^7 drawn on the device from Philox4x32-10
 * keyed by (seed, env_offset + e, t) -- examples/random_actions.py semantics.  t >= 0 (a
 * negative t is rejected). */
int avr_step_random_device(avr_sim *sim, int64_t t, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info);
/* n device-random steps t0 .. t0+n-1, bit-identical to n avr_step_random_device calls.  stacked = 0:
 * every step writes d_obs.. (NULL: the handle's buffers; the last step's outputs remain); stacked = 1:
 * step k writes slot k of d_obs[n][n_envs][obs_dim], d_rew[n][n_envs], d_done[n][n_envs],
 * d_info[n][n_envs][AVR_INFO_DIM] (all four required).  The env groups are joined every 16 steps
 * (not after every step): a group that finishes a step early starts its next one.  Asynchronous;
 * the handle's stream holds the whole rollout. */
int avr_rollout_random_device(avr_sim *sim, int64_t t0, int32_t n, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info, int32_t stacked);
/* Device actions for inspection: d_act[n_envs*7] for step t (same Philox stream). */
int avr_random_actions_device(avr_sim *sim, int64_t t, float *d_act);

/* One Bullet sub-step of length dt for every env, no task glue (known-answer tests). */
int avr_substep(avr_sim *sim, float dt);

int avr_sync(avr_sim *sim);
void *avr_stream(avr_sim *sim);
void *avr_state_device_ptr(avr_sim *sim);
int32_t avr_n_envs(avr_sim *sim);
/* Env groups whose launch sequences run concurrently on separate streams inside each step call
 * (one per 1024 envs, at most 4; AVR_ENV_GROUPS=1..8 in the environment at avr_create overrides).
 * Results do not depend on it.  No reference counterpart (diagnostic). */
int32_t avr_env_groups(avr_sim *sim);
/* Graph captures made by this handle so far (each distinct step key captures once; a few keys
 * are cached).  No reference counterpart (diagnostic). */
int64_t avr_graph_captures(avr_sim *sim);
int32_t avr_state_words(void);          /* FeedingJaco's: avr_task_state_words(AVR_TASK_FEEDING) */
int32_t avr_abi_version(void);
/* Per-task sizes (-1 for an unknown task) and the handle's task. */
int32_t avr_task_state_words(int32_t task);
int32_t avr_task_obs_dim(int32_t task);
int32_t avr_task_act_dim(int32_t task);
int32_t avr_task(avr_sim *sim);
/* Kernel resource usage: [vgprs, 0, lds_bytes, scratch_bytes] of each kernel of a step, in
 * launch order: pairs (kinematics, broadphase, shape-pair list), narrowphase, a (the
 * wave-cooperative GJK/EPA of the rare pairs that need it, manifolds, dynamics, constraint rows),
 * b (PGS + integration), task (the task glue after the frames): out20 holds 5 x 4 ints. */
int avr_kernel_info(avr_sim *sim, int32_t *out20);

/* ---- state queries (device-side gathers; host buffers; block until done) ----
 * The reference reads these through PyBullet every step; here they come out of the state without
 * copying the whole state block to the host.
 * avr_get_q: joint positions / velocities of every articulated DoF, q[n_envs*n_dof],
 *   qd[n_envs*n_dof] (either may be NULL), n_dof = avr_n_dof(sim): the robot's DoFs in URDF DFS
 *   order, then the articulated human chain's (zeros while that chain is static).
 *   Replaces p.getJointStates(robot | human, ...)[0:2] (env.py:320-321, feeding.py:126,
 *   scratch_itch.py:109). */
int32_t avr_n_dof(avr_sim *sim);
int avr_get_q(avr_sim *sim, float *q, float *qd);
/* avr_get_link_pose: world COM frame (x y z, qx qy qz qw) of articulated link `link` of every
 *   env, out7[n_envs*7]; link < 0 selects the robot base.  Forward kinematics on the current
 *   joint positions, as p.getLinkState(robot, link, computeForwardKinematics=True)[0:2]
 *   (feeding.py:124, scratch_itch.py:105; link indices are the compiled robot's, URDF DFS order
 *   within the simulated subtree). */
int avr_get_link_pose(avr_sim *sim, int32_t link, float *out7);
/* avr_get_contact_summary: per env, out4[n_envs*4] = {contact points, sum of normalForce over all
 *   points, over robot-human points, over tool-human points} of the last sub-step's contact set:
 *   the sums p.getContactPoints(...)[9] feeds to get_total_force (feeding.py:83-90,
 *   scratch_itch.py:84-102). */
int avr_get_contact_summary(avr_sim *sim, float *out4);
/* avr_get_flags: per-env health flags, flags[n_envs] (bit0 NaN / failed mass-matrix
 *   factorisation, bit1 contact pool full, bit2 AABB pair list full, bit3 shape pair list full,
 *   bit4 non-contact row buffer full, bit5 more than AVR_COOP_CAP = 4 penetrating hull pairs in
 *   one sub-step: the EPA ran on a rotating window of 4 of them, the others kept their manifold
 *   points -- informational, the env's state is finite); 0 = healthy.  AVR_FLAGS_FAULT_MASK
 *   selects the fault bits (0-4).  No reference counterpart (PyBullet has no
 *   such report); a vectorised trainer polls it instead of the whole state block. */
int avr_get_flags(avr_sim *sim, int32_t *flags);
const char *avr_last_error(avr_sim *sim);

/* ---- device reset (FeedingJaco) ----
 * avr_reset_ik: avr_reset with the reset's inverse kinematics on the device.  Replaces the IK of
 *   FeedingEnv.reset (feeding.py:276-278 -> util.py:34-105 ik_random_restarts) for the masked envs:
 *   host_state rows carry everything the host reset draws (human pose, bowl, impairment, motors;
 *   the arm's joints are overwritten); target7[n_envs*7] is the tool link's COM-frame target
 *   (position, quaternion); init[n_envs*restarts*n_arm] the arm's starting joints of every
 *   restart (drawn by the host from the env's reset stream).  Per env, restarts run in order
 *   with `iters` damped-least-squares updates each until one lands within `tol` (position, m, and
 *   quaternion distance, or a distance within tol of 2: util.py:49) with no robot hull vertex
 *   inside the keep-out box keepout8 = {center xyz, pad, half extents xyz, pad} (NULL: no
 *   screening); else the joints of the restart closest to the target position are kept
 *   (util.py:51-54).  step_sim's self-contact screening (util.py:41-46): alt4[n_envs*restarts*4]
 *   (NULL: none) holds per restart the re-drawn target orientation (the original's Euler angles
 *   +- 45 deg, drawn by the host); a restart whose solution has robot links touching (as
 *   avr_robot_self_contact) switches the target orientation to its alt4 entry, for its own
 *   acceptance check and the later restarts.
 *   The spoon and the food are then placed on the tool frame (world_creation.py:330-343,
 *   feeding.py:291-308) and n_frames settle frames run (feeding.py:319-320), as in avr_reset.
 *   host_ok[n_envs] (may be NULL) receives 1 where a restart was accepted.  Returns -1 for tasks
 *   other than FeedingJaco. */
int avr_reset_ik(avr_sim *sim, const uint8_t *env_mask, const float *host_state, const float *target7, const float *init, const float *alt4,
                 int32_t restarts, int32_t iters, float tol, const float *keepout8, int32_t n_frames, float *host_obs, uint8_t *host_ok);

/* avr_robot_self_contact: len(p.getContactPoints(bodyA=robot, bodyB=robot)) > 0 (util.py:41-46,
 *   63-67) at n joint vectors q[n*avr_n_dof], evaluated at the joint vector itself: the reference
 *   asks after a restart's 5 simulated frames, which are not simulated here -- a known difference,
 *   the same on the host and device IK paths (avr_get_q's layout; everything
 *   else from env 0's state block): out[n] = the robot shape pairs the step's collision pipeline finds
 *   within their contact threshold (compiled robot-robot candidate pairs: the URDF's
 *   URDF_USE_SELF_COLLISION robots, parent-child pairs excluded).  Host screening of the host IK
 *   path (avr/reset.py ik_batch); avr_reset_ik runs the same test on the device. */
int avr_robot_self_contact(avr_sim *sim, int32_t n, const float *q, int32_t *out);

/* avr_narrowphase_query (test hook): the step's narrowphase between shapes pairs[2i] and
 *   pairs[2i+1] (indices into the model's shapes) on body poses poses14[14i..] (A's body:
 *   position, quaternion xyzw; then B's), contact threshold thr -> out8[8i..] = {rc (0 none,
 *   1 contact, 2 unresolved), normal on B xyz, point on B xyz, signed distance}.  The shape-level
 *   counterpart of p.getClosestPoints / the contact a pair adds to its manifold (btGjkEpa2 [ext]);
 *   lets the GJK / EPA be checked against the oracle pair by pair.  Runs the pair as the step
 *   does: a pair whose fp32 lane GJK stalls with an open duality gap is answered by the
 *   cooperative GJK with the double simplex solve, every other pair by the cooperative fp32 path. */
int avr_narrowphase_query(avr_sim *sim, int32_t n, const int32_t *pairs, const float *poses14, float thr, float *out8);

/* ---- device base-pose search (ScratchItchPR2, BedBathingPR2) ----
 * avr_base_search: position_robot_toc (env.py:489-585; scratch_itch.py:189-190,
 *   bed_bathing.py:317) for n envs on the device, one lane per (env, attempt).  Host buffers:
 *   base7[n*attempts*7] each attempt's robot base pose (position, quaternion xyzw; the host draws
 *   the random offset and yaw, env.py:509-511), rest[n*attempts*n_arm] its IK rest pose
 *   (util.py:99), tstart3[n*3] the start goal of the tool link's COM (identity orientation),
 *   goals9[n*9] the shoulder, elbow and wrist positions.  Per attempt: damped-least-squares IK
 *   (`iters` updates, util.py:59-74 ik_jlwki with success threshold `tol`) to the start goal --
 *   missed: the attempt is discarded -- then to each human goal; reached goals add their
 *   joint-limit-weighted kinematic isotropy (env.py:536-553).  Per env the best attempt (most
 *   goals, then manipulability, the first on ties; none reaching the start goal: the closest)
 *   goes to best[n], ok[n] (1: start goal reached) and q_arm[n*n_arm] (its start-goal joints).
 *   res4[n*attempts*4] (may be NULL) receives every attempt's {goals reached or -1,
 *   manipulability, start position error, start quaternion distance}.  The state is not touched.
 *   Returns -1 for FeedingJaco (fixed base). */
int avr_base_search(avr_sim *sim, int32_t n, int32_t attempts, const float *base7, const float *rest, const float *tstart3,
                    const float *goals9, int32_t iters, float tol, int32_t *best, uint8_t *ok, float *q_arm, float *res4);

/* Per-kernel timing on the handle's stream: while enabled, every launch of a step/settle is
 * bracketed by HIP events (adds a little launch overhead; off by default).  avr_kernel_times
 * returns the accumulated milliseconds and launch counts per kernel kind
 * [take_step, substep_a, substep_b, task, substep_pairs, narrowphase, -, -] since enabling
 * (synchronises the stream). */
int avr_profile_kernels(avr_sim *sim, int32_t enable);
int avr_kernel_times(avr_sim *sim, double *ms8, int64_t *count8);

/* Diagnostics (phase-timer builds only, -DAVR_PROF): attach a device buffer of
 * [n_envs][16] uint64 cycle counters.  A no-op for the shipped kernel. */
int avr_set_profile_buffer(avr_sim *sim, void *d_prof);

/* Support-mapping table of one convex hull (host-only utility; avr_create builds one for every
 * hull with more than AVR_TAB_MIN_NV vertices).  Cube map of 6*G*G direction cells; cell c lists,
 * in ascending vertex order, every vertex that can be the support point (first strictly largest
 * projection, as Bullet's btConvexHullShape scan) for some direction of the cell:
 * cell[2c] = offset into idx, cell[2c+1] = count.  idx receives at most cap entries.  Returns the
 * total entry count (allocate that many and call again), or -1 on bad arguments.  Replaces the
 * per-query full vertex scan behind btConvexHullShape::localGetSupportingVertexWithoutMargin
 * (reached from p.stepSimulation, env.py:342) with an exact sub-linear lookup. */
int32_t avr_hull_support_table(const float *verts, int32_t nv, int32_t G, int32_t *cell, int32_t *idx, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif
