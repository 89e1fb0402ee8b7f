// avr_kmodel.h -- device-side scene description (float copies of avr_model_desc) shared by the
// step kernel and the C-ABI host code.
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/avr_model.h"
#include "avr_task.h"

#define MAXL K_MAX_LINKS
#define MAXD K_MAX_DOF
#define MAXF K_MAX_FREE
#define MAXB 48
#define MAXCC 224      // non-static child shapes whose world AABBs are cached per sub-step
#define MAXSH 320      // shapes (the pair kernel stages their packed info in LDS, 16 bits each)
#define MAXSP 256
#define MAXAP 256
#if K_PR2
#define MAXNC 48       // non-contact rows: 21 motors, the 6-row tool weld, violated limits
#else
#define MAXNC 32
#endif
// DoF slots per part-B lane: lane sl (0..15) of an env group holds DoFs sl and (NDL 2) sl + 16
#define NDL (MAXD > 16 ? 2 : 1)
static_assert(MAXD <= 16 * NDL && MAXL <= 32, "DoF slots per lane / 32-bit link masks");
#ifndef SMALL_NV
#define SMALL_NV 64     // hulls with more vertices and no support table take the wave-cooperative narrowphase
#endif
#define GJK_MAX_IT 64
#define GJK_REL_EPS 1e-6f
#define EPA_MAX_IT 64
#define EPA_MAX_V 64
#define EPA_MAX_F 128
#define EPA_EPS 1e-6f
#define BT_BROADPHASE_EXPAND 0.02f
#define BT_DENOM_EPS 1e-12f
#define BT_ANGULAR_MOTION_THRESHOLD (0.5f * 1.5707963267948966f)
#define BIGF 1e30f


// Per-env collision scratch (m.cscr, CS_WORDS floats per env), the hand-over between the three
// kernels of a sub-step's part A: avr_substep_pairs_kernel writes the shape-pair list, the body
// COM frames and the link frames; avr_narrowphase_kernel writes one result per pair;
// avr_substep_a_kernel consumes them.
#define CS_NSP 0                                    // int bits: shape pairs
#define CS_FLAGS 1                                  // int bits: flags raised by the pair kernel
#define CS_N0 2                                     // int bits: sphere-hull pairs (list CS_L0)
#define CS_N1 3                                     // int bits: the other pairs (list CS_L1)
#define CS_PAIRS 4                                  // [MAXSP] (sa | sb << 16, body pair) int bits
#define CS_RES (CS_PAIRS + 2 * MAXSP)               // [MAXSP][8] rc, nB, pB, dist (rc 2: cooperative path)
#define CS_BTF (CS_RES + 8 * MAXSP)                 // [MAXB][8] body COM frames
#define CS_CM (CS_BTF + 8 * MAXB)                   // [MAXL][8] link COM frames
#define CS_AX (CS_CM + 8 * MAXL)                    // [MAXL][4] joint axes (world)
#define CS_ORG (CS_AX + 4 * MAXL)                   // [MAXL][4] joint origins (world)
#define CS_L0 (CS_ORG + 4 * MAXL)                   // [MAXSP][2] the sphere-hull pairs, ascending: (k | ba << 16 | bb << 24, sa | sb << 16)
#define CS_L1 (CS_L0 + 2 * MAXSP)                   // [MAXSP][2] the other pairs, ascending, the same entries
#define CS_COOP (CS_L1 + 2 * MAXSP)                 // nonzero: some pair of this sub-step was left to the coop kernel (rc 2)
#define CS_WORDS (CS_COOP + 4)                      // (keeps every env's CS_RES 16-byte aligned)
static_assert(MAXB <= 256 && MAXSP <= 65536, "narrowphase list entries pack k (16 bits) and two body indices (8 bits each)");

// Articulated links: the robot's nl links, then (impairment 'tremor') the head/neck chain's
// hc_n links with DoFs nd .. nd + hc_n - 1; nla = nl + hc_n.  The chain root's parent is -2:
// the static human slot hc_parent_slot.  Per-link tables are [nla]; the tables that differ by
// gender (joint origins, COM frames, masses, inertias) are [2][nla] (male, female).
struct KModel {
    int nl, nd, nf, nb, ns, np, nh;
    int nla, hc_n, np_base;   // np_base: pairs active in every env (the rest: tremor envs only)
    const int *rl_parent, *rl_jtype, *rl_dof, *rl_has_limit;   // [nla]
    const float *rl_jorig;    // [2][nla][8] p3 q4 pad
    const float *rl_com;      // [2][nla][8]
    const float *rl_axis;     // [nla][4]
    const float *rl_inertia;  // [2][nla][4]
    const float *rl_mass;     // [2][nla]
    const float *rl_lower, *rl_upper;   // [nla]
    float base[8];
    const float *fb_mass, *fb_inertia, *fb_gravity;   // [nf], [nf][4], [nf][4]
    const float *st_pose;                             // [nst][8]
    const int *body_kind, *body_index, *body_shape_start, *body_shape_count, *body_flags;
    const float *body_friction, *body_threshold, *body_aabb;   // [nb][12]
    const float *body_rolling, *body_spinning;                 // [nb] (K_TORSION)
    const int *shape_kind, *shape_body, *shape_gender, *shape_hull;   // hull [ns][4]
    const float *shape_pose, *shape_param, *shape_margin, *shape_aabb; // [ns][8] [ns][4] [ns] [ns][8]
    const float4 *hull_verts;
    const int *shape_tab;       // [ns] first support-table cell of a large hull, -1 without a table
    const int2 *tab_cell;       // [cells] (offset, count) into tab_vert (avr_hulltab.cpp)
    const float4 *tab_vert;     // candidate vertices (x, y, z, vertex index as int bits), ascending per cell
    const int *shape_cidx;      // [ns] index into the per-sub-step child AABB cache, -1 for static shapes
    const float *static_saabb;  // [ns][8] world AABB (min3, pad, max3, pad) of static shapes (host-computed)
    const int *pair_a, *pair_b;
    const int *shape_info;      // [ns] (child AABB cache index + 1, 0 static) | (shape_gender + 1) << 9 | shape_kind << 11
    const int4 *pair_rec;       // [np] (ba | bb << 16, sa0 | na << 16, sb0 | nb << 16, bare | one-by-one << 1)
    int n_arm, arm_dofs[8], n_finger, finger_dofs[4];
    int tool_link, torso_link, head_slot, spoon_free, bowl_free, food_free0, n_food;
    int table_body, bowl_body, spoon_body, food_body0, tool_body;
    float tool_offset[8], mouth[2][4], arm_lower[8], arm_upper[8];
    float time_step;
    int nsub, frame_skip, iters, max_steps;
    float erp, warmstart, lin_damp, ang_damp, max_vel, robot_gain, robot_force, fixed_max_imp;
    float w_distance, w_action, w_food, w_velocity, w_force_nontarget, w_high_forces, w_food_hit,
        w_food_velocities, task_success_threshold;
    unsigned long long seed;
    int env_offset;
    int dof_link[MAXD];        // link owning each DoF
    unsigned anc_mask[MAXL];   // bit k set if link k is on the chain base..link (inclusive)
    unsigned desc_mask[MAXL];  // bit k set if link k is in the subtree of link (inclusive)
    int rl_level[MAXL];        // depth of each link in the tree (roots 0)
    int nlev;                  // number of levels
    int hc_parent_slot, hc_slot[K_HC_N], hc_body[K_HC_N];
    float hc_lower[K_HC_N], hc_upper[K_HC_N], human_gain, human_force;
    float hc_grav[4];          // gravity on the articulated human chain (K_HUMAN_GRAVITY)
    float fix_pivot_b[4];      // fixed constraint: child pivot in the tool body frame
    float tool_tip[4];         // ScratchItch: tool link 1 COM in the tool body frame
    float torso_com[4];        // ScratchItch: PR2 torso link COM in the base frame
    int tool_handle_shapes;    // ScratchItch: leading tool shapes that belong to the handle (link -1)
    float w_tool_force, w_scratch;
    const float4 *bb_tgt;      // BedBathing: wipe targets [2][AVR_BB_MAX_TARGETS] (xyz in the limb frame, limb)
    int bb_ntgt[2][2];         // [gender][limb]
    int bb_limb_slot[2], bb_joint_slot[3];
    float w_wipe, closest_distance;
    float *rows;               // constraint-row scratch: [n_envs][2][rowcap][32] (see solve())
    int rowcap;                // rows per env = MAXNC + K_CROWS * K_MAX_CONTACTS
    int rowstride;             // floats between consecutive envs' row buffers
    int rows_envs;             // envs covered by the row buffer (the handle's n_envs)
    int b4_global;             // diagnostic (AVR_B4_GLOBAL=1): part B reads every row from global memory
    float *ws;                 // per-env workspace between sub-step kernels: [n_envs][128]
    float *cscr;               // per-env collision scratch between the part-A kernels: [n_envs][CS_WORDS]
    unsigned long long *prof;  // diagnostic builds only (AVR_PROF): [n_envs][16] cycle counters
    long long *step_t;         // the step counter of a replayed step graph (take_step reads it when passed t < 0)
};

// Optional event log filled by avr_launch_step (per-kernel timing, see avr_kernel_times):
// an event is recorded before every launch (kind = AVR_K_*) and after the last one (kind -1).
enum { AVR_K_TAKE = 0, AVR_K_A = 1, AVR_K_B = 2, AVR_K_TASK = 3, AVR_K_PAIRS = 4, AVR_K_NARROW = 5, AVR_K_COOP = 6, AVR_K_KINDS = 8 };
struct avr_evlog {
    hipEvent_t *ev;
    int *kind;
    int n, cap;
};
