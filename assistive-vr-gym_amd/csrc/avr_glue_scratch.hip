// avr_glue_scratch.hip -- task glue of the PR2 tasks (included by avr_kernel.hip for
// AVR_TASK_SCRATCH and AVR_TASK_BEDBATH): take_step with the PR2's left arm and the human arm's
// tremor (env.py:274-351; both tasks drive the left arm with gains 0.05 / forces 1.0,
// config.ini:4-5,13-14), then ScratchItchPR2-v0's update_targets (scratch_itch.py:289-293),
// get_total_force (scratch_itch.py:84-102), _get_obs (:104-128) and the reward with
// human_preferences (:47-76, env.py:412-448); BedBathingPR2-v0's are in avr_glue_bedbath.hip.

// take_step (env.py:274-337) for robot_arm='left', gains/forces from config.ini:4-5
// (scratch_itch.py:45).  One thread per env.  The human arm keeps its reactive motors
// (world_creation.py:171-179: targets = the reset pose, gain 0.01, force human_strength) unless the
// impairment is 'tremor': then take_step drives the controllable joints to
// target_human_joint_positions + human_tremors (sign alternating with self.iteration), gain
// human_gains = 0.05 (scratch_itch.py:45), force human_forces (1) x human_strength.
__global__ __launch_bounds__(64) void avr_take_step_kernel(const KModel *__restrict__ mp, float *__restrict__ state, const float *__restrict__ act,
                                                           const unsigned char *__restrict__ mask, int mode, long long t, int env0, int n_envs) {
    const int env = env0 + 512 * (blockIdx.x >> 3) + (blockIdx.x & 7) + 8 * threadIdx.x;
    if (env >= n_envs || (mask && !mask[env])) return;
    const KModel &m = *mp;
    if (t < 0) t = m.step_t[-t - 1];           // graph replay: group -t - 1's counter, written before the launch (run_step, rollout)
    float *st = state + (size_t)env * K_STATE_WORDS;
    float *ws = env_ws(m, env);
    ws[WS_COOPROT] = 0.f;                       // the capped cooperative-pair window restarts every gym step (np_coop)
    float asq = 0.f;
    for (int i = 0; i < m.n_arm; i++) {
        float a_raw = mode == MODE_STEP_RANDOM ? philox_action(m.seed, m.env_offset + env, t, i) : act[(size_t)env * K_ACT_DIM + i];
        asq += a_raw * a_raw;                    // reward_action uses the caller's action (scratch_itch.py:63)
        float a = clampf(a_raw, -1.f, 1.f) * 0.05f;
        const int d = m.arm_dofs[i];
        float qn = st[S_Q + d];
        for (int it = 0; it < m.frame_skip; it++) {
            if (qn + a < m.arm_lower[i]) a = 0.f;
            if (qn + a > m.arm_upper[i]) a = 0.f;
            qn += a;
        }
        st[S_QTGT + d] = qn;
        st[S_KP + d] = m.robot_gain;
        st[S_MAXIMP + d] = m.robot_force * m.time_step;
    }
    if (st[S_TASK + T_TREMOR] != 0.f) {
        const float sg = ((int)st[S_TASK + T_ITER] & 1) ? -1.f : 1.f;
        const float imp = m.human_force * st[S_TASK + T_STRENGTH] * m.time_step;
        for (int c = 0; c < m.hc_n; c++) {
            const int d = m.nd + c;
            st[S_QTGT + d] = st[S_HCH + c] + st[S_HCH + K_HC_N + c] * sg;
            st[S_KP + d] = m.human_gain;
            st[S_MAXIMP + d] = imp;
        }
    }
    ws[WS_ASQ] = asq;
}

#if AVR_TASK == AVR_TASK_SCRATCH
// target_pos = limb frame x target_on_arm (update_targets, scratch_itch.py:289-293); the limb is
// a link of the articulated arm chain, whose frames robot_fk has just computed
AVR_DI void scratch_target(const KModel &m, EnvLDS &L) {
    const int k = (int)L.st[S_TASK + T_LIMB];
    const v3 p = tfpt(ldtf(L.cm[m.nl + k]), ld3(L.st + S_TASK + T_ONARM));
    SYNC();
    if (lane_id() == 0) st3(L.st + S_TASK + T_TARGET, p);
    SYNC();
}

// _get_obs(forces=[tool_force]) (scratch_itch.py:104-128): tool link 1 relative to the PR2 torso
// (link 15, a robot-fixed COM), its orientation, tool - target, target - torso, the left arm's
// joint angles, the human shoulder / elbow / wrist (links 9, 11, 13: arm chain links 2, 4, 6)
// relative to the torso, and the tool's total contact force.  robot_fk must be current.
AVR_DI void scratch_observe(const KModel &m, EnvLDS &L, float tool_force, float *o) {
    if (lane_id() == 0) {
        const v3 torso = tfpt(ldtf(L.st + S_RBASE), V(m.torso_com[0], m.torso_com[1], m.torso_com[2]));
        const tf tb = ldtf(L.st + S_FREE);
        const v3 tool = tfpt(tb, V(m.tool_tip[0], m.tool_tip[1], m.tool_tip[2]));
        const v3 tgt = ld3(L.st + S_TASK + T_TARGET);
        int k = 0;
        v3 a = sub(tool, torso);
        o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        o[k++] = tb.q.x; o[k++] = tb.q.y; o[k++] = tb.q.z; o[k++] = tb.q.w;
        a = sub(tool, tgt);
        o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        a = sub(tgt, torso);
        o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        for (int i = 0; i < m.n_arm; i++) o[k++] = L.st[S_Q + m.arm_dofs[i]];
        for (int j = 2; j <= 6; j += 2) {
            a = sub(ld3(L.cm[m.nl + j]), torso);
            o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        }
        o[k++] = tool_force;
    }
}

// get_total_force (scratch_itch.py:84-102) over the contact pool of the last sub-step, which is
// what p.getContactPoints reports after stepSimulation: per point normalForce = impulse / dt.
//   tool_force        every point of the tool (bodyA=tool);
//   total_on_human    tool-human and robot-human points (the robot: its articulated links and the
//                     robot-fixed geometry);
//   at_target         tool-human points on tool links 0 / 1 (not the handle, linkA -1) whose point
//                     on the human (positionOnB: the manifold's world point at the refresh, from
//                     the body frames of that sub-step's collision pass) is within 0.025 of the
//                     target; target_contact_pos is the last such point in pool order.
// Sums run in lane order (deterministic); `found` is false when no point is at the target.
struct ScratchForces { float tool, total, at; v3 tcp; bool found; };
AVR_DI ScratchForces scratch_forces(const KModel &m, const EnvLDS &L, const float *gcp, const float *btf) {
    const int lane = lane_id();
    const int n = (int)L.st[S_TASK + T_NCP];
    const v3 tgt = ld3(L.st + S_TASK + T_TARGET);
    const int tb = m.tool_body, ts0 = gld(m.body_shape_start + tb);
    float ft = 0.f, fh = 0.f, fa = 0.f;
    int last = -1;
    v3 lp = V(0, 0, 0);
    for (int i = lane; i < n; i += 64) {
        const float *cp = gcp + AVR_CP_WORDS * i;
        const int sa = (int)cp[AVR_CP_SA], sb = (int)cp[AVR_CP_SB];
        const int ba = gld(m.shape_body + sa), bb = gld(m.shape_body + sb);
        const int ka = gld(m.body_kind + ba), kb = gld(m.body_kind + bb);
        const float f = cp[AVR_CP_IMP] / m.time_step;
        const bool ta = ba == tb, tbb = bb == tb;
        const bool ha = ka == AVR_BODY_HUMAN, hb = kb == AVR_BODY_HUMAN;
        const bool ra = ka == AVR_BODY_ROBOT || ka == AVR_BODY_RSTATIC, rb = kb == AVR_BODY_ROBOT || kb == AVR_BODY_RSTATIC;
        const bool toolhum = (ta && hb) || (tbb && ha);
        if (ta || tbb) ft += f;
        if (toolhum || (ra && hb) || (rb && ha)) fh += f;
        if (toolhum && (ta ? sa : sb) - ts0 >= m.tool_handle_shapes) {
            // the point on the human: B's world point if the tool is A, else A's
            const v3 p = ta ? tfpt(ldtf(btf + 8 * bb), ld3(cp + AVR_CP_LB)) : tfpt(ldtf(btf + 8 * ba), ld3(cp + AVR_CP_LA));
            if (len(sub(p, tgt)) < 0.025f) { fa += f; last = i; lp = p; }
        }
    }
    ScratchForces r;
    r.tool = r.total = r.at = 0.f;
    for (int k = 0; k < 64; k++) { r.tool += __shfl(ft, k, 64); r.total += __shfl(fh, k, 64); r.at += __shfl(fa, k, 64); }
    int best = last;
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    r.found = best >= 0;
    const int owner = r.found ? best & 63 : 0;
    r.tcp = V(__shfl(lp.x, owner, 64), __shfl(lp.y, owner, 64), __shfl(lp.z, owner, 64));
    return r;
}

// Task glue after the frames (ScratchEnv.step after take_step, scratch_itch.py:47-82); SETTLE
// mode: target and the reset observation (_get_obs([0], [0, 0]), scratch_itch.py:268).  NaN guard
// for every mode.
__global__ __launch_bounds__(64) void avr_task_kernel(const KModel *__restrict__ mp, float *__restrict__ state, float *__restrict__ obs,
                                                      float *__restrict__ rew, unsigned char *__restrict__ done, float *__restrict__ info,
                                                      const unsigned char *__restrict__ mask, int mode, int env0, int n_envs) {
    __shared__ EnvLDS L;
    AVR_ENV_GUARD();
    const int lane = lane_id();
    float *gst = state + (size_t)env * K_STATE_WORDS;
    const float *gcp = gst + S_CP;
    load_state(m, L, gst);
    robot_fk(m, L);          // arm chain frames (human slots, update_targets) and robot link frames
    scratch_target(m, L);
    if (mode == MODE_SETTLE) {
        if (obs) scratch_observe(m, L, 0.f, obs + (size_t)env * K_OBS_DIM);
    } else if (mode == MODE_STEP || mode == MODE_STEP_RANDOM) {
        if (lane == 0) L.st[S_TASK + T_ITER] += 1.f;
        SYNC();
        const ScratchForces F = scratch_forces(m, L, gcp, env_cs(m, env) + CS_BTF);
        const tf tb = ldtf(L.st + S_FREE);
        const v3 tip = qrot(tb.q, V(m.tool_tip[0], m.tool_tip[1], m.tool_tip[2]));
        const v3 tool = add(tb.p, tip);
        // tool link 1's linear velocity (getLinkState(..., computeLinkVelocity=True)[6], :51)
        const float ee_vel = len(add(ld3(L.st + S_FREE + 7), crs(ld3(L.st + S_FREE + 10), tip)));
        scratch_observe(m, L, F.tool, obs + (size_t)env * K_OBS_DIM);
        const v3 tgt = ld3(L.st + S_TASK + T_TARGET);
        float scratch = 0.f, succ = L.st[S_TASK + T_SUCCESS];
        v3 prev = ld3(L.st + S_TASK + T_PREV);
        if (F.found && len(sub(F.tcp, prev)) > 0.01f && F.at < 10.f) {   // scratch_itch.py:64-68
            scratch = F.at;
            prev = F.tcp;
            succ += 1.f;
        }
        // human_preferences (env.py:412-448), scratching branch
        const float prefs = m.w_velocity * (-ee_vel) + m.w_force_nontarget * (-(F.total - F.at)) + m.w_high_forces * (F.at < 10.f ? 0.f : -F.at);
        const float dist = len(sub(tgt, tool));
        const float asq = env_ws(m, env)[WS_ASQ];
        const float r = m.w_distance * (-dist) + m.w_action * (-asq) + m.w_tool_force * F.at + m.w_scratch * scratch + prefs;
        SYNC();
        if (lane == 0) {
            st3(L.st + S_TASK + T_PREV, prev);
            L.st[S_TASK + T_SUCCESS] = succ;
            rew[env] = r;
            done[env] = (unsigned char)((int)L.st[S_TASK + T_ITER] >= m.max_steps);
            info[(size_t)env * AVR_INFO_DIM + 0] = F.total;
            info[(size_t)env * AVR_INFO_DIM + 1] = succ >= m.task_success_threshold ? 1.f : 0.f;
        }
    }
    SYNC();
    bool bad = false;
    for (int i = lane; i < S_CP; i += 64) bad |= !(L.st[i] == L.st[i]);
    const int ncp = (int)L.st[S_TASK + T_NCP];
    for (int i = lane; i < ncp * AVR_CP_WORDS; i += 64) bad |= !(gcp[i] == gcp[i]);
    bad = __any(bad);
    if (lane == 0) {
        int fl = (int)L.st[S_TASK + T_FLAGS] | L.flags | (bad ? 1 : 0);
        L.st[S_TASK + T_FLAGS] = (float)fl;
    }
    SYNC();
    for (int i = lane; i < S_CP; i += 64) gst[i] = L.st[i];
    prof_flush(m, L, env);
}

#else
#include "avr_glue_bedbath.hip"
#endif  // AVR_TASK_SCRATCH
