/* avr_oracle_scratch.c -- TEST INFRASTRUCTURE ONLY.  ScratchItchPR2-v0 task glue of the CPU
 * oracle (included by avr_oracle.c when AVR_TASK == AVR_TASK_SCRATCH): take_step
 * (env.py:274-351, robot_arm='left', scratch_itch.py:45), update_targets (scratch_itch.py:289-293),
 * get_total_force (:84-102), _get_obs (:104-128), reward + human_preferences (:47-76,
 * env.py:412-448).  Parity vs PyBullet unpinned (see avr_oracle.c). */

/* target_pos = limb frame x target_on_arm; the limb is a link of the articulated arm chain */
static void scratch_target(const model *m, real *st, ws_t *w) {
    int k = (int)st[S_TASK + T_LIMB];
    st3(st + S_TASK + T_TARGET, tfpt(w->cm[m->nl_robot + k], ld3(st + S_TASK + T_ONARM)));
}

static void scratch_observe(const model *m, real *st, ws_t *w, float tool_force, float *o) {
    tf base; base.p = ld3(st + S_RBASE); base.q = ldq(st + S_RBASE + 3);
    v3 torso = tfpt(base, ld3d(m->d.torso_com));                        /* getLinkState(robot, 15)[0] */
    const real *f = st + S_FREE;
    tf tb; tb.p = ld3(f); tb.q = ldq(f + 3);
    v3 tool = tfpt(tb, ld3d(m->d.tool_tip));                             /* getLinkState(tool, 1)[0:2] */
    v3 tgt = ld3(st + S_TASK + T_TARGET);
    int k = 0;
    v3 a = sub(tool, torso);
    o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    o[k++] = (float)tb.q.x; o[k++] = (float)tb.q.y; o[k++] = (float)tb.q.z; o[k++] = (float)tb.q.w;
    a = sub(tool, tgt);
    o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    a = sub(tgt, torso);
    o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    for (int i = 0; i < m->d.n_arm; i++) o[k++] = (float)st[S_Q + m->d.arm_dofs[i]];
    for (int j = 2; j <= 6; j += 2) {                                    /* human links 9, 11, 13 */
        a = sub(w->cm[m->nl_robot + j].p, torso);
        o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    }
    o[k++] = tool_force;
}

static int is_robotlike(const model *m, int b) { int k = m->d.body_kind[b]; return k == AVR_BODY_ROBOT || k == AVR_BODY_RSTATIC; }

/* get_total_force over the last sub-step's contact points (normalForce = impulse / dt); the point
 * on the human is the manifold's world point at that sub-step's collision pass (w->body). */
static void scratch_forces(const model *m, real *st, const ws_t *w, real *tool_force, real *total, real *at, v3 *tcp, int *found) {
    int n = (int)st[S_TASK + T_NCP];
    int tb = m->d.spoon_body, ts0 = m->d.body_shape_start[tb];
    v3 tgt = ld3(st + S_TASK + T_TARGET);
    *tool_force = *total = *at = 0;
    *found = 0;
    for (int i = 0; i < n; i++) {
        real *cp = cp_ptr(st, i);
        int sa = (int)cp[AVR_CP_SA], sb = (int)cp[AVR_CP_SB];
        int ba = m->d.shape_body[sa], bb = m->d.shape_body[sb];
        int ha = m->d.body_kind[ba] == AVR_BODY_HUMAN, hb = m->d.body_kind[bb] == AVR_BODY_HUMAN;
        real f = cp[AVR_CP_IMP] / R(m->d.time_step);
        int ta = ba == tb, tbb = bb == tb;
        int toolhum = (ta && hb) || (tbb && ha);
        if (ta || tbb) *tool_force += f;
        if (toolhum || (is_robotlike(m, ba) && hb) || (is_robotlike(m, bb) && ha)) *total += f;
        if (toolhum && (ta ? sa : sb) - ts0 >= m->d.tool_handle_shapes) {
            v3 p = ta ? tfpt(w->body[bb], ld3(cp + AVR_CP_LB)) : tfpt(w->body[ba], ld3(cp + AVR_CP_LA));
            if (len(sub(p, tgt)) < R(0.025)) { *at += f; *tcp = p; *found = 1; }
        }
    }
}

static int env_step(avr_oracle *o, int e, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    real *st = o->state + (size_t)e * K_STATE_WORDS;
    const model *m = oview(o, st);
    ws_t *w = &o->ws[e];
    w->gender = (int)st[S_TASK + T_GENDER];
    int nsub = m->d.num_sub_steps > 0 ? m->d.num_sub_steps : 1;
    real dt = R(m->d.time_step) / nsub;
    /* take_step: PR2 left arm (env.py:318-335) */
    real a[8], qn[8];
    for (int i = 0; i < m->d.n_arm; i++) {
        real x = act[i];
        x = x < -1 ? -1 : x > 1 ? 1 : x;
        a[i] = (real)((float)x * 0.05f);
        qn[i] = st[S_Q + m->d.arm_dofs[i]];
    }
    for (int it = 0; it < m->d.frame_skip; it++)
        for (int i = 0; i < m->d.n_arm; i++) {
            if (qn[i] + a[i] < R(m->d.arm_lower[i])) a[i] = 0;
            if (qn[i] + a[i] > R(m->d.arm_upper[i])) a[i] = 0;
            qn[i] += a[i];
        }
    for (int i = 0; i < m->d.n_arm; i++) {
        int d = m->d.arm_dofs[i];
        st[S_QTGT + d] = qn[i];
        st[S_KP + d] = R(m->d.robot_gain);
        st[S_MAXIMP + d] = R(m->d.robot_force * m->d.time_step);
    }
    if (st[S_TASK + T_TREMOR] != 0) {
        /* tremor (env.py:327-337): target_human_joint_positions + human_tremors, sign alternating
           with self.iteration; human_gains 0.05, human_forces (1) x human_strength */
        real sg = ((int)st[S_TASK + T_ITER] % 2 == 0) ? 1 : -1;
        real imp = R(m->d.human_force) * st[S_TASK + T_STRENGTH] * R(m->d.time_step);
        for (int k = 0; k < m->d.hc_n; k++) {
            int d = m->nd_robot + k;
            st[S_QTGT + d] = st[S_HCH + k] + st[S_HCH + K_HC_N + k] * sg;
            st[S_KP + d] = R(m->d.human_gain);
            st[S_MAXIMP + d] = imp;
        }
    }
    for (int fr = 0; fr < m->d.frame_skip; fr++) {
        for (int s = 0; s < nsub; s++)
            if (substep(o, st, w, dt)) return -1;
        hard_limits(m, st);                 /* enforce_hard_human_joint_limits (env.py:345) */
    }
    robot_fk(m, st, w);                     /* update_targets (env.py:346) on the final arm pose */
    scratch_target(m, st, w);
    st[S_TASK + T_ITER] += 1;
    real tool_force, total, at;
    v3 tcp = V(0, 0, 0);
    int found;
    scratch_forces(m, st, w, &tool_force, &total, &at, &tcp, &found);
    const real *f = st + S_FREE;
    tf tb; tb.p = ld3(f); tb.q = ldq(f + 3);
    v3 tip = qrot(tb.q, ld3d(m->d.tool_tip));
    v3 tool = add(tb.p, tip);
    real ee_vel = len(add(ld3(f + 7), crs(ld3(f + 10), tip)));   /* tool link 1 velocity (:51) */
    scratch_observe(m, st, w, (float)tool_force, obs);
    v3 tgt = ld3(st + S_TASK + T_TARGET);
    real scratch = 0;
    v3 prev = ld3(st + S_TASK + T_PREV);
    if (found && len(sub(tcp, prev)) > R(0.01) && at < 10) {      /* scratch_itch.py:64-68 */
        scratch = at;
        st3(st + S_TASK + T_PREV, tcp);
        st[S_TASK + T_SUCCESS] += 1;
    }
    real prefs = R(m->d.w_velocity) * (-ee_vel) + R(m->d.w_force_nontarget) * (-(total - at)) + R(m->d.w_high_forces) * (at < 10 ? 0 : -at);
    real asq = 0;
    for (int i = 0; i < m->d.n_arm; i++) asq += (real)act[i] * (real)act[i];   /* unclipped (:63) */
    real r = R(m->d.w_distance) * (-len(sub(tgt, tool))) + R(m->d.w_action) * (-asq) + R(m->d.w_tool_force) * at +
             R(m->d.w_scratch) * scratch + prefs;
    *rew = (float)r;
    *done = (uint8_t)((int)st[S_TASK + T_ITER] >= m->d.max_episode_steps);
    info[0] = (float)total;
    info[1] = (float)(st[S_TASK + T_SUCCESS] >= R(m->d.task_success_threshold) ? 1 : 0);
    for (int i = 0; i < K_STATE_WORDS; i++)
        if (st[i] != st[i]) { st[S_TASK + T_FLAGS] = (real)((int)st[S_TASK + T_FLAGS] | 1); break; }
    return 0;
}
