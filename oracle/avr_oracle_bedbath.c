/* avr_oracle_bedbath.c -- TEST INFRASTRUCTURE ONLY.  BedBathingPR2-v0 task glue of the CPU oracle
 * (included by avr_oracle.c when AVR_TASK == AVR_TASK_BEDBATH): take_step (env.py:274-351,
 * robot_arm='left', bed_bathing.py:46), get_total_force with the wipe targets (:77-127), the
 * tool-human closest distance (getClosestPoints(tool, human, 4.0), :61), _get_obs (:129-153) and
 * the reward + human_preferences (:54-70, env.py:412-448).  Parity vs PyBullet unpinned (see
 * avr_oracle.c). */

static void bb_observe(const model *m, real *st, float tool_force, float *o) {
    tf base; base.p = ld3(st + S_RBASE); base.q = ldq(st + S_RBASE + 3);
    v3 torso = tfpt(base, ld3d(m->d.torso_com));                        /* getLinkState(robot, 15)[0] */
    const real *f = st + S_FREE;
    tf tb; tb.p = ld3(f); tb.q = ldq(f + 3);
    v3 tool = tfpt(tb, ld3d(m->d.tool_tip));                             /* getLinkState(tool, 1)[0:2] */
    int k = 0;
    v3 a = sub(tool, torso);
    o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    o[k++] = (float)tb.q.x; o[k++] = (float)tb.q.y; o[k++] = (float)tb.q.z; o[k++] = (float)tb.q.w;
    for (int i = 0; i < m->d.n_arm; i++) o[k++] = (float)st[S_Q + m->d.arm_dofs[i]];
    for (int j = 0; j < 3; j++) {                                        /* human links 9, 11, 13 */
        a = sub(ld3(st + S_HUMAN + 7 * m->d.bb_joint_slots[j]), torso);
        o[k++] = (float)a.x; o[k++] = (float)a.y; o[k++] = (float)a.z;
    }
    o[k++] = tool_force;
}

static int bb_alive(const real *st, int k) { return ((int)st[S_TASK + T_WIPE + k / 24] >> (k % 24)) & 1; }
static void bb_kill(real *st, int k) {
    int bits = (int)st[S_TASK + T_WIPE + k / 24];
    bits &= ~(1 << (k % 24));
    st[S_TASK + T_WIPE + k / 24] = (real)bits;
}

static int is_robotlike(const model *m, int b) { int k = m->d.body_kind[b]; return k == AVR_BODY_ROBOT || k == AVR_BODY_RSTATIC; }

/* get_total_force (bed_bathing.py:77-127), in the reference's order: the tool-human points one
 * after the other, each deleting the live targets within 0.025 of its point on the human. */
static int bb_forces(const model *m, real *st, const ws_t *w, real *tool_force, real *on_human, real *at) {
    int n = (int)st[S_TASK + T_NCP];
    int tb = m->d.spoon_body, ts0 = m->d.body_shape_start[tb];
    int g = (int)st[S_TASK + T_GENDER];
    int nu = m->d.bb_ntgt[g][0], nt = nu + m->d.bb_ntgt[g][1];
    const real *up = st + S_HUMAN + 7 * m->d.bb_limb_slots[0], *fo = st + S_HUMAN + 7 * m->d.bb_limb_slots[1];
    tf tu, tfo;
    tu.p = ld3(up); tu.q = ldq(up + 3);
    tfo.p = ld3(fo); tfo.q = ldq(fo + 3);
    int wiped = 0;
    *tool_force = *on_human = *at = 0;
    for (int i = 0; i < n; i++) {
        real *cp = cp_ptr(st, i);
        int sa = (int)cp[AVR_CP_SA], sb = (int)cp[AVR_CP_SB];
        int ba = m->d.shape_body[sa], bb = m->d.shape_body[sb];
        int ha = m->d.body_kind[ba] == AVR_BODY_HUMAN, hb = m->d.body_kind[bb] == AVR_BODY_HUMAN;
        real f = cp[AVR_CP_IMP] / R(m->d.time_step);
        int ta = ba == tb, tbb = bb == tb;
        int toolhum = (ta && hb) || (tbb && ha);
        if (ta || tbb) *tool_force += f;
        if (toolhum || (is_robotlike(m, ba) && hb) || (is_robotlike(m, bb) && ha)) *on_human += f;
        if (toolhum && (ta ? sa : sb) - ts0 >= m->d.tool_handle_shapes) {      /* linkA == 1, the cloth */
            *at += f;
            int hbody = ta ? bb : ba;
            if (m->d.body_index[hbody] == 0) continue;                         /* linkB < 0: the base */
            v3 p = ta ? tfpt(w->body[bb], ld3(cp + AVR_CP_LB)) : tfpt(w->body[ba], ld3(cp + AVR_CP_LA));
            for (int k = 0; k < nt; k++) {
                if (!bb_alive(st, k)) continue;
                const double *t = m->d.bb_targets + 4 * ((size_t)g * AVR_BB_MAX_TARGETS + k);
                v3 loc = V(R(t[0]), R(t[1]), R(t[2]));
                v3 tw = tfpt(k < nu ? tu : tfo, loc);
                if (len(sub(p, tw)) < R(0.025)) { bb_kill(st, k); wiped++; }
            }
        }
    }
    return wiped;
}

/* min over getClosestPoints(tool, human, distance=4.0)[8]: every tool shape against every human
 * shape of the env's gender, the narrowphase distance (EPA depth when penetrating); the GJK with
 * the lane path's stall rule, as the kernel's bb_closest + avr_bb_stall_kernel run it */
static real bb_closest(const model *m, real *st, ws_t *w) {
    int tb = m->d.spoon_body, ts0 = m->d.body_shape_start[tb], nts = m->d.body_shape_count[tb];
    int g = (int)st[S_TASK + T_GENDER];
    const real *f = st + S_FREE;
    tf ttf; ttf.p = ld3(f); ttf.q = ldq(f + 3);
    real thr = R(m->d.closest_distance), dmin = R(1e30);
    for (int b = 0; b < m->d.n_bodies; b++) {
        if (m->d.body_kind[b] != AVR_BODY_HUMAN) continue;
        const real *h = st + S_HUMAN + 7 * m->d.body_index[b];
        tf hb; hb.p = ld3(h); hb.q = ldq(h + 3);
        for (int sb = m->d.body_shape_start[b]; sb < m->d.body_shape_start[b] + m->d.body_shape_count[b]; sb++) {
            if (m->d.shape_gender[sb] >= 0 && m->d.shape_gender[sb] != g) continue;
            wshape B = make_wshape(m, sb, hb);
            for (int sa = ts0; sa < ts0 + nts; sa++) {
                wshape A = make_wshape(m, sa, ttf);
                v3 nB, pB;
                real d;
                if (narrowphase(w, &A, &B, thr, &nB, &pB, &d) && d < dmin) dmin = d;
            }
        }
    }
    return dmin < R(1e29) ? dmin : thr;
}

static int env_step(avr_oracle *o, int e, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    real *st = o->state + (size_t)e * K_STATE_WORDS;
    const model *m = oview(o, st);
    ws_t *w = &o->ws[e];
    w->gender = (int)st[S_TASK + T_GENDER];
    int nsub = m->d.num_sub_steps > 0 ? m->d.num_sub_steps : 1;
    real dt = R(m->d.time_step) / nsub;
    /* take_step: PR2 left arm (env.py:318-335); impairment 'none': no human motors change */
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
    for (int fr = 0; fr < m->d.frame_skip; fr++) {
        for (int s = 0; s < nsub; s++)
            if (substep(o, st, w, dt)) return -1;
        /* enforce_hard_human_joint_limits (env.py:345) acts on the controllable joints: none in
           BedBathing's episode (bed_bathing.py:291), the chain is articulated only in the reset */
        if (st[S_TASK + T_HDYN] != 0) hard_limits(m, st);
    }
    robot_fk(m, st, w);
    st[S_TASK + T_ITER] += 1;
    real tool_force, on_human, at;
    int wiped = bb_forces(m, st, w, &tool_force, &on_human, &at);
    real dmin = bb_closest(m, st, w);
    const real *f = st + S_FREE;
    tf tb; tb.p = ld3(f); tb.q = ldq(f + 3);
    v3 tip = qrot(tb.q, ld3d(m->d.tool_tip));
    real ee_vel = len(add(ld3(f + 7), crs(ld3(f + 10), tip)));   /* tool link 1 velocity (:55) */
    bb_observe(m, st, (float)tool_force, obs);
    st[S_TASK + T_SUCCESS] += wiped;
    real prefs = R(m->d.w_velocity) * (-ee_vel) + R(m->d.w_force_nontarget) * (-(on_human - at)) + R(m->d.w_high_forces) * (at < 10 ? 0 : -at);
    real asq = 0;
    for (int i = 0; i < m->d.n_arm; i++) asq += (real)act[i] * (real)act[i];   /* unclipped (:62) */
    real r = R(m->d.w_distance) * (-dmin) + R(m->d.w_action) * (-asq) + R(m->d.w_wipe) * wiped + prefs;
    *rew = (float)r;
    *done = (uint8_t)((int)st[S_TASK + T_ITER] >= m->d.max_episode_steps);
    info[0] = (float)on_human;
    info[1] = (float)(st[S_TASK + T_SUCCESS] >= st[S_TASK + T_NTGT] * R(m->d.task_success_threshold) ? 1 : 0);
    for (int i = 0; i < K_STATE_WORDS; i++)
        if (st[i] != st[i]) { st[S_TASK + T_FLAGS] = (real)((int)st[S_TASK + T_FLAGS] | 1); break; }
    return 0;
}

/* test hook: the closest tool-human distance of env e in its current state */
__attribute__((visibility("default"))) int avr_oracle_bb_closest(avr_oracle *o, int e, double *out) {
    real *st = o->state + (size_t)e * K_STATE_WORDS;
    const model *m = oview(o, st);
    ws_t *w = &o->ws[e];
    w->gender = (int)st[S_TASK + T_GENDER];
    *out = (double)bb_closest(m, st, w);
    return 0;
}
