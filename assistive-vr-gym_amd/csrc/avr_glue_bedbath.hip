// avr_glue_bedbath.hip -- BedBathingPR2-v0 task glue (included by avr_glue_scratch.hip for
// AVR_TASK_BEDBATH, after the PR2 take_step it shares with ScratchItch): get_total_force with the
// wipe-target bookkeeping (bed_bathing.py:77-127), the tool-human closest distance
// (p.getClosestPoints(tool, human, distance=4.0), :61), _get_obs (:129-153) and the reward with
// human_preferences (:54-70, env.py:412-448).  The human is static during the episode, so the
// targets' world positions (update_targets, :382-394) follow from the limb slots directly.

// _get_obs(forces=[tool_force]) (bed_bathing.py:129-153): tool link 1 (the cloth) relative to the
// PR2 torso (link 15, robot-fixed), its orientation, the left arm's joint angles, the human
// shoulder / elbow / wrist (links 9, 11, 13) relative to the torso, the tool's contact force.
AVR_DI void bb_observe(const KModel &m, const EnvLDS &L, float tool_force, float *o) {
    if (lane_id() == 0) {
        const v3 torso = tfpt(ldtf(L.st + S_RBASE), V(m.torso_com[0], m.torso_com[1], m.torso_com[2]));
        const tf tb = ldtf(L.st + S_FREE);
        const v3 tool = tfpt(tb, V(m.tool_tip[0], m.tool_tip[1], m.tool_tip[2]));
        int k = 0;
        v3 a = sub(tool, torso);
        o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        o[k++] = tb.q.x; o[k++] = tb.q.y; o[k++] = tb.q.z; o[k++] = tb.q.w;
        for (int i = 0; i < m.n_arm; i++) o[k++] = L.st[S_Q + m.arm_dofs[i]];
        for (int j = 0; j < 3; j++) {
            a = sub(ld3(L.st + S_HUMAN + 7 * m.bb_joint_slot[j]), torso);
            o[k++] = a.x; o[k++] = a.y; o[k++] = a.z;
        }
        o[k++] = tool_force;
    }
}

// wipe target k still on the arm: bit k % 24 of task word T_WIPE + k / 24
AVR_DI bool bb_alive(const float *st, int k) { return ((int)st[S_TASK + T_WIPE + k / 24] >> (k % 24)) & 1; }

struct BBShared {
    float pts[K_MAX_CONTACTS][4];   // wiping contact points (world, on the human), pool order
    unsigned char kill[AVR_BB_MAX_TARGETS];
    int npts, wiped;
};

// get_total_force (bed_bathing.py:77-127) over the contact pool of the last sub-step (normalForce
// = impulse / dt):
//   tool        every point of the tool (bodyA=tool, :83-85) -- the observation's force;
//   on_human    robot-human and tool-human points (:90-96);
//   at          tool-human points on tool link 1, the cloth (:97-98);
//   wiping      those of them on a human link (linkB >= 0: not the base, :100-101) delete every
//               remaining target within 0.025 of their point on the human (positionOnB, :104-125).
// Deletions only remove targets, so the set deleted in a step -- and its count, new_contact_points
// -- is every live target within reach of any wiping point, whatever the pool order.
struct BBForces { float tool, on_human, at; int wiped; };
AVR_DI BBForces bb_forces(const KModel &m, EnvLDS &L, BBShared &B, const float *gcp, const float *btf) {
    const int lane = lane_id();
    const int n = (int)L.st[S_TASK + T_NCP];
    const int tb = m.tool_body, ts0 = gld(m.body_shape_start + tb);
    float ft = 0.f, fh = 0.f, fa = 0.f;
    bool wp = false;
    v3 p = V(0, 0, 0);
    if (lane < n) {        // (K_MAX_CONTACTS == 64: one point per lane)
        const float *cp = gcp + AVR_CP_WORDS * lane;
        const int sa = (int)cp[AVR_CP_SA], sb = (int)cp[AVR_CP_SB];
        const int ba = gld(m.shape_body + sa), bb = gld(m.shape_body + sb);
        const int ka = gld(m.body_kind + ba), kb = gld(m.body_kind + bb);
        const float f = cp[AVR_CP_IMP] / m.time_step;
        const bool ta = ba == tb, tbb = bb == tb;
        const bool ha = ka == AVR_BODY_HUMAN, hb = kb == AVR_BODY_HUMAN;
        const bool ra = ka == AVR_BODY_ROBOT || ka == AVR_BODY_RSTATIC, rb = kb == AVR_BODY_ROBOT || kb == AVR_BODY_RSTATIC;
        const bool toolhum = (ta && hb) || (tbb && ha);
        if (ta || tbb) ft = f;
        if (toolhum || (ra && hb) || (rb && ha)) fh = f;
        if (toolhum && (ta ? sa : sb) - ts0 >= m.tool_handle_shapes) {
            fa = f;
            const int hbody = ta ? bb : ba;
            if (gld(m.body_index + hbody) != 0) {          // human slot 0 is the base (link -1)
                wp = true;
                p = ta ? tfpt(ldtf(btf + 8 * bb), ld3(cp + AVR_CP_LB)) : tfpt(ldtf(btf + 8 * ba), ld3(cp + AVR_CP_LA));
            }
        }
    }
    static_assert(K_MAX_CONTACTS <= 64, "one contact point per lane");
    int tot = 0;
    const int j = ballot_prefix(wp, &tot);
    if (wp) { B.pts[j][0] = p.x; B.pts[j][1] = p.y; B.pts[j][2] = p.z; }
    BBForces r;
    r.tool = r.on_human = r.at = 0.f;
    for (int k = 0; k < 64; k++) { r.tool += __shfl(ft, k, 64); r.on_human += __shfl(fh, k, 64); r.at += __shfl(fa, k, 64); }
    SYNC();
    // targets: world position = limb slot frame x the target's limb-frame position
    const int g = L.gender;
    const int nu = m.bb_ntgt[g][0], nt = nu + m.bb_ntgt[g][1];
    const tf up = ldtf(L.st + S_HUMAN + 7 * m.bb_limb_slot[0]), fo = ldtf(L.st + S_HUMAN + 7 * m.bb_limb_slot[1]);
    for (int k = lane; k < AVR_BB_MAX_TARGETS; k += 64) {
        bool kill = false;
        if (k < nt && bb_alive(L.st, k)) {
            const float4 t = m.bb_tgt[g * AVR_BB_MAX_TARGETS + k];
            const v3 w = tfpt(k < nu ? up : fo, V(t.x, t.y, t.z));
            for (int q = 0; q < tot; q++)
                kill |= len(sub(ld3(B.pts[q]), w)) < 0.025f;
        }
        B.kill[k] = kill ? 1 : 0;
    }
    SYNC();
    if (lane == 0) {
        int wiped = 0;
        for (int w = 0; w < 6; w++) {
            int bits = (int)L.st[S_TASK + T_WIPE + w];
            for (int b = 0; b < 24; b++)
                if (B.kill[24 * w + b]) { bits &= ~(1 << b); wiped++; }
            L.st[S_TASK + T_WIPE + w] = (float)bits;
        }
        B.wiped = wiped;
    }
    SYNC();
    r.wiped = B.wiped;
    return r;
}

// min over the closest points of the tool and the human (bed_bathing.py:61): every tool shape
// against every human shape of the env's gender, the signed distance of each pair (negative:
// penetration) when within `closest_distance` (4.0); the narrowphase's lane path, then the
// wave-cooperative path (EPA) for the penetrating pairs it hands on.  A lane GJK that stalls with
// an open duality gap (rc 4) is queued in the env's workspace (WS_BB_*) for avr_bb_stall_kernel,
// which reruns it with the double simplex solve (gjk_coop_d, as the step's narrowphase does) and
// finishes the reward: the double code here would take this kernel from 211 to 256 VGPRs.  Pairs
// past the queue's capacity rerun on the fp32 cooperative GJK.  Poses: the state after the step
// (the tool's body frame, the human slots).
#define WS_BB_N 64          // int bits: queued stalled pairs
#define WS_BB_DMIN 65       // the minimum over the other pairs (BIGF: none within reach)
#define WS_BB_WIPED 66      // the step's wiped-target count
#define WS_BB_PREFS 67      // the human-preference terms
#define WS_BB_PAIRS 68      // int bits: sa | sb << 16 of each queued pair
#define WS_BB_CAP (WS_WORDS - WS_BB_PAIRS)
static_assert(WS_FW + 4 * MAXF <= WS_BB_N, "the stalled-pair queue lies past the velocity words");
AVR_DI float bb_closest(const KModel &m, const EnvLDS &L, EpaBuf &E, float *ws, int &nq) {
    const int lane = lane_id();
    nq = 0;
    const int tb = m.tool_body, ts0 = gld(m.body_shape_start + tb), nts = gld(m.body_shape_count + tb);
    int hs0 = 1 << 30, hs1 = 0;
    for (int b = 0; b < m.nb; b++)
        if (gld(m.body_kind + b) == AVR_BODY_HUMAN) {
            hs0 = min(hs0, gld(m.body_shape_start + b));
            hs1 = max(hs1, gld(m.body_shape_start + b) + gld(m.body_shape_count + b));
        }
    const tf ttf = ldtf(L.st + S_FREE);
    const float thr = m.closest_distance;
    const int npair = nts * max(hs1 - hs0, 0);
    float dmin = BIGF;
    for (int c0 = 0; c0 < npair; c0 += 64) {
        const int idx = c0 + lane;
        int sa = -1, sb = -1;
        bool coop = false, stall = false;
        if (idx < npair) {
            sb = hs0 + idx / nts;
            sa = ts0 + idx % nts;
            const int g = gld(m.shape_gender + sb);
            if (g >= 0 && g != L.gender) sa = -1;
        }
        if (sa >= 0) {
            const int bb = gld(m.shape_body + sb);
            const WShape A = make_wshape(m, sa, ttf), Bs = make_wshape(m, sb, ldtf(L.st + S_HUMAN + 7 * gld(m.body_index + bb)));
            if ((A.nv > SMALL_NV && A.tab < 0) || (Bs.nv > SMALL_NV && Bs.tab < 0)) coop = true;
            else {
                v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
                float d = 0.f;
                int nit, nk;
                const int rc = narrowphase<false>(m, E, A, Bs, thr, nB, pB, d, nit, nk);
                if (rc == 1) dmin = fminf(dmin, d);
                else if (rc == 4) stall = true;
                else if (rc == 2) coop = true;
            }
        }
        // stalled pairs into the queue, in order; past its capacity onto the fp32 cooperative path
        {
            int tot;
            const int pre = ballot_prefix(stall, &tot);
            if (stall) {
                if (nq + pre < WS_BB_CAP) ws[WS_BB_PAIRS + nq + pre] = __int_as_float(sa | sb << 16);
                else coop = true;
            }
            nq = min(nq + tot, WS_BB_CAP);
        }
        unsigned long long cm = __ballot(coop);
        while (cm) {
            const int l = __ffsll((long long)cm) - 1;
            cm &= cm - 1;
            const int csa = __shfl(sa, l, 64), csb = __shfl(sb, l, 64);
            const int bb = gld(m.shape_body + csb);
            const WShape A = make_wshape(m, csa, ttf), Bs = make_wshape(m, csb, ldtf(L.st + S_HUMAN + 7 * gld(m.body_index + bb)));
            v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
            float d = 0.f;
            int nit, nk;
            const int rc = narrowphase<true>(m, E, A, Bs, thr, nB, pB, d, nit, nk);
            SYNC();
            if (lane == 0 && rc == 1) dmin = fminf(dmin, d);
        }
    }
    for (int o = 32; o > 0; o >>= 1) dmin = fminf(dmin, __shfl_xor(dmin, o, 64));
    return dmin;
}

// the reward (bed_bathing.py:64-66, env.py:412-448), from the closest distance and the step's
// other terms; one expression for the task kernel and avr_bb_stall_kernel
AVR_DI float bb_reward(const KModel &m, float dmin, float asq, float wiped, float prefs) {
    dmin = dmin < BIGF ? dmin : m.closest_distance;      // (no pair within reach: the query's own bound)
    return m.w_distance * (-dmin) + m.w_action * (-asq) + m.w_wipe * wiped + prefs;
}

// Task glue after the frames (BedBathingEnv.step after take_step, bed_bathing.py:54-75); SETTLE
// mode: the reset observation (_get_obs([0], [0, 0]), :351).  NaN guard for every mode.
__global__ __launch_bounds__(64) void avr_task_kernel(const KModel *__restrict__ mp, float *__restrict__ state, float *__restrict__ obs,
                                                      float *__restrict__ rew, unsigned char *__restrict__ done, float *__restrict__ info,
                                                      const unsigned char *__restrict__ mask, int mode, int env0, int n_envs) {
    __shared__ EnvLDS L;
    __shared__ BBShared B;
    __shared__ EpaBuf E;
    AVR_ENV_GUARD();
    const int lane = lane_id();
    float *gst = state + (size_t)env * K_STATE_WORDS;
    const float *gcp = gst + S_CP;
    load_state(m, L, gst);
    robot_fk(m, L);          // robot link frames; the arm chain's slots while it is articulated (reset settle)
    if (mode == MODE_SETTLE) {
        if (obs) bb_observe(m, L, 0.f, obs + (size_t)env * K_OBS_DIM);
    } else if (mode == MODE_STEP || mode == MODE_STEP_RANDOM) {
        if (lane == 0) L.st[S_TASK + T_ITER] += 1.f;
        SYNC();
        const BBForces F = bb_forces(m, L, B, gcp, env_cs(m, env) + CS_BTF);
        float *ws = env_ws(m, env);
        int nq;
        const float dmin = bb_closest(m, L, E, ws, nq);
        const tf tb = ldtf(L.st + S_FREE);
        const v3 tip = qrot(tb.q, V(m.tool_tip[0], m.tool_tip[1], m.tool_tip[2]));
        // tool link 1's linear velocity (getLinkState(tool, 1, computeLinkVelocity=True)[6], :55)
        const float ee_vel = len(add(ld3(L.st + S_FREE + 7), crs(ld3(L.st + S_FREE + 10), tip)));
        bb_observe(m, L, F.tool, obs + (size_t)env * K_OBS_DIM);
        // human_preferences (env.py:412-448), wiping branch: tool_force_at_target = tool force on the human
        const float prefs = m.w_velocity * (-ee_vel) + m.w_force_nontarget * (-(F.on_human - F.at)) + m.w_high_forces * (F.at < 10.f ? 0.f : -F.at);
        const float asq = ws[WS_ASQ];
        const float r = bb_reward(m, dmin, asq, (float)F.wiped, prefs);
        SYNC();
        if (lane == 0) {
            // (avr_bb_stall_kernel finishes the reward of an env with queued pairs)
            ws[WS_BB_N] = __int_as_float(nq);
            ws[WS_BB_DMIN] = dmin;
            ws[WS_BB_WIPED] = (float)F.wiped;
            ws[WS_BB_PREFS] = prefs;
            const float succ = L.st[S_TASK + T_SUCCESS] + (float)F.wiped;
            L.st[S_TASK + T_SUCCESS] = succ;
            rew[env] = r;
            done[env] = (unsigned char)((int)L.st[S_TASK + T_ITER] >= m.max_steps);
            info[(size_t)env * AVR_INFO_DIM + 0] = F.on_human;
            info[(size_t)env * AVR_INFO_DIM + 1] = succ >= L.st[S_TASK + T_NTGT] * m.task_success_threshold ? 1.f : 0.f;
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

// The closest-distance pairs whose lane GJK stalled (bb_closest's queue), rerun with the
// cooperative GJK's double simplex solve -- the step narrowphase's treatment of the same stop --
// and the reward finished from the full minimum (bb_reward).  One wave per env; an env with an
// empty queue (nearly all) returns at once.
__global__ __launch_bounds__(64) void avr_bb_stall_kernel(const KModel *__restrict__ mp, float *__restrict__ state, float *__restrict__ rew,
                                                          const unsigned char *__restrict__ mask, int env0, int n_envs) {
    __shared__ EpaBuf E;
    const int env = env0 + blockIdx.x;
    if (env >= n_envs || (mask && !mask[env])) return;
    const KModel &m = *mp;
    float *ws = env_ws(m, env);
    const int nq = __float_as_int(ws[WS_BB_N]);
    if (nq <= 0) return;
    const float *gst = state + (size_t)env * K_STATE_WORDS;
    const tf ttf = ldtf(gst + S_FREE);
    const float thr = m.closest_distance;
    float dmin = ws[WS_BB_DMIN];
    for (int k = 0; k < nq; k++) {
        const int key = __float_as_int(ws[WS_BB_PAIRS + k]);
        const int sa = key & 0xffff, sb = key >> 16;
        const int bb = gld(m.shape_body + sb);
        const WShape A = make_wshape(m, sa, ttf), Bs = make_wshape(m, sb, ldtf(gst + S_HUMAN + 7 * gld(m.body_index + bb)));
        v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
        float d = 0.f;
        int nit, nk;
        const int rc = narrowphase<true>(m, E, A, Bs, thr, nB, pB, d, nit, nk, nullptr, true);
        SYNC();
        if (rc == 1) dmin = fminf(dmin, d);
    }
    if (lane_id() == 0) rew[env] = bb_reward(m, dmin, ws[WS_ASQ], ws[WS_BB_WIPED], ws[WS_BB_PREFS]);
}
