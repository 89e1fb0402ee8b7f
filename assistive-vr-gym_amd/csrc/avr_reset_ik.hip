// avr_reset_ik.hip -- batched reset IK on the device (avr_reset_ik, include/avr.h).
//
// Restates the reset's inverse kinematics with random restarts (util.py:34-105
// ik_random_restarts; feeding.py:276-278 for FeedingJaco: the tool link's COM frame to the
// spoon-above-bowl target) as damped least squares, one 64-lane block per env:
//   per restart r: the arm DoFs start from init[env][r] (the host draws them from the env's
//   reset stream, so the restart sequence is the host reset's); `iters` DLS updates
//     dq = J^T (J J^T + 1e-4 I)^-1 [p* - p; rot_err(q*, q)],  q <- clamp(q + dq, lower, upper)
//   with an early exit at every 10th iteration once |dp| < 1e-5 and |rot_err| < 1e-4;
//   step_sim's self-contact screening (util.py:41-46): when the robot's links touch each other at
//   the solution, the target orientation becomes alt[env][r] (the orientation re-drawn +-45 deg
//   about the original's Euler angles, drawn by the host) for this restart's check and the later
//   restarts; accept when |p* - p| < tol and |q* - q| < tol or |q* - q| within tol of 2
//   (util.py:49, np.isclose), and no robot hull vertex lies inside the keep-out box (the reset's
//   table screening, avr/reset.py table_clear); when no restart is accepted, the restart closest
//   to the target position is kept (util.py:51-54).
// The same rules as the host path's ik_batch (avr/reset.py) run on one env at a time; the host
// path is the checker of this kernel (tests/test_reset_ik.py).
// After the IK the task places the tool-attached free bodies (FeedingJaco: the spoon on the
// tool frame, world_creation.py:330-343, and the food spheres above it, feeding.py:291-308).

// Robot self-contact at the pose in L (robot FK done): what p.getContactPoints(robot, robot)
// reports (the Jaco is loaded with URDF_USE_SELF_COLLISION, world_creation.py:282), at the IK
// solution itself -- the reference asks after a restart's 5 simulated frames (util.py:41-46);
// these are not simulated here, a known difference (host and device alike).  The step's
// collision pipeline on the compiled robot-robot candidate pairs (parent-child pairs are not
// candidates): fattened body AABBs, child AABB culling (bare pairs unculled), the lane
// narrowphase within the pair's contact threshold, one lane per candidate pair; the pairs the
// lane path hands on (rc 2: penetrating cores or a hull without a support table, rc 4: a stalled
// GJK) are appended to Q and resolved by the wave-cooperative narrowphase (EPA, double GJK), as
// the step resolves them.  A pair beyond Q's capacity counts as touching.  Returns the number of
// touching shape pairs in every lane.
struct SelfQ {
    static constexpr int CAP = 64;
    int n;
    int2 e[CAP];       // (sa | sb << 16, ba | bb << 16 | rc 4 << 31)
};
template <class LT>
AVR_DI int robot_self_contacts(const KModel &m, const LT &L, EpaBuf &E, SelfQ &Q) {
    const int lane = lane_id();
    int cnt = 0;
    if (lane == 0) Q.n = 0;
    SYNC();
    for (int p0 = 0; p0 < m.np; p0 += 64) {
        const int p = p0 + lane;
        if (p >= m.np) continue;
        const int4 r = m.pair_rec[p];
        const int ba = r.x & 0xffff, bb = r.x >> 16;
        if (gld(m.body_kind + ba) != AVR_BODY_ROBOT || gld(m.body_kind + bb) != AVR_BODY_ROBOT) continue;
        const tf ta = body_tf(m, L, ba), tb = body_tf(m, L, bb);
        const v3 e = V(BT_BROADPHASE_EXPAND, BT_BROADPHASE_EXPAND, BT_BROADPHASE_EXPAND);
        v3 amn, amx, bmn, bmx;
        aabb_of(ta, gld3(m.body_aabb + 12 * ba), gld3(m.body_aabb + 12 * ba + 3), amn, amx);
        aabb_of(tb, gld3(m.body_aabb + 12 * bb), gld3(m.body_aabb + 12 * bb + 3), bmn, bmx);
        if (!overlap(sub(amn, e), add(amx, e), sub(bmn, e), add(bmx, e))) continue;
        const float thr = fminf(gld(m.body_threshold + ba), gld(m.body_threshold + bb));
        const bool bare = (r.w & 1) != 0;
        const int sa0 = r.y & 0xffff, na = r.y >> 16, sb0 = r.z & 0xffff, nb = r.z >> 16;
        for (int i = 0; i < na; i++) {
            v3 a0, a1;
            shape_aabb(m, sa0 + i, ta, a0, a1);
            for (int j = 0; j < nb; j++) {
                v3 b0, b1;
                shape_aabb(m, sb0 + j, tb, b0, b1);
                if (!bare && !overlap(a0, a1, b0, b1)) continue;
                const WShape A = make_wshape(m, sa0 + i, ta), B = make_wshape(m, sb0 + j, tb);
                int rc = 2;     // (a hull the lane GJK cannot take)
                if (!((A.nv > SMALL_NV && A.tab < 0) || (B.nv > SMALL_NV && B.tab < 0))) {
                    v3 nB, pB;
                    float d;
                    int nit, nk;
                    rc = narrowphase<false>(m, E, A, B, thr, nB, pB, d, nit, nk);   // (the lane path never touches the EPA buffer)
                }
                if (rc == 2 || rc == 4) {
                    const int k = atomicAdd(&Q.n, 1);
                    if (k < SelfQ::CAP) Q.e[k] = make_int2((sa0 + i) | (sb0 + j) << 16, ba | bb << 16 | (rc == 4 ? (int)0x80000000u : 0));
                    else cnt++;
                } else cnt += rc != 0;
            }
        }
    }
    for (int o = 32; o; o >>= 1) cnt += __shfl_xor(cnt, o);
    SYNC();
    const int nq = min(Q.n, SelfQ::CAP);
    for (int k = 0; k < nq; k++) {
        const int2 q = Q.e[k];
        const int ba = q.y & 0x7fff, bb = (q.y >> 16) & 0x7fff;
        const float thr = fminf(gld(m.body_threshold + ba), gld(m.body_threshold + bb));
        const WShape A = make_wshape(m, q.x & 0xffff, body_tf(m, L, ba)), B = make_wshape(m, q.x >> 16, body_tf(m, L, bb));
        v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
        float d = 0.f;
        int nit, nk;
        const int rc = narrowphase<true>(m, E, A, B, thr, nB, pB, d, nit, nk, nullptr, q.y < 0);
        SYNC();
        cnt += rc == 1;
    }
    return cnt;
}

struct IkLDS {
    float J[8][8];     // [arm column][6 rows] (+ pad)
    float err[8];
    float y[8];
    float JJ[36];
    float pe, qe;
    int stop, clear;
};

// |J J^T + 1e-4 I| y = err by Cholesky (6 x 6, lane 0)
AVR_DI void ik_solve6(const float *A_, const float *b, float *y) {
    float Lm[36];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j <= i; j++) {
            float s = A_[6 * i + j];
            for (int k = 0; k < j; k++) s -= Lm[6 * i + k] * Lm[6 * j + k];
            Lm[6 * i + j] = i == j ? sqrtf(fmaxf(s, 1e-20f)) : s / Lm[6 * j + j];
        }
    float z[6];
    for (int i = 0; i < 6; i++) {
        float s = b[i];
        for (int k = 0; k < i; k++) s -= Lm[6 * i + k] * z[k];
        z[i] = s / Lm[6 * i + i];
    }
    for (int i = 5; i >= 0; i--) {
        float s = z[i];
        for (int k = i + 1; k < 6; k++) s -= Lm[6 * k + i] * y[k];
        y[i] = s / Lm[6 * i + i];
    }
}

// rotation error of q_cur towards q_tgt as a rotation vector (avr/reset.py _rot_err)
AVR_DI v3 ik_rot_err(qt tgt, qt cur) {
    qt d = qmul(tgt, qconj(cur));
    if (d.w < 0.f) d = Q(-d.x, -d.y, -d.z, -d.w);
    const float s = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
    if (!(s > 1e-12f)) return V(0, 0, 0);
    const float ang = 2.f * atan2f(s, d.w);
    return scl(V(d.x, d.y, d.z), ang / s);
}

__global__ __launch_bounds__(64) void avr_reset_ik_kernel(const KModel *__restrict__ mp, float *__restrict__ state, const unsigned char *__restrict__ mask,
                                                          const float *__restrict__ target, const float *__restrict__ init, const float *__restrict__ alt, int R,
                                                          int iters, float tol, float4 box_c, float4 box_he, unsigned char *__restrict__ ok,
                                                          int n_envs) {
    __shared__ PairsLDS L;
    __shared__ IkLDS K;
    __shared__ EpaBuf E;
    __shared__ SelfQ SQ;
    const int env = blockIdx.x;
    if (env >= n_envs || !mask[env]) return;     // uniform over the block
    const KModel &m = *mp;
    const int lane = lane_id();
    float *gst = state + (size_t)env * K_STATE_WORDS;
    load_state(m, L, gst);
    const int link = m.tool_link, na = m.n_arm;
    const v3 tp = V(target[7 * env + 0], target[7 * env + 1], target[7 * env + 2]);
    qt tq = Q(target[7 * env + 3], target[7 * env + 4], target[7 * env + 5], target[7 * env + 6]);
    // this lane's arm column: DoF, the link that owns it (if on the tool link's chain), limits
    int cdof = -1, clink = -1;
    float lo = 0.f, hi = 0.f;
    if (lane < na) {
        cdof = m.arm_dofs[lane];
        const int l = m.dof_link[cdof];
        clink = is_ancestor(m, link, l) ? l : -1;
        lo = m.arm_lower[lane] > -1e9f ? m.arm_lower[lane] : -6.283185307179586f;
        hi = m.arm_upper[lane] < 1e9f ? m.arm_upper[lane] : 6.283185307179586f;
    }
    bool accepted = false;
    float best_pe = 3.4e38f, bestq = 0.f;      // the restart closest to the target position (util.py:51-54)
    for (int r = 0; r < R; r++) {
        if (lane < na) L.st[S_Q + cdof] = init[((size_t)env * R + r) * na + lane];
        SYNC();
        for (int it = 0; it < iters; it++) {
            robot_fk(m, L);
            const v3 cp = ld3(L.cm[link]);
            if (lane == 0) {
                const v3 ep = sub(tp, cp);
                const v3 er = ik_rot_err(tq, ldq(L.cm[link] + 3));
                K.err[0] = ep.x; K.err[1] = ep.y; K.err[2] = ep.z;
                K.err[3] = er.x; K.err[4] = er.y; K.err[5] = er.z;
                K.stop = (it % 10 == 9) && len(ep) < 1e-5f && len(er) < 1e-4f;
            }
            if (lane < na) {
                float *c = K.J[lane];
                if (clink >= 0) {
                    const v3 ax = ld3(L.ax[clink]);
                    st3(c, crs(ax, sub(cp, ld3(L.org[clink]))));
                    st3(c + 3, ax);
                } else {
                    for (int i = 0; i < 6; i++) c[i] = 0.f;
                }
            }
            SYNC();
            if (K.stop) break;
            if (lane < 36) {
                const int i = lane / 6, j = lane - 6 * (lane / 6);
                float s = i == j ? 1e-4f : 0.f;
                for (int c = 0; c < na; c++) s += K.J[c][i] * K.J[c][j];
                K.JJ[lane] = s;
            }
            SYNC();
            if (lane == 0) ik_solve6(K.JJ, K.err, K.y);
            SYNC();
            if (lane < na) {
                float dq = 0.f;
                for (int i = 0; i < 6; i++) dq += K.J[lane][i] * K.y[i];
                L.st[S_Q + cdof] = clampf(L.st[S_Q + cdof] + dq, lo, hi);
            }
            SYNC();
        }
        robot_fk(m, L);
        // step_sim's self-contact screening: a touching solution re-orients the target
        if (alt && robot_self_contacts(m, L, E, SQ) > 0) {
            const float *a = alt + ((size_t)env * R + r) * 4;
            tq = Q(a[0], a[1], a[2], a[3]);
        }
        if (lane == 0) {
            const qt cq = ldq(L.cm[link] + 3);
            K.pe = len(sub(tp, ld3(L.cm[link])));
            K.qe = sqrtf((tq.x - cq.x) * (tq.x - cq.x) + (tq.y - cq.y) * (tq.y - cq.y) + (tq.z - cq.z) * (tq.z - cq.z) + (tq.w - cq.w) * (tq.w - cq.w));
            K.clear = 1;
        }
        SYNC();
        if (K.pe < best_pe) {       // (wave-uniform)
            best_pe = K.pe;
            if (lane < na) bestq = L.st[S_Q + cdof];
        }
        // util.py:49: |dq| < tol, or np.isclose(|dq|, 2, atol=tol) (the other cover of the rotation)
        if (K.pe < tol && (K.qe < tol || fabsf(K.qe - 2.f) <= tol + 2e-5f)) {
            // keep-out screening: every hull vertex of every robot link outside the box
            if (box_he.x >= 0.f) {
                bool inside = false;
                for (int b = 0; b < m.nb; b++) {
                    if (m.body_kind[b] != AVR_BODY_ROBOT) continue;
                    const tf lc = ldtf(L.cm[m.body_index[b]]);
                    const int s0 = m.body_shape_start[b], s1 = s0 + m.body_shape_count[b];
                    for (int s = s0; s < s1; s++) {
                        if (m.shape_kind[s] != 3) continue;          // convex hulls
                        const tf w = tfmul(lc, gldtf(m.shape_pose + 8 * s));
                        const int v0 = m.shape_hull[4 * s], nv = m.shape_hull[4 * s + 1];
                        for (int v = lane; v < nv; v += 64) {
                            const float4 hv = m.hull_verts[v0 + v];
                            const v3 p = tfpt(w, V(hv.x, hv.y, hv.z));
                            inside |= fabsf(p.x - box_c.x) <= box_he.x && fabsf(p.y - box_c.y) <= box_he.y && fabsf(p.z - box_c.z) <= box_he.z;
                        }
                    }
                }
                if (inside) K.clear = 0;       // benign race: every writer stores 0
            }
            SYNC();
            accepted = K.clear != 0;
        }
        if (accepted) break;
    }
    if (!accepted) {
        if (lane < na) L.st[S_Q + cdof] = bestq;
        SYNC();
        robot_fk(m, L);                 // (the tool frame of the kept joints places the spoon)
    }
    if (lane < na) gst[S_Q + cdof] = L.st[S_Q + cdof];
    if (lane == 0) ok[env] = accepted ? 1 : 0;
#if AVR_TASK == AVR_TASK_FEEDING
    // spoon on the tool frame, food spheres of radius 0.005 stacked above it, all at rest
    if (lane == 0) {
        const tf sp = tfmul(ldtf(L.cm[link]), gldtf(m.tool_offset));
        float *f = gst + S_FREE + AVR_FB_WORDS * m.spoon_free;
        sttf(f, sp);
        for (int k = 7; k < AVR_FB_WORDS; k++) f[k] = 0.f;
        const float r = 0.005f;
        for (int k = 0; k < m.n_food; k++) {
            const int i = k >> 2, j = (k >> 1) & 1, kk = k & 1;
            float *g = gst + S_FREE + AVR_FB_WORDS * (m.food_free0 + k);
            st3(g, add(sp.p, V(i * 2 * r - 0.005f, j * 2 * r, kk * 2 * r + 0.02f)));
            stq(g + 3, Q(0, 0, 0, 1));
            for (int q = 7; q < AVR_FB_WORDS; q++) g[q] = 0.f;
        }
    }
#endif
}

hipError_t avr_launch_reset_ik(const KModel *d_m, float *state, const unsigned char *mask, const float *target, const float *init, const float *alt, int R,
                               int iters, float tol, const float *box8, unsigned char *ok, int n_envs, hipStream_t st) {
    if (n_envs <= 0) return hipSuccess;
    const float4 c = box8 ? make_float4(box8[0], box8[1], box8[2], 0.f) : make_float4(0, 0, 0, 0);
    const float4 he = box8 ? make_float4(box8[4], box8[5], box8[6], 0.f) : make_float4(-1, -1, -1, 0);
    hipLaunchKernelGGL(avr_reset_ik_kernel, dim3(n_envs), dim3(64), 0, st, d_m, state, mask, target, init, alt, R, iters, tol, c, he, ok, n_envs);
    return hipGetLastError();
}

// avr_robot_self_contact: the screening above at n given joint vectors (q: n x avr_n_dof, the
// rest of each pose from env 0's state block); out[i] = touching robot shape pairs
__global__ __launch_bounds__(64) void avr_self_contact_kernel(const KModel *__restrict__ mp, const float *__restrict__ state, const float *__restrict__ q,
                                                              int *__restrict__ out, int n) {
    __shared__ PairsLDS L;
    __shared__ EpaBuf E;
    __shared__ SelfQ SQ;
    const int i = blockIdx.x;
    if (i >= n) return;
    const KModel &m = *mp;
    load_state(m, L, state);
    SYNC();
    const int nq = m.nd + m.hc_n;      // (avr_n_dof: robot DoFs, then the human chain's)
    for (int d = lane_id(); d < nq; d += 64) L.st[S_Q + d] = q[(size_t)i * nq + d];
    SYNC();
    robot_fk(m, L);
    const int c = robot_self_contacts(m, L, E, SQ);
    if (lane_id() == 0) out[i] = c;
}

hipError_t avr_launch_self_contact(const KModel *d_m, const float *state, const float *q, int *out, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_self_contact_kernel, dim3(n), dim3(64), 0, st, d_m, state, q, out, n);
    return hipGetLastError();
}

// avr_narrowphase_query (test hook): the step's wave-cooperative narrowphase (closed forms, GJK
// with margins, EPA for penetrating cores) between shapes sa and sb at given body poses, one
// wave per query -> {rc, normal on B xyz, point on B xyz, distance}
__global__ __launch_bounds__(64) void avr_np_query_kernel(const KModel *__restrict__ mp, const int *__restrict__ pairs, const float *__restrict__ poses,
                                                          float thr, float *__restrict__ out, int n) {
    __shared__ EpaBuf E;
    const int q = blockIdx.x;
    if (q >= n) return;
    const KModel &m = *mp;
    const float *pa = poses + 14 * (size_t)q, *pb = pa + 7;
    tf ta, tb;
    ta.p = V(pa[0], pa[1], pa[2]); ta.q = Q(pa[3], pa[4], pa[5], pa[6]);
    tb.p = V(pb[0], pb[1], pb[2]); tb.q = Q(pb[3], pb[4], pb[5], pb[6]);
    const WShape A = make_wshape(m, pairs[2 * q], ta), B = make_wshape(m, pairs[2 * q + 1], tb);
    v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
    float d = 0.f;
    int nit, nk;
    // as the step runs it: a lane GJK that stalls with an open duality gap (rc 4) hands the pair
    // to the cooperative GJK in double (np_coop); every other pair gets the cooperative fp32 path
    // (sphere-hull pairs take the point-core lane GJK, ph_step, which hands nothing over this way)
    const bool big = (A.nv > SMALL_NV && A.tab < 0) || (B.nv > SMALL_NV && B.tab < 0);
    const bool sph = (A.kind == AVR_SPHERE && B.kind == AVR_HULL) || (A.kind == AVR_HULL && B.kind == AVR_SPHERE);
    const bool dbl = !big && !sph && narrowphase<false>(m, E, A, B, thr, nB, pB, d, nit, nk) == 4;
    nB = V(0, 0, 0); pB = V(0, 0, 0); d = 0.f;
    const int rc = narrowphase<true>(m, E, A, B, thr, nB, pB, d, nit, nk, nullptr, dbl);
    if (lane_id() == 0) {
        float *o = out + 8 * (size_t)q;
        o[0] = (float)rc; o[1] = nB.x; o[2] = nB.y; o[3] = nB.z; o[4] = pB.x; o[5] = pB.y; o[6] = pB.z; o[7] = d;
    }
}

hipError_t avr_launch_np_query(const KModel *d_m, const int *pairs, const float *poses, float thr, float *out, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_np_query_kernel, dim3(n), dim3(64), 0, st, d_m, pairs, poses, thr, out, n);
    return hipGetLastError();
}
