// avr_base_search.hip -- the PR2 tasks' base-pose search on the device (avr_base_search,
// include/avr.h).
//
// Restates position_robot_toc (env.py:489-585; scratch_itch.py:189-190, bed_bathing.py:317) as
// avr/reset_scratch.position_robot_toc does on the host, with one lane per (env, attempt):
//   the attempt's base pose (drawn by the host) and its IK rest pose start four damped-least-
//   squares solves of the tool link's COM frame (util.py:59-74 ik_jlwki, success threshold tol):
//   the start goal (position and the identity orientation; a failure discards the attempt), then
//   the shoulder, elbow and wrist positions; each reached goal adds its joint-limit-weighted
//   kinematic isotropy (JLWKI, env.py:466-477,536-553) to the attempt's manipulability.
//   DLS update: dq = J^T (J J^T + 1e-4 I)^-1 err, q <- clamp(q + dq, lower, upper); a lane stops
//   a solve at an iteration it % 10 == 9 where every |err| component is below 1e-6.
// A second kernel (one thread per env) picks the best attempt: most goals reached, then the
// largest manipulability, the first on ties; with no start goal reached, the attempt that came
// closest to it.  The host path (reset_scratch.position_robot_toc, fp64) is this kernel's checker
// (tests/test_base_search.py).

#define BS_MAXC 8        // arm columns (n_arm <= 8)

// per lane (private LDS rows, no sharing): the arm's joints and, per arm column on the tool
// link's chain, the joint origin and world axis of the last FK
struct BsLane { float q[BS_MAXC]; float oa[BS_MAXC][6]; };

// FK of the tool link's chain on base `t`: COM frame of the tool link; origin / world axis of
// every arm column on the chain into W.oa (the same products as reset_scratch.arm_fk)
AVR_DI tf bs_fk(const KModel &m, const int *colof, tf t, BsLane &W) {
    const int link = m.tool_link;
    for (unsigned b = m.anc_mask[link]; b; b &= b - 1u) {
        const int k = __builtin_ctz(b);
        const tf jo = gldtf(m.rl_jorig + 8 * k);
        const v3 ax = gld3(m.rl_axis + 4 * k);
        const int jt = gld(m.rl_jtype + k), c = colof[k];
        const float qv = c >= 0 ? W.q[c] : 0.f;
        t = tfmul(t, jo);
        const v3 aw = qrot(t.q, ax);
        if (c >= 0) { W.oa[c][0] = t.p.x; W.oa[c][1] = t.p.y; W.oa[c][2] = t.p.z; W.oa[c][3] = aw.x; W.oa[c][4] = aw.y; W.oa[c][5] = aw.z; }
        if (jt == AVR_J_REVOLUTE) t.q = qmul(t.q, qaxis(ax, qv));
        else if (jt == AVR_J_PRISMATIC) t.p = add(t.p, scl(aw, qv));
    }
    return tfmul(t, gldtf(m.rl_com + 8 * link));
}

// the Jacobian of the tool link's COM at cp: column c = [ax_c x (cp - o_c); ax_c] (0 past na)
AVR_DI void bs_jac(const BsLane &W, int na, v3 cp, float (&J)[6][BS_MAXC]) {
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++) {
        const v3 o = V(W.oa[c][0], W.oa[c][1], W.oa[c][2]), a = V(W.oa[c][3], W.oa[c][4], W.oa[c][5]);
        const v3 l = crs(a, sub(cp, o));
        const bool on = c < na;
        J[0][c] = on ? l.x : 0.f; J[1][c] = on ? l.y : 0.f; J[2][c] = on ? l.z : 0.f;
        J[3][c] = on ? a.x : 0.f; J[4][c] = on ? a.y : 0.f; J[5][c] = on ? a.z : 0.f;
    }
}

// y = (A)^-1 b for the symmetric positive definite R x R matrix A (Cholesky, registers);
// returns the product of the factor's diagonal (det A = that squared), 0 if A is not positive
template <int R>
AVR_DI float bs_chol_solve(float (&A)[6][6], const float *b, float *y) {
    float Lm[R][R], z[R];
    float pd = 1.f;
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) {
            float s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= Lm[i][k] * Lm[j][k];
            if (i == j) {
                if (!(s > 0.f)) pd = 0.f;
                Lm[i][i] = sqrtf(fmaxf(s, 1e-30f));
                pd *= Lm[i][i];
            } else Lm[i][j] = s / Lm[j][j];
        }
    if (b) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            float s = b[i];
#pragma unroll
            for (int k = 0; k < i; k++) s -= Lm[i][k] * z[k];
            z[i] = s / Lm[i][i];
        }
#pragma unroll
        for (int i = R - 1; i >= 0; i--) {
            float s = z[i];
#pragma unroll
            for (int k = i + 1; k < R; k++) s -= Lm[k][i] * y[k];
            y[i] = s / Lm[i][i];
        }
    }
    return pd;
}

// one DLS solve from the rest pose towards tp (and the identity orientation when ORIENT); returns
// the tool link's final COM frame (W.q holds the joints, W.oa the final FK's columns)
template <bool ORIENT>
AVR_DI tf bs_ik(const KModel &m, const int *colof, tf base, BsLane &W, const float *rest, const float *lo, const float *hi, int na, v3 tp,
                int iters) {
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++) W.q[c] = c < na ? rest[c] : 0.f;
    constexpr int R = ORIENT ? 6 : 3;
    for (int it = 0; it < iters; it++) {
        const tf cf = bs_fk(m, colof, base, W);
        float err[6];
        const v3 ep = sub(tp, cf.p);
        err[0] = ep.x; err[1] = ep.y; err[2] = ep.z;
        if (ORIENT) {
            const v3 er = ik_rot_err(Q(0, 0, 0, 1), cf.q);
            err[3] = er.x; err[4] = er.y; err[5] = er.z;
        }
        if (it % 10 == 9) {
            bool conv = true;
#pragma unroll
            for (int i = 0; i < R; i++) conv = conv && fabsf(err[i]) < 1e-6f;
            if (conv) break;
        }
        float J[6][BS_MAXC];
        bs_jac(W, na, cf.p, J);
        float A[6][6], y[6];
#pragma unroll
        for (int i = 0; i < R; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) {
                float s = i == j ? 1e-4f : 0.f;
#pragma unroll
                for (int c = 0; c < BS_MAXC; c++) s += J[i][c] * J[j][c];
                A[i][j] = s;
            }
        (void)bs_chol_solve<R>(A, err, y);
#pragma unroll
        for (int c = 0; c < BS_MAXC; c++) {
            if (c >= na) continue;
            float dq = 0.f;
#pragma unroll
            for (int i = 0; i < R; i++) dq += J[i][c] * y[i];
            W.q[c] = clampf(W.q[c] + dq, lo[c], hi[c]);
        }
    }
    return bs_fk(m, colof, base, W);
}

// JLWKI of the current joints: det(J W J^T)^(1/6) / (trace(J W J^T) / 6), W = diag of the
// joint-limit weights 1 - 0.5^((r - |r - q + lower|) / (0.05 r) + 1) >= 0.001, r = (upper - lower) / 2
AVR_DI float bs_jlwki(const BsLane &W, int na, v3 cp, const float *lo, const float *hi) {
    float J[6][BS_MAXC], w[BS_MAXC];
    bs_jac(W, na, cp, J);
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++) {
        const float qr = 0.5f * (hi[c] - lo[c]);
        const float e = (qr - fabsf(qr - W.q[c] + lo[c])) / (0.05f * qr) + 1.f;
        w[c] = c < na ? fmaxf(1.f - exp2f(-e), 0.001f) : 0.f;
    }
    float A[6][6];
    float tr = 0.f;
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) {
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < BS_MAXC; c++) s += J[i][c] * w[c] * J[j][c];
            A[i][j] = s;
            if (i == j) tr += s;
        }
    const float pd = bs_chol_solve<6>(A, nullptr, nullptr);     // sqrt(det)
    // det^(1/6) = pd^(1/3)
    return pd > 0.f ? cbrtf(pd) / (tr / 6.f) : 0.f;
}

// res[item] = {goals reached (-1: start goal missed), manipulability, start-goal position error,
// start-goal quaternion distance}; q[item][c] the start solve's joints
__global__ __launch_bounds__(64) void avr_base_search_kernel(const KModel *__restrict__ mp, const float *__restrict__ base7, const float *__restrict__ rest,
                                                             const float *__restrict__ tstart, const float *__restrict__ goals, int attempts, int iters,
                                                             float tol, float4 *__restrict__ res, float *__restrict__ qout, int n_items) {
    const KModel &m = *mp;
    __shared__ int colof[MAXL];
    __shared__ BsLane WL[64];
    const int lane = lane_id();
    for (int k = lane; k < MAXL; k += 64) {
        int c = -1;
        if (k < m.nla) {
            const int d = gld(m.rl_dof + k);
            for (int a = 0; a < m.n_arm; a++)
                if (d >= 0 && m.arm_dofs[a] == d) c = a;
        }
        colof[k] = c;
    }
    __syncthreads();
    const int item = blockIdx.x * 64 + lane;
    if (item >= n_items) return;
    BsLane &W = WL[lane];
    // arm columns off the tool link's chain keep a zero origin and axis: zero Jacobian columns
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++)
#pragma unroll
        for (int r = 0; r < 6; r++) W.oa[c][r] = 0.f;
    const int env = item / attempts, na = m.n_arm;
    float lo[BS_MAXC], hi[BS_MAXC], r0[BS_MAXC];
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++) {
        lo[c] = c < na ? (m.arm_lower[c] > -1e9f ? m.arm_lower[c] : -6.283185307179586f) : 0.f;
        hi[c] = c < na ? (m.arm_upper[c] < 1e9f ? m.arm_upper[c] : 6.283185307179586f) : 0.f;
        r0[c] = c < na ? rest[(size_t)item * na + c] : 0.f;
    }
    const float *b = base7 + (size_t)item * 7;
    const tf base = {V(b[0], b[1], b[2]), Q(b[3], b[4], b[5], b[6])};
    const v3 ts = V(tstart[3 * env], tstart[3 * env + 1], tstart[3 * env + 2]);
    // start goal: position and the identity orientation (util.py:72: quaternion distance within
    // tol of 0 or of 2, as the host path tests it)
    const tf s = bs_ik<true>(m, colof, base, W, r0, lo, hi, na, ts, iters);
    const float pe = len(sub(ts, s.p));
    const float qe = sqrtf(s.q.x * s.q.x + s.q.y * s.q.y + s.q.z * s.q.z + (1.f - s.q.w) * (1.f - s.q.w));
    const bool ok0 = pe < tol && (qe < tol || fabsf(qe - 2.f) < tol);
#pragma unroll
    for (int c = 0; c < BS_MAXC; c++)
        if (c < na) qout[(size_t)item * na + c] = W.q[c];
    int ng = -1;
    float man = 0.f;
    if (ok0) {
        ng = 1;
        man = bs_jlwki(W, na, s.p, lo, hi);
        for (int g = 0; g < 3; g++) {         // shoulder, elbow, wrist: positions only
            const float *gp = goals + 9 * env + 3 * g;
            const v3 tg = V(gp[0], gp[1], gp[2]);
            const tf f = bs_ik<false>(m, colof, base, W, r0, lo, hi, na, tg, iters);
            if (len(sub(tg, f.p)) < tol) {
                ng++;
                man += bs_jlwki(W, na, f.p, lo, hi);
            }
        }
    }
    res[item] = make_float4((float)ng, man, pe, qe);
}

// best attempt per env (one thread per env): most goals, then manipulability, the first on ties;
// none with the start goal: the smallest start-goal position error.  best[env] = attempt,
// ok[env] = 1 when the start goal was reached
__global__ void avr_base_pick_kernel(const float4 *__restrict__ res, int attempts, int *__restrict__ best, unsigned char *__restrict__ ok, int n_envs) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= n_envs) return;
    const float4 *r = res + (size_t)env * attempts;
    int bi = -1, ci = 0;
    for (int a = 0; a < attempts; a++) {
        const float4 x = r[a];
        if (x.x > 0.f && (bi < 0 || x.x > r[bi].x || (x.x == r[bi].x && x.y > r[bi].y))) bi = a;
        if (x.z < r[ci].z) ci = a;
    }
    best[env] = bi >= 0 ? bi : ci;
    ok[env] = bi >= 0 ? 1 : 0;
}

hipError_t avr_launch_base_search(const KModel *h_m, const KModel *d_m, const float *base7, const float *rest, const float *tstart, const float *goals,
                                  int attempts, int iters, float tol, float4 *res, float *qout, int *best, unsigned char *ok, int n_envs, hipStream_t st) {
    (void)h_m;
    const int n_items = n_envs * attempts;
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_base_search_kernel, dim3((n_items + 63) / 64), dim3(64), 0, st, d_m, base7, rest, tstart, goals, attempts, iters, tol, res,
                       qout, n_items);
    hipLaunchKernelGGL(avr_base_pick_kernel, dim3((n_envs + 63) / 64), dim3(64), 0, st, res, attempts, best, ok, n_envs);
    return hipGetLastError();
}
