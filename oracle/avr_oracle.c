/* avr_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement (double precision) of the
 * reference's hot path: one `gym.step` of FeedingJaco-v0 = AssistiveEnv.take_step
 * (env.py:274-351) around 5 x p.stepSimulation (env.py:342), each stepSimulation running
 * numSubSteps=2 Bullet sub-steps (feeding.py:289), followed by the task glue
 * get_total_force / get_food_rewards / _get_obs / reward (feeding.py:56-142) and
 * human_preferences (env.py:412-448).
 *
 * PARITY STATUS: PyBullet (bullet3) is an un-vendored third-party dependency that is absent
 * from this image.  The physics below restates Bullet's published algorithm from
 * its documented behaviour (btMultiBody ABA dynamics, btMultiBodyJointMotor /
 * JointLimitConstraint / FixedConstraint rows, btPersistentManifold, btGjkPairDetector,
 * btSequentialImpulse/btMultiBodyConstraintSolver PGS); every assumed default is a named
 * constant.  Against real PyBullet this oracle is *parity unpinned*; it is pinned by analytic
 * known-answer tests (tests/test_oracle_kat.py) and it pins the HIP path (GPU == oracle).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * library; the product (libavr.so) never links it.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/avr_model.h"

/* Task layout (include/avr_model.h): one build per task, AVR_TASK selects it (Makefile). */
#ifndef AVR_TASK
#define AVR_TASK AVR_TASK_FEEDING
#endif
#define T_TARGET 0
#define T_ITER 3
#define T_SUCCESS 4
#define T_GENDER 7
#define T_FLAGS 8
#define T_NCP 9
#define T_HDYN 10
#if AVR_TASK == AVR_TASK_FEEDING
#define K_MAX_LINKS AVR_MAX_LINKS
#define K_MAX_DOF AVR_MAX_DOF
#define K_HC_N AVR_HC_N
#define K_MAX_FREE AVR_MAX_FREE
#define K_MAX_HUMAN AVR_MAX_HUMAN
#define K_MAX_CONTACTS AVR_MAX_CONTACTS
#define K_ACT_DIM AVR_ACT_DIM
#define K_OBS_DIM AVR_OBS_DIM
#define S_Q AVR_S_Q
#define S_QD AVR_S_QD
#define S_QTGT AVR_S_QTGT
#define S_KP AVR_S_KP
#define S_MAXIMP AVR_S_MAXIMP
#define S_FREE AVR_S_FREE
#define S_TASK AVR_S_TASK
#define S_HUMAN AVR_S_HUMAN
#define S_HCH AVR_S_HCH
#define S_CP AVR_S_CP
#define K_STATE_WORDS AVR_STATE_WORDS
#define T_ALIVE AVR_T_ALIVE
#define T_HIT AVR_T_HIT
#else
#define K_MAX_LINKS AVR_SI_MAX_LINKS
#define K_MAX_DOF AVR_SI_MAX_DOF
#define K_HC_N AVR_SI_HC_N
#define K_MAX_FREE AVR_SI_MAX_FREE
#define K_MAX_HUMAN AVR_SI_MAX_HUMAN
#define K_MAX_CONTACTS AVR_SI_MAX_CONTACTS
#define K_ACT_DIM AVR_SI_ACT_DIM
#if AVR_TASK == AVR_TASK_BEDBATH
#define K_OBS_DIM AVR_BB_OBS_DIM
#define T_WIPE AVR_BB_T_WIPE
#define T_NTGT AVR_BB_T_NTGT
#else
#define K_OBS_DIM AVR_SI_OBS_DIM
#endif
#define S_Q AVR_SI_S_Q
#define S_QD AVR_SI_S_QD
#define S_QTGT AVR_SI_S_QTGT
#define S_KP AVR_SI_S_KP
#define S_MAXIMP AVR_SI_S_MAXIMP
#define S_FREE AVR_SI_S_FREE
#define S_RBASE AVR_SI_S_RBASE
#define S_TASK AVR_SI_S_TASK
#define S_HUMAN AVR_SI_S_HUMAN
#define S_HCH AVR_SI_S_HCH
#define S_CP AVR_SI_S_CP
#define K_STATE_WORDS AVR_SI_STATE_WORDS
#define T_LIMB AVR_SI_T_LIMB
#define T_STRENGTH AVR_SI_T_STRENGTH
#define T_PREV AVR_SI_T_PREV
#define T_TREMOR AVR_SI_T_TREMOR
#define T_ONARM AVR_SI_T_ONARM
#endif
#define SCRATCH (AVR_TASK == AVR_TASK_SCRATCH)
#define BEDBATH (AVR_TASK == AVR_TASK_BEDBATH)
#define PR2F (AVR_TASK != AVR_TASK_FEEDING)     /* the PR2 tasks: per-env base, composite tool, arm chain */

#ifdef AVR_ORACLE_FLOAT
typedef float real;
#define R(x) ((float)(x))
#else
typedef double real;
#define R(x) ((double)(x))
#endif

/* ---------------------------------------------------------------- assumed Bullet constants */
/* Precision probe build (-DAVR_ORACLE_PROBE, tools only): the fp64 oracle with chosen stage
 * outputs rounded to float (avr_oracle_probe_mask bits), to find where fp32 rounding is amplified */
#ifdef AVR_ORACLE_PROBE
static unsigned probe_mask;
#define PRB(k, x) ((probe_mask >> (k) & 1) ? (real)(float)(x) : (x))
#else
#define PRB(k, x) (x)
#endif
#define PRB3(k, v) V(PRB(k, (v).x), PRB(k, (v).y), PRB(k, (v).z))
#define BT_ANGULAR_MOTION_THRESHOLD (0.5 * 1.5707963267948966) /* btMultiBody quat update   */
#define BT_BROADPHASE_EXPAND 0.02      /* gContactBreakingThreshold AABB fattening           */
#define BT_DENOM_EPS 1e-12             /* SIMD_EPSILON guard on jacDiagABInv (double build)  */
/* PyBullet's solverResidualThreshold (btContactSolverInfo::m_leastSquaresResidualThreshold, which
 * PhysicsServerCommandProcessor sets to 1e-7 [ext]): the PGS stops after the first iteration whose
 * largest squared row residual -- the row's impulse change times its effective mass denominator,
 * max over every row resolved in that iteration -- is at most this
 * (btSequentialImpulseConstraintSolver::solveGroupCacheFriendlyIterations,
 * btMultiBodyConstraintSolver::solveSingleIteration [ext]).  One solve group per env. */
#define BT_RESIDUAL_THRESHOLD 1e-7
#define BT_LARGE 1e18
#define GJK_MAX_IT 64
#define GJK_REL_EPS 1e-6
#define EPA_MAX_IT 64
#define EPA_MAX_V 64
#define EPA_MAX_F 128
#define EPA_EPS 1e-6

typedef struct { real x, y, z; } v3;
typedef struct { real x, y, z, w; } qt;

static inline v3 V(real x, real y, real z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scl(v3 a, real s) { return V(a.x * s, a.y * s, a.z * s); }
static inline real dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 crs(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline real len2(v3 a) { return dot(a, a); }
static inline real len(v3 a) { return sqrt(dot(a, a)); }
static inline v3 ld3(const real *p) { return V(p[0], p[1], p[2]); }
static inline v3 ld3d(const double *p) { return V(R(p[0]), R(p[1]), R(p[2])); }
static inline void st3(real *p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
static inline qt Q(real x, real y, real z, real w) { qt r = {x, y, z, w}; return r; }
static inline qt ldq(const real *p) { return Q(p[0], p[1], p[2], p[3]); }
static inline qt ldqd(const double *p) { return Q(R(p[0]), R(p[1]), R(p[2]), R(p[3])); }
static inline void stq(real *p, qt a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; }
static inline qt qmul(qt a, qt b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
             a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
static inline qt qconj(qt a) { return Q(-a.x, -a.y, -a.z, a.w); }
static inline v3 qrot(qt q, v3 v) {
    v3 u = V(q.x, q.y, q.z);
    v3 t = scl(crs(u, v), R(2));
    return add(add(v, scl(t, q.w)), crs(u, t));
}
static inline qt qnorm(qt q) {
    real n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Q(q.x / n, q.y / n, q.z / n, q.w / n);
}
static inline qt qaxis(v3 a, real ang) {
    real s = sin(R(0.5) * ang);
    return Q(a.x * s, a.y * s, a.z * s, cos(R(0.5) * ang));
}
typedef struct { real m[3][3]; } m3;
static m3 qmat(qt q) {
    m3 r;
    real x = q.x, y = q.y, z = q.z, w = q.w;
    r.m[0][0] = 1 - 2 * (y * y + z * z); r.m[0][1] = 2 * (x * y - z * w); r.m[0][2] = 2 * (x * z + y * w);
    r.m[1][0] = 2 * (x * y + z * w); r.m[1][1] = 1 - 2 * (x * x + z * z); r.m[1][2] = 2 * (y * z - x * w);
    r.m[2][0] = 2 * (x * z - y * w); r.m[2][1] = 2 * (y * z + x * w); r.m[2][2] = 1 - 2 * (x * x + y * y);
    return r;
}
static inline v3 mv(const m3 *a, v3 v) {
    return V(a->m[0][0] * v.x + a->m[0][1] * v.y + a->m[0][2] * v.z, a->m[1][0] * v.x + a->m[1][1] * v.y + a->m[1][2] * v.z,
             a->m[2][0] * v.x + a->m[2][1] * v.y + a->m[2][2] * v.z);
}
static inline v3 mtv(const m3 *a, v3 v) {
    return V(a->m[0][0] * v.x + a->m[1][0] * v.y + a->m[2][0] * v.z, a->m[0][1] * v.x + a->m[1][1] * v.y + a->m[2][1] * v.z,
             a->m[0][2] * v.x + a->m[1][2] * v.y + a->m[2][2] * v.z);
}
/* world inertia R diag(I) R^T applied to v */
static inline v3 inertia_mul(qt q, v3 I, v3 v) {
    v3 l = qrot(qconj(q), v);
    return qrot(q, V(I.x * l.x, I.y * l.y, I.z * l.z));
}
static inline v3 inertia_inv_mul(qt q, v3 I, v3 v) {
    v3 l = qrot(qconj(q), v);
    return qrot(q, V(I.x > 0 ? l.x / I.x : 0, I.y > 0 ? l.y / I.y : 0, I.z > 0 ? l.z / I.z : 0));
}

typedef struct { v3 p; qt q; } tf;
static inline tf tfmul(tf a, tf b) { tf r; r.p = add(a.p, qrot(a.q, b.p)); r.q = qmul(a.q, b.q); return r; }
static inline v3 tfpt(tf a, v3 p) { return add(a.p, qrot(a.q, p)); }
static inline v3 tfinvpt(tf a, v3 p) { return qrot(qconj(a.q), sub(p, a.p)); }
static inline tf ldtf(const double *p) { tf r; r.p = ld3d(p); r.q = ldqd(p + 3); return r; }

/* ---------------------------------------------------------------- model (converted) */
/* A model view: the articulated system an env simulates.  View 0 is the robot alone (the
 * human is static: impairments none / limits / weakness, feeding.py:244 passes no controllable
 * joints); views 1 and 2 (male, female) append the tremor head/neck chain -- human joints
 * 24..27 as links nl_robot.. with DoFs nd_robot.. hanging off the static chest slot
 * (parent -2), plus the chain-vs-static body pairs (np = n_pairs). */
#define MAX_BODIES 64
typedef struct {
    avr_model_desc d;                 /* arrays point into the copies below */
    int nl, nd, nf, nb, ns, np;
    int nl_robot, nd_robot, hc;       /* hc: this view articulates the head chain */
    int parent[K_MAX_LINKS], jtype[K_MAX_LINKS], dof[K_MAX_LINKS], has_limit[K_MAX_LINKS];
    real lower[K_MAX_LINKS], upper[K_MAX_LINKS];
    int body_link[MAX_BODIES];        /* articulated link of a collision body, -1 if none */
    tf jorig[K_MAX_LINKS], com[K_MAX_LINKS];
    v3 axis[K_MAX_LINKS], inertia[K_MAX_LINKS];
    real mass[K_MAX_LINKS];
    tf base;
    real *hv;                         /* hull verts (real) */
    real *hp;                         /* hull planes       */
} model;

/* ---------------------------------------------------------------- per-env workspace */
#define MAX_ROWS 512
#define MAX_SHAPES 512
#define MAX_SPAIRS 256

typedef struct {
    int kindA, idxA, kindB, idxB;     /* endpoint kind: 0 none, 1 robot, 2 free */
    real JA[K_MAX_DOF], JB[K_MAX_DOF];      /* robot: ndof entries; free: 6 (lin, ang) */
    real MA[K_MAX_DOF], MB[K_MAX_DOF];      /* M^-1 J^T */
    real inv, rhs, lo, hi, imp, fric;
    int normal_row;                   /* friction rows: index into normal rows */
    int cp;                           /* contact point index (normal rows)     */
} row_t;

typedef struct {
    tf lk[K_MAX_LINKS];             /* link (URDF) frames */
    tf cm[K_MAX_LINKS];             /* COM frames         */
    v3 ax[K_MAX_LINKS], org[K_MAX_LINKS];
    tf body[MAX_BODIES];
    v3 bmin[MAX_BODIES], bmax[MAX_BODIES];
    real Mi[K_MAX_DOF][K_MAX_DOF];    /* Cholesky factor of M */
    real vq[K_MAX_DOF];                 /* robot velocity (post unconstrained) */
    v3 fv[K_MAX_FREE], fw[K_MAX_FREE];
    real dq[K_MAX_DOF];                 /* solver delta velocities */
    v3 dfv[K_MAX_FREE], dfw[K_MAX_FREE];
    row_t rows[MAX_ROWS];
    int nrows, n_nc, n_nrm, n_fr, n_tor;
    int nc_idx[64], nrm_idx[MAX_ROWS / 3 + 8], fr_idx[MAX_ROWS], tor_idx[MAX_ROWS];
    int sp_a[MAX_SPAIRS], sp_b[MAX_SPAIRS], sp_pair[MAX_SPAIRS];
    int nsp;
    int gender;
    real oldcp[K_MAX_CONTACTS * AVR_CP_WORDS];
    long long stats_gjk, stats_epa, stats_rows, stats_iters, stats_solves, stats_stall;
    int np_plain;          /* narrowphase without the lane GJK's stall rule (bb_closest) */
    int island_exit;       /* test-only: the PGS residual exit per island (solve_islands) */
} ws_t;

typedef struct avr_oracle {
    model m;             /* view 0 (static human) */
    model mv[2];         /* tremor views: male, female */
    int n_envs;
    real *state;         /* n_envs * K_STATE_WORDS */
    ws_t *ws;
    char err[256];
    int threads;
} avr_oracle;

/* the view an env simulates: T_HDYN (impairment 'tremor') selects the head-chain view */
static const model *oview(const avr_oracle *o, const real *st) {
    if (o->m.d.hc_n > 0 && st[S_TASK + T_HDYN] != 0) return &o->mv[(int)st[S_TASK + T_GENDER] ? 1 : 0];
    return &o->m;
}

/* ---------------------------------------------------------------- kinematics */
static tf slot_pose(const real *st, int slot) {
    const real *h = st + S_HUMAN + 7 * slot;
    tf t; t.p = ld3(h); t.q = ldq(h + 3);
    return t;
}

/* Link frames of the view's articulated links.  The head chain's root hangs off the chest slot
 * (parent -2); its link frames are its COM frames and are published into the human slot poses
 * so that collision and the task glue (getLinkState(human, 27), feeding.py:134,254) see them. */
static void robot_fk(const model *m, real *st, ws_t *w) {
    for (int i = 0; i < m->nl; i++) {
        int p = m->parent[i];
#if PR2F
        tf base; base.p = ld3(st + S_RBASE); base.q = ldq(st + S_RBASE + 3);   /* position_robot_toc: per env */
#else
        tf base = m->base;
#endif
        tf par = p == -2 ? slot_pose(st, m->d.hc_parent_slot) : p < 0 ? base : w->lk[p];
        tf t = tfmul(par, m->jorig[i]);
        w->org[i] = t.p;
        w->ax[i] = qrot(t.q, m->axis[i]);
        int dof = m->dof[i];
        if (m->jtype[i] == AVR_J_REVOLUTE) t.q = qmul(t.q, qaxis(m->axis[i], st[S_Q + dof]));
        else if (m->jtype[i] == AVR_J_PRISMATIC) t.p = add(t.p, scl(w->ax[i], st[S_Q + dof]));
        w->lk[i] = t;
        w->cm[i] = tfmul(t, m->com[i]);
#ifdef AVR_ORACLE_PROBE
        w->org[i] = PRB3(0, w->org[i]); w->ax[i] = PRB3(0, w->ax[i]);
        w->cm[i].p = PRB3(0, w->cm[i].p);
        w->cm[i].q = Q(PRB(0, w->cm[i].q.x), PRB(0, w->cm[i].q.y), PRB(0, w->cm[i].q.z), PRB(0, w->cm[i].q.w));
#endif
    }
    if (m->hc)
        for (int k = 0; k < m->d.hc_n; k++) {
            int slot = m->d.hc_slot[k];
            if (slot < 0) continue;
            real *h = st + S_HUMAN + 7 * slot;
            st3(h, w->cm[m->nl_robot + k].p);
            stq(h + 3, w->cm[m->nl_robot + k].q);
        }
}

static int is_ancestor_dof(const model *m, int link, int dof_link) {
    for (int k = link; k >= 0; k = m->parent[k])
        if (k == dof_link) return 1;
    return 0;
}

/* Jacobian column of DoF owned by link j for a point p (world) on a body downstream. */
static void dof_col(const model *m, const ws_t *w, int j, v3 p, v3 *lin, v3 *ang) {
    if (m->jtype[j] == AVR_J_REVOLUTE) {
        *ang = w->ax[j];
        *lin = crs(w->ax[j], sub(p, w->org[j]));
    } else {
        *ang = V(0, 0, 0);
        *lin = w->ax[j];
    }
}

/* Joint-space mass matrix (CRBA via Jacobians), Cholesky-factored in place. Equivalent to
 * btMultiBody's ABA solve for the same articulated inertia (fixed base). */
static int robot_mass_matrix(const model *m, ws_t *w) {
    int nd = m->nd;
    real M[K_MAX_DOF][K_MAX_DOF];
    memset(M, 0, sizeof(M));
    int dl[K_MAX_DOF];
    for (int j = 0; j < m->nl; j++)
        if (m->dof[j] >= 0) dl[m->dof[j]] = j;
    for (int i = 0; i < m->nl; i++) {
        real mi = m->mass[i];
        if (mi <= 0) continue;
        v3 c = w->cm[i].p;
        v3 lin[K_MAX_DOF], ang[K_MAX_DOF];
        int use[K_MAX_DOF];
        for (int a = 0; a < nd; a++) {
            use[a] = is_ancestor_dof(m, i, dl[a]);
            if (use[a]) dof_col(m, w, dl[a], c, &lin[a], &ang[a]);
        }
        for (int a = 0; a < nd; a++) {
            if (!use[a]) continue;
            v3 Ia = inertia_mul(w->cm[i].q, m->inertia[i], ang[a]);
            for (int b = 0; b <= a; b++) {
                if (!use[b]) continue;
                M[a][b] += mi * dot(lin[a], lin[b]) + dot(Ia, ang[b]);
            }
        }
    }
#ifdef AVR_ORACLE_PROBE
    for (int a = 0; a < nd; a++) for (int b = 0; b <= a; b++) M[a][b] = PRB(2, M[a][b]);
#endif
    /* Cholesky M = L L^T (lower) */
    for (int j = 0; j < nd; j++) {
        real s = M[j][j];
        for (int k = 0; k < j; k++) s -= w->Mi[j][k] * w->Mi[j][k];
        if (s <= 0) return -1;
        real d = sqrt(s);
        w->Mi[j][j] = d;
        for (int i = j + 1; i < nd; i++) {
            real t = M[i][j];
            for (int k = 0; k < j; k++) t -= w->Mi[i][k] * w->Mi[j][k];
            w->Mi[i][j] = t / d;
        }
    }
#ifdef AVR_ORACLE_PROBE
    for (int a = 0; a < nd; a++) for (int b = 0; b <= a; b++) w->Mi[a][b] = PRB(3, w->Mi[a][b]);
#endif
    return 0;
}

static void chol_solve(const model *m, const ws_t *w, const real *b, real *x) {
    int nd = m->nd;
    real y[K_MAX_DOF];
    for (int i = 0; i < nd; i++) {
        real s = b[i];
        for (int k = 0; k < i; k++) s -= w->Mi[i][k] * y[k];
        y[i] = s / w->Mi[i][i];
    }
    for (int i = nd - 1; i >= 0; i--) {
        real s = y[i];
        for (int k = i + 1; k < nd; k++) s -= w->Mi[k][i] * x[k];
        x[i] = s / w->Mi[i][i];
    }
#ifdef AVR_ORACLE_PROBE
    for (int i = 0; i < nd; i++) x[i] = PRB(4, x[i]);
#endif
}

/* Bias forces h(q,qd) by recursive Newton-Euler in world frame: Coriolis/centrifugal,
 * gyroscopic w x Iw, btMultiBody damping -(k1+k2|v|) m v, -(k1+k2|w|) I w (robot gravity is
 * zeroed per body in Feeding, feeding.py:285). */
static void robot_bias(const model *m, const real *st, ws_t *w, real *h) {
    int nl = m->nl;
    v3 om[K_MAX_LINKS], vc[K_MAX_LINKS], al[K_MAX_LINKS], ac[K_MAX_LINKS];
    v3 F[K_MAX_LINKS], N[K_MAX_LINKS];
    real k1l = R(m->d.linear_damping), k1a = R(m->d.angular_damping);
    for (int i = 0; i < nl; i++) {
        int p = m->parent[i];
        v3 omp = p < 0 ? V(0, 0, 0) : om[p];
        v3 vp = p < 0 ? V(0, 0, 0) : vc[p];
        v3 alp = p < 0 ? V(0, 0, 0) : al[p];
        v3 acp = p < 0 ? V(0, 0, 0) : ac[p];
        v3 cp = p < 0 ? m->base.p : w->cm[p].p;
        int dof = m->dof[i];
        real qd = dof >= 0 ? st[S_QD + dof] : 0;
        v3 o = w->org[i], c = w->cm[i].p;
        v3 rpo = sub(o, cp), roc = sub(c, o);
        v3 vo = add(vp, crs(omp, rpo));                               /* joint point velocity */
        v3 ao = add(acp, add(crs(alp, rpo), crs(omp, crs(omp, rpo))));
        if (m->jtype[i] == AVR_J_REVOLUTE) {
            v3 wj = scl(w->ax[i], qd);
            om[i] = add(omp, wj);
            al[i] = add(alp, crs(omp, wj));
            vc[i] = add(vo, crs(om[i], roc));
            ac[i] = add(ao, add(crs(al[i], roc), crs(om[i], crs(om[i], roc))));
        } else if (m->jtype[i] == AVR_J_PRISMATIC) {
            v3 vj = scl(w->ax[i], qd);
            om[i] = omp;
            al[i] = alp;
            vc[i] = add(add(vo, vj), crs(om[i], roc));
            ac[i] = add(add(ao, scl(crs(omp, vj), 2)), add(crs(al[i], roc), crs(om[i], crs(om[i], roc))));
        } else {
            om[i] = omp;
            al[i] = alp;
            vc[i] = add(vo, crs(om[i], roc));
            ac[i] = add(ao, add(crs(al[i], roc), crs(om[i], crs(om[i], roc))));
        }
        real mi = m->mass[i];
        qt q = w->cm[i].q;
        v3 Iw = inertia_mul(q, m->inertia[i], om[i]);
        real vn = len(vc[i]), wn = len(om[i]);
        v3 fdamp = scl(vc[i], -mi * (k1l + k1l * vn));
        v3 tdamp = scl(Iw, -(k1a + k1a * wn));
        /* gravity: F = m (a - g), the human chain's (ScratchItch -1 z) on links after the robot's,
           the robot's (0 in both tasks; known-answer tests set it) on the robot's */
        v3 g = i >= m->nl_robot ? ld3d(m->d.human_gravity) : ld3d(m->d.robot_gravity);
        F[i] = (g.x != 0 || g.y != 0 || g.z != 0) ? sub(scl(sub(ac[i], g), mi), fdamp) : sub(scl(ac[i], mi), fdamp);
        N[i] = sub(add(inertia_mul(q, m->inertia[i], al[i]), crs(om[i], Iw)), tdamp);
    }
    for (int d = 0; d < m->nd; d++) h[d] = 0;
    for (int i = nl - 1; i >= 0; i--) {
        int dof = m->dof[i];
        v3 o = w->org[i], c = w->cm[i].p;
        if (dof >= 0) {
            if (m->jtype[i] == AVR_J_REVOLUTE) h[dof] = dot(w->ax[i], add(N[i], crs(sub(c, o), F[i])));
            else h[dof] = dot(w->ax[i], F[i]);
        }
        int p = m->parent[i];
        if (p >= 0) {
            F[p] = add(F[p], F[i]);
            N[p] = add(N[p], add(N[i], crs(sub(c, w->cm[p].p), F[i])));
        }
    }
}

/* ---------------------------------------------------------------- shapes & support */
typedef struct {
    int kind;
    tf t;          /* world */
    real margin;
    v3 he;         /* box core half extents / capsule: (r, halfheight, 0) */
    const real *v; /* hull verts */
    int nv;
} wshape;

static wshape make_wshape(const model *m, int s, tf body) {
    wshape w;
    w.kind = m->d.shape_kind[s];
    w.t = tfmul(body, ldtf(m->d.shape_pose + 7 * s));
    w.margin = R(m->d.shape_margin[s]);
    const double *pa = m->d.shape_param + 4 * s;
    w.v = 0;
    w.nv = 0;
    if (w.kind == AVR_BOX) {
        w.he = V(fmax(R(pa[0]) - w.margin, 0), fmax(R(pa[1]) - w.margin, 0), fmax(R(pa[2]) - w.margin, 0));
    } else if (w.kind == AVR_CAPSULE) {
        w.he = V(R(pa[0]), R(pa[1]), 0);
    } else {
        w.he = V(R(pa[0]), 0, 0);
    }
    if (w.kind == AVR_HULL) {
        w.v = m->hv + 3 * m->d.shape_hull[4 * s + 0];
        w.nv = m->d.shape_hull[4 * s + 1];
    }
    return w;
}

/* support point of the shape CORE (no margin) in world direction d */
static v3 support(const wshape *s, v3 d) {
    v3 l = qrot(qconj(s->t.q), d);
    v3 r;
    switch (s->kind) {
    case AVR_SPHERE: r = V(0, 0, 0); break;
    case AVR_CAPSULE: r = V(0, 0, l.z >= 0 ? s->he.y : -s->he.y); break;
    case AVR_BOX: r = V(l.x >= 0 ? s->he.x : -s->he.x, l.y >= 0 ? s->he.y : -s->he.y, l.z >= 0 ? s->he.z : -s->he.z); break;
    default: {
        real best = -BT_LARGE;
        int bi = 0;
        for (int i = 0; i < s->nv; i++) {
            real dd = l.x * s->v[3 * i] + l.y * s->v[3 * i + 1] + l.z * s->v[3 * i + 2];
            if (dd > best) { best = dd; bi = i; }
        }
        r = V(s->v[3 * bi], s->v[3 * bi + 1], s->v[3 * bi + 2]);
    }
    }
    return tfpt(s->t, r);
}

/* ---------------------------------------------------------------- GJK (cores) */
typedef struct { v3 w[4], a[4], b[4]; int n; } simplex;

/* closest point on simplex to origin; reduces simplex to the supporting feature; returns
 * barycentric weights in lam; returns 1 if origin is inside a full tetrahedron */
static int simplex_closest(simplex *S, v3 *vout, real lam[4]) {
    if (S->n == 1) { lam[0] = 1; *vout = S->w[0]; return 0; }
    if (S->n == 2) {
        v3 A = S->w[0], B = S->w[1], ab = sub(B, A);
        real t = -dot(A, ab), dd = dot(ab, ab);
        if (t <= 0 || dd <= 0) { S->n = 1; lam[0] = 1; *vout = A; return 0; }
        if (t >= dd) { S->w[0] = S->w[1]; S->a[0] = S->a[1]; S->b[0] = S->b[1]; S->n = 1; lam[0] = 1; *vout = B; return 0; }
        t /= dd;
        lam[0] = 1 - t; lam[1] = t;
        *vout = add(A, scl(ab, t));
        return 0;
    }
    if (S->n == 3) {
        /* Ericson, closest point on triangle ABC to P = origin */
        v3 A = S->w[0], B = S->w[1], C = S->w[2];
        v3 ab = sub(B, A), ac = sub(C, A), ap = scl(A, -1);
        real d1 = dot(ab, ap), d2 = dot(ac, ap);
        if (d1 <= 0 && d2 <= 0) { S->n = 1; lam[0] = 1; *vout = A; return 0; }
        v3 bp = scl(B, -1);
        real d3 = dot(ab, bp), d4 = dot(ac, bp);
        if (d3 >= 0 && d4 <= d3) { S->w[0] = B; S->a[0] = S->a[1]; S->b[0] = S->b[1]; S->n = 1; lam[0] = 1; *vout = B; return 0; }
        real vc = d1 * d4 - d3 * d2;
        if (vc <= 0 && d1 >= 0 && d3 <= 0) {
            real v = d1 / (d1 - d3);
            S->n = 2; lam[0] = 1 - v; lam[1] = v; *vout = add(A, scl(ab, v)); return 0;
        }
        v3 cp = scl(C, -1);
        real d5 = dot(ab, cp), d6 = dot(ac, cp);
        if (d6 >= 0 && d5 <= d6) { S->w[0] = C; S->a[0] = S->a[2]; S->b[0] = S->b[2]; S->n = 1; lam[0] = 1; *vout = C; return 0; }
        real vb = d5 * d2 - d1 * d6;
        if (vb <= 0 && d2 >= 0 && d6 <= 0) {
            real wv = d2 / (d2 - d6);
            S->w[1] = C; S->a[1] = S->a[2]; S->b[1] = S->b[2]; S->n = 2;
            lam[0] = 1 - wv; lam[1] = wv; *vout = add(A, scl(ac, wv)); return 0;
        }
        real va = d3 * d6 - d5 * d4;
        if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
            real wv = (d4 - d3) / ((d4 - d3) + (d5 - d6));
            S->w[0] = B; S->a[0] = S->a[1]; S->b[0] = S->b[1];
            S->w[1] = C; S->a[1] = S->a[2]; S->b[1] = S->b[2]; S->n = 2;
            lam[0] = 1 - wv; lam[1] = wv; *vout = add(B, scl(sub(C, B), wv)); return 0;
        }
        real den = 1 / (va + vb + vc);
        real v = vb * den, wv = vc * den;
        lam[0] = 1 - v - wv; lam[1] = v; lam[2] = wv;
        *vout = add(A, add(scl(ab, v), scl(ac, wv)));
        return 0;
    }
    /* tetrahedron: test the faces that can see the origin */
    static const int F[4][4] = {{0, 1, 2, 3}, {0, 3, 1, 2}, {0, 2, 3, 1}, {1, 3, 2, 0}};
    real best = BT_LARGE;
    simplex bestS;
    real bestL[4] = {0, 0, 0, 0};
    v3 bestv = V(0, 0, 0);
    int outside_any = 0;
    for (int f = 0; f < 4; f++) {
        v3 A = S->w[F[f][0]], B = S->w[F[f][1]], C = S->w[F[f][2]], D = S->w[F[f][3]];
        v3 n = crs(sub(B, A), sub(C, A));
        real sp = dot(scl(A, -1), n), sd = dot(sub(D, A), n);
        if (sd * sd < 1e-30) continue;          /* degenerate tetra face */
        if (sp * sd < 0) {                      /* origin and D on opposite sides */
            outside_any = 1;
            simplex T;
            for (int k = 0; k < 3; k++) { T.w[k] = S->w[F[f][k]]; T.a[k] = S->a[F[f][k]]; T.b[k] = S->b[F[f][k]]; }
            T.n = 3;
            real L[4];
            v3 v;
            simplex_closest(&T, &v, L);
            real d2 = len2(v);
            if (d2 < best) { best = d2; bestS = T; bestv = v; for (int k = 0; k < 4; k++) bestL[k] = L[k]; }
        }
    }
    if (!outside_any) { lam[0] = lam[1] = lam[2] = lam[3] = 0; *vout = V(0, 0, 0); return 1; }
    *S = bestS;
    for (int k = 0; k < 4; k++) lam[k] = bestL[k];
    *vout = bestv;
    return 0;
}

/* The closest point of the simplex to the origin with the Voronoi tests and the barycentric solve
 * in double, the results rounded to `real` (the kernel's simplex_closest_d, avr_kernel.hip: float
 * supports, double algebra -- the fp32 GJK's rerun after a stall, see gjk()).  A tetrahedron's
 * faces compete by their distance rounded to `real`, the lowest face index on ties.  In the fp64
 * build this is simplex_closest() itself. */
typedef struct { double x, y, z; } d3_t;
static d3_t D3(v3 a) { d3_t r = {(double)a.x, (double)a.y, (double)a.z}; return r; }
static d3_t dadd(d3_t a, d3_t b) { d3_t r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static d3_t dsub(d3_t a, d3_t b) { d3_t r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static d3_t dscl(d3_t a, double k) { d3_t r = {a.x * k, a.y * k, a.z * k}; return r; }
static d3_t dcrs(d3_t a, d3_t b) { d3_t r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; return r; }
static double ddot(d3_t a, d3_t b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 dtor(d3_t a) { return V((real)a.x, (real)a.y, (real)a.z); }

/* Ericson's triangle test in double; used: 1 A, 2 B, 4 C, 3 AB, 5 AC, 6 BC, 7 ABC */
static d3_t tri_cp_dbl(d3_t A, d3_t B, d3_t C, int *used, double *la, double *lb, double *lc) {
    d3_t ab = dsub(B, A), ac = dsub(C, A), ap = dscl(A, -1.0);
    double d1 = ddot(ab, ap), d2 = ddot(ac, ap);
    *la = *lb = *lc = 0.0;
    if (d1 <= 0.0 && d2 <= 0.0) { *used = 1; *la = 1.0; return A; }
    d3_t bp = dscl(B, -1.0);
    double d3 = ddot(ab, bp), d4 = ddot(ac, bp);
    if (d3 >= 0.0 && d4 <= d3) { *used = 2; *lb = 1.0; return B; }
    double vc = d1 * d4 - d3 * d2;
    if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
        double v = d1 / (d1 - d3);
        *used = 3; *la = 1.0 - v; *lb = v; return dadd(A, dscl(ab, v));
    }
    d3_t cp = dscl(C, -1.0);
    double d5 = ddot(ab, cp), d6 = ddot(ac, cp);
    if (d6 >= 0.0 && d5 <= d6) { *used = 4; *lc = 1.0; return C; }
    double vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
        double wv = d2 / (d2 - d6);
        *used = 5; *la = 1.0 - wv; *lc = wv; return dadd(A, dscl(ac, wv));
    }
    double va = d3 * d6 - d5 * d4;
    if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
        double wv = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        *used = 6; *lb = 1.0 - wv; *lc = wv; return dadd(B, dscl(dsub(C, B), wv));
    }
    double den = 1.0 / (va + vb + vc);
    double v = vb * den, wv = vc * den;
    *used = 7; *la = 1.0 - v - wv; *lb = v; *lc = wv;
    return dadd(A, dadd(dscl(ab, v), dscl(ac, wv)));
}

static void sx_move(simplex *S, int to, int from) { S->w[to] = S->w[from]; S->a[to] = S->a[from]; S->b[to] = S->b[from]; }

/* keep the triangle's feature `used` in slots 0.. in order; weights rounded to real */
static void tri_compact_dbl(simplex *S, int used, double la, double lb, double lc, real lam[4]) {
    switch (used) {
    case 1: S->n = 1; lam[0] = (real)la; break;
    case 2: sx_move(S, 0, 1); S->n = 1; lam[0] = (real)lb; break;
    case 4: sx_move(S, 0, 2); S->n = 1; lam[0] = (real)lc; break;
    case 3: S->n = 2; lam[0] = (real)la; lam[1] = (real)lb; break;
    case 5: sx_move(S, 1, 2); S->n = 2; lam[0] = (real)la; lam[1] = (real)lc; break;
    case 6: sx_move(S, 0, 1); sx_move(S, 1, 2); S->n = 2; lam[0] = (real)lb; lam[1] = (real)lc; break;
    default: S->n = 3; lam[0] = (real)la; lam[1] = (real)lb; lam[2] = (real)lc; break;
    }
}

static int simplex_closest_dbl(simplex *S, v3 *vout, real lam[4]) {
    if (S->n == 1) { lam[0] = 1; *vout = S->w[0]; return 0; }
    if (S->n == 2) {
        d3_t A = D3(S->w[0]), B = D3(S->w[1]), ab = dsub(B, A);
        double t = -ddot(A, ab), dd = ddot(ab, ab);
        if (t <= 0.0 || dd <= 0.0) { S->n = 1; lam[0] = 1; *vout = S->w[0]; return 0; }
        if (t >= dd) { sx_move(S, 0, 1); S->n = 1; lam[0] = 1; *vout = S->w[0]; return 0; }
        t /= dd;
        lam[0] = (real)(1.0 - t); lam[1] = (real)t;
        *vout = dtor(dadd(A, dscl(ab, t)));
        return 0;
    }
    if (S->n == 3) {
        int used;
        double la, lb, lc;
        d3_t cv = tri_cp_dbl(D3(S->w[0]), D3(S->w[1]), D3(S->w[2]), &used, &la, &lb, &lc);
        *vout = dtor(cv);
        tri_compact_dbl(S, used, la, lb, lc, lam);
        return 0;
    }
    static const int F[4][4] = {{0, 1, 2, 3}, {0, 3, 1, 2}, {0, 2, 3, 1}, {1, 3, 2, 0}};
    int bf = -1, bused = 7;
    real best = (real)BT_LARGE;
    double bla = 0, blb = 0, blc = 0;
    d3_t bcv = {0, 0, 0};
    for (int f = 0; f < 4; f++) {
        d3_t A = D3(S->w[F[f][0]]), B = D3(S->w[F[f][1]]), C = D3(S->w[F[f][2]]), D = D3(S->w[F[f][3]]);
        d3_t n = dcrs(dsub(B, A), dsub(C, A));
        double sp = ddot(dscl(A, -1.0), n), sd = ddot(dsub(D, A), n);
        if (sd * sd < 1e-30 || !(sp * sd < 0.0)) continue;
        int used;
        double la, lb, lc;
        d3_t cv = tri_cp_dbl(A, B, C, &used, &la, &lb, &lc);
        real d2 = (real)ddot(cv, cv);
        if (bf < 0 || d2 < best) { best = d2; bf = f; bused = used; bla = la; blb = lb; blc = lc; bcv = cv; }
    }
    if (bf < 0) { lam[0] = lam[1] = lam[2] = lam[3] = 0; *vout = V(0, 0, 0); return 1; }
    simplex T = *S;
    for (int k = 0; k < 3; k++) { T.w[k] = S->w[F[bf][k]]; T.a[k] = S->a[F[bf][k]]; T.b[k] = S->b[F[bf][k]]; }
    *S = T;
    S->n = 3;
    *vout = dtor(bcv);
    tri_compact_dbl(S, bused, bla, blb, blc, lam);
    return 0;
}

enum { GJK_SEPARATED = 0, GJK_FAR = 1, GJK_PENETRATING = 2 };
#define GJK_NP_GAP 1e-4     /* largest duality gap (m) a no-progress stop may leave (kernel: gjk_lane) */
enum { GJK_PLAIN = 0, GJK_LANE_RULE = 1, GJK_DOUBLE_SOLVE = 2 };

/* GJK on the shape cores (btGjkPairDetector's loop).  mode GJK_LANE_RULE restates the kernel's
 * lane path (gjk_lane, avr_kernel.hip): a step that makes no progress ends the GJK only when the
 * duality gap at the final direction is closed (|v|^2 - v.w <= GJK_NP_GAP |v|, one more support
 * query); otherwise the fp32 GJK has stalled on a thin simplex (its closest-point algebra cancelled),
 * and the GJK is rerun from the start with that algebra in double (GJK_DOUBLE_SOLVE: the kernel's
 * gjk_coop_d).  GJK_PLAIN: the sphere-hull point-core GJK (ph_step), which the kernel runs without
 * the rule.  In the fp64 build the rerun repeats the
 * first pass's arithmetic exactly, so the rule changes nothing there. */
static int gjk_mode(const wshape *A, const wshape *B, real maxdist2, v3 *pa, v3 *pb, real *dist, simplex *S, int mode, int *stalled) {
    v3 v = sub(A->t.p, B->t.p);
    if (len2(v) < R(1e-20)) v = V(1, 0, 0);
    S->n = 0;
    real lam[4] = {1, 0, 0, 0};
    real prev = BT_LARGE;
    int status = GJK_SEPARATED;
    for (int it = 0; it < GJK_MAX_IT; it++) {
        v3 sa = support(A, scl(v, -1)), sb = support(B, v);
        v3 wv = sub(sa, sb);
        real vv = len2(v), vw = dot(v, wv);
        if (vw > 0 && vw * vw > vv * maxdist2) return GJK_FAR;
        int dup = 0;
        for (int k = 0; k < S->n; k++)
            if (S->w[k].x == wv.x && S->w[k].y == wv.y && S->w[k].z == wv.z) dup = 1;
        if (dup && S->n > 0) break;
        if (S->n > 0 && vv - vw <= R(GJK_REL_EPS) * vv) break;
        S->w[S->n] = wv; S->a[S->n] = sa; S->b[S->n] = sb; S->n++;
        v3 nv;
        if (mode == GJK_DOUBLE_SOLVE ? simplex_closest_dbl(S, &nv, lam) : simplex_closest(S, &nv, lam)) { status = GJK_PENETRATING; break; }
        real nvv = len2(nv);
        if (nvv < R(1e-14) * (1 + len2(wv))) { status = GJK_PENETRATING; break; }
        if (nvv >= prev) {
            v = nv;
            if (mode == GJK_LANE_RULE && it + 1 < GJK_MAX_IT) {     /* (the kernel's next iteration: its support query) */
                v3 w2 = sub(support(A, scl(v, -1)), support(B, v));
                real vv2 = len2(v), gap = vv2 - dot(v, w2);
                if (gap > 0 && gap * gap > (R(GJK_NP_GAP) * R(GJK_NP_GAP)) * vv2) {
                    *stalled = 1;
                    return gjk_mode(A, B, maxdist2, pa, pb, dist, S, GJK_DOUBLE_SOLVE, stalled);
                }
            }
            break;
        }
        prev = nvv;
        v = nv;
    }
    if (status == GJK_PENETRATING) return GJK_PENETRATING;
    v3 a = V(0, 0, 0), b = V(0, 0, 0);
    for (int k = 0; k < S->n; k++) { a = add(a, scl(S->a[k], lam[k])); b = add(b, scl(S->b[k], lam[k])); }
    *pa = a; *pb = b;
    *dist = len(sub(a, b));
    return GJK_SEPARATED;
}

/* ---------------------------------------------------------------- EPA */
typedef struct { int i, j, k; v3 n; real d; int alive; } epa_face;

static int epa_add_face(epa_face *F, int *nf, const v3 *W, int i, int j, int k) {
    if (*nf >= EPA_MAX_F) return -1;
    v3 n = crs(sub(W[j], W[i]), sub(W[k], W[i]));
    real l = len(n);
    if (l < R(1e-18)) return -2;
    n = scl(n, 1 / l);
    epa_face *f = &F[(*nf)++];
    f->i = i; f->j = j; f->k = k; f->n = n; f->d = dot(n, W[i]); f->alive = 1;
    return 0;
}

static int epa(const wshape *A, const wshape *B, simplex *S, v3 *normal_out, real *depth, v3 *pa, v3 *pb) {
    v3 W[EPA_MAX_V], PA[EPA_MAX_V], PB[EPA_MAX_V];
    int nv = 0;
    for (int k = 0; k < S->n; k++) { W[nv] = S->w[k]; PA[nv] = S->a[k]; PB[nv] = S->b[k]; nv++; }
    /* blow up lower-dimensional simplices to a tetrahedron */
    static const real dirs[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
    for (int di = 0; di < 6 && nv < 4; di++) {
        v3 d = V(dirs[di][0], dirs[di][1], dirs[di][2]);
        if (nv == 2) {
            v3 e = sub(W[1], W[0]);
            v3 c = crs(e, d);
            if (len2(c) < R(1e-12)) continue;
            d = c;
        } else if (nv == 3) {
            d = crs(sub(W[1], W[0]), sub(W[2], W[0]));
            if (di & 1) d = scl(d, -1);
            if (len2(d) < R(1e-24)) continue;
        }
        v3 sa = support(A, d), sb = support(B, scl(d, -1));
        v3 wv = sub(sa, sb);
        int dup = 0;
        for (int k = 0; k < nv; k++)
            if (len2(sub(W[k], wv)) < R(1e-20)) dup = 1;
        if (dup) continue;
        W[nv] = wv; PA[nv] = sa; PB[nv] = sb; nv++;
    }
    if (nv < 4) return -1;
    /* orient tetrahedron */
    if (dot(crs(sub(W[1], W[0]), sub(W[2], W[0])), sub(W[3], W[0])) > 0) {
        v3 t = W[1]; W[1] = W[2]; W[2] = t;
        t = PA[1]; PA[1] = PA[2]; PA[2] = t;
        t = PB[1]; PB[1] = PB[2]; PB[2] = t;
    }
    epa_face F[EPA_MAX_F];
    int nf = 0;
    if (epa_add_face(F, &nf, W, 0, 1, 2) || epa_add_face(F, &nf, W, 0, 3, 1) ||
        epa_add_face(F, &nf, W, 0, 2, 3) || epa_add_face(F, &nf, W, 1, 3, 2))
        return -1;
    int best = -1;
    for (int it = 0; it < EPA_MAX_IT; it++) {
        best = -1;
        real bd = BT_LARGE;
        for (int f = 0; f < nf; f++)
            if (F[f].alive && F[f].d < bd) { bd = F[f].d; best = f; }
        if (best < 0) return -1;
        v3 n = F[best].n;
        v3 sa = support(A, n), sb = support(B, scl(n, -1));
        v3 wv = sub(sa, sb);
        real dist = dot(wv, n);
        if (dist - F[best].d < R(EPA_EPS) || nv >= EPA_MAX_V) break;
        int vi = nv++;
        W[vi] = wv; PA[vi] = sa; PB[vi] = sb;
        /* remove visible faces, collect horizon */
        int edges[EPA_MAX_F * 3][2];
        int ne = 0;
        for (int f = 0; f < nf; f++) {
            if (!F[f].alive) continue;
            if (dot(F[f].n, sub(wv, W[F[f].i])) > 0) {
                F[f].alive = 0;
                int e3[3][2] = {{F[f].i, F[f].j}, {F[f].j, F[f].k}, {F[f].k, F[f].i}};
                for (int e = 0; e < 3; e++) {
                    int found = -1;
                    for (int q = 0; q < ne; q++)
                        if (edges[q][0] == e3[e][1] && edges[q][1] == e3[e][0]) { found = q; break; }
                    if (found >= 0) { edges[found][0] = edges[ne - 1][0]; edges[found][1] = edges[ne - 1][1]; ne--; }
                    else { edges[ne][0] = e3[e][0]; edges[ne][1] = e3[e][1]; ne++; }
                }
            }
        }
        /* compact dead faces */
        int k = 0;
        for (int f = 0; f < nf; f++)
            if (F[f].alive) F[k++] = F[f];
        nf = k;
        for (int e = 0; e < ne; e++)
            if (epa_add_face(F, &nf, W, edges[e][0], edges[e][1], vi) == -1) return -1;
    }
    if (best < 0) return -1;
    epa_face *f = &F[best];
    v3 n = f->n;
    v3 p = scl(n, f->d);
    /* barycentric of p in triangle */
    v3 a = W[f->i], b = W[f->j], c = W[f->k];
    v3 v0 = sub(b, a), v1 = sub(c, a), v2 = sub(p, a);
    real d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
    real den = d00 * d11 - d01 * d01;
    real lv = 0, lw = 0;
    if (fabs(den) > R(1e-30)) { lv = (d11 * d20 - d01 * d21) / den; lw = (d00 * d21 - d01 * d20) / den; }
    real lu = 1 - lv - lw;
    *pa = add(add(scl(PA[f->i], lu), scl(PA[f->j], lv)), scl(PA[f->k], lw));
    *pb = add(add(scl(PB[f->i], lu), scl(PB[f->j], lv)), scl(PB[f->k], lw));
    *normal_out = n;
    *depth = f->d;
    return 0;
}

/* ---------------------------------------------------------------- narrowphase */
/* returns 1 and (normalOnB, pointOnB, distance) if a contact within `thr` exists */
static int narrowphase(ws_t *o, const wshape *A, const wshape *B, real thr, v3 *nB, v3 *pB, real *dist) {
    int ka = A->kind, kb = B->kind;
    if (ka == AVR_SPHERE && kb == AVR_SPHERE) {               /* btSphereSphereCollisionAlgorithm */
        v3 diff = sub(A->t.p, B->t.p);
        real l = len(diff), ra = A->he.x, rb = B->he.x;
        if (l > ra + rb) return 0;
        real d = l - (ra + rb);
        v3 n = V(1, 0, 0);
        if (l > R(1.1920928955078125e-07)) n = scl(diff, 1 / l);
        *nB = n; *pB = add(B->t.p, scl(n, rb)); *dist = d;
        return d <= thr;
    }
    if ((ka == AVR_SPHERE && kb == AVR_BOX) || (ka == AVR_BOX && kb == AVR_SPHERE)) {  /* btSphereBoxCollisionAlgorithm */
        int swapped = ka == AVR_BOX;
        const wshape *S = swapped ? B : A, *X = swapped ? A : B;
        v3 rel = tfinvpt(X->t, S->t.p);
        v3 he = X->he;
        v3 cp = V(fmin(he.x, fmax(-he.x, rel.x)), fmin(he.y, fmax(-he.y, rel.y)), fmin(he.z, fmax(-he.z, rel.z)));
        real r = S->he.x, inter = r + X->margin, cdist = inter + thr;
        v3 n = sub(rel, cp);
        real d2 = len2(n), d;
        if (d2 > cdist * cdist) return 0;
        if (d2 <= R(1.1920928955078125e-07)) {
            real fd = he.x - rel.x, md = fd;
            cp = rel; cp.x = he.x; n = V(1, 0, 0);
            fd = he.x + rel.x; if (fd < md) { md = fd; cp = rel; cp.x = -he.x; n = V(-1, 0, 0); }
            fd = he.y - rel.y; if (fd < md) { md = fd; cp = rel; cp.y = he.y; n = V(0, 1, 0); }
            fd = he.y + rel.y; if (fd < md) { md = fd; cp = rel; cp.y = -he.y; n = V(0, -1, 0); }
            fd = he.z - rel.z; if (fd < md) { md = fd; cp = rel; cp.z = he.z; n = V(0, 0, 1); }
            fd = he.z + rel.z; if (fd < md) { md = fd; cp = rel; cp.z = -he.z; n = V(0, 0, -1); }
            d = -md;
        } else {
            d = sqrt(d2);
            n = scl(n, 1 / d);
        }
        v3 pbox = tfpt(X->t, add(cp, scl(n, X->margin)));
        v3 nw = qrot(X->t.q, n);
        real pen = d - inter;
        if (pen > thr) return 0;
        if (!swapped) { *nB = nw; *pB = pbox; *dist = pen; }           /* box is B */
        else { *nB = scl(nw, -1); *pB = add(pbox, scl(nw, pen)); *dist = pen; } /* sphere is B */
        return 1;
    }
    if ((ka == AVR_SPHERE || ka == AVR_CAPSULE) && (kb == AVR_SPHERE || kb == AVR_CAPSULE) && !(ka == AVR_CAPSULE && kb == AVR_CAPSULE)) {
        /* point vs segment closed form (equivalent to GJK on these cores) */
        int swapped = ka == AVR_CAPSULE;
        const wshape *S = swapped ? B : A, *C = swapped ? A : B;
        v3 az = qrot(C->t.q, V(0, 0, 1));
        v3 p0 = sub(C->t.p, scl(az, C->he.y)), p1 = add(C->t.p, scl(az, C->he.y));
        v3 e = sub(p1, p0);
        real t = dot(sub(S->t.p, p0), e) / fmax(dot(e, e), R(1e-30));
        t = fmin(R(1), fmax(R(0), t));
        v3 q = add(p0, scl(e, t));
        v3 diff = sub(S->t.p, q);
        real l = len(diff);
        v3 n = l > R(1e-12) ? scl(diff, 1 / l) : V(1, 0, 0);
        real d = l - S->he.x - C->he.x;
        if (d > thr) return 0;
        if (!swapped) { *nB = n; *pB = add(q, scl(n, C->he.x)); *dist = d; }
        else { *nB = scl(n, -1); *pB = sub(S->t.p, scl(n, S->he.x)); *dist = d; }
        return 1;
    }
    /* general convex-convex: GJK on cores, EPA when the cores overlap (btGjkPairDetector) */
    real ma = A->margin, mb = B->margin;
    real maxd = ma + mb + thr;
    v3 pa, pb;
    real cd;
    simplex S;
    o->stats_gjk++;
    /* the kernel's lane rule for every general pair except sphere-hull (its point-core list);
     * o->np_plain (unset by the shipped paths) switches it off for experiments */
    const int sph_hull = (ka == AVR_SPHERE && kb == AVR_HULL) || (ka == AVR_HULL && kb == AVR_SPHERE);
    int stalled = 0;
    int st = gjk_mode(A, B, maxd * maxd, &pa, &pb, &cd, &S, (sph_hull || o->np_plain) ? GJK_PLAIN : GJK_LANE_RULE, &stalled);
    o->stats_stall += stalled;
    if (st == GJK_FAR) return 0;
    v3 n;
    real d;
    if (st == GJK_SEPARATED && cd > R(1e-9)) {
        n = scl(sub(pa, pb), 1 / cd);
        d = cd - ma - mb;
    } else {
        real depth;
        v3 en;
        o->stats_epa++;
        if (epa(A, B, &S, &en, &depth, &pa, &pb)) return 0;
        n = scl(en, -1);
        d = -depth - ma - mb;
    }
    if (d > thr) return 0;
    *nB = n;
    *pB = add(pb, scl(n, mb));
    *dist = d;
    return 1;
}

/* ---------------------------------------------------------------- body transforms & AABBs */
static tf body_tf(const model *m, const real *st, const ws_t *w, int b) {
    int kind = m->d.body_kind[b], idx = m->d.body_index[b];
    tf t;
    if (kind == AVR_BODY_ROBOT) return w->cm[idx];
    if (kind == AVR_BODY_FREE) {
        const real *f = st + S_FREE + AVR_FB_WORDS * idx;
        t.p = ld3(f); t.q = ldq(f + 3);
        return t;
    }
    if (kind == AVR_BODY_STATIC) return ldtf(m->d.st_pose + 7 * idx);
#if PR2F
    if (kind == AVR_BODY_RSTATIC) { t.p = ld3(st + S_RBASE); t.q = ldq(st + S_RBASE + 3); return t; }
#endif
    const real *h = st + S_HUMAN + 7 * idx;
    t.p = ld3(h); t.q = ldq(h + 3);
    return t;
}

static void aabb_of(tf t, v3 c, v3 h, v3 *mn, v3 *mx) {
    m3 Rm = qmat(t.q);
    v3 cw = tfpt(t, c);
    v3 hw = V(fabs(Rm.m[0][0]) * h.x + fabs(Rm.m[0][1]) * h.y + fabs(Rm.m[0][2]) * h.z,
              fabs(Rm.m[1][0]) * h.x + fabs(Rm.m[1][1]) * h.y + fabs(Rm.m[1][2]) * h.z,
              fabs(Rm.m[2][0]) * h.x + fabs(Rm.m[2][1]) * h.y + fabs(Rm.m[2][2]) * h.z);
    *mn = sub(cw, hw);
    *mx = add(cw, hw);
}

static inline int aabb_overlap(v3 a0, v3 a1, v3 b0, v3 b1) {
    return a0.x <= b1.x && a1.x >= b0.x && a0.y <= b1.y && a1.y >= b0.y && a0.z <= b1.z && a1.z >= b0.z;
}

static int shape_enabled(const model *m, int s, int gender) {
    int g = m->d.shape_gender[s];
    return g < 0 || g == gender;
}

static void shape_aabb(const model *m, int s, tf body, v3 *mn, v3 *mx) {
    tf t = tfmul(body, ldtf(m->d.shape_pose + 7 * s));
    const double *a = m->d.shape_aabb + 6 * s;
    aabb_of(t, ld3d(a), ld3d(a + 3), mn, mx);
}

/* ---------------------------------------------------------------- contact manifolds */
static real *cp_ptr(real *st, int i) { return st + S_CP + AVR_CP_WORDS * i; }

/* One btPersistentManifold (<= 4 points) of a shape pair, held locally while it is updated. */
typedef struct { real p[AVR_MANIFOLD_POINTS][AVR_CP_WORDS]; int n; } manifold_t;

/* btPersistentManifold::sortCachedPoints */
static int sort_cached(const manifold_t *M, v3 la_new, real d_new) {
    int maxi = -1;
    real maxpen = d_new;
    for (int i = 0; i < 4; i++)
        if (M->p[i][AVR_CP_DIST] < maxpen) { maxi = i; maxpen = M->p[i][AVR_CP_DIST]; }
    v3 p[4];
    for (int i = 0; i < 4; i++) p[i] = ld3(M->p[i] + AVR_CP_LA);
    real res[4] = {0, 0, 0, 0};
    if (maxi != 0) res[0] = len2(crs(sub(la_new, p[1]), sub(p[3], p[2])));
    if (maxi != 1) res[1] = len2(crs(sub(la_new, p[0]), sub(p[3], p[2])));
    if (maxi != 2) res[2] = len2(crs(sub(la_new, p[0]), sub(p[3], p[1])));
    if (maxi != 3) res[3] = len2(crs(sub(la_new, p[0]), sub(p[2], p[1])));
    int bi = 0;
    real bv = -1;
    for (int i = 0; i < 4; i++)
        if (fabs(res[i]) > bv) { bv = fabs(res[i]); bi = i; }
    return bi;
}

/* btManifoldResult::addContactPoint -> getCacheEntry / replaceContactPoint / addManifoldPoint */
static void manifold_add(manifold_t *M, int sa, int sb, int pair, tf ta, tf tb, v3 nB, v3 pB, real dist, real thr) {
    if (dist > thr) return;
    v3 pA = add(pB, scl(nB, dist));
    v3 la = tfinvpt(ta, pA), lb = tfinvpt(tb, pB);
    real shortest = thr * thr;
    int near = -1;
    for (int k = 0; k < M->n; k++) {
        real d2 = len2(sub(ld3(M->p[k] + AVR_CP_LA), la));
        if (d2 < shortest) { shortest = d2; near = k; }
    }
    real *c;
    if (near >= 0) {                               /* replace: keep impulse + lifetime */
        c = M->p[near];
    } else if (M->n == AVR_MANIFOLD_POINTS) {      /* full: area-maximising replacement */
        c = M->p[sort_cached(M, la, dist)];
        c[AVR_CP_IMP] = 0; c[AVR_CP_LIFE] = 0;
    } else {
        c = M->p[M->n++];
        c[AVR_CP_IMP] = 0; c[AVR_CP_LIFE] = 0;
    }
    c[AVR_CP_SA] = (real)sa; c[AVR_CP_SB] = (real)sb; c[AVR_CP_PAIR] = (real)pair; c[AVR_CP_SLOT] = 0;
    st3(c + AVR_CP_LA, la); st3(c + AVR_CP_LB, lb); st3(c + AVR_CP_N, nB);
    c[AVR_CP_DIST] = dist;
}

/* btPersistentManifold::refreshContactPoints */
static void manifold_refresh(manifold_t *M, tf ta, tf tb, real thr) {
    for (int k = M->n - 1; k >= 0; k--) {
        real *c = M->p[k];
        v3 pa = tfpt(ta, ld3(c + AVR_CP_LA)), pb = tfpt(tb, ld3(c + AVR_CP_LB));
        c[AVR_CP_DIST] = dot(sub(pa, pb), ld3(c + AVR_CP_N));
        c[AVR_CP_LIFE] += 1;
    }
    for (int k = M->n - 1; k >= 0; k--) {
        real *c = M->p[k];
        int rm = 0;
        if (c[AVR_CP_DIST] > thr) rm = 1;
        else {
            v3 pa = tfpt(ta, ld3(c + AVR_CP_LA)), pb = tfpt(tb, ld3(c + AVR_CP_LB));
            v3 nrm = ld3(c + AVR_CP_N);
            v3 dd = sub(pb, sub(pa, scl(nrm, c[AVR_CP_DIST])));
            if (len2(dd) > thr * thr) rm = 1;
        }
        if (rm) {                                  /* removeContactPoint: swap last in */
            if (k != M->n - 1) memcpy(c, M->p[M->n - 1], sizeof(real) * AVR_CP_WORDS);
            M->n--;
        }
    }
}

/* ---------------------------------------------------------------- constraint rows */
static void add_endpoint_jac(const model *m, const ws_t *w, int link, v3 p, v3 lin, v3 ang, real *J) {
    /* J[d] = d(lin . v(p) + ang . omega)/dqd for dofs in the chain of `link` */
    for (int d = 0; d < m->nd; d++) J[d] = 0;
    for (int k = link; k >= 0; k = m->parent[k]) {
        int dof = m->dof[k];
        if (dof < 0) continue;
        v3 cl, ca;
        dof_col(m, w, k, p, &cl, &ca);
        J[dof] = dot(lin, cl) + dot(ang, ca);
    }
}

/* Fill endpoint (side 0=A, 1=B) of a row for body b at point p with linear dir `lin` and
 * angular dir `ang` (world). */
static void row_endpoint(const model *m, const real *st, ws_t *w, row_t *r, int side, int b, v3 p, v3 lin, v3 ang) {
    int kind = m->d.body_kind[b], idx = m->d.body_index[b];
    int *pk = side ? &r->kindB : &r->kindA, *pi = side ? &r->idxB : &r->idxA;
    real *J = side ? r->JB : r->JA, *MJ = side ? r->MB : r->MA;
    if (m->body_link[b] >= 0) {      /* robot link, or head-chain link in a tremor view */
        idx = m->body_link[b];
        *pk = 1; *pi = idx;
        add_endpoint_jac(m, w, idx, p, lin, ang, J);
        chol_solve(m, w, J, MJ);
    } else if (kind == AVR_BODY_FREE) {
        *pk = 2; *pi = idx;
        const real *f = st + S_FREE + AVR_FB_WORDS * idx;
        v3 c = ld3(f);
        qt q = ldq(f + 3);
        v3 angt = add(crs(sub(p, c), lin), ang);
        st3(J, lin); st3(J + 3, angt);
        real im = m->d.fb_mass[idx] > 0 ? 1 / R(m->d.fb_mass[idx]) : 0;
        v3 I = ld3d(m->d.fb_inertia + 3 * idx);
        st3(MJ, scl(lin, im));
        st3(MJ + 3, inertia_inv_mul(q, I, angt));
    } else {
        *pk = 0; *pi = 0;
    }
}

static real ep_dot(const model *m, const ws_t *w, int kind, int idx, const real *J, int use_delta) {
    if (kind == 1) {
        real s = 0;
        for (int d = 0; d < m->nd; d++) s += J[d] * (use_delta ? w->dq[d] : w->vq[d]);
        return s;
    }
    if (kind == 2) {
        v3 v = use_delta ? w->dfv[idx] : w->fv[idx], om = use_delta ? w->dfw[idx] : w->fw[idx];
        return J[0] * v.x + J[1] * v.y + J[2] * v.z + J[3] * om.x + J[4] * om.y + J[5] * om.z;
    }
    return 0;
}

static real ep_denom(const model *m, int kind, const real *J, const real *MJ) {
    int n = kind == 1 ? m->nd : kind == 2 ? 6 : 0;
    real s = 0;
    for (int i = 0; i < n; i++) s += J[i] * MJ[i];
    return s;
}

static void ep_apply(const model *m, ws_t *w, int kind, int idx, const real *MJ, real imp) {
    if (kind == 1) {
        for (int d = 0; d < m->nd; d++) w->dq[d] = PRB(8, w->dq[d] + MJ[d] * imp);
    } else if (kind == 2) {
        w->dfv[idx] = add(w->dfv[idx], scl(ld3(MJ), imp));
        w->dfw[idx] = add(w->dfw[idx], scl(ld3(MJ + 3), imp));
    }
}

static void row_finish(const model *m, ws_t *w, row_t *r) {
#ifdef AVR_ORACLE_PROBE
    for (int i = 0; i < K_MAX_DOF; i++) { r->JA[i] = PRB(6, r->JA[i]); r->JB[i] = PRB(6, r->JB[i]); r->MA[i] = PRB(6, r->MA[i]); r->MB[i] = PRB(6, r->MB[i]); }
#endif
    real den = ep_denom(m, r->kindA, r->JA, r->MA) + ep_denom(m, r->kindB, r->JB, r->MB);
    r->inv = den > R(BT_DENOM_EPS) ? PRB(6, 1 / den) : 1;
}

static real row_relvel(const model *m, const ws_t *w, const row_t *r) {
    return ep_dot(m, w, r->kindA, r->idxA, r->JA, 0) + ep_dot(m, w, r->kindB, r->idxB, r->JB, 0);
}

static row_t *new_row(ws_t *w) {
    row_t *r = &w->rows[w->nrows++];
    memset(r, 0, sizeof(*r));
    r->normal_row = -1;
    r->cp = -1;
    return r;
}

/* btMultiBodyJointLimitConstraint + btMultiBodyJointMotor + btMultiBodyFixedConstraint rows */
static void build_noncontact_rows(const model *m, const real *st, ws_t *w, real dt) {
    real erp = R(m->d.erp);
    /* joint limits (created at URDF load, link order); a row exists only when violated */
    for (int i = 0; i < m->nl; i++) {
        if (!m->has_limit[i]) continue;
        int dof = m->dof[i];
        real q = st[S_Q + dof];
        real lo = m->lower[i], hi = m->upper[i];
#if PR2F
        if (i >= m->nl_robot) {   /* human arm limits x the env's limit_scale (human_creation.py:226) */
            lo = st[S_HCH + 2 * K_HC_N + (i - m->nl_robot)];
            hi = st[S_HCH + 3 * K_HC_N + (i - m->nl_robot)];
        }
#endif
        for (int side = 0; side < 2; side++) {
            real pen = side == 0 ? q - lo : hi - q;
            if (pen > 0) continue;
            row_t *r = new_row(w);
            r->kindA = 1; r->idxA = i;
            for (int d = 0; d < m->nd; d++) r->JA[d] = 0;
            r->JA[dof] = side == 0 ? 1 : -1;
            chol_solve(m, w, r->JA, r->MA);
            row_finish(m, w, r);
            real rel = row_relvel(m, w, r);
            real pos = -pen * erp / dt, vel = -rel;
            r->rhs = (pos + vel) * r->inv;
            r->lo = 0; r->hi = R(100.0);                       /* btMultiBodyConstraint default max impulse */
            w->nc_idx[w->n_nc++] = w->nrows - 1;
        }
    }
    /* joint motors (createJointMotors order = link order) */
    for (int i = 0; i < m->nl; i++) {
        int dof = m->dof[i];
        if (dof < 0) continue;
        row_t *r = new_row(w);
        r->kindA = 1; r->idxA = i;
        for (int d = 0; d < m->nd; d++) r->JA[d] = 0;
        r->JA[dof] = 1;
        chol_solve(m, w, r->JA, r->MA);
        row_finish(m, w, r);
        real q = st[S_Q + dof], cur = w->vq[dof];
        real kp = st[S_KP + dof], kd = 1;                  /* pybullet default velocityGain 1 */
        real desired = kp * (st[S_QTGT + dof] - q) / dt + cur + kd * (0 - cur);
        real rel = row_relvel(m, w, r);
        r->rhs = (desired - rel) * r->inv;
        real mi = st[S_MAXIMP + dof];
        r->lo = -mi; r->hi = mi;
        w->nc_idx[w->n_nc++] = w->nrows - 1;
    }
    /* fixed constraint: robot tool link <-> spoon base (world_creation.py:363-364) */
    {
        int link = m->d.tool_link;
        int fb = m->d.spoon_free;
        tf ta = w->cm[link];
        tf off = ldtf(m->d.tool_offset);
        v3 pivA = tfpt(ta, off.p);
        qt frA = qmul(ta.q, off.q);
        const real *f = st + S_FREE + AVR_FB_WORDS * fb;
        tf tb; tb.p = ld3(f); tb.q = ldq(f + 3);
#if PR2F
        v3 pivB = tfpt(tb, ld3d(m->d.fix_pivot_b));   /* the composite tool's base (handle) COM */
#else
        v3 pivB = tb.p;
#endif
        m3 FA = qmat(frA), FB = qmat(tb.q);
        /* relRot = FA^-1 FB; matrixToEulerXYZ with btGetMatrixElem(mat, i) = mat[i%3][i/3] */
        m3 rr;
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) {
                real s = 0;
                for (int k = 0; k < 3; k++) s += FA.m[k][a] * FB.m[k][b];
                rr.m[a][b] = s;
            }
#define ME(i) rr.m[(i) % 3][(i) / 3]
        v3 ang;
        real fi = ME(2);
        if (fi < 1) {
            if (fi > -1) ang = V(atan2(-ME(5), ME(8)), asin(ME(2)), atan2(-ME(1), ME(0)));
            else ang = V(-atan2(ME(3), ME(4)), -R(1.5707963267948966), 0);
        } else ang = V(atan2(ME(3), ME(4)), R(1.5707963267948966), 0);
#undef ME
        real mi = R(m->d.fixed_max_force * m->d.time_step);
        int bodyA = -1, bodyB = m->d.spoon_body;
        for (int b = 0; b < m->nb; b++)
            if (m->d.body_kind[b] == AVR_BODY_ROBOT && m->d.body_index[b] == link) bodyA = b;
        for (int i = 0; i < 6; i++) {
            row_t *r = new_row(w);
            v3 lin = V(0, 0, 0), an = V(0, 0, 0);
            real pos;
            if (i < 3) {
                if (i == 0) lin.x = 1; else if (i == 1) lin.y = 1; else lin.z = 1;
                pos = dot(sub(pivA, pivB), lin);
                if (bodyA >= 0) row_endpoint(m, st, w, r, 0, bodyA, pivA, lin, V(0, 0, 0));
                else { r->kindA = 1; r->idxA = link; add_endpoint_jac(m, w, link, pivA, lin, V(0, 0, 0), r->JA); chol_solve(m, w, r->JA, r->MA); }
                row_endpoint(m, st, w, r, 1, bodyB, pivB, scl(lin, -1), V(0, 0, 0));
            } else {
                an = V(FA.m[0][i - 3], FA.m[1][i - 3], FA.m[2][i - 3]);
                pos = i == 3 ? ang.x : i == 4 ? ang.y : ang.z;
                r->kindA = 1; r->idxA = link;
                add_endpoint_jac(m, w, link, pivA, V(0, 0, 0), an, r->JA);
                chol_solve(m, w, r->JA, r->MA);
                row_endpoint(m, st, w, r, 1, bodyB, pivB, V(0, 0, 0), scl(an, -1));
                /* free-body angular-only row: J = (0, -an) */
                st3(r->JB, V(0, 0, 0));
                st3(r->JB + 3, scl(an, -1));
                {
                    const real *ff = st + S_FREE + AVR_FB_WORDS * fb;
                    st3(r->MB, V(0, 0, 0));
                    st3(r->MB + 3, inertia_inv_mul(ldq(ff + 3), ld3d(m->d.fb_inertia + 3 * fb), scl(an, -1)));
                }
            }
            row_finish(m, w, r);
            real rel = row_relvel(m, w, r);
            r->rhs = (-pos * erp / dt - rel) * r->inv;
            r->lo = -mi; r->hi = mi;
            w->nc_idx[w->n_nc++] = w->nrows - 1;
        }
    }
}

/* btPlaneSpace1 */
static void plane_space(v3 n, v3 *p, v3 *q) {
    if (fabs(n.z) > R(0.7071067811865475244)) {
        real a = n.y * n.y + n.z * n.z, k = 1 / sqrt(a);
        *p = V(0, -n.z * k, n.y * k);
        *q = V(a * k, -n.x * p->z, n.x * p->y);
    } else {
        real a = n.x * n.x + n.y * n.y, k = 1 / sqrt(a);
        *p = V(-n.y * k, n.x * k, 0);
        *q = V(-n.z * p->y, n.z * p->x, a * k);
    }
}

/* btManifoldResult::calculateCombinedRollingFriction / ...SpinningFriction [ext]: the coefficient of
 * one body times the other's lateral friction, summed both ways, clamped to +-10 (Bullet's
 * MAX_FRICTION) */
static real torsion_coeff(const model *m, int ba, int bb, const double *c) {
    if (!c) return 0;
    real x = R(c[ba] * m->d.body_friction[bb] + c[bb] * m->d.body_friction[ba]);
    return x > 10 ? 10 : x < -10 ? -10 : x;
}

static void build_contact_rows(const model *m, real *st, ws_t *w, real dt) {
    int ncp = (int)st[S_TASK + T_NCP];
    real erp = R(m->d.erp), ws = R(m->d.warmstart);
    for (int i = 0; i < ncp; i++) {
        real *c = cp_ptr(st, i);
        int sa = (int)c[AVR_CP_SA], sb = (int)c[AVR_CP_SB];
        int ba = m->d.shape_body[sa], bb = m->d.shape_body[sb];
        tf ta = body_tf(m, st, w, ba), tb = body_tf(m, st, w, bb);
        v3 pa = tfpt(ta, ld3(c + AVR_CP_LA)), pb = tfpt(tb, ld3(c + AVR_CP_LB));
        v3 n = ld3(c + AVR_CP_N);
        real fric = R(m->d.body_friction[ba] * m->d.body_friction[bb]);
        if (fric > 10) fric = 10;
        /* normal row */
        row_t *r = new_row(w);
        row_endpoint(m, st, w, r, 0, ba, pa, n, V(0, 0, 0));
        row_endpoint(m, st, w, r, 1, bb, pb, scl(n, -1), V(0, 0, 0));
        row_finish(m, w, r);
        real rel = row_relvel(m, w, r);
        real pen = c[AVR_CP_DIST];
        real velerr = -rel, poserr = 0;
        if (pen > 0) velerr -= pen / dt;
        else poserr = -pen * erp / dt;
        r->rhs = PRB(9, (poserr + velerr) * r->inv);
        r->lo = 0; r->hi = R(1e10);
        r->cp = i;
        r->imp = c[AVR_CP_IMP] * ws;                               /* warm start */
        int nrow = w->nrows - 1;
        int nidx = w->n_nrm;
        w->nrm_idx[w->n_nrm++] = nrow;
        if (r->imp != 0) {
            ep_apply(m, w, r->kindA, r->idxA, r->MA, r->imp);
            ep_apply(m, w, r->kindB, r->idxB, r->MB, r->imp);
        }
        v3 t1, t2;
        plane_space(n, &t1, &t2);
        for (int k = 0; k < 2; k++) {
            v3 t = k ? t2 : t1;
            row_t *f = new_row(w);
            row_endpoint(m, st, w, f, 0, ba, pa, t, V(0, 0, 0));
            row_endpoint(m, st, w, f, 1, bb, pb, scl(t, -1), V(0, 0, 0));
            row_finish(m, w, f);
            real rv = row_relvel(m, w, f);
            f->rhs = -rv * f->inv;
            f->fric = fric;
            f->normal_row = nidx;
            w->fr_idx[w->n_fr++] = w->nrows - 1;
        }
        /* torsional friction (btMultiBodyConstraintSolver::convertMultiBodyContact [ext]): with a
         * combined spinning friction a row about the normal, with a combined rolling friction two
         * rows about plane_space(n) -- angular-only Jacobians, no positional term, no warm start,
         * in that order; Bullet adds them for the first 4 points of a manifold (rollingFriction
         * counter), i.e. every point here (manifolds hold <= 4) */
        real spin = torsion_coeff(m, ba, bb, m->d.body_spinning), roll = torsion_coeff(m, ba, bb, m->d.body_rolling);
        for (int k = 0; k < 3; k++) {
            if (k == 0 ? !(spin > 0) : !(roll > 0)) continue;
            v3 ax = k == 0 ? n : k == 1 ? t1 : t2;
            row_t *f = new_row(w);
            row_endpoint(m, st, w, f, 0, ba, pa, V(0, 0, 0), ax);
            row_endpoint(m, st, w, f, 1, bb, pb, V(0, 0, 0), scl(ax, -1));
            row_finish(m, w, f);
            real rv = row_relvel(m, w, f);
            f->rhs = -rv * f->inv;
            f->fric = k == 0 ? spin : roll;
            f->normal_row = nidx;
            w->tor_idx[w->n_tor++] = w->nrows - 1;
        }
    }
}

/* one row resolve (btMultiBodyConstraintSolver::resolveSingleConstraintRowGeneric [ext]); returns
 * the row's squared residual: (impulse change / jacDiagABInv)^2 */
static real resolve(const model *m, ws_t *w, row_t *r) {
    real dv = PRB(7, ep_dot(m, w, r->kindA, r->idxA, r->JA, 1) + ep_dot(m, w, r->kindB, r->idxB, r->JB, 1));
    real delta = PRB(7, r->rhs - dv * r->inv);
    real sum = r->imp + delta;
    if (sum < r->lo) { delta = r->lo - r->imp; r->imp = r->lo; }
    else if (sum > r->hi) { delta = r->hi - r->imp; r->imp = r->hi; }
    else r->imp = sum;
    ep_apply(m, w, r->kindA, r->idxA, r->MA, delta);
    ep_apply(m, w, r->kindB, r->idxB, r->MB, delta);
    const real res = delta / r->inv;
    return res * res;
}

/* Test-only variant (avr_oracle_set_island_exit): the residual exit per island instead of per env.
 * An island is a connected set of bodies through the rows -- nodes: the robot multibody, the human
 * chain, each free body (static geometry joins nothing).  Each island leaves the PGS after its own
 * first iteration whose largest squared row residual is within the threshold; the other islands go
 * on.  This is what Bullet does when it solves islands as separate groups (splitIslands with
 * islands of at least minimumSolverBatchSize rows, btSimulationIslandManager [ext]); the build's
 * default treats the env as one group (tests/test_oracle_kat.py bounds the difference). */
static int isl_find(int *par, int x) { while (par[x] != x) x = par[x] = par[par[x]]; return x; }
static int row_node(const model *m, int kind, int idx) {
    if (kind == 1) return idx < m->nl_robot ? 0 : 1;
    if (kind == 2) return 2 + idx;
    return -1;
}
static void solve_islands(const model *m, ws_t *w) {
    int iters = m->d.solver_iterations;
    w->stats_solves++;
    enum { NN = 2 + K_MAX_FREE };
    int par[NN];
    for (int k = 0; k < NN; k++) par[k] = k;
    for (int r = 0; r < w->nrows; r++) {
        const int a = row_node(m, w->rows[r].kindA, w->rows[r].idxA), b = row_node(m, w->rows[r].kindB, w->rows[r].idxB);
        if (a >= 0 && b >= 0) par[isl_find(par, a)] = isl_find(par, b);
    }
    int isl[MAX_ROWS];
    for (int r = 0; r < w->nrows; r++) {
        const int a = row_node(m, w->rows[r].kindA, w->rows[r].idxA), b = row_node(m, w->rows[r].kindB, w->rows[r].idxB);
        isl[r] = isl_find(par, a >= 0 ? a : b >= 0 ? b : 0);
    }
    int done[NN] = {0};
    for (int it = 0; it < iters; it++) {
        real res[NN];
        for (int k = 0; k < NN; k++) res[k] = 0;
#define RESI(r, x) do { const real r_ = (x); if (r_ > res[isl[r]]) res[isl[r]] = r_; } while (0)
        for (int j = 0; j < w->n_nc; j++) {
            int k = (it & 1) ? j : w->n_nc - 1 - j;
            const int r = w->nc_idx[k];
            if (!done[isl[r]]) RESI(r, resolve(m, w, &w->rows[r]));
        }
        for (int j = 0; j < w->n_nrm; j++) {
            const int r = w->nrm_idx[j];
            if (!done[isl[r]]) RESI(r, resolve(m, w, &w->rows[r]));
        }
        for (int j = 0; j < w->n_fr; j++) {
            const int r = w->fr_idx[j];
            row_t *f = &w->rows[r];
            real nimp = w->rows[w->nrm_idx[f->normal_row]].imp;
            if (nimp > 0 && !done[isl[r]]) {
                f->lo = -f->fric * nimp;
                f->hi = f->fric * nimp;
                RESI(r, resolve(m, w, f));
            }
        }
        for (int j = 0; j < w->n_tor; j++) {
            const int r = w->tor_idx[j];
            row_t *f = &w->rows[r];
            real nimp = w->rows[w->nrm_idx[f->normal_row]].imp;
            if (nimp > 0 && !done[isl[r]]) {
                f->lo = -f->fric * nimp;
                f->hi = f->fric * nimp;
                RESI(r, resolve(m, w, f));
            }
        }
#undef RESI
        w->stats_iters++;
        int all = 1;
        for (int r = 0; r < w->nrows; r++) {
            if (!done[isl[r]] && res[isl[r]] <= R(BT_RESIDUAL_THRESHOLD)) done[isl[r]] = 1;
        }
        for (int r = 0; r < w->nrows; r++) all &= done[isl[r]];
        if (all) break;
    }
}

static void solve(const model *m, ws_t *w) {
    if (w->island_exit) { solve_islands(m, w); return; }
    int iters = m->d.solver_iterations;
    w->stats_solves++;
#define RES(x) do { const real r_ = (x); if (r_ > res) res = r_; } while (0)
    for (int it = 0; it < iters; it++) {
        real res = 0;                       /* largest squared residual of this iteration */
        for (int j = 0; j < w->n_nc; j++) {
            int k = (it & 1) ? j : w->n_nc - 1 - j;
            RES(resolve(m, w, &w->rows[w->nc_idx[k]]));
        }
        for (int j = 0; j < w->n_nrm; j++) RES(resolve(m, w, &w->rows[w->nrm_idx[j]]));
        for (int j = 0; j < w->n_fr; j++) {
            row_t *f = &w->rows[w->fr_idx[j]];
            real nimp = w->rows[w->nrm_idx[f->normal_row]].imp;
            if (nimp > 0) {
                f->lo = -f->fric * nimp;
                f->hi = f->fric * nimp;
                RES(resolve(m, w, f));
            }
        }
        /* torsional friction rows after the lateral ones (solveSingleIteration [ext]), limits
         * +-coefficient x the contact's current normal impulse */
        for (int j = 0; j < w->n_tor; j++) {
            row_t *f = &w->rows[w->tor_idx[j]];
            real nimp = w->rows[w->nrm_idx[f->normal_row]].imp;
            if (nimp > 0) {
                f->lo = -f->fric * nimp;
                f->hi = f->fric * nimp;
                RES(resolve(m, w, f));
            }
        }
        w->stats_iters++;
        if (res <= R(BT_RESIDUAL_THRESHOLD)) break;     /* solverResidualThreshold */
    }
#undef RES
}

/* ---------------------------------------------------------------- collision detection */
static void collide(avr_oracle *o, real *st, ws_t *w) {
    const model *m = oview(o, st);
    int gender = w->gender;
    for (int b = 0; b < m->nb; b++) {
        w->body[b] = body_tf(m, st, w, b);
        int g = m->d.body_kind[b] == AVR_BODY_HUMAN ? gender : 0;
        const double *a = m->d.body_aabb + 12 * b + 6 * g;
        aabb_of(w->body[b], ld3d(a), ld3d(a + 3), &w->bmin[b], &w->bmax[b]);
        v3 e = V(R(BT_BROADPHASE_EXPAND), R(BT_BROADPHASE_EXPAND), R(BT_BROADPHASE_EXPAND));
        w->bmin[b] = sub(w->bmin[b], e);
        w->bmax[b] = add(w->bmax[b], e);
    }
    /* child-level overlapping shape pairs, in candidate order (i-major, j-minor) */
    w->nsp = 0;
    for (int p = 0; p < m->np; p++) {
        int ba = m->d.pair_a[p], bb = m->d.pair_b[p];
        if (!aabb_overlap(w->bmin[ba], w->bmax[ba], w->bmin[bb], w->bmax[bb])) continue;
        int sa0 = m->d.body_shape_start[ba], na = m->d.body_shape_count[ba];
        int sb0 = m->d.body_shape_start[bb], nb = m->d.body_shape_count[bb];
        for (int i = 0; i < na; i++) {
            int sa = sa0 + i;
            if (!shape_enabled(m, sa, gender)) continue;
            v3 a0, a1;
            shape_aabb(m, sa, w->body[ba], &a0, &a1);
            int bare = (m->d.body_flags[ba] & 1) && (m->d.body_flags[bb] & 1);
            for (int j = 0; j < nb; j++) {
                int sb = sb0 + j;
                if (!shape_enabled(m, sb, gender)) continue;
                v3 b0, b1;
                shape_aabb(m, sb, w->body[bb], &b0, &b1);
                /* compound children are culled by child AABB (btCompoundCollisionAlgorithm);
                   two bare convex shapes keep their manifold while the broadphase pair lives */
                if (!bare && !aabb_overlap(a0, a1, b0, b1)) continue;
                if (w->nsp < MAX_SPAIRS) { w->sp_a[w->nsp] = sa; w->sp_b[w->nsp] = sb; w->sp_pair[w->nsp] = p; w->nsp++; }
            }
        }
    }
    /* Rebuild the contact pool: for each overlapping shape pair, in order, take its old
     * manifold (points in slot order), run narrowphase + add + refresh, append the survivors.
     * Points of pairs that stopped overlapping are dropped (child algorithm destroyed). */
    int nold = (int)st[S_TASK + T_NCP];
    real *oldcp = w->oldcp;
    memcpy(oldcp, st + S_CP, sizeof(real) * AVR_CP_WORDS * nold);
    int nnew = 0;
    for (int q = 0; q < w->nsp; q++) {
        int sa = w->sp_a[q], sb = w->sp_b[q], p = w->sp_pair[q];
        int ba = m->d.shape_body[sa], bb = m->d.shape_body[sb];
        real thr = R(fmin(m->d.body_threshold[ba], m->d.body_threshold[bb]));
        manifold_t M;
        M.n = 0;
        for (int i = 0; i < nold && M.n < AVR_MANIFOLD_POINTS; i++) {
            const real *c = oldcp + AVR_CP_WORDS * i;
            if ((int)c[AVR_CP_SA] == sa && (int)c[AVR_CP_SB] == sb) memcpy(M.p[M.n++], c, sizeof(real) * AVR_CP_WORDS);
        }
        wshape A = make_wshape(m, sa, w->body[ba]), B = make_wshape(m, sb, w->body[bb]);
        v3 nB, pB;
        real d;
        int hit = narrowphase(w, &A, &B, thr, &nB, &pB, &d);
#ifdef AVR_ORACLE_PROBE
        nB = PRB3(1, nB); pB = PRB3(1, pB); d = PRB(1, d);
#endif
        if (hit) manifold_add(&M, sa, sb, p, w->body[ba], w->body[bb], nB, pB, d, thr);
        manifold_refresh(&M, w->body[ba], w->body[bb], thr);
        for (int k = 0; k < M.n; k++) {
            if (nnew >= K_MAX_CONTACTS) { st[S_TASK + T_FLAGS] = (real)((int)st[S_TASK + T_FLAGS] | 2); break; }
            memcpy(cp_ptr(st, nnew++), M.p[k], sizeof(real) * AVR_CP_WORDS);
        }
    }
    st[S_TASK + T_NCP] = (real)nnew;
}

/* ---------------------------------------------------------------- one Bullet sub-step */
static int substep(avr_oracle *o, real *st, ws_t *w, real dt) {
    const model *m = oview(o, st);
    robot_fk(m, st, w);
    collide(o, st, w);
    /* unconstrained velocities (btMultiBody::computeAccelerationsArticulatedBodyAlgorithmMultiDof) */
    if (robot_mass_matrix(m, w)) return -1;
    real h[K_MAX_DOF] = {0}, qdd[K_MAX_DOF] = {0}, nh[K_MAX_DOF] = {0};
    robot_bias(m, st, w, h);
    for (int d = 0; d < m->nd; d++) nh[d] = -PRB(5, h[d]);
    chol_solve(m, w, nh, qdd);
    real vmax = R(m->d.max_coord_vel);
    for (int d = 0; d < m->nd; d++) {
        real v = st[S_QD + d] + dt * qdd[d];
        w->vq[d] = fmin(vmax, fmax(-vmax, v));
        w->dq[d] = 0;
    }
    real k1l = R(m->d.linear_damping), k1a = R(m->d.angular_damping);
    for (int f = 0; f < m->nf; f++) {
        const real *fb = st + S_FREE + AVR_FB_WORDS * f;
        v3 v = ld3(fb + 7), om = ld3(fb + 10);
        qt q = ldq(fb + 3);
        real mass = R(m->d.fb_mass[f]);
        v3 I = ld3d(m->d.fb_inertia + 3 * f), g = ld3d(m->d.fb_gravity + 3 * f);
        v3 Iw = inertia_mul(q, I, om);
        v3 F = sub(scl(g, mass), scl(v, mass * (k1l + k1l * len(v))));
        v3 T = sub(scl(Iw, -(k1a + k1a * len(om))), crs(om, Iw));
        v3 nv = add(v, scl(F, dt / mass));
        v3 nw = add(om, scl(inertia_inv_mul(q, I, T), dt));
        w->fv[f] = V(fmin(vmax, fmax(-vmax, nv.x)), fmin(vmax, fmax(-vmax, nv.y)), fmin(vmax, fmax(-vmax, nv.z)));
        w->fw[f] = V(fmin(vmax, fmax(-vmax, nw.x)), fmin(vmax, fmax(-vmax, nw.y)), fmin(vmax, fmax(-vmax, nw.z)));
        w->dfv[f] = V(0, 0, 0);
        w->dfw[f] = V(0, 0, 0);
    }
    /* constraint rows + PGS */
    w->nrows = w->n_nc = w->n_nrm = w->n_fr = w->n_tor = 0;
    build_noncontact_rows(m, st, w, dt);
    build_contact_rows(m, st, w, dt);
    w->stats_rows += w->nrows;
    solve(m, w);
    for (int j = 0; j < w->n_nrm; j++) {
        row_t *r = &w->rows[w->nrm_idx[j]];
        cp_ptr(st, r->cp)[AVR_CP_IMP] = r->imp;
    }
    /* velocities, then positions (semi-implicit Euler; btMultiBody::stepPositionsMultiDof) */
    for (int d = 0; d < m->nd; d++) {
        real v = w->vq[d] + w->dq[d];
        v = fmin(vmax, fmax(-vmax, v));
        st[S_QD + d] = v;
        st[S_Q + d] += dt * v;
    }
    for (int f = 0; f < m->nf; f++) {
        real *fb = st + S_FREE + AVR_FB_WORDS * f;
        v3 v = add(w->fv[f], w->dfv[f]), om = add(w->fw[f], w->dfw[f]);
        v = V(fmin(vmax, fmax(-vmax, v.x)), fmin(vmax, fmax(-vmax, v.y)), fmin(vmax, fmax(-vmax, v.z)));
        om = V(fmin(vmax, fmax(-vmax, om.x)), fmin(vmax, fmax(-vmax, om.y)), fmin(vmax, fmax(-vmax, om.z)));
        st3(fb + 7, v);
        st3(fb + 10, om);
        st3(fb, add(ld3(fb), scl(v, dt)));
        /* quaternion exponential update with Bullet's angular motion clamp */
        real ang = len(om);
        if (ang * dt > R(BT_ANGULAR_MOTION_THRESHOLD)) ang = R(0.5 * 1.5707963267948966) / dt;
        v3 ax;
        if (ang < R(0.001)) ax = scl(om, R(0.5) * dt - (dt * dt * dt) * R(0.020833333333) * ang * ang);
        else ax = scl(om, sin(R(0.5) * ang * dt) / ang);
        qt dq = Q(ax.x, ax.y, ax.z, cos(ang * dt * R(0.5)));
        stq(fb + 3, qnorm(qmul(dq, ldq(fb + 3))));
    }
    return 0;
}

/* ---------------------------------------------------------------- task glue (FeedingJaco) */
static real contact_force(const model *m, real *st, int (*pred)(const model *, int, int, void *), void *ctx, int *count) {
    int n = (int)st[S_TASK + T_NCP];
    real s = 0;
    int c = 0;
    for (int i = 0; i < n; i++) {
        real *cp = cp_ptr(st, i);
        int ba = m->d.shape_body[(int)cp[AVR_CP_SA]], bb = m->d.shape_body[(int)cp[AVR_CP_SB]];
        if (pred(m, ba, bb, ctx)) { s += cp[AVR_CP_IMP] / R(m->d.time_step); c++; }
    }
    if (count) *count = c;
    return s;
}

#if !PR2F
static int is_robot(const model *m, int b) { return m->d.body_kind[b] == AVR_BODY_ROBOT; }
static int is_human(const model *m, int b) { return m->d.body_kind[b] == AVR_BODY_HUMAN; }
static int pred_robot_human(const model *m, int a, int b, void *c) { (void)c; return (is_robot(m, a) && is_human(m, b)) || (is_robot(m, b) && is_human(m, a)); }
static int pred_spoon_human(const model *m, int a, int b, void *c) { (void)c; int s = m->d.spoon_body; return (a == s && is_human(m, b)) || (b == s && is_human(m, a)); }
static int pred_body_pair(const model *m, int a, int b, void *c) { int *p = (int *)c; (void)m; return (a == p[0] && b == p[1]) || (a == p[1] && b == p[0]); }
static int pred_body_human(const model *m, int a, int b, void *c) { int f = *(int *)c; return (a == f && is_human(m, b)) || (b == f && is_human(m, a)); }

static void mouth_target(const model *m, const real *st, real *out) {
    const real *h = st + S_HUMAN + 7 * m->d.head_slot;
    tf t; t.p = ld3(h); t.q = ldq(h + 3);
    int g = (int)st[S_TASK + T_GENDER];
    v3 p = tfpt(t, ld3d(m->d.mouth_offset[g]));
    st3(out, p);
}

static void observe(const model *m, real *st, ws_t *w, float spoon_force, float *obs) {
    robot_fk(m, st, w);
    v3 torso = w->cm[m->d.torso_link].p;
    const real *sp = st + S_FREE + AVR_FB_WORDS * m->d.spoon_free;
    v3 spos = ld3(sp);
    v3 tgt = ld3(st + S_TASK + T_TARGET);
    const real *h = st + S_HUMAN + 7 * m->d.head_slot;
    int k = 0;
    v3 a = sub(spos, torso);
    obs[k++] = (float)a.x; obs[k++] = (float)a.y; obs[k++] = (float)a.z;
    for (int i = 0; i < 4; i++) obs[k++] = (float)sp[3 + i];
    a = sub(spos, tgt);
    obs[k++] = (float)a.x; obs[k++] = (float)a.y; obs[k++] = (float)a.z;
    for (int i = 0; i < m->d.n_arm; i++) obs[k++] = (float)st[S_Q + m->d.arm_dofs[i]];
    a = sub(ld3(h), torso);
    obs[k++] = (float)a.x; obs[k++] = (float)a.y; obs[k++] = (float)a.z;
    for (int i = 0; i < 4; i++) obs[k++] = (float)h[3 + i];
    obs[k++] = spoon_force;
}

#endif

/* enforce_hard_human_joint_limits (env.py:389-410): after every stepSimulation a head-chain
 * joint outside its limits is reset onto the limit with zero velocity (resetJointState). */
static void hard_limits(const model *m, real *st) {
    for (int k = 0; k < m->d.hc_n; k++) {
        int d = m->nd_robot + k;
#if PR2F
        real lo = st[S_HCH + 2 * K_HC_N + k], hi = st[S_HCH + 3 * K_HC_N + k];
#else
        real lo = R(m->d.hc_lower[k]), hi = R(m->d.hc_upper[k]);
#endif
        if (st[S_Q + d] < lo) { st[S_Q + d] = lo; st[S_QD + d] = 0; }
        else if (st[S_Q + d] > hi) { st[S_Q + d] = hi; st[S_QD + d] = 0; }
    }
}

#if !PR2F
static int env_step(avr_oracle *o, int e, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    real *st = o->state + (size_t)e * K_STATE_WORDS;
    const model *m = oview(o, st);
    ws_t *w = &o->ws[e];
    w->gender = (int)st[S_TASK + T_GENDER];
    real dt = R(m->d.time_step) / (m->d.num_sub_steps > 0 ? m->d.num_sub_steps : 1);
    int nsub = m->d.num_sub_steps > 0 ? m->d.num_sub_steps : 1;
    /* take_step (env.py:274-337) */
    real a[8], qn[8];
    for (int i = 0; i < m->d.n_arm; i++) {
        real x = act[i];
        x = x < -1 ? -1 : x > 1 ? 1 : x;
        a[i] = (real)((float)x * 0.05f);                  /* float32 action space */
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
    if (m->hc) {
        /* tremor (env.py:327-337): position targets target_human_joint_positions + human_tremors,
           the tremor's sign alternating with self.iteration; gains human_gains, forces
           human_forces * human_strength (strength 1: 'tremor' is not 'weakness') */
        real sg = ((int)st[S_TASK + T_ITER] % 2 == 0) ? 1 : -1;
        for (int k = 0; k < m->d.hc_n; k++) {
            int d = m->nd_robot + k;
            st[S_QTGT + d] = st[S_HCH + k] + st[S_HCH + K_HC_N + k] * sg;
            st[S_KP + d] = R(m->d.human_gain);
            st[S_MAXIMP + d] = R(m->d.human_force * m->d.time_step);
        }
    }
    for (int fr = 0; fr < m->d.frame_skip; fr++) {
        for (int s = 0; s < nsub; s++)
            if (substep(o, st, w, dt)) return -1;
        /* enforce_hard_human_joint_limits (a no-op while the human is static), then
           update_targets (feeding.py:345-349) on the current head pose */
        if (m->hc) {
            hard_limits(m, st);
            robot_fk(m, st, w);
        }
        mouth_target(m, st, st + S_TASK + T_TARGET);
    }
    st[S_TASK + T_ITER] += 1;
    /* get_total_force (feeding.py:83-90) */
    real robot_force = contact_force(m, st, pred_robot_human, 0, 0);
    real spoon_force = contact_force(m, st, pred_spoon_human, 0, 0);
    /* get_food_rewards (feeding.py:92-121) */
    real food_reward = 0, hit_reward = 0, mouth_vel = 0;
    int alive = (int)st[S_TASK + T_ALIVE], hit = (int)st[S_TASK + T_HIT];
    v3 tgt = ld3(st + S_TASK + T_TARGET);
    for (int k = 0; k < m->d.n_food; k++) {
        if (!(alive >> k & 1)) continue;
        real *fb = st + S_FREE + AVR_FB_WORDS * (m->d.food_free0 + k);
        v3 fp = ld3(fb);
        int fbody = m->d.food_body0 + k;
        if (len(sub(tgt, fp)) < R(0.02)) {
            food_reward += 20;
            st[S_TASK + T_SUCCESS] += 1;
            mouth_vel += len(ld3(fb + 7));
            alive &= ~(1 << k);
            /* teleported far away (feeding.py:109); the draw U(1000,2000) is replaced by a fixed spot */
            st3(fb, V(R(1500 + 10 * k), 1500, 1500));
            continue;
        }
        int ctab = 0, cbowl = 0, chum = 0;
        int pt[2] = {fbody, m->d.table_body}, pb[2] = {fbody, m->d.bowl_body};
        contact_force(m, st, pred_body_pair, pt, &ctab);
        contact_force(m, st, pred_body_pair, pb, &cbowl);
        if (fp.z < R(0.5) || ctab > 0 || cbowl > 0) {
            food_reward -= 5;
            alive &= ~(1 << k);
            continue;
        }
        contact_force(m, st, pred_body_human, &fbody, &chum);
        if (chum > 0 && !(hit >> k & 1)) { hit |= 1 << k; hit_reward -= 1; }
    }
    st[S_TASK + T_ALIVE] = (real)alive;
    st[S_TASK + T_HIT] = (real)hit;
    const real *sp = st + S_FREE + AVR_FB_WORDS * m->d.spoon_free;
    real ee_vel = len(ld3(sp + 7));
    observe(m, st, w, (float)spoon_force, obs);
    /* human_preferences (env.py:412-448), feeding branch */
    real prefs = R(m->d.w_velocity) * (-ee_vel) + R(m->d.w_force_nontarget) * (-robot_force) +
                 R(m->d.w_high_forces) * (spoon_force < 10 ? 0 : -spoon_force) + R(m->d.w_food_hit) * hit_reward +
                 R(m->d.w_food_velocities) * (-mouth_vel);
    real dist = len(sub(tgt, ld3(sp)));
    real asq = 0;
    for (int i = 0; i < m->d.n_arm; i++) asq += (real)act[i] * (real)act[i];    /* unclipped (feeding.py:69) */
    real r = R(m->d.w_distance) * (-dist) + R(m->d.w_action) * (-asq) + R(m->d.w_food) * food_reward + prefs;
    *rew = (float)r;
    int it = (int)st[S_TASK + T_ITER];
    *done = (uint8_t)(it >= m->d.max_episode_steps);
    info[0] = (float)(robot_force + spoon_force);
    info[1] = (float)(st[S_TASK + T_SUCCESS] >= R(m->d.n_food) * R(m->d.task_success_threshold) ? 1 : 0);
    for (int i = 0; i < K_STATE_WORDS; i++)
        if (st[i] != st[i]) { st[S_TASK + T_FLAGS] = (real)((int)st[S_TASK + T_FLAGS] | 1); break; }
    return 0;
}

#elif SCRATCH
#include "avr_oracle_scratch.c"
#else
#include "avr_oracle_bedbath.c"
#endif

/* ---------------------------------------------------------------- public API */
#define EXPORT __attribute__((visibility("default")))
#ifdef AVR_ORACLE_PROBE
EXPORT void avr_oracle_probe_mask(unsigned m) { probe_mask = m; }
#endif

static void *dupa(const void *p, size_t n) {
    void *r = malloc(n ? n : 1);
    if (p && n) memcpy(r, p, n);
    return r;
}

EXPORT int avr_oracle_create(const avr_model_desc *d, int n_envs, avr_oracle **out) {
    if (!d || !out || n_envs <= 0) return -1;
    if (d->n_links + d->hc_n > K_MAX_LINKS || d->n_dof + d->hc_n > K_MAX_DOF || d->n_free > K_MAX_FREE ||
        d->n_human > K_MAX_HUMAN || d->n_bodies > MAX_BODIES || d->n_shapes > MAX_SHAPES || d->hc_n > K_HC_N)
        return -2;
    avr_oracle *o = (avr_oracle *)calloc(1, sizeof(avr_oracle));
    model *m = &o->m;
    m->d = *d;
    /* deep-copy arrays so the caller's buffers can go away */
#define CP(field, n, T) m->d.field = (const T *)dupa(d->field, sizeof(T) * (size_t)(n))
    int L = d->n_links, B = d->n_bodies, S = d->n_shapes;
    CP(rl_parent, L, int32_t); CP(rl_jtype, L, int32_t); CP(rl_dof, L, int32_t); CP(rl_has_limit, L, int32_t);
    CP(rl_jpos, 3 * L, double); CP(rl_jquat, 4 * L, double); CP(rl_axis, 3 * L, double);
    CP(rl_com_pos, 3 * L, double); CP(rl_com_quat, 4 * L, double); CP(rl_mass, L, double); CP(rl_inertia, 3 * L, double);
    CP(rl_lower, L, double); CP(rl_upper, L, double); CP(robot_base, 7, double);
    CP(fb_mass, d->n_free, double); CP(fb_inertia, 3 * d->n_free, double); CP(fb_gravity, 3 * d->n_free, double);
    CP(st_pose, 7 * d->n_static, double);
    CP(body_kind, B, int32_t); CP(body_flags, B, int32_t); CP(body_index, B, int32_t); CP(body_shape_start, B, int32_t); CP(body_shape_count, B, int32_t);
    CP(body_friction, B, double); CP(body_threshold, B, double); CP(body_aabb, 12 * B, double);
    if (d->body_rolling) CP(body_rolling, B, double);       /* (NULL: no rolling / spinning friction) */
    if (d->body_spinning) CP(body_spinning, B, double);
    CP(shape_kind, S, int32_t); CP(shape_body, S, int32_t); CP(shape_gender, S, int32_t); CP(shape_hull, 4 * S, int32_t);
    CP(shape_pose, 7 * S, double); CP(shape_param, 4 * S, double); CP(shape_margin, S, double); CP(shape_aabb, 6 * S, double);
    CP(hull_verts, 3 * d->n_hull_verts, double); CP(hull_planes, 4 * d->n_hull_planes, double);
    CP(pair_a, d->n_pairs, int32_t); CP(pair_b, d->n_pairs, int32_t);
#if BEDBATH
    if (!d->bb_targets) { free(o); return -2; }
    CP(bb_targets, 2 * 4 * AVR_BB_MAX_TARGETS, double);
#endif
#undef CP
    m->nl = L; m->nd = d->n_dof; m->nf = d->n_free; m->nb = B; m->ns = S;
    m->np = d->hc_n > 0 ? d->n_pairs_base : d->n_pairs;
    m->nl_robot = L; m->nd_robot = d->n_dof; m->hc = 0;
    for (int i = 0; i < L; i++) {
        m->parent[i] = d->rl_parent[i]; m->jtype[i] = d->rl_jtype[i]; m->dof[i] = d->rl_dof[i];
        m->has_limit[i] = d->rl_has_limit[i]; m->lower[i] = R(d->rl_lower[i]); m->upper[i] = R(d->rl_upper[i]);
        m->jorig[i].p = ld3d(d->rl_jpos + 3 * i); m->jorig[i].q = ldqd(d->rl_jquat + 4 * i);
        m->com[i].p = ld3d(d->rl_com_pos + 3 * i); m->com[i].q = ldqd(d->rl_com_quat + 4 * i);
        m->axis[i] = ld3d(d->rl_axis + 3 * i);
        m->inertia[i] = ld3d(d->rl_inertia + 3 * i);
        m->mass[i] = R(d->rl_mass[i]);
    }
    for (int b = 0; b < B; b++) m->body_link[b] = d->body_kind[b] == AVR_BODY_ROBOT ? d->body_index[b] : -1;
    m->base = ldtf(d->robot_base);
    m->hv = (real *)malloc(sizeof(real) * 3 * (size_t)(d->n_hull_verts + 1));
    for (int i = 0; i < 3 * d->n_hull_verts; i++) m->hv[i] = R(d->hull_verts[i]);
    m->hp = 0;
    /* tremor views: the head chain appended to the robot (links nl.., DoFs nd..) */
    for (int g = 0; g < 2; g++) {
        model *v = &o->mv[g];
        *v = *m;
        if (d->hc_n <= 0) continue;
        v->hc = 1;
        v->np = d->n_pairs;
        for (int k = 0; k < d->hc_n; k++) {
            int i = L + k;
            v->parent[i] = k == 0 ? -2 : i - 1;
            v->jtype[i] = AVR_J_REVOLUTE; v->dof[i] = d->n_dof + k; v->has_limit[i] = 1;
            v->lower[i] = R(d->hc_lower[k]); v->upper[i] = R(d->hc_upper[k]);
            v->jorig[i].p = ld3d(d->hc_jpos[g][k]); v->jorig[i].q = Q(0, 0, 0, 1);
            v->com[i].p = V(0, 0, 0); v->com[i].q = Q(0, 0, 0, 1);
            v->axis[i] = ld3d(d->hc_axis[k]);
            v->inertia[i] = ld3d(d->hc_inertia[g][k]);
            v->mass[i] = R(d->hc_mass[g][k]);
            if (d->hc_body[k] >= 0) v->body_link[d->hc_body[k]] = i;
        }
        v->nl = L + d->hc_n; v->nd = d->n_dof + d->hc_n;
    }
    o->n_envs = n_envs;
    o->threads = 1;
    o->state = (real *)calloc((size_t)n_envs * K_STATE_WORDS, sizeof(real));
    o->ws = (ws_t *)calloc((size_t)n_envs, sizeof(ws_t));
    *out = o;
    return 0;
}

EXPORT int avr_oracle_destroy(avr_oracle *o) {
    if (!o) return -1;
    model *m = &o->m;
    free((void *)m->d.rl_parent); free((void *)m->d.rl_jtype); free((void *)m->d.rl_dof); free((void *)m->d.rl_has_limit);
    free((void *)m->d.rl_jpos); free((void *)m->d.rl_jquat); free((void *)m->d.rl_axis); free((void *)m->d.rl_com_pos);
    free((void *)m->d.rl_com_quat); free((void *)m->d.rl_mass); free((void *)m->d.rl_inertia); free((void *)m->d.rl_lower);
    free((void *)m->d.rl_upper); free((void *)m->d.robot_base); free((void *)m->d.fb_mass); free((void *)m->d.fb_inertia);
    free((void *)m->d.fb_gravity); free((void *)m->d.st_pose); free((void *)m->d.body_kind); free((void *)m->d.body_flags); free((void *)m->d.body_index);
    free((void *)m->d.body_shape_start); free((void *)m->d.body_shape_count); free((void *)m->d.body_friction);
    free((void *)m->d.body_threshold); free((void *)m->d.body_aabb); free((void *)m->d.shape_kind); free((void *)m->d.shape_body);
    free((void *)m->d.shape_gender); free((void *)m->d.shape_hull); free((void *)m->d.shape_pose); free((void *)m->d.shape_param);
    free((void *)m->d.shape_margin); free((void *)m->d.shape_aabb); free((void *)m->d.hull_verts); free((void *)m->d.hull_planes);
    free((void *)m->d.pair_a); free((void *)m->d.pair_b);
    free((void *)m->d.body_rolling); free((void *)m->d.body_spinning);
    free(m->hv);
    free(o->state);
    free(o->ws);
    free(o);
    return 0;
}

EXPORT int avr_oracle_state_words(void) { return K_STATE_WORDS; }

EXPORT int avr_oracle_set_state(avr_oracle *o, const double *state) {
    for (size_t i = 0; i < (size_t)o->n_envs * K_STATE_WORDS; i++) o->state[i] = R(state[i]);
    return 0;
}

EXPORT int avr_oracle_get_state(avr_oracle *o, double *state) {
    for (size_t i = 0; i < (size_t)o->n_envs * K_STATE_WORDS; i++) state[i] = (double)o->state[i];
    return 0;
}

/* reset-path settle: n_frames x stepSimulation with the current motor settings, no task glue
 * (feeding.py:319-320), then the reset observation (feeding.py:325). */
EXPORT int avr_oracle_settle(avr_oracle *o, int n_frames, float *obs) {
    const model *m0 = &o->m;
    real dt = R(m0->d.time_step) / (m0->d.num_sub_steps > 0 ? m0->d.num_sub_steps : 1);
    int nsub = m0->d.num_sub_steps > 0 ? m0->d.num_sub_steps : 1;
    for (int e = 0; e < o->n_envs; e++) {
        real *st = o->state + (size_t)e * K_STATE_WORDS;
        const model *m = oview(o, st);
        ws_t *w = &o->ws[e];
        w->gender = (int)st[S_TASK + T_GENDER];
        for (int f = 0; f < n_frames; f++)
            for (int s = 0; s < nsub; s++)
                if (substep(o, st, w, dt)) return -1;
        /* reset drops the food with plain stepSimulation calls: no hard human limits here */
        robot_fk(m, st, w);
#if SCRATCH
        scratch_target(m, st, w);
        if (obs) scratch_observe(m, st, w, 0.0f, obs + (size_t)e * K_OBS_DIM);   /* _get_obs([0], [0, 0]) */
#elif BEDBATH
        if (obs) bb_observe(m, st, 0.0f, obs + (size_t)e * K_OBS_DIM);           /* _get_obs([0], [0, 0]) (bed_bathing.py:351) */
#else
        mouth_target(m, st, st + S_TASK + T_TARGET);
        if (obs) observe(m, st, w, 0.0f, obs + (size_t)e * K_OBS_DIM);
#endif
    }
    return 0;
}

EXPORT int avr_oracle_step(avr_oracle *o, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    int bad = -1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(o->threads) if (o->threads > 1)
    for (int e = 0; e < o->n_envs; e++)
        if (env_step(o, e, act + (size_t)e * K_ACT_DIM, obs + (size_t)e * K_OBS_DIM, rew + e, done + e, info + (size_t)e * AVR_INFO_DIM))
            bad = e;
    if (bad >= 0) {
        snprintf(o->err, sizeof(o->err), "env %d: mass matrix not positive definite", bad);
        return -1;
    }
    return 0;
}

/* single sub-step without task glue (KAT tests) */
EXPORT int avr_oracle_substep(avr_oracle *o, double dt) {
    for (int e = 0; e < o->n_envs; e++) {
        real *st = o->state + (size_t)e * K_STATE_WORDS;
        o->ws[e].gender = (int)st[S_TASK + T_GENDER];
        if (substep(o, st, &o->ws[e], R(dt))) return -1;
    }
    return 0;
}

/* counters since creation: GJK runs, EPA runs, constraint rows built, PGS iterations run, PGS solves,
 * GJK runs rerun with the double simplex solve after a stall (gjk_mode) */
EXPORT void avr_oracle_stats(avr_oracle *o, long long *out6) {
    for (int k = 0; k < 6; k++) out6[k] = 0;
    for (int e = 0; e < o->n_envs; e++) {
        out6[0] += o->ws[e].stats_gjk; out6[1] += o->ws[e].stats_epa; out6[2] += o->ws[e].stats_rows;
        out6[3] += o->ws[e].stats_iters; out6[4] += o->ws[e].stats_solves; out6[5] += o->ws[e].stats_stall;
    }
}

/* threads used by avr_oracle_step / avr_oracle_settle (OpenMP over envs; 1 = serial) */
EXPORT void avr_oracle_set_threads(avr_oracle *o, int n) { o->threads = n > 0 ? n : 1; }
/* test-only: the PGS residual exit per island instead of per env (solve_islands) */
EXPORT void avr_oracle_set_island_exit(avr_oracle *o, int on) {
    for (int e = 0; e < o->n_envs; e++) o->ws[e].island_exit = on;
}

/* geometry query for tests: narrowphase between shapes sa (on body pose pa[7]) and sb (pb[7]) */
EXPORT int avr_oracle_narrowphase(avr_oracle *o, int sa, const double *pa, int sb, const double *pb, double thr, double *out7) {
    tf ta = ldtf(pa), tb = ldtf(pb);
    wshape A = make_wshape(&o->m, sa, ta), B = make_wshape(&o->m, sb, tb);
    v3 n, p;
    real d;
    int r = narrowphase(&o->ws[0], &A, &B, R(thr), &n, &p, &d);
    out7[0] = n.x; out7[1] = n.y; out7[2] = n.z; out7[3] = p.x; out7[4] = p.y; out7[5] = p.z; out7[6] = d;
    return r;
}

/* forward kinematics for tests: COM frames of robot links -> out[n_links*7] */
EXPORT int avr_oracle_robot_fk(avr_oracle *o, int env, double *out) {
    ws_t *w = &o->ws[env];
    real *st = o->state + (size_t)env * K_STATE_WORDS;
    robot_fk(oview(o, st), st, w);
    for (int i = 0; i < o->m.nl_robot; i++) {
        out[7 * i + 0] = w->cm[i].p.x; out[7 * i + 1] = w->cm[i].p.y; out[7 * i + 2] = w->cm[i].p.z;
        out[7 * i + 3] = w->cm[i].q.x; out[7 * i + 4] = w->cm[i].q.y; out[7 * i + 5] = w->cm[i].q.z; out[7 * i + 6] = w->cm[i].q.w;
    }
    return 0;
}

/* robot self-contact for the reset IK's step_sim screening (util.py:41-46, 63-67:
 * p.getContactPoints(robot, robot) after a restart's frames): at each of n joint vectors
 * q[n*(n_dof+hc_n)] (env 0's state block otherwise), the robot shape pairs the collision pipeline
 * (collide: fattened body AABBs, child AABB culling, narrowphase within the pair's threshold)
 * finds on the robot-robot candidate pairs -> out[n] */
EXPORT int avr_oracle_robot_self_contact(avr_oracle *o, int n, const double *q, int *out) {
    if (!o || n < 0 || (n > 0 && (!q || !out))) return -1;
    const int nq = o->m.d.n_dof + o->m.d.hc_n;
    real *st = (real *)malloc(sizeof(real) * K_STATE_WORDS);
    ws_t *w = (ws_t *)calloc(1, sizeof(ws_t));
    for (int i = 0; i < n; i++) {
        memcpy(st, o->state, sizeof(real) * K_STATE_WORDS);
        for (int d = 0; d < nq; d++) st[S_Q + d] = R(q[(size_t)i * nq + d]);
        const model *m = oview(o, st);
        robot_fk(m, st, w);
        int cnt = 0;
        for (int p = 0; p < m->np; p++) {
            int ba = m->d.pair_a[p], bb = m->d.pair_b[p];
            if (m->d.body_kind[ba] != AVR_BODY_ROBOT || m->d.body_kind[bb] != AVR_BODY_ROBOT) continue;
            tf ta = body_tf(m, st, w, ba), tb = body_tf(m, st, w, bb);
            v3 a0, a1, b0, b1, e = V(R(BT_BROADPHASE_EXPAND), R(BT_BROADPHASE_EXPAND), R(BT_BROADPHASE_EXPAND));
            aabb_of(ta, ld3d(m->d.body_aabb + 12 * ba), ld3d(m->d.body_aabb + 12 * ba + 3), &a0, &a1);
            aabb_of(tb, ld3d(m->d.body_aabb + 12 * bb), ld3d(m->d.body_aabb + 12 * bb + 3), &b0, &b1);
            if (!aabb_overlap(sub(a0, e), add(a1, e), sub(b0, e), add(b1, e))) continue;
            real thr = R(fmin(m->d.body_threshold[ba], m->d.body_threshold[bb]));
            int bare = (m->d.body_flags[ba] & 1) && (m->d.body_flags[bb] & 1);
            for (int sa = m->d.body_shape_start[ba]; sa < m->d.body_shape_start[ba] + m->d.body_shape_count[ba]; sa++) {
                v3 c0, c1;
                shape_aabb(m, sa, ta, &c0, &c1);
                for (int sb = m->d.body_shape_start[bb]; sb < m->d.body_shape_start[bb] + m->d.body_shape_count[bb]; sb++) {
                    v3 d0, d1;
                    shape_aabb(m, sb, tb, &d0, &d1);
                    if (!bare && !aabb_overlap(c0, c1, d0, d1)) continue;
                    wshape A = make_wshape(m, sa, ta), B = make_wshape(m, sb, tb);
                    v3 nB, pB;
                    real dd;
                    cnt += narrowphase(w, &A, &B, thr, &nB, &pB, &dd) != 0;
                }
            }
        }
        out[i] = cnt;
    }
    free(st);
    free(w);
    return 0;
}

EXPORT const char *avr_oracle_last_error(avr_oracle *o) { return o ? o->err : "null handle"; }
