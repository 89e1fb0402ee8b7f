// avr_kernel.hip -- MI355X (gfx950) step kernel for the Assistive Gym FeedingJaco-v0 hot path.
//
// One environment per wavefront (workgroup = 64 lanes).  A launch advances every env by one
// gym step: take_step glue (env.py:274-337), frame_skip x numSubSteps Bullet sub-steps
// (env.py:341-349, feeding.py:289), then get_total_force / get_food_rewards / _get_obs / reward
// (feeding.py:56-142, env.py:412-448).  The per-env state block (avr_model.h) is staged in LDS
// for the whole launch and written back once; model data (hull vertices, link tables) is
// read-only global memory shared by all envs and stays L2/MALL resident.
//
// Work decomposition inside a wave:
//   * lanes over bodies / candidate pairs / child-shape pairs (broadphase, AABB culling);
//   * one lane per child-shape pair for the narrowphase of small shapes (spheres, capsules,
//     boxes, hulls <= SMALL_NV vertices), the whole wave per pair for large hulls (support
//     mapping = parallel vertex scan + wave argmax) and for EPA;
//   * one lane per manifold for the persistent-manifold update (prefix-sum compaction);
//   * lanes over mass-matrix entries, over constraint rows (Jacobians, M^-1 J^T);
//   * the projected Gauss-Seidel sweep is inherently sequential (Bullet semantics): it runs
//     wave-uniform out of LDS.
// No MFMA: this is branchy small-body dynamics.  The algorithm is identical to the CPU oracle
// (oracle/avr_oracle.c), which cites the Bullet/PyBullet behaviour it restates.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/avr.h"
#include <cstring>
#include <cstdlib>
#include "avr_math.h"

#include "avr_kmodel.h"

// explicitly addressed memory: LDS (ds_read / ds_write) and global (global_load) pointers, so that
// no hot loop goes through flat instructions (a flat load makes every wait cover both counters)
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) float lds_f;
// Model and scratch arrays live in global memory, but a pointer loaded from the KModel is generic
// to the compiler: its loads become flat loads, whose waits also drain every LDS access in
// flight.  Hot reads name the address space (gld: global; the model arrays are never written).
#define AVR_GA __attribute__((address_space(1)))
template <class T> __device__ __forceinline__ T gld(const T *p) { return *(const AVR_GA T *)p; }
__device__ __forceinline__ int2 gld(const int2 *p) { const AVR_GA int *q = (const AVR_GA int *)p; return make_int2(q[0], q[1]); }
__device__ __forceinline__ float2 gld(const float2 *p) { const f2v x = *(const AVR_GA f2v *)p; return make_float2(x.x, x.y); }
__device__ __forceinline__ float4 gld(const float4 *p) { const f4v x = *(const AVR_GA f4v *)p; return make_float4(x.x, x.y, x.z, x.w); }
__device__ __forceinline__ v3 gld3(const float *p) { const AVR_GA float *q = (const AVR_GA float *)p; return V(q[0], q[1], q[2]); }
__device__ __forceinline__ qt gldq(const float *p) { const AVR_GA float *q = (const AVR_GA float *)p; return Q(q[0], q[1], q[2], q[3]); }
__device__ __forceinline__ tf gldtf(const float *p) { tf r; r.p = gld3(p); r.q = gldq(p + 3); return r; }
typedef __attribute__((address_space(3))) f2v lds_f2;
typedef __attribute__((address_space(3))) f4v lds_f4;
typedef __attribute__((address_space(3))) int lds_i;
typedef const __attribute__((address_space(1))) float *gfp;
typedef const __attribute__((address_space(1))) f4v *gf4p;
typedef const __attribute__((address_space(1))) f2v *gf2p;

// --------------------------------------------------------------------------- device model


// --------------------------------------------------------------------------- LDS layout
#define AVR_PROF_SLOTS 48   // diagnostic build: per-env cycle / event counters (tools/prof_phases.py)
struct EnvLDS {
    float st[S_CP];     // state words before the contact cache; the cache lives in global memory
    float cm[MAXL][8], ax[MAXL][4], org[MAXL][4];
    float btf[MAXB][8];
    float vq[MAXD];
    float fv[MAXF][4], fw[MAXF][4];
    float Iinv[MAXF][12];   // world inverse inertia (row-major 3x3)
    float gsc[MAXF][4];     // 1/sqrt(m), sqrt of the inverse principal inertias (mass-normalised rows)
    float h[MAXD], qdd[MAXD];
    int nsp, nap, n_nc, n_c, flags, gender;
    int n_t;                // (K_TORSION) contacts with torsional rows
    int nla, nda;           // articulated links / DoFs of this env (the head chain counts under 'tremor')
#ifdef AVR_PROF
    unsigned long long prof[AVR_PROF_SLOTS];
#endif
#ifdef AVR_PAD_A_WORDS
    float pad_a[AVR_PAD_A_WORDS];   // (occupancy experiments: extra LDS per kernel-a block)
#endif
    // Phase-overlaid storage (kernel a's LDS footprint sets how many env groups' launches can be
    // resident at once): the contact update's pool is dead once the new pool is
    // in global memory; the mass matrix's Cholesky factor is dead once M^-1 is formed, before the
    // RNEA (and the row enumeration after it) uses its temporaries; M^-1 lives until the rows.
    // robot_fk's joint frames (lk) are its own scratch (dead when it returns; kernel a, which gets
    // its frames from the pair kernel, never runs it, and no caller holds u data across it).
    union __attribute__((aligned(16))) {
        float lk[MAXL][8];                 // robot_fk: joint frames + joint value
        struct {                           // contact update (part A3)
            float ocp[K_MAX_CONTACTS * AVR_CP_WORDS];   // previous contact pool, updated in place
            int okey[K_MAX_CONTACTS];                   // its (sa | sb << 16) keys
        } k;
        struct {                           // dynamics and rows
            union {
                float rn[6][MAXL][4];      // RNEA temporaries: omega, v_com, alpha, a_com, F, N
                float Mi[MAXD][MAXD];      // Cholesky factor of the mass matrix (lower)
            };
            float iw[MAXL][8];             // world inertia (xx yy zz xy xz yz), mass
            float Minv[MAXD][MAXD];        // M^-1
        } d;
    } u;
};

// LDS of the pair kernel (avr_substep_pairs_kernel), <= 10 KB so that 16 blocks (a 4096-env
// launch) are resident at once.  The state words and link frames are dead once the body frames
// exist, so the collision scratch overlays them.
struct PairsLDS {
    float btf[MAXB][8];
    unsigned short sinfo[MAXSH];   // m.shape_info (13 bits: child index + 1, gender + 1, kind)
    int flags, gender, nla, nda;
#ifdef AVR_PROF
    unsigned long long prof[AVR_PROF_SLOTS];
#endif
    union __attribute__((aligned(16))) {
        struct {                           // forward kinematics and body frames
            float st[S_CP];
            float lk[MAXL][8], cm[MAXL][8], ax[MAXL][4], org[MAXL][4];
        };
        struct {
            struct {                       // collision detection
                float bmin[MAXB][4], bmax[MAXB][4];
                unsigned short apair[MAXAP];        // active body pairs (broadphase output, in pair order)
                unsigned short candA[128], candB[128];   // children of A (B) whose AABB meets B's (A's) body AABB
                float caabb[MAXCC][6];     // world AABBs of the non-static shapes (min3, max3)
            } c;
        } u;
    };
};
#ifndef AVR_PROF
static_assert(sizeof(PairsLDS) <= 10240, "pair kernel: 16 blocks per CU");
static_assert(MAXSH % 64 == 0, "shape info staged 64 per pass");
#endif

// Intra-env synchronisation.  An env is one wavefront, so a workgroup fence -- this wave's memory
// operations complete and are visible -- plus a compiler barrier is enough; no s_barrier (the
// kernels' bodies are device functions that a multi-env block could run one wave per env).
#define SYNC()                                          \
    do {                                                \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); \
        __builtin_amdgcn_wave_barrier();                \
    } while (0)

// Diagnostic phase timers (separate AVR_PROF build only; the shipped kernel has none).
#ifdef AVR_PROF
#define PROF_START(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_STOP(slot, v) \
    do { unsigned long long _n = __builtin_amdgcn_s_memtime(); if (lane_id() == 0) L.prof[slot] += _n - (v); v = _n; } while (0)
#else
#define PROF_START(v) (void)0
#define PROF_STOP(slot, v) (void)0
#endif

// --------------------------------------------------------------------------- kinematics
// robot_fk: link frames published in LDS.  Every link (lane i) first publishes its joint's local
// data (origin frame, joint rotation, axis, displacement); then each lane composes the local
// frames of its own chain root first -- the same transform products in the same order as a
// level-by-level pass over the tree, without a barrier per level.  Under 'tremor' the head chain
// follows the robot's links: its root hangs off the static chest slot (parent -2) and its link
// frames (== COM frames) are published into the human slot poses, where collision and the task
// glue (getLinkState(human, 27), feeding.py:134,254) read them.
template <class LT>
AVR_DI int lgo(const LT &L, const KModel &m) { return L.gender * m.nla; }   // gendered table offset

// robot_fk's joint-frame scratch: a member of EnvLDS's phase union, of PairsLDS's FK struct
AVR_DI float (*lk_of(EnvLDS &L))[8] { return L.u.lk; }
AVR_DI float (*lk_of(PairsLDS &L))[8] { return L.lk; }

template <class LT>
AVR_DI void robot_fk(const KModel &m, LT &L) {
    const int i = lane_id();
    const bool mine = i < L.nla;
    unsigned am = 0;
    tf com;
    v3 axl = V(0, 0, 0);
    // local joint data in LDS (lk: origin frame + displacement in word 7; cm: joint rotation,
    // axis, joint type), overwritten by the results once every lane has composed its chain
    if (mine) {
        const int go = lgo(L, m);
        const int jt = gld(m.rl_jtype + (i));
        am = gld(m.anc_mask + (i));
        const tf jo = gldtf(m.rl_jorig + 8 * (go + i));
        com = gldtf(m.rl_com + 8 * (go + i));
        axl = gld3(m.rl_axis + 4 * i);
        const int dof = gld(m.rl_dof + (i));
        const float qv = dof >= 0 ? L.st[S_Q + dof] : 0.f;
        const qt qj = jt == AVR_J_REVOLUTE ? qaxis(axl, qv) : Q(0, 0, 0, 1);
        sttf(lk_of(L)[i], jo);
        lk_of(L)[i][7] = qv;
        stq(L.cm[i], qj);
        st3(L.cm[i] + 4, axl);
        L.cm[i][7] = (float)jt;
    }
    SYNC();
    tf t;
    v3 org = V(0, 0, 0), axw = V(0, 0, 0);
    if (mine) {
        const int r = __builtin_ctz(am);                       // the chain's root link
#if K_RBASE_IN_STATE
        t = gld(m.rl_parent + (r)) == -2 ? ldtf(L.st + S_HUMAN + 7 * m.hc_parent_slot) : ldtf(L.st + S_RBASE);
#else
        t = gld(m.rl_parent + (r)) == -2 ? ldtf(L.st + S_HUMAN + 7 * m.hc_parent_slot) : gldtf(m.base);
#endif
        for (unsigned b = am; b; b &= b - 1u) {
            const int k = __builtin_ctz(b);
            const tf jo = ldtf(lk_of(L)[k]);
            const float qv = lk_of(L)[k][7];
            const qt qj = ldq(L.cm[k]);
            const v3 ax = ld3(L.cm[k] + 4);
            const int jt = (int)L.cm[k][7];
            t = tfmul(t, jo);
            const v3 aw = qrot(t.q, ax);
            if (k == i) { org = t.p; axw = aw; }
            if (jt == AVR_J_REVOLUTE) t.q = qmul(t.q, qj);
            else if (jt == AVR_J_PRISMATIC) t.p = add(t.p, scl(aw, qv));
        }
    }
    SYNC();
    if (mine) {
        st3(L.org[i], org);
        st3(L.ax[i], axw);
        sttf(lk_of(L)[i], t);
        sttf(L.cm[i], tfmul(t, com));
    }
    SYNC();
    const int c = i - m.nl;
    if (mine && c >= 0) {
        const int slot = gld(m.hc_slot + (c));
        if (slot >= 0) {
            float *h = L.st + S_HUMAN + 7 * slot;
            st3(h, ld3(L.cm[i]));
            stq(h + 3, ldq(L.cm[i] + 3));
        }
    }
    SYNC();
}

AVR_DI bool is_ancestor(const KModel &m, int link, int anc) { return (gld(m.anc_mask + (link)) >> anc) & 1u; }

AVR_DI void dof_col(const KModel &m, const EnvLDS &L, int j, v3 p, v3 &lin, v3 &ang) {
    v3 a = ld3(L.ax[j]);
    if (gld(m.rl_jtype + (j)) == AVR_J_REVOLUTE) {
        ang = a;
        lin = crs(a, sub(p, ld3(L.org[j])));
    } else {
        ang = V(0, 0, 0);
        lin = a;
    }
}

// Mass matrix: one lane per lower-triangle entry (a,b), then the Cholesky factor in LDS.  Rows and
// columns beyond nd are padded with the identity so M^-1 solves run over MAXD unrolled.

// x = M^-1 e_c for a column c of the block [B0, B1) of the block-diagonal factor (entries of x
// outside the block are 0): forward / back substitution over the block only -- the full-size solve
// on e_c adds nothing but products with exact zeros (the other block, the zero head of y)
template <int B0, int B1>
AVR_DI void chol_solve_block(const EnvLDS &L, int c, float *x) {
    float y[MAXD];
#pragma unroll
    for (int i = 0; i < MAXD; i++) { y[i] = 0.f; x[i] = 0.f; }
#pragma unroll
    for (int i = B0; i < B1; i++) {
        float s = i == c ? 1.f : 0.f;
#pragma unroll
        for (int k = B0; k < i; k++) s -= L.u.d.Mi[i][k] * y[k];
        y[i] = s / L.u.d.Mi[i][i];
    }
#pragma unroll
    for (int i = B1 - 1; i >= B0; i--) {
        float s = y[i];
#pragma unroll
        for (int k = i + 1; k < B1; k++) s -= L.u.d.Mi[k][i] * x[k];
        x[i] = s / L.u.d.Mi[i][i];
    }
}

AVR_DI bool robot_mass_matrix(const KModel &m, EnvLDS &L) {
    PROF_START(pm);
    const int nd = L.nda;
    const int go = lgo(L, m);
    const int lane = lane_id();
    if (lane < L.nla) {   // world inertia R diag(I) R^T and mass of link `lane`
        const m3 R = qmat(ldq(L.cm[lane] + 3));
        const v3 I = gld3(m.rl_inertia + 4 * (go + lane));
        float *w = L.u.d.iw[lane];
#define AVR_IW(a, b) (R.m[a][0] * R.m[b][0] * I.x + R.m[a][1] * R.m[b][1] * I.y + R.m[a][2] * R.m[b][2] * I.z)
        w[0] = AVR_IW(0, 0); w[1] = AVR_IW(1, 1); w[2] = AVR_IW(2, 2);
        w[3] = AVR_IW(0, 1); w[4] = AVR_IW(0, 2); w[5] = AVR_IW(1, 2);
#undef AVR_IW
        w[6] = gld(m.rl_mass + (go + lane));
    }
    SYNC();
    const int ne = MAXD * (MAXD + 1) / 2;
    for (int e = lane; e < ne; e += 64) {
        int a = 0, rem = e;
        while (rem > a) { rem -= a + 1; a++; }
        int b = rem;
        float s = 0.f;
        if (a < nd && b < nd) {
            const int la = gld(m.dof_link + (a)), lb = gld(m.dof_link + (b));
            const v3 axa = ld3(L.ax[la]), oa = ld3(L.org[la]), axb = ld3(L.ax[lb]), ob = ld3(L.org[lb]);
            const bool ra = gld(m.rl_jtype + (la)) == AVR_J_REVOLUTE, rb = gld(m.rl_jtype + (lb)) == AVR_J_REVOLUTE;
            // links in both subtrees, ascending (a per-lane bit loop: no scalar load per link)
            for (unsigned dm = gld(m.desc_mask + (la)) & gld(m.desc_mask + (lb)); dm; dm &= dm - 1u) {
                const int i = __builtin_ctz(dm);
                const float *w = L.u.d.iw[i];
                const float mi = w[6];
                if (mi <= 0.f) continue;
                const v3 c = ld3(L.cm[i]);
                const v3 lina = ra ? crs(axa, sub(c, oa)) : axa, linb = rb ? crs(axb, sub(c, ob)) : axb;
                const v3 anga = ra ? axa : V(0, 0, 0), angb = rb ? axb : V(0, 0, 0);
                const v3 Ia = V(w[0] * anga.x + w[3] * anga.y + w[4] * anga.z, w[3] * anga.x + w[1] * anga.y + w[5] * anga.z,
                                w[4] * anga.x + w[5] * anga.y + w[2] * anga.z);
                s += mi * dot(lina, linb) + dot(Ia, angb);
            }
        } else if (a == b) s = 1.f;
        L.u.d.Mi[a][b] = s;
        if (a != b) L.u.d.Mi[b][a] = 0.f;
    }
    SYNC();
    PROF_STOP(24, pm);
    // column Cholesky, rows of each column in parallel (one lane per row).  M is block diagonal:
    // the robot's K_ND DoFs, then the articulated human chain's (and identity padding), which share
    // no link.  The two blocks factor side by side -- iteration j takes robot column j and chain
    // column K_ND + j -- and skip the cross-block terms, which are exact zeros: the same values,
    // bit for bit, as the full column loop.
    static_assert(K_ND <= MAXD, "robot block");
    constexpr int NH = MAXD - K_ND;
    constexpr int NJ = K_ND > NH ? K_ND : NH;
    int ok = 1;
    {
        const int i = lane;
        const bool rob = i < K_ND;
        const int k0 = rob ? 0 : K_ND;         // the first column of this lane's block
        for (int jj = 0; jj < NJ; jj++) {
            const int j = rob ? jj : K_ND + jj;    // this lane's block's column
            const bool live = rob ? jj < K_ND : (jj < NH && i < MAXD);
            float s = 0.f, t = 0.f;
            if (live) {
                s = L.u.d.Mi[j][j];
                for (int k = k0; k < j; k++) s -= L.u.d.Mi[j][k] * L.u.d.Mi[j][k];
                if (i > j) {
                    t = L.u.d.Mi[i][j];
                    for (int k = k0; k < j; k++) t -= L.u.d.Mi[i][k] * L.u.d.Mi[j][k];
                }
            }
            // every column's diagonal is positive in exact arithmetic; a lane of either block reports
            const int bad = __any(live && s <= 0.f);
            if (bad) ok = 0;
            const float d = sqrtf(fmaxf(s, 1e-30f));
            SYNC();
            if (live && i > j) L.u.d.Mi[i][j] = t / d;
            if (live && i == j) L.u.d.Mi[j][j] = d;
            SYNC();
        }
    }
    PROF_STOP(25, pm);
    // columns of M^-1 (one lane per DoF), each within its block: every robot row gets M^-1 J^T
    // from these
    if (lane < MAXD) {
        float x[MAXD];
        if (lane < K_ND) chol_solve_block<0, K_ND>(L, lane, x);
        else chol_solve_block<K_ND, MAXD>(L, lane, x);
#pragma unroll
        for (int k = 0; k < MAXD; k++) L.u.d.Minv[k][lane] = x[k];
    }
    SYNC();
    PROF_STOP(26, pm);
    return ok != 0;
}

// y = M^-1 x (padding DoFs have identity rows)
#ifndef AVR_MINV_LAUNDER
#define AVR_MINV_LAUNDER 1
#endif
AVR_DI void minv_mul(const EnvLDS &L, const float *x, float *y) {
#if AVR_MINV_LAUNDER
    // keep the MAXD^2 M^-1 loads inside the caller's loops: hoisted, they pin ~200 VGPRs (the PR2
    // tasks' kernel a 281 -> 190 VGPRs, two waves per SIMD instead of one: ScratchItch 1.16M ->
    // 1.31M env-steps/s, BedBathing 1.35M -> 1.55M; FeedingJaco unchanged)
    int z = 0;
    asm volatile("" : "+v"(z));
    const float *Mv = &L.u.d.Minv[0][0] + z;
#else
    const float *Mv = &L.u.d.Minv[0][0];
#endif
#pragma unroll
    for (int i = 0; i < MAXD; i++) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < MAXD; k++) s += Mv[i * MAXD + k] * x[k];
        y[i] = s;
    }
}

// y = M^-1 x for an endpoint on articulated link `link`, within the link's block of M: a robot
// link's Jacobian is zero on the human chain's DoFs (no chain DoF is an ancestor of a robot link)
// and a chain link's on the robot's, and M^-1 is block diagonal with exact zeros off the blocks
// (chol_solve_block), so the terms skipped are products of zeros that minv_mul would add to its
// sums, leaving them unchanged: the same bits with K_ND^2 (robot) instead of MAXD^2 products -- the
// serial tail of an env's contact rows when one lane holds a robot contact (FeedingJaco: 100 of 196
// products per row; the PR2 tasks 196 of 576)
template <int LO, int HI>
AVR_DI void minv_mul_blk(const EnvLDS &L, const float *x, float *y) {
#if AVR_MINV_LAUNDER
    int z = 0;
    asm volatile("" : "+v"(z));
    const float *Mv = &L.u.d.Minv[0][0] + z;
#else
    const float *Mv = &L.u.d.Minv[0][0];
#endif
#pragma unroll
    for (int i = 0; i < MAXD; i++) {
        if (i < LO || i >= HI) { y[i] = 0.f; continue; }
        float s = 0.f;
#pragma unroll
        for (int k = LO; k < HI; k++) s = fmaf(Mv[i * MAXD + k], x[k], s);
        y[i] = s;
    }
}
AVR_DI void minv_mul_link(const KModel &m, const EnvLDS &L, int link, const float *x, float *y) {
    if (link < m.nl) minv_mul_blk<0, K_ND>(L, x, y);
    else minv_mul_blk<K_ND, MAXD>(L, x, y);
}

// the second robot endpoint of a row whose first endpoint's (J, M^-1 J^T) are in J, MJ: y = M^-1 x
// row by row (minv_mul's sums), each y_i added to MJ_i and x_i y_i, x_i vq_i to den, rel in DoF
// order, then x added to J -- the same roundings as storing the first endpoint's part and adding
// the second's to it (add_robot) without the read-back of the first from memory
template <int LO, int HI>
AVR_DI void minv_mul_add_blk(const EnvLDS &L, const float *x, float *J, float *MJ, float &den, float &rel) {
#if AVR_MINV_LAUNDER
    int z = 0;
    asm volatile("" : "+v"(z));
    const float *Mv = &L.u.d.Minv[0][0] + z;
#else
    const float *Mv = &L.u.d.Minv[0][0];
#endif
#pragma unroll
    for (int i = 0; i < MAXD; i++) {
        // (outside x's block: s = 0 and x_i = 0 exactly, so den, rel and MJ_i keep their values)
        if (i < LO || i >= HI) continue;
        float s = 0.f;
#pragma unroll
        for (int k = LO; k < HI; k++) s = fmaf(Mv[i * MAXD + k], x[k], s);
        den = fmaf(x[i], s, den); rel = fmaf(x[i], L.vq[i], rel);
        MJ[i] += s;
    }
#pragma unroll
    for (int i = 0; i < MAXD; i++) J[i] += x[i];
}
AVR_DI void minv_mul_add(const KModel &m, const EnvLDS &L, int link, const float *x, float *J, float *MJ, float &den, float &rel) {
    if (link < m.nl) minv_mul_add_blk<0, K_ND>(L, x, J, MJ, den, rel);
    else minv_mul_add_blk<K_ND, MAXD>(L, x, J, MJ, den, rel);
}

// entry d of M^-1 x within the block [LO, HI) of M (minv_mul_blk's sum for row d; one lane per row)
template <int LO, int HI>
AVR_DI float minv_entry(const EnvLDS &L, const float *x, int d) {
    if (d < LO || d >= HI) return 0.f;
    const float *Mv = &L.u.d.Minv[0][0] + d * MAXD;
    float s = 0.f;
#pragma unroll
    for (int k = LO; k < HI; k++) s = fmaf(Mv[k], x[k], s);
    return s;
}

// Recursive Newton-Euler bias forces (Coriolis, gyroscopic, btMultiBody damping), result in L.h.
// The forward recursion (parent p of link i, joint origin o_i, COM c_i):
//   om_i = om_p + w_i                       (w_i = axis qd, revolute; 0 otherwise)
//   al_i = al_p + om_p x w_i
//   vc_i = ((vc_p + om_p x (o_i - c_p)) + v_i) + om_i x (c_i - o_i)          (v_i = axis qd, prismatic)
//   ac_i = ((ac_p + (al_p x (o_i - c_p) + om_p x (om_p x (o_i - c_p)))) + 2 om_p x v_i)
//          + (al_i x (c_i - o_i) + om_i x (om_i x (c_i - o_i)))
// is a sum of per-link terms over the root-to-i path, so every link forms its own terms once its
// parent's om (then al) are known and sums its ancestors' terms root first (links are numbered
// parents first): the same additions in the same order as the level-by-level recursion, in three
// passes instead of one per tree level.  The backward force accumulation is summed per DoF: the
// DoF of link j sees the moment about its joint origin of every force in its subtree,
// h_j = ax_j . sum_k (N_k + (c_k - o_j) x F_k) (revolute; ax_j . sum_k F_k prismatic), which is what
// the recursion (F_p += F_k, N_p += N_k + (c_k - c_p) x F_k) evaluates.
// (the ancestors of a link, root first: a per-lane bit loop over its ancestor mask, whose trip
// count is the link's depth rather than the link count; kernel a 0.182 -> 0.178 ms per 4096-env
// launch, bit-identical)
AVR_DI v3 anc_sum(const KModel &m, unsigned am, const float (*T)[4], int nla, v3 acc) {
    (void)m; (void)nla;
    for (unsigned dm = am; dm; dm &= dm - 1u) {
        const f4v t = *(const lds_f4 *)T[__builtin_ctz(dm)];
        acc = add(acc, V(t.x, t.y, t.z));
    }
    return acc;
}
AVR_DI v3 anc_sum3(const KModel &m, unsigned am, const float (*A)[4], const float (*B)[4], const float (*C)[4], int nla, v3 acc) {
    (void)m; (void)nla;
    for (unsigned dm = am; dm; dm &= dm - 1u) {
        const int k = __builtin_ctz(dm);
        const f4v a = *(const lds_f4 *)A[k], b = *(const lds_f4 *)B[k], c = *(const lds_f4 *)C[k];
        acc = add(add(add(acc, V(a.x, a.y, a.z)), V(b.x, b.y, b.z)), V(c.x, c.y, c.z));
    }
    return acc;
}

AVR_DI void robot_bias(const KModel &m, EnvLDS &L) {
    float (*R0)[4] = L.u.d.rn[0], (*R1)[4] = L.u.d.rn[1], (*R2)[4] = L.u.d.rn[2], (*R3)[4] = L.u.d.rn[3], (*R4)[4] = L.u.d.rn[4], (*R5)[4] = L.u.d.rn[5];
    const float k1l = m.lin_damp, k1a = m.ang_damp;
    const int i = lane_id();
    const int nla = L.nla;
    const bool mine = i < nla;
    int p = -3, jt = AVR_J_FIXED;
    unsigned am = 0;
    float mi = 0.f, qd = 0.f;
    v3 I = V(0, 0, 0), o = V(0, 0, 0), c = V(0, 0, 0), axw = V(0, 0, 0);
    qt q = Q(0, 0, 0, 1);
    if (mine) {
        const int go = lgo(L, m);
        p = gld(m.rl_parent + (i));          // < 0: fixed robot base or (-2) the static chest slot
        jt = gld(m.rl_jtype + (i));
        am = gld(m.anc_mask + (i));
        const int dof = gld(m.rl_dof + (i));
        qd = dof >= 0 ? L.st[S_QD + dof] : 0.f;
        o = ld3(L.org[i]); c = ld3(L.cm[i]); axw = ld3(L.ax[i]);
        q = ldq(L.cm[i] + 3);
        mi = gld(m.rl_mass + (go + i));
        I = gld3(m.rl_inertia + 4 * (go + i));
    }
    const bool rev = jt == AVR_J_REVOLUTE, pri = jt == AVR_J_PRISMATIC;
    const v3 wj = rev ? scl(axw, qd) : V(0, 0, 0), vj = pri ? scl(axw, qd) : V(0, 0, 0);
    const v3 cp = p < 0 ? gld3(m.base) : ld3(L.cm[p > 0 ? p : 0]);
    const v3 rpo = sub(o, cp), roc = sub(c, o);
    // pass 1: angular velocities
    if (mine) st3(R1[i], wj);
    SYNC();
    const v3 om = anc_sum(m, am, R1, nla, V(0, 0, 0));
    if (mine) st3(R0[i], om);
    SYNC();
    // pass 2: angular accelerations, COM velocities
    const v3 omp = p < 0 ? V(0, 0, 0) : ld3(R0[p]);
    if (mine) {
        st3(R2[i], crs(omp, wj));
        st3(R3[i], crs(omp, rpo)); st3(R4[i], vj); st3(R5[i], crs(om, roc));
    }
    SYNC();
    const v3 al = anc_sum(m, am, R2, nla, V(0, 0, 0));
    const v3 vc = anc_sum3(m, am, R3, R4, R5, nla, V(0, 0, 0));
    if (mine) st3(R1[i], al);
    SYNC();
    // pass 3: COM accelerations
    const v3 alp = p < 0 ? V(0, 0, 0) : ld3(R1[p]);
    SYNC();
    if (mine) {
        st3(R2[i], add(crs(alp, rpo), crs(omp, crs(omp, rpo))));
        st3(R3[i], scl(crs(omp, vj), 2.f));
        st3(R4[i], add(crs(al, roc), crs(om, crs(om, roc))));
    }
    SYNC();
    const v3 ac = anc_sum3(m, am, R2, R3, R4, nla, V(0, 0, 0));
    // forces: FF = R1, NN = R5 (every lane is past its pass-3 reads of R2..R4 only after the sync below)
    if (mine) {
        const v3 Iw = inertia_mul(q, I, om);
        const float vn = len(vc), wn = len(om);
        const v3 fdamp = scl(vc, -mi * (k1l + k1l * vn));
        const v3 tdamp = scl(Iw, -(k1a + k1a * wn));
#if K_HUMAN_GRAVITY
        // gravity of the articulated human chain (its links follow the robot's): F = m (a - g)
        const v3 ga = i >= m.nl ? V(ac.x - m.hc_grav[0], ac.y - m.hc_grav[1], ac.z - m.hc_grav[2]) : ac;
        st3(R1[i], sub(scl(ga, mi), fdamp));
#else
        st3(R1[i], sub(scl(ac, mi), fdamp));
#endif
        st3(R5[i], sub(add(inertia_mul(q, I, al), crs(om, Iw)), tdamp));
    }
    SYNC();
    if (i < MAXD) {
        float h = 0.f;
        if (i < L.nda) {
            const int j = gld(m.dof_link + (i));
            const v3 aj = ld3(L.ax[j]), oj = ld3(L.org[j]);
            const bool rj = gld(m.rl_jtype + (j)) == AVR_J_REVOLUTE;
            v3 acc = V(0, 0, 0);
            for (unsigned dm = gld(m.desc_mask + (j)); dm; dm &= dm - 1u) {     // the subtree of j, ascending
                const int k = __builtin_ctz(dm);
                const v3 F = ld3(R1[k]);
                acc = add(acc, rj ? add(ld3(R5[k]), crs(sub(ld3(L.cm[k]), oj), F)) : F);
            }
            h = dot(aj, acc);
        }
        L.h[i] = h;
    }
    SYNC();
}

// --------------------------------------------------------------------------- shapes
struct WShape {
    int kind, nv, vs, tab;
    tf t;
    float margin;
    v3 he;
};

AVR_DI WShape make_wshape(const KModel &m, int s, tf body) {
    WShape w;
    w.kind = gld(m.shape_kind + (s));
    w.t = tfmul(body, gldtf(m.shape_pose + 8 * s));
    w.margin = gld(m.shape_margin + (s));
    const v3 pa = gld3(m.shape_param + 4 * s);
    if (w.kind == AVR_BOX) w.he = V(fmaxf(pa.x - w.margin, 0.f), fmaxf(pa.y - w.margin, 0.f), fmaxf(pa.z - w.margin, 0.f));
    else if (w.kind == AVR_CAPSULE) w.he = V(pa.x, pa.y, 0.f);
    else w.he = V(pa.x, 0.f, 0.f);
    w.vs = gld(m.shape_hull + (4 * s + 0));
    w.nv = w.kind == AVR_HULL ? gld(m.shape_hull + (4 * s + 1)) : 0;
    w.tab = w.kind == AVR_HULL ? gld(m.shape_tab + (s)) : -1;
    return w;
}

// support point of the CORE in world direction d; COOP: the whole wave scans a big hull
// read-only float4 array accessed through the global address space (global_load, not flat)
struct GlobalF4 {
    const float4 *p;
    AVR_DI float4 operator[](int i) const {
#if defined(__HIP_DEVICE_COMPILE__)
        return ((const __attribute__((address_space(1))) float4 *)p)[i];
#else
        return p[i];
#endif
    }
};

template <bool COOP, int NB = 8>
AVR_DI v3 support(const KModel &m, const WShape &s, v3 d) {
    v3 l = qrot(qconj(s.t.q), d);
    v3 r;
    if (s.kind == AVR_SPHERE) r = V(0, 0, 0);
    else if (s.kind == AVR_CAPSULE) r = V(0, 0, l.z >= 0.f ? s.he.y : -s.he.y);
    else if (s.kind == AVR_BOX) r = V(l.x >= 0.f ? s.he.x : -s.he.x, l.y >= 0.f ? s.he.y : -s.he.y, l.z >= 0.f ? s.he.z : -s.he.z);
    else if (s.tab >= 0) {
        // support table (avr_hulltab.cpp): the candidates of l's cube-map cell, ascending
        // vertex order, hold the first strictly largest projection of the whole hull
        const GlobalF4 tv{m.tab_vert};
        const float ax = fabsf(l.x), ay = fabsf(l.y), az = fabsf(l.z);
        const float mx = fmaxf(ax, fmaxf(ay, az));
        if (!(mx > 0.f)) {               // zero / NaN direction: the scan keeps vertex 0
            const float4 v = GlobalF4{m.hull_verts + s.vs}[0];
            r = V(v.x, v.y, v.z);
        } else {
            int f;
            float u, w;
            if (ax >= ay && ax >= az) { f = l.x < 0.f; u = l.y; w = l.z; }
            else if (ay >= az) { f = 2 + (l.y < 0.f); u = l.x; w = l.z; }
            else { f = 4 + (l.z < 0.f); u = l.x; w = l.y; }
            const float sc = 0.5f * (float)AVR_TAB_G / mx;
            const int i = min(AVR_TAB_G - 1, max(0, (int)((u + mx) * sc)));
            const int j = min(AVR_TAB_G - 1, max(0, (int)((w + mx) * sc)));
            const int2 oc = gld(m.tab_cell + (s.tab + (f * AVR_TAB_G + i) * AVR_TAB_G + j));
            // batches of 4 candidates in flight; a short last batch re-reads the last candidate,
            // which cannot displace an earlier winner under the strict ">" (exact)
            float best = -BIGF;
            float4 bv = tv[oc.x];
            const int last = oc.x + oc.y - 1;
            for (int k = 0; k < oc.y; k += 4) {
                float4 v[4];
#pragma unroll
                for (int q = 0; q < 4; q++) v[q] = tv[min(oc.x + k + q, last)];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float dd = l.x * v[q].x + l.y * v[q].y + l.z * v[q].z;
                    if (dd > best) { best = dd; bv = v[q]; }
                }
            }
            r = V(bv.x, bv.y, bv.z);
        }
    } else {
        // vertices through the global address space, several loads in flight per pass; the
        // first vertex with the strictly largest projection wins (index order), as before
        const GlobalF4 hv{m.hull_verts + s.vs};
        if (COOP) {
            float best = -BIGF;
            int bi = 0x7fffffff;
            int i = lane_id();
            for (; i + 192 < s.nv; i += 256) {
                const float4 v0 = hv[i], v1 = hv[i + 64], v2 = hv[i + 128], v3_ = hv[i + 192];
                float d0 = l.x * v0.x + l.y * v0.y + l.z * v0.z, d1 = l.x * v1.x + l.y * v1.y + l.z * v1.z;
                float d2 = l.x * v2.x + l.y * v2.y + l.z * v2.z, d3 = l.x * v3_.x + l.y * v3_.y + l.z * v3_.z;
                if (d0 > best) { best = d0; bi = i; }
                if (d1 > best) { best = d1; bi = i + 64; }
                if (d2 > best) { best = d2; bi = i + 128; }
                if (d3 > best) { best = d3; bi = i + 192; }
            }
            for (; i < s.nv; i += 64) {
                const float4 v = hv[i];
                const float dd = l.x * v.x + l.y * v.y + l.z * v.z;
                if (dd > best) { best = dd; bi = i; }
            }
            bi = wave_argmax(best, bi);
            const float4 v = hv[bi];
            r = V(v.x, v.y, v.z);
        } else {
            // batches of NB vertices in flight, ceil(nv / NB) round trips; a short last batch
            // re-reads vertex nv - 1, which cannot displace an earlier winner under the strict ">"
            float best = -BIGF;
            float4 bv = hv[0];
            const int last = s.nv - 1;
            for (int i = 0; i < s.nv; i += NB) {
                float4 v[NB];
#pragma unroll
                for (int k = 0; k < NB; k++) v[k] = hv[min(i + k, last)];
#pragma unroll
                for (int k = 0; k < NB; k++) {
                    const float dd = l.x * v[k].x + l.y * v[k].y + l.z * v[k].z;
                    if (dd > best) { best = dd; bv = v[k]; }
                }
            }
            r = V(bv.x, bv.y, bv.z);
        }
    }
    return tfpt(s.t, r);
}

// cube-map cell of a table hull for the local direction l (support(): mx > 0)
AVR_DI int2 tab_cell_of(const KModel &m, int tab, v3 l, float mx) {
    const float ax = fabsf(l.x), ay = fabsf(l.y), az = fabsf(l.z);
    int f;
    float u, w;
    if (ax >= ay && ax >= az) { f = l.x < 0.f; u = l.y; w = l.z; }
    else if (ay >= az) { f = 2 + (l.y < 0.f); u = l.x; w = l.z; }
    else { f = 4 + (l.z < 0.f); u = l.x; w = l.y; }
    const float sc = 0.5f * (float)AVR_TAB_G / mx;
    const int i = min(AVR_TAB_G - 1, max(0, (int)((u + mx) * sc)));
    const int j = min(AVR_TAB_G - 1, max(0, (int)((w + mx) * sc)));
    return gld(m.tab_cell + (tab + (f * AVR_TAB_G + i) * AVR_TAB_G + j));
}

// support(A, da) and support(B, db) together: when both are table hulls, the two cell lookups
// and then the two candidate scans are issued side by side (two dependent round trips instead of
// four).  Exactly support()'s results: the same candidates, the same strict ">" in ascending
// order, and a scan past a list's end re-reads its last candidate, which cannot displace a winner.
template <bool COOP>
AVR_DI void support2(const KModel &m, const WShape &A, v3 da, const WShape &B, v3 db, v3 &ra, v3 &rb) {
    const v3 la = qrot(qconj(A.t.q), da), lb = qrot(qconj(B.t.q), db);
    const float mxa = fmaxf(fabsf(la.x), fmaxf(fabsf(la.y), fabsf(la.z))), mxb = fmaxf(fabsf(lb.x), fmaxf(fabsf(lb.y), fabsf(lb.z)));
    if (!(A.tab >= 0 && B.tab >= 0 && mxa > 0.f && mxb > 0.f)) {
        ra = support<COOP>(m, A, da);
        rb = support<COOP>(m, B, db);
        return;
    }
    const GlobalF4 tv{m.tab_vert};
    const int2 ca = tab_cell_of(m, A.tab, la, mxa), cb = tab_cell_of(m, B.tab, lb, mxb);
    float besta = -BIGF, bestb = -BIGF;
    float4 bva = tv[ca.x], bvb = tv[cb.x];
    const int lasta = ca.x + ca.y - 1, lastb = cb.x + cb.y - 1, n = max(ca.y, cb.y);
    for (int k = 0; k < n; k += 4) {
        float4 va[4], vb[4];
#pragma unroll
        for (int q = 0; q < 4; q++) { va[q] = tv[min(ca.x + k + q, lasta)]; vb[q] = tv[min(cb.x + k + q, lastb)]; }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float d1 = la.x * va[q].x + la.y * va[q].y + la.z * va[q].z;
            if (d1 > besta) { besta = d1; bva = va[q]; }
            const float d2 = lb.x * vb[q].x + lb.y * vb[q].y + lb.z * vb[q].z;
            if (d2 > bestb) { bestb = d2; bvb = vb[q]; }
        }
    }
    ra = tfpt(A.t, V(bva.x, bva.y, bva.z));
    rb = tfpt(B.t, V(bvb.x, bvb.y, bvb.z));
}

// --------------------------------------------------------------------------- GJK
// GJK simplex: Minkowski vertices w = a - b with their support points on A and B
struct Simplex { v3 w[4], a[4], b[4]; int n; };
// GJK simplex of a point core (sphere) against a hull: only w and the hull's support points h
// are kept (the point's side is the constant core)
struct SimplexP { v3 w[4], h[4]; int n; };

AVR_DI void sx_copy(Simplex &S, int dst, int src) { S.w[dst] = S.w[src]; S.a[dst] = S.a[src]; S.b[dst] = S.b[src]; }
AVR_DI void sx_copy(SimplexP &S, int dst, int src) { S.w[dst] = S.w[src]; S.h[dst] = S.h[src]; }
// vertices (1, 2, 3) -> (3, 1, .): the tetrahedron face 1 moved to slots 0, 1, 2
AVR_DI void sx_face1(Simplex &S) { const v3 w1 = S.w[1], a1 = S.a[1], b1 = S.b[1]; sx_copy(S, 1, 3); S.w[2] = w1; S.a[2] = a1; S.b[2] = b1; }
AVR_DI void sx_face1(SimplexP &S) { const v3 w1 = S.w[1], h1 = S.h[1]; sx_copy(S, 1, 3); S.w[2] = w1; S.h[2] = h1; }

// Closest point of triangle ABC to the origin (Ericson 5.1.5).  used: bit mask of the vertices
// spanning the closest feature (1=A 2=B 4=C); l*: barycentric weights.
AVR_DI v3 tri_cp(v3 A, v3 B, v3 C, int &used, float &la, float &lb, float &lc) {
    v3 ab = sub(B, A), ac = sub(C, A), ap = scl(A, -1.f);
    float d1 = dot(ab, ap), d2 = dot(ac, ap);
    la = lb = lc = 0.f;
    if (d1 <= 0.f && d2 <= 0.f) { used = 1; la = 1.f; return A; }
    v3 bp = scl(B, -1.f);
    float d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.f && d4 <= d3) { used = 2; lb = 1.f; return B; }
    float vc = d1 * d4 - d3 * d2;
    if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
        float v = d1 / (d1 - d3);
        used = 3; la = 1.f - v; lb = v; return add(A, scl(ab, v));
    }
    v3 cp = scl(C, -1.f);
    float d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0.f && d5 <= d6) { used = 4; lc = 1.f; return C; }
    float vb = d5 * d2 - d1 * d6;
    if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
        float wv = d2 / (d2 - d6);
        used = 5; la = 1.f - wv; lc = wv; return add(A, scl(ac, wv));
    }
    float va = d3 * d6 - d5 * d4;
    if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
        float wv = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        used = 6; lb = 1.f - wv; lc = wv; return add(B, scl(sub(C, B), wv));
    }
    float den = 1.f / (va + vb + vc);
    float v = vb * den, wv = vc * den;
    used = 7; la = 1.f - v - wv; lb = v; lc = wv;
    return add(A, add(scl(ab, v), scl(ac, wv)));
}

// keep the vertices of slots 0..2 selected by `used`, compacted in order; lam in slot order
template <class SX>
AVR_DI void tri_compact(SX &S, int used, float la, float lb, float lc, float lam[4]) {
    switch (used) {
    case 1: S.n = 1; lam[0] = la; break;
    case 2: sx_copy(S, 0, 1); S.n = 1; lam[0] = lb; break;
    case 4: sx_copy(S, 0, 2); S.n = 1; lam[0] = lc; break;
    case 3: S.n = 2; lam[0] = la; lam[1] = lb; break;
    case 5: sx_copy(S, 1, 2); S.n = 2; lam[0] = la; lam[1] = lc; break;
    case 6: sx_copy(S, 0, 1); sx_copy(S, 1, 2); S.n = 2; lam[0] = lb; lam[1] = lc; break;
    default: S.n = 3; lam[0] = la; lam[1] = lb; lam[2] = lc; break;
    }
}

template <class SX>
AVR_DI int tri_closest(SX &S, v3 &vout, float lam[4]) {
    int used;
    float la, lb, lc;
    vout = tri_cp(S.w[0], S.w[1], S.w[2], used, la, lb, lc);
    tri_compact(S, used, la, lb, lc, lam);
    return 0;
}

// one face (i0,i1,i2) of the tetrahedron, opposite vertex i3 (literal indices at every call)
template <class SX>
AVR_DI void tetra_face(const SX &S, int f, int i0, int i1, int i2, int i3, bool &outside_any, float &best, int &bf, int &bused,
                       float &bla, float &blb, float &blc, v3 &bestv) {
    v3 A = S.w[i0], B = S.w[i1], C = S.w[i2], D = S.w[i3];
    v3 n = crs(sub(B, A), sub(C, A));
    float sp = dot(scl(A, -1.f), n), sd = dot(sub(D, A), n);
    if (sd * sd < 1e-30f) return;
    if (sp * sd < 0.f) {
        outside_any = true;
        int used;
        float la, lb, lc;
        v3 v = tri_cp(A, B, C, used, la, lb, lc);
        float d2 = len2(v);
        if (d2 < best) { best = d2; bf = f; bused = used; bla = la; blb = lb; blc = lc; bestv = v; }
    }
}

template <class SX>
AVR_DI int simplex_closest(SX &S, v3 &vout, float lam[4]) {
    if (S.n == 1) { lam[0] = 1.f; vout = S.w[0]; return 0; }
    if (S.n == 2) {
        v3 A = S.w[0], B = S.w[1], ab = sub(B, A);
        float t = -dot(A, ab), dd = dot(ab, ab);
        if (t <= 0.f || dd <= 0.f) { S.n = 1; lam[0] = 1.f; vout = A; return 0; }
        if (t >= dd) { sx_copy(S, 0, 1); S.n = 1; lam[0] = 1.f; vout = B; return 0; }
        t /= dd;
        lam[0] = 1.f - t; lam[1] = t;
        vout = add(A, scl(ab, t));
        return 0;
    }
    if (S.n == 3) return tri_closest(S, vout, lam);
    float best = BIGF;
    int bf = -1, bused = 0;
    float bla = 0.f, blb = 0.f, blc = 0.f;
    v3 bestv = V(0, 0, 0);
    bool outside_any = false;
    tetra_face(S, 0, 0, 1, 2, 3, outside_any, best, bf, bused, bla, blb, blc, bestv);
    tetra_face(S, 1, 0, 3, 1, 2, outside_any, best, bf, bused, bla, blb, blc, bestv);
    tetra_face(S, 2, 0, 2, 3, 1, outside_any, best, bf, bused, bla, blb, blc, bestv);
    tetra_face(S, 3, 1, 3, 2, 0, outside_any, best, bf, bused, bla, blb, blc, bestv);
    if (!outside_any || bf < 0) { lam[0] = lam[1] = lam[2] = lam[3] = 0.f; vout = V(0, 0, 0); return 1; }
    // move the winning face's vertices to slots 0,1,2 (in face order), then compact
    switch (bf) {
    case 0: break;
    case 1: sx_face1(S); break;
    case 2: sx_copy(S, 1, 2); sx_copy(S, 2, 3); break;
    default: sx_copy(S, 0, 1); sx_copy(S, 1, 3); break;
    }
    S.n = 3;
    tri_compact(S, bused, bla, blb, blc, lam);
    vout = bestv;
    return 0;
}

// The cooperative GJK for the pairs whose fp32 lane GJK stalled (rc 4: hulls, boxes and capsules
// against each other) solves for the simplex's closest point in double precision.
// Its Voronoi-region tests and barycentric weights on thin simplices -- a scratcher or wiper lying
// along a limb capsule, a box edge along a segment -- cancel catastrophically in fp32: the fp32
// GJK stops on "no progress" with a wrong witness for ~3 % of such poses (normals off by up to 50
// degrees, distances by a centimetre; tools/dbg_np_state.py, kernel and fp32 oracle alike at
// different poses), where the fp64 oracle -- PyBullet itself runs in double -- converges.  The
// simplex vertices (float supports, exactly representable in double) are unchanged; the Voronoi
// tests and the barycentric solve run in double, and the closest point and its weights are
// rounded to float (the rest of the iteration is the fp32 GJK's).
struct d3 { double x, y, z; };
AVR_DI d3 D3(v3 a) { return d3{(double)a.x, (double)a.y, (double)a.z}; }
AVR_DI d3 dadd(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
AVR_DI d3 dsub(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
AVR_DI d3 dscl(d3 a, double s) { return d3{a.x * s, a.y * s, a.z * s}; }
AVR_DI d3 dcrs(d3 a, d3 b) { return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
AVR_DI double ddot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
AVR_DI v3 dtof(d3 a) { return V((float)a.x, (float)a.y, (float)a.z); }

AVR_DI d3 tri_cp_d(d3 A, d3 B, d3 C, int &used, double &la, double &lb, double &lc) {
    d3 ab = dsub(B, A), ac = dsub(C, A), ap = dscl(A, -1.0);
    double d1 = ddot(ab, ap), d2 = ddot(ac, ap);
    la = lb = lc = 0.0;
    if (d1 <= 0.0 && d2 <= 0.0) { used = 1; la = 1.0; return A; }
    d3 bp = dscl(B, -1.0);
    double d3_ = ddot(ab, bp), d4 = ddot(ac, bp);
    if (d3_ >= 0.0 && d4 <= d3_) { used = 2; lb = 1.0; return B; }
    double vc = d1 * d4 - d3_ * d2;
    if (vc <= 0.0 && d1 >= 0.0 && d3_ <= 0.0) {
        double v = d1 / (d1 - d3_);
        used = 3; la = 1.0 - v; lb = v; return dadd(A, dscl(ab, v));
    }
    d3 cp = dscl(C, -1.0);
    double d5 = ddot(ab, cp), d6 = ddot(ac, cp);
    if (d6 >= 0.0 && d5 <= d6) { used = 4; lc = 1.0; return C; }
    double vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
        double wv = d2 / (d2 - d6);
        used = 5; la = 1.0 - wv; lc = wv; return dadd(A, dscl(ac, wv));
    }
    double va = d3_ * d6 - d5 * d4;
    if (va <= 0.0 && (d4 - d3_) >= 0.0 && (d5 - d6) >= 0.0) {
        double wv = (d4 - d3_) / ((d4 - d3_) + (d5 - d6));
        used = 6; lb = 1.0 - wv; lc = wv; return dadd(B, dscl(dsub(C, B), wv));
    }
    double den = 1.0 / (va + vb + vc);
    double v = vb * den, wv = vc * den;
    used = 7; la = 1.0 - v - wv; lb = v; lc = wv;
    return dadd(A, dadd(dscl(ab, v), dscl(ac, wv)));
}

AVR_DI void tri_compact_d(Simplex &S, int used, double la, double lb, double lc, float lam[4]) {
    switch (used) {
    case 1: S.n = 1; lam[0] = (float)la; break;
    case 2: sx_copy(S, 0, 1); S.n = 1; lam[0] = (float)lb; break;
    case 4: sx_copy(S, 0, 2); S.n = 1; lam[0] = (float)lc; break;
    case 3: S.n = 2; lam[0] = (float)la; lam[1] = (float)lb; break;
    case 5: sx_copy(S, 1, 2); S.n = 2; lam[0] = (float)la; lam[1] = (float)lc; break;
    case 6: sx_copy(S, 0, 1); sx_copy(S, 1, 2); S.n = 2; lam[0] = (float)lb; lam[1] = (float)lc; break;
    default: S.n = 3; lam[0] = (float)la; lam[1] = (float)lb; lam[2] = (float)lc; break;
    }
}

// the closest point of the simplex to the origin and its weights, computed in double and rounded
// to float (the fp32 GJK's state; only the Voronoi tests and the barycentric solve need the
// digits).  Wave-cooperative (every lane holds the same simplex): a tetrahedron's faces are tested
// one per lane (lane f & 3: face f) and share one triangle solve with the 3-simplex case.
AVR_DI int simplex_closest_d(Simplex &S, v3 &vout, float lam[4]) {
    if (S.n == 1) { lam[0] = 1.f; vout = S.w[0]; return 0; }
    if (S.n == 2) {
        d3 A = D3(S.w[0]), B = D3(S.w[1]), ab = dsub(B, A);
        double t = -ddot(A, ab), dd = ddot(ab, ab);
        if (t <= 0.0 || dd <= 0.0) { S.n = 1; lam[0] = 1.f; vout = S.w[0]; return 0; }
        if (t >= dd) { sx_copy(S, 0, 1); S.n = 1; lam[0] = 1.f; vout = S.w[0]; return 0; }
        t /= dd;
        lam[0] = (float)(1.0 - t); lam[1] = (float)t;
        vout = dtof(dadd(A, dscl(ab, t)));
        return 0;
    }
    const bool tet = S.n == 4;
    // faces (0 1 2 | 3), (0 3 1 | 2), (0 2 3 | 1), (1 3 2 | 0); a triangle is face 0.  Vertices by
    // selects between registers, not a lane-dependent index (that would put the simplex in scratch)
    const int f = tet ? (lane_id() & 3) : 0;
    const d3 W0 = D3(S.w[0]), W1 = D3(S.w[1]), W2 = D3(S.w[2]), W3 = D3(S.w[3]);
    const bool f0 = f == 0, f1 = f == 1, f2 = f == 2;
    const d3 A = f0 || f1 || f2 ? W0 : W1;
    const d3 B = f0 ? W1 : f2 ? W2 : W3;
    const d3 C = f0 ? W2 : f1 ? W1 : f2 ? W3 : W2;
    bool outside = true;
    if (tet) {
        const d3 D = f0 ? W3 : f1 ? W2 : f2 ? W1 : W0;
        const d3 n = dcrs(dsub(B, A), dsub(C, A));
        const double sp = ddot(dscl(A, -1.0), n), sd = ddot(dsub(D, A), n);
        outside = !(sd * sd < 1e-30) && sp * sd < 0.0;
    }
    int used;
    double la, lb, lc;
    const d3 cv = tri_cp_d(A, B, C, used, la, lb, lc);
    if (!tet) {
        vout = dtof(cv);
        tri_compact_d(S, used, la, lb, lc, lam);
        return 0;
    }
    if (!(__ballot(outside) & 0xfull)) { lam[0] = lam[1] = lam[2] = lam[3] = 0.f; vout = V(0, 0, 0); return 1; }
    // the face with the smallest distance wins, the lowest index on ties (the serial loop's d2 <
    // best over faces 0..3; a strict minimum in double that rounds to a float tie keeps the lower
    // face, as a tie does)
    const float d2 = outside ? (float)ddot(cv, cv) : BIGF;
    float m = fminf(d2, __shfl_xor(d2, 1));
    m = fminf(m, __shfl_xor(m, 2));
    // no outside face attains m when every outside face's distance is NaN / inf: answer as the
    // fp32 solve does for a simplex with no usable face (penetrating), not with ctz of an empty mask
    const unsigned long long bmask = __ballot(outside && d2 == m) & 0xfull;
    if (!bmask) { lam[0] = lam[1] = lam[2] = lam[3] = 0.f; vout = V(0, 0, 0); return 1; }
    const int bf = __builtin_ctzll(bmask);
    const int bused = __shfl(used, bf);
    const double bla = __shfl(la, bf), blb = __shfl(lb, bf), blc = __shfl(lc, bf);
    vout = V(__shfl((float)cv.x, bf), __shfl((float)cv.y, bf), __shfl((float)cv.z, bf));
    switch (bf) {
    case 0: break;
    case 1: sx_face1(S); break;
    case 2: sx_copy(S, 1, 2); sx_copy(S, 2, 3); break;
    default: sx_copy(S, 0, 1); sx_copy(S, 1, 3); break;
    }
    S.n = 3;
    tri_compact_d(S, bused, bla, blb, blc, lam);
    return 0;
}

#define GJK_NP_GAP 1e-4f     // lane GJK: largest duality gap (m) a no-progress stop may leave (gjk_lane)
#define GJK_SEPARATED 0
#define GJK_FAR 1
#define GJK_PENETRATING 2
#define GJK_UNFINISHED 3        // lane path only: iteration cap hit, finish on the cooperative path
#define GJK_STALLED 4           // lane path only: no progress with an open duality gap, rerun in double (gjk_coop_d)
// The lane-per-pair path runs at the pace of its slowest lane: pairs that have not converged
// after GJK_LANE_IT iterations are handed to the wave-cooperative path, which reruns the same
// GJK (same support tie-break, same arithmetic) to completion -- identical results.
#ifndef GJK_LANE_IT
#define GJK_LANE_IT GJK_MAX_IT     // measured: a cap of 4..16 does not pay on this scene
#endif

// hull vertices in flight per support scan of the lane GJK (hull-hull pairs: two scans per
// iteration; 4 keeps the narrowphase kernel within 128 VGPRs)
#ifndef GJK_NB
#define GJK_NB 4
#endif
AVR_DI int gjk_coop_d(const KModel &m, const WShape &A, const WShape &B, float maxdist2, v3 &pa, v3 &pb, float &dist, Simplex &S, int &nit) {
    v3 v = sub(A.t.p, B.t.p);
    if (len2(v) < 1e-20f) v = V(1, 0, 0);
    S.n = 0;
    float lam[4] = {1, 0, 0, 0};
    float prev = BIGF;
    int status = GJK_SEPARATED;
    for (int it = 0; it < GJK_MAX_IT; it++) {
        nit = it + 1;
        v3 sa, sb;
        support2<true>(m, A, scl(v, -1.f), B, v, sa, sb);
        v3 wv = sub(sa, sb);
        float vv = len2(v), vw = dot(v, wv);
        if (vw > 0.f && vw * vw > vv * maxdist2) return GJK_FAR;
        bool dup = false;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < S.n && S.w[k].x == wv.x && S.w[k].y == wv.y && S.w[k].z == wv.z) dup = true;
        if (dup && S.n > 0) break;
        if (S.n > 0 && vv - vw <= GJK_REL_EPS * vv) break;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k == S.n) { S.w[k] = wv; S.a[k] = sa; S.b[k] = sb; }
        S.n++;
        v3 nv;
        if (simplex_closest_d(S, nv, lam)) { status = GJK_PENETRATING; break; }
        float nvv = len2(nv);
        if (nvv < 1e-14f * (1.f + len2(wv))) { status = GJK_PENETRATING; break; }
        if (nvv >= prev) { v = nv; break; }
        prev = nvv;
        v = nv;
    }
    if (status == GJK_PENETRATING) return GJK_PENETRATING;
    v3 a = V(0, 0, 0), b = V(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < S.n) { a = add(a, scl(S.a[k], lam[k])); b = add(b, scl(S.b[k], lam[k])); }
    pa = a; pb = b;
    dist = len(sub(a, b));
    return GJK_SEPARATED;
}

// the cooperative GJK in fp32 (pairs the lane path hands over for EPA or a big hull): the lane
// path's arithmetic with both supports of an iteration issued together
AVR_DI int gjk_coop_f(const KModel &m, const WShape &A, const WShape &B, float maxdist2, v3 &pa, v3 &pb, float &dist, Simplex &S, int &nit) {
    v3 v = sub(A.t.p, B.t.p);
    if (len2(v) < 1e-20f) v = V(1, 0, 0);
    S.n = 0;
    float lam[4] = {1, 0, 0, 0};
    float prev = BIGF;
    int status = GJK_SEPARATED;
    for (int it = 0; it < GJK_MAX_IT; it++) {
        nit = it + 1;
        v3 sa, sb;
        support2<true>(m, A, scl(v, -1.f), B, v, sa, sb);
        v3 wv = sub(sa, sb);
        float vv = len2(v), vw = dot(v, wv);
        if (vw > 0.f && vw * vw > vv * maxdist2) return GJK_FAR;
        bool dup = false;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < S.n && S.w[k].x == wv.x && S.w[k].y == wv.y && S.w[k].z == wv.z) dup = true;
        if (dup && S.n > 0) break;
        if (S.n > 0 && vv - vw <= GJK_REL_EPS * vv) break;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k == S.n) { S.w[k] = wv; S.a[k] = sa; S.b[k] = sb; }
        S.n++;
        v3 nv;
        if (simplex_closest(S, nv, lam)) { status = GJK_PENETRATING; break; }
        float nvv = len2(nv);
        if (nvv < 1e-14f * (1.f + len2(wv))) { status = GJK_PENETRATING; break; }
        if (nvv >= prev) { v = nv; break; }
        prev = nvv;
        v = nv;
    }
    if (status == GJK_PENETRATING) return GJK_PENETRATING;
    v3 a = V(0, 0, 0), b = V(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < S.n) { a = add(a, scl(S.a[k], lam[k])); b = add(b, scl(S.b[k], lam[k])); }
    pa = a; pb = b;
    dist = len(sub(a, b));
    return GJK_SEPARATED;
}

// Lane path (one pair per lane, fp32).  A step that makes no progress ends it as in the oracle
// only when the duality gap at the final direction is closed: the distance's upper and lower
// bounds (|v| and v.w / |v|, one more support query) within GJK_NP_GAP.  Otherwise -- the fp32
// symptom of a thin simplex whose closest point has lost its digits, see gjk_coop_d -- the pair is
// handed to the cooperative GJK in double (rc 4).  Measured with the fp32 oracle: on the ScratchItch
// state-27 neighbourhood (4000 jittered poses, tools/dbg_np_state.py) the 132 wrong answers all
// stop on no progress with gaps of 1.3 - 37 mm, 90 % of the correct no-progress stops below 0.6 um;
// in FeedingJaco runs 4.5 % of the no-progress stops (~0.1 % of GJK calls) exceed 0.1 mm.
AVR_DI int gjk_lane(const KModel &m, const WShape &A, const WShape &B, float maxdist2, v3 &pa, v3 &pb, float &dist, Simplex &S, int &nit) {
    v3 v = sub(A.t.p, B.t.p);
    if (len2(v) < 1e-20f) v = V(1, 0, 0);
    S.n = 0;
    float lam[4] = {1, 0, 0, 0};
    float prev = BIGF;
    int status = GJK_SEPARATED;
    bool converged = false, npc = false;
    for (int it = 0; it < GJK_LANE_IT; it++) {
        nit = it + 1;
        v3 sa = support<false, GJK_NB>(m, A, scl(v, -1.f)), sb = support<false, GJK_NB>(m, B, v);
        v3 wv = sub(sa, sb);
        float vv = len2(v), vw = dot(v, wv);
        if (npc) {      // the step before made no progress: keep its simplex if the gap is closed
            const float gap = vv - vw;     // (|v| times the gap between the distance's bounds)
            if (gap > 0.f && gap * gap > (GJK_NP_GAP * GJK_NP_GAP) * vv) return GJK_STALLED;
            converged = true;
            break;
        }
        if (vw > 0.f && vw * vw > vv * maxdist2) return GJK_FAR;
        bool dup = false;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < S.n && S.w[k].x == wv.x && S.w[k].y == wv.y && S.w[k].z == wv.z) dup = true;
        if (dup && S.n > 0) { converged = true; break; }
        if (S.n > 0 && vv - vw <= GJK_REL_EPS * vv) { converged = true; break; }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k == S.n) { S.w[k] = wv; S.a[k] = sa; S.b[k] = sb; }
        S.n++;
        v3 nv;
        if (simplex_closest(S, nv, lam)) { status = GJK_PENETRATING; converged = true; break; }
        float nvv = len2(nv);
        if (nvv < 1e-14f * (1.f + len2(wv))) { status = GJK_PENETRATING; converged = true; break; }
        if (nvv >= prev) { v = nv; npc = true; continue; }     // (the gap check takes the next support)
        prev = nvv;
        v = nv;
    }
    if (!converged) return GJK_UNFINISHED;
    if (status == GJK_PENETRATING) return GJK_PENETRATING;
    v3 a = V(0, 0, 0), b = V(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < S.n) { a = add(a, scl(S.a[k], lam[k])); b = add(b, scl(S.b[k], lam[k])); }
    pa = a; pb = b;
    dist = len(sub(a, b));
    return GJK_SEPARATED;
}

template <bool COOP>
AVR_DI int gjk(const KModel &m, const WShape &A, const WShape &B, float maxdist2, v3 &pa, v3 &pb, float &dist, Simplex &S, int &nit, bool dbl) {
    if constexpr (COOP) return dbl ? gjk_coop_d(m, A, B, maxdist2, pa, pb, dist, S, nit) : gjk_coop_f(m, A, B, maxdist2, pa, pb, dist, S, nit);
    else return gjk_lane(m, A, B, maxdist2, pa, pb, dist, S, nit);
}

// --------------------------------------------------------------------------- EPA (wave-cooperative)
// The polytope lives in a per-env global scratch buffer (EPA runs only when shape cores
// overlap, which is rare; keeping it out of LDS buys occupancy for everything else).
struct EpaBuf {
    float eW[EPA_MAX_V][9];        // minkowski vertex + support on A + support on B
    int eFi[EPA_MAX_F][4];         // i j k alive
    float eFn[EPA_MAX_F][4];       // normal + d
    int eEdge[EPA_MAX_F * 3][2];
};
AVR_DI int epa_add_face(EpaBuf &L, int &nf, int i, int j, int k) {
    if (nf >= EPA_MAX_F) return -1;
    v3 Wi = ld3(L.eW[i]), Wj = ld3(L.eW[j]), Wk = ld3(L.eW[k]);
    v3 n = crs(sub(Wj, Wi), sub(Wk, Wi));
    float l = len(n);
    if (l < 1e-18f) return -2;
    n = scl(n, 1.f / l);
    SYNC();
    if (lane_id() == 0) {
        L.eFi[nf][0] = i; L.eFi[nf][1] = j; L.eFi[nf][2] = k; L.eFi[nf][3] = 1;
        st3(L.eFn[nf], n);
        L.eFn[nf][3] = dot(n, Wi);
    }
    SYNC();
    nf++;
    return 0;
}

AVR_DI void epa_set_vert(EpaBuf &L, int vi, v3 w, v3 a, v3 b) {
    SYNC();
    if (lane_id() == 0) { st3(L.eW[vi], w); st3(L.eW[vi] + 3, a); st3(L.eW[vi] + 6, b); }
    SYNC();
}

AVR_DI int epa(const KModel &m, EpaBuf &L, const WShape &A, const WShape &B, const Simplex &S, v3 &normal_out, float &depth, v3 &pa, v3 &pb) {
    int nv = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < S.n) { epa_set_vert(L, nv, S.w[k], S.a[k], S.b[k]); nv++; }
    for (int di = 0; di < 6 && nv < 4; di++) {
        float sg = (di & 1) ? -1.f : 1.f;
        v3 d = V(di < 2 ? sg : 0.f, (di >> 1) == 1 ? sg : 0.f, di >= 4 ? sg : 0.f);
        if (nv == 2) {
            v3 e = sub(ld3(L.eW[1]), ld3(L.eW[0]));
            v3 c = crs(e, d);
            if (len2(c) < 1e-12f) continue;
            d = c;
        } else if (nv == 3) {
            v3 W0 = ld3(L.eW[0]);
            d = crs(sub(ld3(L.eW[1]), W0), sub(ld3(L.eW[2]), W0));
            if (di & 1) d = scl(d, -1.f);
            if (len2(d) < 1e-24f) continue;
        }
        v3 sa, sb;
        support2<true>(m, A, d, B, scl(d, -1.f), sa, sb);
        v3 wv = sub(sa, sb);
        bool dup = false;
        for (int k = 0; k < nv; k++)
            if (len2(sub(ld3(L.eW[k]), wv)) < 1e-20f) dup = true;
        if (dup) continue;
        epa_set_vert(L, nv++, wv, sa, sb);
    }
    if (nv < 4) return -1;
    {
        v3 W0 = ld3(L.eW[0]), W1 = ld3(L.eW[1]), W2 = ld3(L.eW[2]), W3 = ld3(L.eW[3]);
        if (dot(crs(sub(W1, W0), sub(W2, W0)), sub(W3, W0)) > 0.f) {
            float t1[9], t2[9];
            for (int k = 0; k < 9; k++) { t1[k] = L.eW[1][k]; t2[k] = L.eW[2][k]; }
            SYNC();
            if (lane_id() == 0)
                for (int k = 0; k < 9; k++) { L.eW[1][k] = t2[k]; L.eW[2][k] = t1[k]; }
            SYNC();
        }
    }
    int nf = 0;
    if (epa_add_face(L, nf, 0, 1, 2) || epa_add_face(L, nf, 0, 3, 1) || epa_add_face(L, nf, 0, 2, 3) || epa_add_face(L, nf, 1, 3, 2)) return -1;
    int best = -1;
    const int lane = lane_id();
    for (int it = 0; it < EPA_MAX_IT; it++) {
        // closest alive face: the first strictly smallest d (wave argmin, lowest index on ties)
        float bd = BIGF;
        int bf = 0x7fffffff;
        for (int f = lane; f < nf; f += 64)
            if (L.eFi[f][3] && L.eFn[f][3] < bd) { bd = L.eFn[f][3]; bf = f; }
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o, 64);
            const int of = __shfl_xor(bf, o, 64);
            if (od < bd || (od == bd && of < bf)) { bd = od; bf = of; }
        }
        best = bf == 0x7fffffff ? -1 : bf;
        if (best < 0) return -1;
        v3 n = ld3(L.eFn[best]);
        v3 sa, sb;
        support2<true>(m, A, n, B, scl(n, -1.f), sa, sb);
        v3 wv = sub(sa, sb);
        float dist = dot(wv, n);
        if (dist - L.eFn[best][3] < EPA_EPS || nv >= EPA_MAX_V) break;
        int vi = nv++;
        epa_set_vert(L, vi, wv, sa, sb);
        // visible faces die and leave the horizon edge list.  A face's visibility depends on that
        // face alone, so every lane tests one face; lane 0 then walks the visible faces in face
        // order and edits the edge list serially (the order of the list, with its swap-with-last
        // removals, is that of the CPU restatement)
        int ne = 0;
        for (int base = 0; base < nf; base += 64) {
            const int fl = base + lane;
            bool vis = false;
            if (fl < nf && L.eFi[fl][3]) vis = dot(ld3(L.eFn[fl]), sub(wv, ld3(L.eW[L.eFi[fl][0]]))) > 0.f;
            unsigned long long vm = __ballot(vis);
            if (lane != 0) continue;
            while (vm) {
                const int f = base + __ffsll((long long)vm) - 1;
                vm &= vm - 1;
                {
                    const int fi = L.eFi[f][0], fj = L.eFi[f][1], fk = L.eFi[f][2];
                    L.eFi[f][3] = 0;
                    const int e3[3][2] = {{fi, fj}, {fj, fk}, {fk, fi}};
                    for (int e = 0; e < 3; e++) {
                        int found = -1;
                        for (int q = 0; q < ne; q++)
                            if (L.eEdge[q][0] == e3[e][1] && L.eEdge[q][1] == e3[e][0]) { found = q; break; }
                        if (found >= 0) { L.eEdge[found][0] = L.eEdge[ne - 1][0]; L.eEdge[found][1] = L.eEdge[ne - 1][1]; ne--; }
                        else { L.eEdge[ne][0] = e3[e][0]; L.eEdge[ne][1] = e3[e][1]; ne++; }
                    }
                }
            }
        }
        ne = __shfl(ne, 0, 64);
        SYNC();
        // compact the dead faces away, in order (lane-parallel: reads of a chunk precede its writes,
        // which land at or below the chunk)
        int k = 0;
        for (int base = 0; base < nf; base += 64) {
            const int f = base + lane;
            const bool alive = f < nf && L.eFi[f][3];
            int fi0 = 0, fi1 = 0, fi2 = 0;
            float fn0 = 0.f, fn1 = 0.f, fn2 = 0.f, fn3 = 0.f;
            if (alive) { fi0 = L.eFi[f][0]; fi1 = L.eFi[f][1]; fi2 = L.eFi[f][2]; fn0 = L.eFn[f][0]; fn1 = L.eFn[f][1]; fn2 = L.eFn[f][2]; fn3 = L.eFn[f][3]; }
            int tot;
            const int pre = ballot_prefix(alive, &tot);
            SYNC();
            if (alive) {
                L.eFi[k + pre][0] = fi0; L.eFi[k + pre][1] = fi1; L.eFi[k + pre][2] = fi2; L.eFi[k + pre][3] = 1;
                L.eFn[k + pre][0] = fn0; L.eFn[k + pre][1] = fn1; L.eFn[k + pre][2] = fn2; L.eFn[k + pre][3] = fn3;
            }
            k += tot;
            SYNC();
        }
        nf = k;
        // the new faces (horizon edge, new vertex), in edge order; a degenerate one is skipped, a
        // full face array ends EPA (epa_add_face semantics, lane-parallel)
        const v3 Wv = ld3(L.eW[vi]);
        for (int e0 = 0; e0 < ne; e0 += 64) {
            const int e = e0 + lane;
            int ei = 0, ej = 0;
            v3 fn = V(0, 0, 0);
            bool ok = false;
            if (e < ne) {
                ei = L.eEdge[e][0]; ej = L.eEdge[e][1];
                const v3 Wi = ld3(L.eW[ei]), Wj = ld3(L.eW[ej]);
                fn = crs(sub(Wj, Wi), sub(Wv, Wi));
                const float l = len(fn);
                ok = !(l < 1e-18f);
                if (ok) fn = scl(fn, 1.f / l);
            }
            int tot;
            const int pre = ballot_prefix(ok, &tot);
            const int last = min(ne - e0, 64) - 1;          // the chunk's last edge: the fullest array it meets
            const int before_last = __shfl(pre, last, 64);
            if (nf + before_last >= EPA_MAX_F) return -1;
            SYNC();
            if (ok) {
                const int f = nf + pre;
                L.eFi[f][0] = ei; L.eFi[f][1] = ej; L.eFi[f][2] = vi; L.eFi[f][3] = 1;
                st3(L.eFn[f], fn);
                L.eFn[f][3] = dot(fn, ld3(L.eW[ei]));
            }
            nf += tot;
            SYNC();
        }
    }
    if (best < 0) return -1;
    v3 n = ld3(L.eFn[best]);
    float fd = L.eFn[best][3];
    v3 p = scl(n, fd);
    int fi = L.eFi[best][0], fj = L.eFi[best][1], fk = L.eFi[best][2];
    v3 a = ld3(L.eW[fi]), b = ld3(L.eW[fj]), c = ld3(L.eW[fk]);
    v3 v0 = sub(b, a), v1 = sub(c, a), v2 = sub(p, a);
    float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
    float den = d00 * d11 - d01 * d01;
    float lv = 0.f, lw = 0.f;
    if (fabsf(den) > 1e-30f) { lv = (d11 * d20 - d01 * d21) / den; lw = (d00 * d21 - d01 * d20) / den; }
    float lu = 1.f - lv - lw;
    pa = add(add(scl(ld3(L.eW[fi] + 3), lu), scl(ld3(L.eW[fj] + 3), lv)), scl(ld3(L.eW[fk] + 3), lw));
    pb = add(add(scl(ld3(L.eW[fi] + 6), lu), scl(ld3(L.eW[fj] + 6), lv)), scl(ld3(L.eW[fk] + 6), lw));
    normal_out = n;
    depth = fd;
    return 0;
}

// --------------------------------------------------------------------------- narrowphase
// returns: 0 no contact, 1 contact (nB, pB, dist), 2 needs the cooperative path
// (nit, kind: diagnostic out-parameters -- GJK iterations, and 0 sphere-sphere, 1 sphere-box,
// 2 sphere-capsule, 3 GJK; unused outside the AVR_PROF build)
template <bool COOP>
AVR_DI int narrowphase(const KModel &m, EpaBuf &E, const WShape &A, const WShape &B, float thr, v3 &nB, v3 &pB, float &dist, int &nit, int &kind,
                       int *epa_budget = nullptr, bool dbl = false) {
    int ka = A.kind, kb = B.kind;
    nit = 0;
    kind = 3;
    if (ka == AVR_SPHERE && kb == AVR_SPHERE) {
        kind = 0;
        v3 diff = sub(A.t.p, B.t.p);
        float l = len(diff), ra = A.he.x, rb = B.he.x;
        if (l > ra + rb) return 0;
        float d = l - (ra + rb);
        v3 n = V(1, 0, 0);
        if (l > 1.1920928955078125e-07f) n = scl(diff, 1.f / l);
        nB = n; pB = add(B.t.p, scl(n, rb)); dist = d;
        return d <= thr ? 1 : 0;
    }
    if ((ka == AVR_SPHERE && kb == AVR_BOX) || (ka == AVR_BOX && kb == AVR_SPHERE)) {
        bool swapped = ka == AVR_BOX;
        kind = 1;
        const WShape Sp = swapped ? B : A;
        const WShape X = swapped ? A : B;
        v3 rel = tfinvpt(X.t, Sp.t.p);
        v3 he = X.he;
        v3 cp = V(fminf(he.x, fmaxf(-he.x, rel.x)), fminf(he.y, fmaxf(-he.y, rel.y)), fminf(he.z, fmaxf(-he.z, rel.z)));
        float r = Sp.he.x, inter = r + X.margin, cdist = inter + thr;
        v3 n = sub(rel, cp);
        float d2 = len2(n), d;
        if (d2 > cdist * cdist) return 0;
        if (d2 <= 1.1920928955078125e-07f) {
            float fd = he.x - rel.x, md = fd;
            cp = rel; cp.x = he.x; n = V(1, 0, 0);
            fd = he.x + rel.x; if (fd < md) { md = fd; cp = rel; cp.x = -he.x; n = V(-1, 0, 0); }
            fd = he.y - rel.y; if (fd < md) { md = fd; cp = rel; cp.y = he.y; n = V(0, 1, 0); }
            fd = he.y + rel.y; if (fd < md) { md = fd; cp = rel; cp.y = -he.y; n = V(0, -1, 0); }
            fd = he.z - rel.z; if (fd < md) { md = fd; cp = rel; cp.z = he.z; n = V(0, 0, 1); }
            fd = he.z + rel.z; if (fd < md) { md = fd; cp = rel; cp.z = -he.z; n = V(0, 0, -1); }
            d = -md;
        } else {
            d = sqrtf(d2);
            n = scl(n, 1.f / d);
        }
        v3 pbox = tfpt(X.t, add(cp, scl(n, X.margin)));
        v3 nw = qrot(X.t.q, n);
        float pen = d - inter;
        if (pen > thr) return 0;
        if (!swapped) { nB = nw; pB = pbox; dist = pen; }
        else { nB = scl(nw, -1.f); pB = add(pbox, scl(nw, pen)); dist = pen; }
        return 1;
    }
    if ((ka == AVR_SPHERE || ka == AVR_CAPSULE) && (kb == AVR_SPHERE || kb == AVR_CAPSULE) && !(ka == AVR_CAPSULE && kb == AVR_CAPSULE)) {
        bool swapped = ka == AVR_CAPSULE;
        kind = 2;
        const WShape Sp = swapped ? B : A;
        const WShape Cp = swapped ? A : B;
        v3 az = qrot(Cp.t.q, V(0, 0, 1));
        v3 p0 = sub(Cp.t.p, scl(az, Cp.he.y)), p1 = add(Cp.t.p, scl(az, Cp.he.y));
        v3 e = sub(p1, p0);
        float t = dot(sub(Sp.t.p, p0), e) / fmaxf(dot(e, e), 1e-30f);
        t = fminf(1.f, fmaxf(0.f, t));
        v3 q = add(p0, scl(e, t));
        v3 diff = sub(Sp.t.p, q);
        float l = len(diff);
        v3 n = l > 1e-12f ? scl(diff, 1.f / l) : V(1, 0, 0);
        float d = l - Sp.he.x - Cp.he.x;
        if (d > thr) return 0;
        if (!swapped) { nB = n; pB = add(q, scl(n, Cp.he.x)); dist = d; }
        else { nB = scl(n, -1.f); pB = sub(Sp.t.p, scl(n, Sp.he.x)); dist = d; }
        return 1;
    }
    float ma = A.margin, mb = B.margin;
    float maxd = ma + mb + thr;
    v3 pa, pb;
    float cd;
    Simplex S;
    int st = gjk<COOP>(m, A, B, maxd * maxd, pa, pb, cd, S, nit, dbl);
    if (st == GJK_FAR) return 0;
    if (st == GJK_UNFINISHED) return 2;
    if (st == GJK_STALLED) return 4;
    v3 n;
    float d;
    if (st == GJK_SEPARATED && cd > 1e-9f) {
        n = scl(sub(pa, pb), 1.f / cd);
        d = cd - ma - mb;
    } else {
        if (!COOP) return 2;
        if (epa_budget) {           // (np_coop's per-sub-step EPA cap: 3 = penetrating, not solved)
            if (*epa_budget <= 0) return 3;
            --*epa_budget;
        }
        float depth;
        v3 en;
        if (epa(m, E, A, B, S, en, depth, pa, pb)) return 0;
        n = scl(en, -1.f);
        d = -depth - ma - mb;
    }
    if (d > thr) return 0;
    nB = n;
    pB = add(pb, scl(n, mb));
    dist = d;
    return 1;
}

// --------------------------------------------------------------------------- bodies
template <class LT>
AVR_DI tf body_tf(const KModel &m, const LT &L, int b) {
    int kind = gld(m.body_kind + (b)), idx = gld(m.body_index + (b));
    if (kind == AVR_BODY_ROBOT) return ldtf(L.cm[idx]);
    if (kind == AVR_BODY_FREE) return ldtf(L.st + S_FREE + AVR_FB_WORDS * idx);
    if (kind == AVR_BODY_STATIC) return gldtf(m.st_pose + 8 * idx);
#if K_RBASE_IN_STATE
    if (kind == AVR_BODY_RSTATIC) return ldtf(L.st + S_RBASE);
#endif
    return ldtf(L.st + S_HUMAN + 7 * idx);
}

AVR_DI void aabb_of(tf t, v3 c, v3 h, v3 &mn, v3 &mx) {
    m3 R = qmat(t.q);
    v3 cw = tfpt(t, c);
    v3 hw = V(fabsf(R.m[0][0]) * h.x + fabsf(R.m[0][1]) * h.y + fabsf(R.m[0][2]) * h.z,
              fabsf(R.m[1][0]) * h.x + fabsf(R.m[1][1]) * h.y + fabsf(R.m[1][2]) * h.z,
              fabsf(R.m[2][0]) * h.x + fabsf(R.m[2][1]) * h.y + fabsf(R.m[2][2]) * h.z);
    mn = sub(cw, hw);
    mx = add(cw, hw);
}

AVR_DI bool overlap(v3 a0, v3 a1, v3 b0, v3 b1) {
    return a0.x <= b1.x && a1.x >= b0.x && a0.y <= b1.y && a1.y >= b0.y && a0.z <= b1.z && a1.z >= b0.z;
}

AVR_DI void shape_aabb(const KModel &m, int s, tf body, v3 &mn, v3 &mx) {
    tf t = tfmul(body, gldtf(m.shape_pose + 8 * s));
    const float *a = m.shape_aabb + 8 * s;
    aabb_of(t, gld3(a), gld3(a + 4), mn, mx);
}

AVR_DI bool shape_enabled(const KModel &m, int s, int gender) {
    int g = m.shape_gender[s];
    return g < 0 || g == gender;
}

// --------------------------------------------------------------------------- manifolds (one lane per shape pair)
// A manifold is <= 4 points of the OLD contact pool (each point belongs to exactly one shape
// pair, so lanes update disjoint LDS words in place) plus at most one NEW point held in
// registers.  Slot order is kept as 8-bit indices packed in one register (255 = the new point).
#define MF_NEW 255
struct MfNew { float p[AVR_CP_WORDS]; };

AVR_DI int mf_idx(unsigned pk, int j) { return (int)((pk >> (8 * j)) & 255u); }
AVR_DI unsigned mf_set(unsigned pk, int j, int v) { return (pk & ~(255u << (8 * j))) | ((unsigned)v << (8 * j)); }
// (branch-free: the pool word is read at a clamped index either way and the register word
// selected, so a refresh over a manifold holding the new point runs no divergent branches)
AVR_DI float mf_rd(const lds_f *cp, const MfNew &nw, int idx, int w) {
    const bool nu = idx == MF_NEW;
    const float x = cp[AVR_CP_WORDS * (nu ? 0 : idx) + w];
    return nu ? nw.p[w] : x;
}
AVR_DI v3 cp_rd3(const lds_f *cp, int idx, int w) {
    const lds_f *q = cp + AVR_CP_WORDS * idx + w;
    return V(q[0], q[1], q[2]);
}
AVR_DI v3 mf_rd3(const lds_f *cp, const MfNew &nw, int idx, int w) {
    return V(mf_rd(cp, nw, idx, w), mf_rd(cp, nw, idx, w + 1), mf_rd(cp, nw, idx, w + 2));
}
AVR_DI void mf_wr(lds_f *cp, MfNew &nw, int idx, int w, float x) {
    if (idx == MF_NEW) {
#pragma unroll
        for (int k = 0; k < AVR_CP_WORDS; k++)
            if (k == w) nw.p[k] = x;
    } else cp[AVR_CP_WORDS * idx + w] = x;
}

// btPersistentManifold::sortCachedPoints
AVR_DI int sort_cached(const lds_f *cp, const MfNew &nw, unsigned pk, v3 la_new, float d_new) {
    int maxi = -1;
    float maxpen = d_new;
    v3 p[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int id = mf_idx(pk, i);                 // (a full manifold holds old points only)
        float d = cp[AVR_CP_WORDS * id + AVR_CP_DIST];
        if (d < maxpen) { maxi = i; maxpen = d; }
        p[i] = cp_rd3(cp, id, AVR_CP_LA);
    }
    float res[4] = {0, 0, 0, 0};
    if (maxi != 0) res[0] = len2(crs(sub(la_new, p[1]), sub(p[3], p[2])));
    if (maxi != 1) res[1] = len2(crs(sub(la_new, p[0]), sub(p[3], p[2])));
    if (maxi != 2) res[2] = len2(crs(sub(la_new, p[0]), sub(p[3], p[1])));
    if (maxi != 3) res[3] = len2(crs(sub(la_new, p[0]), sub(p[2], p[1])));
    int bi = 0;
    float bv = -1.f;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (fabsf(res[i]) > bv) { bv = fabsf(res[i]); bi = i; }
    return bi;
}

// btManifoldResult::addContactPoint (getCacheEntry / replaceContactPoint / addManifoldPoint).  The
// manifold holds old points only when a pair's one narrowphase point arrives: a replaced point is
// rewritten in the LDS pool, an appended one goes to the registers (nw).
AVR_DI void manifold_add(lds_f *cp, MfNew &nw, unsigned &pk, int &n, int sa, int sb, int pair, tf ta, tf tb, v3 nB, v3 pB,
                         float dist, float thr) {
    if (dist > thr) return;
    v3 pA = add(pB, scl(nB, dist));
    v3 la = tfinvpt(ta, pA), lb = tfinvpt(tb, pB);
    float shortest = thr * thr;
    int near = -1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < n) {
            float d2 = len2(sub(cp_rd3(cp, mf_idx(pk, k), AVR_CP_LA), la));
            if (d2 < shortest) { shortest = d2; near = k; }
        }
    }
    if (near >= 0 || n == AVR_MANIFOLD_POINTS) {
        const int id = mf_idx(pk, near >= 0 ? near : sort_cached(cp, nw, pk, la, dist));
        lds_f *q = cp + AVR_CP_WORDS * id;
        if (near < 0) { q[AVR_CP_IMP] = 0.f; q[AVR_CP_LIFE] = 0.f; }
        q[AVR_CP_SA] = (float)sa; q[AVR_CP_SB] = (float)sb; q[AVR_CP_PAIR] = (float)pair; q[AVR_CP_SLOT] = 0.f;
        q[AVR_CP_LA + 0] = la.x; q[AVR_CP_LA + 1] = la.y; q[AVR_CP_LA + 2] = la.z;
        q[AVR_CP_LB + 0] = lb.x; q[AVR_CP_LB + 1] = lb.y; q[AVR_CP_LB + 2] = lb.z;
        q[AVR_CP_N + 0] = nB.x; q[AVR_CP_N + 1] = nB.y; q[AVR_CP_N + 2] = nB.z;
        q[AVR_CP_DIST] = dist;
    } else {
        pk = mf_set(pk, n, MF_NEW);
        n++;
        nw.p[AVR_CP_IMP] = 0.f; nw.p[AVR_CP_LIFE] = 0.f;
        nw.p[AVR_CP_SA] = (float)sa; nw.p[AVR_CP_SB] = (float)sb; nw.p[AVR_CP_PAIR] = (float)pair; nw.p[AVR_CP_SLOT] = 0.f;
        nw.p[AVR_CP_LA + 0] = la.x; nw.p[AVR_CP_LA + 1] = la.y; nw.p[AVR_CP_LA + 2] = la.z;
        nw.p[AVR_CP_LB + 0] = lb.x; nw.p[AVR_CP_LB + 1] = lb.y; nw.p[AVR_CP_LB + 2] = lb.z;
        nw.p[AVR_CP_N + 0] = nB.x; nw.p[AVR_CP_N + 1] = nB.y; nw.p[AVR_CP_N + 2] = nB.z;
        nw.p[AVR_CP_DIST] = dist;
    }
}

// btPersistentManifold::refreshContactPoints.  Its second sweep (removal, last slot moved into the
// removed one, from the top slot down) decides each point on that point's own refreshed data, and a
// moved point has been decided already, so the decisions are taken in the first sweep with the
// world points it computes, and the second sweep only compacts.
AVR_DI void manifold_refresh(lds_f *cp, MfNew &nw, unsigned &pk, int &n, tf ta, tf tb, float thr) {
    bool rm[4];
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        rm[k] = false;
        if (k < n) {
            int id = mf_idx(pk, k);
            v3 pa = tfpt(ta, mf_rd3(cp, nw, id, AVR_CP_LA)), pb = tfpt(tb, mf_rd3(cp, nw, id, AVR_CP_LB));
            const v3 nrm = mf_rd3(cp, nw, id, AVR_CP_N);
            const float dd = dot(sub(pa, pb), nrm);
            mf_wr(cp, nw, id, AVR_CP_DIST, dd);
            mf_wr(cp, nw, id, AVR_CP_LIFE, mf_rd(cp, nw, id, AVR_CP_LIFE) + 1.f);
            if (dd > thr) rm[k] = true;
            else {
                v3 df = sub(pb, sub(pa, scl(nrm, dd)));
                if (len2(df) > thr * thr) rm[k] = true;
            }
        }
    }
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        if (k < n && rm[k]) {   // removeContactPoint: the last slot moves into slot k
            pk = mf_set(pk, k, mf_idx(pk, n - 1));
            n--;
        }
    }
}

// --------------------------------------------------------------------------- collision detection
// Per sub-step (btCollisionWorld::performDiscreteCollisionDetection restated):
//   1. body transforms and fattened AABBs (btDbvtBroadphase, margin 0.02);
//   2. broadphase over the compiled candidate body pairs, order-preserving compaction;
//   3. world AABBs of every non-static child shape, cached in LDS (static ones are precomputed
//      on the host, m.static_saabb);
//   4. child shape pairs (compound culling, i-major / j-minor within a body pair) stream through
//      a 128-entry LDS queue; every 64 pairs form a batch that is finished right away:
//      narrowphase one lane per pair (small shapes), wave-cooperative narrowphase for big hulls
//      and EPA (in pair order), then the persistent-manifold update one lane per pair with an
//      order-preserving append of the surviving points to the new contact pool.
// The previous contact pool stays in the env's global state (read, and updated in place by the
// single lane that owns each point); the new pool is appended to global scratch and copied
// over the old one at the end.

AVR_DI float *env_cs(const KModel &m, int env) { return m.cscr + (size_t)env * CS_WORDS; }

// world AABB of child shape s from its packed info (m.shape_info): the per-sub-step cache for a
// non-static shape, the host-precomputed box for a static one
template <class LT>
AVR_DI void child_aabb(const KModel &m, const LT &L, int s, int info, v3 &mn, v3 &mx) {
    const int c = (info & 511) - 1;
    if (c >= 0) { mn = ld3(L.u.c.caabb[c]); mx = ld3(L.u.c.caabb[c] + 3); }
    else { const gf4p a = (gf4p)(m.static_saabb + 8 * s); const f4v x = a[0], y = a[1]; mn = V(x.x, x.y, x.z); mx = V(y.x, y.y, y.z); }
}
AVR_DI bool info_enabled(int info, int gender) { const int g = (info >> 9 & 3) - 1; return g < 0 || g == gender; }
AVR_DI int info_kind(int info) { return (info >> 11) & 3; }
// a sphere against a convex hull: the narrowphase kernel runs these on the point-core GJK
AVR_DI bool sphere_hull(int ia, int ib) {
    const int ka = info_kind(ia), kb = info_kind(ib);
    return (ka == AVR_SPHERE && kb == AVR_HULL) || (ka == AVR_HULL && kb == AVR_SPHERE);
}

// manifold update for the nq (<= 64) shape pairs k0 .. k0 + nq - 1 of the list, lane q <-> pair
// k0 + q, from the narrowphase results of avr_narrowphase_kernel
// one lane's shape pair k (clamped into the list) and its narrowphase result, loaded a batch
// ahead of its use so that the loads overlap the previous batch's pool stores
struct PairIn { float2 kw; float4 r0, r1; };
AVR_DI void pair_in(const float *cs, int k, int nsp, PairIn &P) {
    k = min(k, max(nsp - 1, 0));
    P.kw = gld((const float2 *)(cs + CS_PAIRS) + k);
    P.r0 = gld((const float4 *)(cs + CS_RES) + 2 * k);
    P.r1 = gld((const float4 *)(cs + CS_RES) + 2 * k + 1);
}

static_assert(K_MAX_CONTACTS % 4 == 0, "the old pool's keys are read four at a time");
AVR_DI void collide_batch(const KModel &m, EnvLDS &L, const PairIn &in, int k0, int nq, lds_f *oldcp, int nold, float *newcp, int &nnew) {
    const int lane = lane_id();
    PROF_START(pb);
    int sa = 0, sb = 0, p = 0, ba = 0, bb = 0;
    int rc = 0;
    v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
    float d = 0.f;
    if (lane < nq) {
        const int k = __float_as_int(in.kw.x);
        sa = k & 0xffff; sb = k >> 16;
        const int w = __float_as_int(in.kw.y);     // body pair | ba << 16 | bb << 24
        p = w & 0xffff; ba = (w >> 16) & 0xff; bb = (w >> 24) & 0xff;
        rc = __float_as_int(in.r0.x);   // (0 or 1: the narrowphase and coop kernels finished every pair)
        nB = V(in.r0.y, in.r0.z, in.r0.w); pB = V(in.r1.x, in.r1.y, in.r1.z); d = in.r1.w;
    }
    PROF_STOP(17, pb);

    // manifold update (one lane per pair)
    unsigned pk = 0u;
    int n = 0;
    MfNew nw;
#pragma unroll
    for (int k = 0; k < AVR_CP_WORDS; k++) nw.p[k] = 0.f;
    if (lane < nq) {
        float thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
        const int key = sa | (sb << 16);
        // the old pool's points of this pair: a bit mask over the pool (keys read four at a time,
        // every read in flight together), then its first AVR_MANIFOLD_POINTS set bits in pool order
        // -- the points the in-order scan would take, at ~3 VALU per old point instead of ~10
        const lds_f4 *ok = (const lds_f4 *)L.u.k.okey;
        constexpr int NW = (K_MAX_CONTACTS + 31) / 32;
        unsigned mb[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) {
            unsigned b = 0u;
            if (32 * w < nold) {
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    if (32 * w + 4 * c < K_MAX_CONTACTS) {
                        const f4v q = ok[8 * w + c];
                        b |= (__float_as_int(q.x) == key ? 1u : 0u) << (4 * c) | (__float_as_int(q.y) == key ? 2u : 0u) << (4 * c)
                           | (__float_as_int(q.z) == key ? 4u : 0u) << (4 * c) | (__float_as_int(q.w) == key ? 8u : 0u) << (4 * c);
                    }
                }
                const int r = nold - 32 * w;      // (keys past the pool are stale)
                if (r < 32) b &= (1u << r) - 1u;
            }
            mb[w] = b;
        }
#pragma unroll
        for (int t = 0; t < AVR_MANIFOLD_POINTS; t++) {
            int ws = -1;
            unsigned bw = 0u;
#pragma unroll
            for (int w = NW - 1; w >= 0; w--)
                if (mb[w]) { ws = w; bw = mb[w]; }
            if (ws >= 0) {
                pk |= (unsigned)(32 * ws + __builtin_ctz(bw)) << (8 * t);
                n = t + 1;
#pragma unroll
                for (int w = 0; w < NW; w++)
                    if (w == ws) mb[w] &= mb[w] - 1u;
            }
        }
#ifdef AVR_PROF
    }
    PROF_STOP(40, pb);
    if (lane < nq) {
        float thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
#endif
        tf ta = ldtf(L.btf[ba]), tb = ldtf(L.btf[bb]);
        if (rc == 1) manifold_add(oldcp, nw, pk, n, sa, sb, p, ta, tb, nB, pB, d, thr);
#ifdef AVR_PROF
    }
    PROF_STOP(41, pb);
    if (lane < nq) {
        float thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
        tf ta = ldtf(L.btf[ba]), tb = ldtf(L.btf[bb]);
#endif
        manifold_refresh(oldcp, nw, pk, n, ta, tb, thr);
    }
    PROF_STOP(42, pb);
    int incl = n;
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int excl = incl - n;
    const int tot = __shfl(incl, 63, 64);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < n) {
            int dst = nnew + excl + k;
            int id = mf_idx(pk, k);
            if (dst < K_MAX_CONTACTS) {
                // 16-word point record: the new point from registers or an old one from memory
                float4 *o = (float4 *)(newcp + AVR_CP_WORDS * dst);
                if (id == MF_NEW) {
                    o[0] = make_float4(nw.p[0], nw.p[1], nw.p[2], nw.p[3]);
                    o[1] = make_float4(nw.p[4], nw.p[5], nw.p[6], nw.p[7]);
                    o[2] = make_float4(nw.p[8], nw.p[9], nw.p[10], nw.p[11]);
                    o[3] = make_float4(nw.p[12], nw.p[13], nw.p[14], nw.p[15]);
                } else {
                    const lds_f4 *q = (const lds_f4 *)(oldcp + AVR_CP_WORDS * id);
                    const f4v q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
                    o[0] = make_float4(q0.x, q0.y, q0.z, q0.w);
                    o[1] = make_float4(q1.x, q1.y, q1.z, q1.w);
                    o[2] = make_float4(q2.x, q2.y, q2.z, q2.w);
                    o[3] = make_float4(q3.x, q3.y, q3.z, q3.w);
                }
            }
        }
    }
    nnew += tot;
    PROF_STOP(18, pb);
}

// Part A1 (avr_substep_pairs_kernel): body frames, fattened AABBs, broadphase and the ordered
// shape-pair list, written to the env's collision scratch.
template <class LT>
AVR_DI void collide_pairs(const KModel &m, LT &L, float *cs) {
    const int lane = lane_id();
    const int gender = L.gender;
    PROF_START(pt);
    // body transforms + fattened AABBs (one lane per body: nb <= MAXB < 64)
    v3 bmn = V(0, 0, 0), bmx = V(0, 0, 0);
    if (lane < m.nb) {
        const int b = lane;
        tf t = body_tf(m, L, b);
        int g = gld(m.body_kind + (b)) == AVR_BODY_HUMAN ? gender : 0;
        const float *a = m.body_aabb + 12 * b + 6 * g;
        v3 mn, mx;
        aabb_of(t, ld3(a), ld3(a + 3), mn, mx);
        v3 e = V(BT_BROADPHASE_EXPAND, BT_BROADPHASE_EXPAND, BT_BROADPHASE_EXPAND);
        sttf(L.btf[b], t);
        sttf(cs + CS_BTF + 8 * b, t);
        bmn = sub(mn, e);
        bmx = add(mx, e);
    }
    SYNC();     // the state words and link frames are dead: the collision scratch overlays them
    if (lane < m.nb) {
        st3(L.u.c.bmin[lane], bmn);
        st3(L.u.c.bmax[lane], bmx);
    }
    SYNC();
    // world AABBs of the non-static child shapes (child index from the staged shape info; the
    // shape records are read unconditionally, clamped into the table, so the unrolled passes'
    // loads are not held behind each other's branches)
#pragma unroll
    for (int q = 0; q < MAXSH / 64; q++) {
        const int s = lane + 64 * q, sc = min(s, m.ns - 1);
        const int c = s < m.ns ? (int)(L.sinfo[sc] & 511) - 1 : -1;
        v3 mn, mx;
        shape_aabb(m, sc, ldtf(L.btf[gld(m.shape_body + sc)]), mn, mx);
        if (c >= 0) {
            st3(L.u.c.caabb[c], mn);
            st3(L.u.c.caabb[c] + 3, mx);
        }
    }
    // broadphase over the candidate pair list, order-preserving compaction; the body indices of
    // BP_BATCH rounds of 64 pairs are loaded together (one round trip per batch, not per round)
    int nap = 0;
    const int npe = L.nla > m.nl ? m.np : m.np_base;   // chain-vs-static pairs: 'tremor' envs only
    constexpr int BP_BATCH = 8;
    for (int b0 = 0; b0 < npe; b0 += 64 * BP_BATCH) {
        int pa[BP_BATCH], pb[BP_BATCH];
#pragma unroll
        for (int q = 0; q < BP_BATCH; q++) {
            const int p = min(b0 + 64 * q + lane, npe - 1);
            pa[q] = gld(m.pair_a + p);
            pb[q] = gld(m.pair_b + p);
        }
#pragma unroll
        for (int q = 0; q < BP_BATCH; q++) {
            const int base = b0 + 64 * q;
            if (base >= npe) break;
            const int p = base + lane;
            const int ba = pa[q], bb = pb[q];
            const bool act = p < npe && overlap(ld3(L.u.c.bmin[ba]), ld3(L.u.c.bmax[ba]), ld3(L.u.c.bmin[bb]), ld3(L.u.c.bmax[bb]));
            int tot;
            int pre = ballot_prefix(act, &tot);
            if (act && nap + pre < MAXAP) L.u.c.apair[nap + pre] = p;
            nap += tot;
        }
    }
    if (nap > MAXAP) { if (lane == 0) L.flags |= 4; nap = MAXAP; }
    SYNC();
    // the active pairs' records, loaded once (every round trip in flight together): lane l of
    // slot q holds active pair 64 q + l's; the rounds below read them across lanes rather than
    // from global memory each time
    static_assert(MAXAP == 256, "four record slots");
    auto rec_load = [&](int q) {
        const int a = 64 * q + lane;
        const int ap = L.u.c.apair[min(a, max(nap - 1, 0))];
        const int4 r = m.pair_rec[ap];
        return a < nap ? r : make_int4(0, 0, 0, 0);
    };
    const int4 rq0 = rec_load(0), rq1 = rec_load(1), rq2 = rec_load(2), rq3 = rec_load(3);
    PROF_STOP(1, pt);
    // Child shape pairs, in pair order (i-major, j-minor within a body pair), appended to the
    // list.  A child's world AABB lies inside its body's fattened AABB, so children of A that
    // miss B's body AABB cannot meet any child of B: the child lists are culled against the other
    // body first, which leaves the set of overlapping child pairs and its order unchanged.
    // Pairs are produced 64 at a time from either a run of consecutive single-child pairs (1 x 1:
    // food-food, robot link-link, ...; 80 % of the active pairs), one lane per pair, or one culled
    // compound pair, one lane per item.
    int nsp = 0;
    int k = 0;                                      // next active pair
    int gp = 0, gsa0 = 0, gsb0 = 0, gncB = 1, gn = 0, gbase = 0;
    bool gcull = false, gbare = false;
    float grcpB = 1.f;
    int n0 = 0, n1 = 0;                             // sphere-hull / other pairs
    int gbab = 0;                                   // the compound pair's bodies (ba | bb << 8)
    for (;;) {
        bool act = false, last = false;
        int sa = 0, sb = 0, q = gp, ia = 0, ib = 0, bab = gbab;
        if (gbase < gn) {                           // the compound pair in progress
            const int it = gbase + lane;
            if (it < gn) {
                const int i = (int)(((float)it + 0.5f) * grcpB);     // exact: it < 2^14, ncB <= 128
                const int j = it - i * gncB;
                if (gcull) {
                    sa = L.u.c.candA[i];
                    sb = L.u.c.candB[j];
                    ia = L.sinfo[sa]; ib = L.sinfo[sb];
                    v3 a0, a1, b0, b1;
                    child_aabb(m, L, sa, ia, a0, a1);
                    child_aabb(m, L, sb, ib, b0, b1);
                    act = overlap(a0, a1, b0, b1);
                } else {
                    sa = gsa0 + i;
                    sb = gsb0 + j;
                    ia = L.sinfo[sa]; ib = L.sinfo[sb];
                    if (info_enabled(ia, gender) && info_enabled(ib, gender)) {
                        if (gbare) act = true;
                        else {
                            v3 a0, a1, b0, b1;
                            child_aabb(m, L, sa, ia, a0, a1);
                            child_aabb(m, L, sb, ib, b0, b1);
                            act = overlap(a0, a1, b0, b1);
                        }
                    }
                }
            }
            gbase += 64;
        } else if (k < nap) {
            if (gcull) { SYNC(); gcull = false; }   // candA / candB are rewritten below
            const int kk = k + lane;
            int4 rec;
            {
                // record of active pair kk: slot kk / 64 (k / 64 or the next) of lane kk % 64
                const int s0 = k >> 6;
                const int4 lo = s0 == 0 ? rq0 : s0 == 1 ? rq1 : s0 == 2 ? rq2 : rq3;
                const int4 hi = s0 == 0 ? rq1 : s0 == 1 ? rq2 : rq3;
                const int src = kk & 63;
                const bool up = (kk >> 6) != s0;
                const int4 a = make_int4(__shfl(lo.x, src), __shfl(lo.y, src), __shfl(lo.z, src), __shfl(lo.w, src));
                const int4 b = make_int4(__shfl(hi.x, src), __shfl(hi.y, src), __shfl(hi.z, src), __shfl(hi.w, src));
                rec = kk < nap ? (up ? b : a) : make_int4(0, 0, 0, 0);
            }
            const unsigned long long bm = __ballot(kk < nap && (rec.w & 2));
            const int run = bm == ~0ull ? 64 : __ffsll((long long)~bm) - 1;
            if (run > 0) {                          // a run of 1 x 1 pairs
                if (lane < run) {
                    q = L.u.c.apair[kk];
                    sa = rec.y & 0xffff;
                    sb = rec.z & 0xffff;
                    bab = (rec.x & 0xffff) | (rec.x >> 16) << 8;
                    ia = L.sinfo[sa]; ib = L.sinfo[sb];
                    if (info_enabled(ia, gender) && info_enabled(ib, gender)) {
                        if (rec.w & 1) act = true;
                        else {
                            v3 a0, a1, b0, b1;
                            child_aabb(m, L, sa, ia, a0, a1);
                            child_aabb(m, L, sb, ib, b0, b1);
                            act = overlap(a0, a1, b0, b1);
                        }
                    }
                }
#ifdef AVR_PROF
                if (lane == 0) L.prof[4] += run;
#endif
                k += run;
            } else {                                // set up compound pair k (lane 0's record, loaded above)
                gp = L.u.c.apair[k];
                const int4 r0 = make_int4(__builtin_amdgcn_readfirstlane(rec.x), __builtin_amdgcn_readfirstlane(rec.y),
                                          __builtin_amdgcn_readfirstlane(rec.z), __builtin_amdgcn_readfirstlane(rec.w));
                const int ba = r0.x & 0xffff, bb = r0.x >> 16;
                gbab = ba | bb << 8;
                const int na = r0.y >> 16, nb = r0.z >> 16;
                gsa0 = r0.y & 0xffff;
                gsb0 = r0.z & 0xffff;
                gbare = r0.w & 1;
                // a single child against at most 64 (food against the spoon pieces): its items are
                // tested directly, in one round, rather than after a culling round.  The same set
                // in the same order: child AABBs lie inside their bodies' fattened AABBs, so an
                // overlapping child pair passes both body culls.  (Measured: extending this to 128
                // children -- the bowl, the wheelchair -- made the kernel slower, 0.080 -> 0.083 ms.)
                gcull = !gbare && na * nb > 1 && !((na == 1 || nb == 1) && na * nb <= 64);
                int ncA = na, ncB = nb;
                if (gcull) {
                    const v3 bAmn = ld3(L.u.c.bmin[ba]), bAmx = ld3(L.u.c.bmax[ba]);
                    const v3 bBmn = ld3(L.u.c.bmin[bb]), bBmx = ld3(L.u.c.bmax[bb]);
                    ncA = 0;
                    for (int base = 0; base < na; base += 64) {
                        const int i = base + lane;
                        bool a = false;
                        if (i < na) {
                            const int ia = L.sinfo[gsa0 + i];
                            if (info_enabled(ia, gender)) {
                                v3 a0, a1;
                                child_aabb(m, L, gsa0 + i, ia, a0, a1);
                                a = overlap(a0, a1, bBmn, bBmx);
                            }
                        }
                        int tot;
                        int pre = ballot_prefix(a, &tot);
                        if (a) L.u.c.candA[ncA + pre] = gsa0 + i;
                        ncA += tot;
                    }
                    ncB = 0;
                    for (int base = 0; base < nb; base += 64) {
                        const int j = base + lane;
                        bool a = false;
                        if (j < nb) {
                            const int ib = L.sinfo[gsb0 + j];
                            if (info_enabled(ib, gender)) {
                                v3 b0, b1;
                                child_aabb(m, L, gsb0 + j, ib, b0, b1);
                                a = overlap(b0, b1, bAmn, bAmx);
                            }
                        }
                        int tot;
                        int pre = ballot_prefix(a, &tot);
                        if (a) L.u.c.candB[ncB + pre] = gsb0 + j;
                        ncB += tot;
                    }
                    SYNC();
                }
                gn = ncA * ncB;
                gncB = ncB > 0 ? ncB : 1;
                grcpB = 1.f / (float)gncB;
                gbase = 0;
#ifdef AVR_PROF
                if (lane == 0) L.prof[4] += gn;
#endif
                k++;
                continue;
            }
        } else last = true;
        // append in lane order; the restated pipeline keeps at most MAXSP shape pairs per
        // sub-step (flag 8)
        int tot;
        int pre = ballot_prefix(act, &tot);
        const int kq = nsp + pre;
        const bool ok = act && kq < MAXSP;
        if (ok) {
            cs[CS_PAIRS + 2 * kq] = __int_as_float(sa | (sb << 16));
            cs[CS_PAIRS + 2 * kq + 1] = __int_as_float(q | bab << 16);
        }
        // the narrowphase kernel's two work lists (pair indices, ascending)
        const bool sh = ok && sphere_hull(ia, ib);
        int t0, t1;
        const int p0 = ballot_prefix(sh, &t0), p1 = ballot_prefix(ok && !sh, &t1);
        // (entries carry the shape and body indices, so the narrowphase reads no pair record)
        if (ok) {
            const int l = sh ? CS_L0 + 2 * (n0 + p0) : CS_L1 + 2 * (n1 + p1);
            *(float2 *)(cs + l) = make_float2(__int_as_float(kq | bab << 16), __int_as_float(sa | (sb << 16)));
        }
        n0 += t0;
        n1 += t1;
        nsp += tot;
        if (last) break;
    }
    if (nsp > MAXSP) { if (lane == 0) L.flags |= 8; nsp = MAXSP; }
#ifdef AVR_PROF
    if (lane == 0) { L.prof[14] += nsp; L.prof[15] += nap; }
#endif
    if (lane == 0) {
        cs[CS_NSP] = __int_as_float(nsp); cs[CS_FLAGS] = __int_as_float(L.flags);
        cs[CS_N0] = __int_as_float(n0); cs[CS_N1] = __int_as_float(n1);
        cs[CS_COOP] = 0.f;
    }
    PROF_STOP(2, pt);
}

// Part A3 (avr_substep_a_kernel): manifold update of every listed shape pair from its
// narrowphase result, 64 pairs at a time, and the new contact pool.  The previous contact pool
// is copied into LDS first (read, and updated in place by the single lane that owns each point),
// so the new pool is appended straight into the env's state.
AVR_DI void collide_contacts(const KModel &m, EnvLDS &L, const float *cs, float *gcp) {
    const int lane = lane_id();
    float *newcp = gcp;
    PROF_START(pt);
    // the previous contact pool in LDS (the manifold update reads and updates it in place) and
    // its keys (matching in the manifold update)
    const int nold = (int)L.st[S_TASK + T_NCP];
    lds_f *ocp = (lds_f *)L.u.k.ocp;      // (staged by load_a)
    for (int i = lane; i < nold; i += 64)
        L.u.k.okey[i] = (int)ocp[AVR_CP_WORDS * i + AVR_CP_SA] | ((int)ocp[AVR_CP_WORDS * i + AVR_CP_SB] << 16);
    if (lane == 0) L.flags |= __float_as_int(gld(cs + CS_FLAGS));
    __builtin_amdgcn_s_waitcnt(0);     // (every read of the old pool has returned before the new one overwrites it)
    SYNC();
    const int nsp = __float_as_int(gld(cs + CS_NSP));
    int nnew = 0;
    PairIn cur, nxt;
    pair_in(cs, lane, nsp, cur);
    for (int k0 = 0; k0 < nsp; k0 += 64) {
        pair_in(cs, k0 + 64 + lane, nsp, nxt);
        collide_batch(m, L, cur, k0, min(64, nsp - k0), ocp, nold, newcp, nnew);
        SYNC();
        cur = nxt;
    }
    if (nnew > K_MAX_CONTACTS) { if (lane == 0) L.flags |= 2; nnew = K_MAX_CONTACTS; }
    SYNC();
    if (lane == 0) L.st[S_TASK + T_NCP] = (float)nnew;
    SYNC();
    PROF_STOP(3, pt);
}

// --------------------------------------------------------------------------- constraint rows
// Jacobian entry of DoF d (< MAXD) for a point p on the link with ancestor mask am, direction
// (lin, ang): lin . (axis x (p - origin)) + ang . axis (revolute), lin . axis (prismatic).  The
// multiply-adds are spelled out (fmaf) so that the contact's lane (robot_jac, all DoFs unrolled)
// and the wave-cooperative row (one DoF per lane) round alike: left to contraction, the compiler
// fuses different products of the two forms (which product of a sum it fuses depends on how
// often each is used after CSE).
AVR_DI float jac_entry(const KModel &m, const EnvLDS &L, unsigned am, int d, v3 p, v3 lin, v3 ang) {
    float v = 0.f;
    if (d < m.nd + m.hc_n) {               // chain DoFs are never ancestors of a robot link
        const int k = gld(m.dof_link + (d));
        if ((am >> k) & 1u) {
            const v3 a = ld3(L.ax[k]);
            if (gld(m.rl_jtype + (k)) == AVR_J_REVOLUTE) {
                const v3 r = sub(p, ld3(L.org[k]));
                const v3 cl = V(fmaf(a.y, r.z, -(a.z * r.y)), fmaf(a.z, r.x, -(a.x * r.z)), fmaf(a.x, r.y, -(a.y * r.x)));
                v = fmaf(lin.z, cl.z, fmaf(lin.y, cl.y, lin.x * cl.x)) + fmaf(ang.z, a.z, fmaf(ang.y, a.y, ang.x * a.x));
            } else {
                v = fmaf(lin.z, a.z, fmaf(lin.y, a.y, lin.x * a.x)) + fmaf(ang.z, 0.f, fmaf(ang.y, 0.f, ang.x * 0.f));
            }
        }
    }
    return v;
}
AVR_DI void robot_jac(const KModel &m, const EnvLDS &L, int link, v3 p, v3 lin, v3 ang, float *J) {
    const unsigned am = gld(m.anc_mask + (link));
#pragma unroll
    for (int d = 0; d < MAXD; d++) J[d] = jac_entry(m, L, am, d, p, lin, ang);
}

AVR_DI float free_dot(const EnvLDS &L, int f, v3 lin, v3 ang) {
    return dot(lin, ld3(L.fv[f])) + dot(ang, ld3(L.fw[f]));
}

AVR_DI v3 iinv_mul(const EnvLDS &L, int f, v3 a) {
    const float *I = L.Iinv[f];
    return V(I[0] * a.x + I[1] * a.y + I[2] * a.z, I[3] * a.x + I[4] * a.y + I[5] * a.z, I[6] * a.x + I[7] * a.y + I[8] * a.z);
}


// Constraint rows live in a per-env buffer in global memory, in solve order [non-contact]
// [normals][frictions].  A row's ownership mask (own_mask) names its free-body endpoints: 2 bits
// per free body f, 1 = endpoint A, 2 = endpoint B (part B's lane f holds body f); an all-zero
// header is a null row (no endpoint, inv = rhs = lo = hi = 0).
// Non-contact rows have 20-word records at word 20 r:
//   w0 ownership mask   w1 robot slot + 1 (int bits, 0: none)   w2 inv   w3 rhs   w4 lo   w5 hi
//   w8..13 free A Jacobian (lin, ang)   w14..19 free B Jacobian
// Contact rows (row n_nc + k, k = c for contact c's normal, n_c + 2c + {0,1} for its frictions)
// have 16-word records at word CR_BASE + 16 k:
//   w0 ownership mask | (robot slot + 1) << 20   w1 inv   w2 rhs   w3 see below
//   w4..9 free A Jacobian   w10..15 free B Jacobian
// w3: normal rows the residual limit (BT_RESIDUAL_SQRT inv), a friction unit's first row its
// friction coefficient, its second row its own residual limit (and the second row's w0, which the
// resolve does not read, the first row's limit); torsional rows their coefficient.  (K_TORSION) a
// normal record's w0 also carries the contact's torsional index + 1 in bits 2..19 (0: none).
// (normal rows clamp to [0, 1e10], frictions to +-friction * normal impulse; the normal row's
// starting impulse is the manifold point's cached impulse x warm-start factor, read by part B
// from the contact pool).  Rows with an articulated endpoint own a robot part (slot): 16 (J[d],
// M^-1 J^T[d]) pairs, A and B endpoints combined.  Non-contact rows take slots 0 .. n_nc-1,
// robot contacts 3 consecutive slots each.  The free bodies' M^-1 J^T is not stored: part B
// forms it on the owner lane from the mass-normalised part (see put_free).
#define RW 32       // allocation unit of the per-env row buffer (2 * rowcap * RW floats)
#define RWC 20      // words per non-contact record
#define CRW 16      // words per contact record
#define CR_BASE (MAXNC * RWC)
#define CI_SLOT 20  // contact header word 0: robot slot + 1 from this bit
#if NDL == 2
#define ROBW 64     // words per robot part: lane sl's (J, M^-1 J^T) of DoFs sl and sl + 16
#else
#define ROBW 32     // words per robot part: lane sl's (J, M^-1 J^T) of DoF sl
#endif
// per-env workspace between the sub-step kernels: [n_envs][WS_WORDS] floats
#define WS_WORDS 128
#define WS_NNC 0     // int bits: non-contact rows
#define WS_NC 1      // int bits: contact points (rows n_nc .. n_nc + K_CROWS n_c)
#define WS_ASQ 2     // sum of squared caller actions (take_step -> task glue)
#define WS_XCC 3     // diagnostic builds: XCD that ran part A
#define WS_NROB 4    // int bits: robot parts (slots) of the row set
#define WS_COOPROT 5 // int bits: rotation of the capped cooperative-pair window (np_coop)
#define WS_NT 6      // int bits: (K_TORSION) contacts with torsional rows (rows n_nc + 3 n_c ..)
#define WS_VQ 16     // [MAXD] unconstrained robot velocities
#define WS_FV (WS_VQ + 16 * NDL)     // [MAXF][4] unconstrained free-body linear velocities
#define WS_FW (WS_FV + 4 * MAXF)     // [MAXF][4] angular
static_assert(MAXD <= 16 * NDL && WS_FW + 4 * MAXF <= WS_WORDS, "workspace layout");
// A row's ownership mask: 2 bits per free body f (= part-B lane f): 1 endpoint A, 2 endpoint B
AVR_DI int own_mask(int fa, int fb) { return (fa >= 0 ? 1 << (2 * fa) : 0) | (fb >= 0 ? 2 << (2 * fb) : 0); }
static_assert(CR_BASE + K_CROWS * K_MAX_CONTACTS * CRW <= (MAXNC + K_CROWS * K_MAX_CONTACTS) * RWC, "contact records fit below the robot parts");

AVR_DI float *row_rec(const KModel &m, float *base, int r) { (void)m; return base + r * RWC; }
AVR_DI float *row_crec(float *base, int k) { return base + CR_BASE + k * CRW; }
AVR_DI float *row_rob(const KModel &m, float *base, int slot) { return base + m.rowcap * RWC + slot * ROBW; }

// A free endpoint's part is stored mass-normalised: g = (jl / sqrt(m), D^1/2 R^T ja) with
// R D R^T the world inverse inertia.  Part B then keeps the body's velocity increment in the
// same coordinates (dv = v~ / sqrt(m) ... ) so that J.dv = g.v~ and M^-1 J^T delta = g delta:
// one 6-vector per endpoint serves both halves of a row resolve.
#ifndef B4_PK
#define B4_PK 1     // free parts stored as (linear, angular) pairs per axis: packed-f32 row resolves (0: scalar layout)
#endif
// Friction units resolved as a pair through their coupling (go4_pair, -DB4_FPAIR=1): the same
// Gauss-Seidel step in exact arithmetic, ~1 % faster part B, but rounded differently from the
// sequential resolve -- and where a contact's normal impulse sits at 0 (a point at the contact
// threshold), that rounding decides whether its friction unit is active in an iteration, so the
// two orders end sub-steps apart by up to 5e-2 m/s on the BedBathing wiping states
// (tools/dbg_torsion.py; the sequential resolve matches the oracle to 1e-6 there).  Off: parity
// with the oracle's sequential order first.
#ifndef B4_FPAIR
#define B4_FPAIR 0
#endif
#if B4_FPAIR
#error "B4_FPAIR: the second friction row's 4th header word now holds its residual limit, not the coupling"
#endif
static_assert(!K_TORSION || MAXF == 1, "the torsional index shares the normal header's word 0 with a 1-body ownership mask");
AVR_DI void put_free(const EnvLDS &L, int f, float *w, v3 jl, v3 ja) {
    const float *g = L.gsc[f];
    const qt q = ldq(L.st + S_FREE + AVR_FB_WORDS * f + 3);
    const v3 b = qrot(qconj(q), ja);
#if B4_PK
    w[0] = jl.x * g[0]; w[1] = b.x * g[1]; w[2] = jl.y * g[0];
    w[3] = b.y * g[2]; w[4] = jl.z * g[0]; w[5] = b.z * g[3];
#else
    w[0] = jl.x * g[0]; w[1] = jl.y * g[0]; w[2] = jl.z * g[0];
    w[3] = b.x * g[1]; w[4] = b.y * g[2]; w[5] = b.z * g[3];
#endif
}
AVR_DI void put_free_zero(float *w) {
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = 0.f;
}
// PyBullet's solverResidualThreshold (1e-7 on the largest squared row residual of a PGS iteration,
// the row's impulse change over its jacDiagABInv; oracle/avr_oracle.c BT_RESIDUAL_THRESHOLD): a row
// has converged when |delta| <= sqrt(1e-7) inv.  Kernel a stores that limit with every row.
#define BT_RESIDUAL_SQRT 3.16227766e-4f
AVR_DI void put_hdr(float *w, int info, float inv, float rhs, float lo, float hi, int slot) {
    w[0] = __int_as_float(info); w[1] = __int_as_float(slot + 1); w[2] = inv; w[3] = rhs; w[4] = lo; w[5] = hi; w[6] = BT_RESIDUAL_SQRT * inv; w[7] = 0.f;
}
AVR_DI void put_robot(float *w, const float *J, const float *MJ) {
#if NDL == 2
#pragma unroll
    for (int d = 0; d < 16; d++) {
        w[4 * d] = J[d]; w[4 * d + 1] = MJ[d];
        w[4 * d + 2] = d + 16 < MAXD ? J[d + 16] : 0.f; w[4 * d + 3] = d + 16 < MAXD ? MJ[d + 16] : 0.f;
    }
#else
#pragma unroll
    for (int d = 0; d < 16; d++) { w[2 * d] = d < MAXD ? J[d] : 0.f; w[2 * d + 1] = d < MAXD ? MJ[d] : 0.f; }
#endif
}


#ifdef AVR_COOP_CHECK
__device__ int g_coop_check;     // (diagnostic build: mismatches reported)
#endif
// Non-contact rows (limits, motors, fixed constraint), one lane per row.
// Row order restates btMultiBodyConstraintSolver's setup order: joint-limit rows
// of violated limits (link order, lower then upper), motor rows (link order), fixed rows.
AVR_DI int build_noncontact_rows(const KModel &m, EnvLDS &L, float *rows, float dt) {
    const int lane = lane_id();
    const float erp = m.erp;
    // enumerate in parallel (lane l = link l: its violated limits, then its motor), number the rows
    // by ballot prefix and hand each row's description to the lane of that row through LDS
    int nrow, kind = -1, dof = 0, fix = 0;
    float pen = 0.f;
    {
        float (*desc)[4] = L.u.d.rn[0];        // [MAXNC] (kind, dof, pen); the RNEA temporaries are dead
        const bool lk = lane < L.nla;
        const int ld = lk ? gld(m.rl_dof + (lane)) : -1;
        const bool hl = lk && gld(m.rl_has_limit + (lane));
        float plo = 1.f, phi = 1.f;
        if (hl) {
            const float q = L.st[S_Q + ld];
#if K_CHAIN_LIMITS_IN_STATE
            // the human chain's limits carry the env's limit_scale (state); the robot's are the model's
            const int c = lane - m.nl;
            plo = q - (c >= 0 ? L.st[S_HCH + 2 * K_HC_N + c] : gld(m.rl_lower + (lane)));
            phi = (c >= 0 ? L.st[S_HCH + 3 * K_HC_N + c] : gld(m.rl_upper + (lane))) - q;
#else
            plo = q - gld(m.rl_lower + (lane));
            phi = gld(m.rl_upper + (lane)) - q;
#endif
        }
        const bool vlo = hl && !(plo > 0.f), vhi = hl && !(phi > 0.f), mot = ld >= 0;
        const unsigned long long blo = __ballot(vlo), bhi = __ballot(vhi), bmo = __ballot(mot), lt = (1ull << lane) - 1ull;
        const int nlim = __popcll(blo) + __popcll(bhi);
        const int rlo = __popcll(blo & lt) + __popcll(bhi & lt), rmo = nlim + __popcll(bmo & lt);
        if (vlo && rlo < MAXNC) st3(desc[rlo], V(0.f, (float)ld, plo));
        if (vhi && rlo + vlo < MAXNC) st3(desc[rlo + vlo], V(1.f, (float)ld, phi));
        if (mot && rmo < MAXNC) st3(desc[rmo], V(2.f, (float)ld, 0.f));
        nrow = nlim + __popcll(bmo);
        SYNC();
        if (lane < nrow && lane < MAXNC) {
            const v3 t = ld3(desc[lane]);
            kind = (int)t.x; dof = (int)t.y; pen = t.z;
        }
    }
    if (lane >= nrow && lane < nrow + 6) { kind = 3; fix = lane - nrow; }
    nrow += 6;
    if (lane >= MAXNC) kind = -1;
    // fixed constraint robot tool link <-> spoon (uniform geometry)
    const int link = m.tool_link, fb = m.spoon_free;
    const tf ta = ldtf(L.cm[link]);
    const tf off = gldtf(m.tool_offset);
    const v3 pivA = tfpt(ta, off.p);
    const qt frA = qmul(ta.q, off.q);
    const tf tb = ldtf(L.st + S_FREE + AVR_FB_WORDS * fb);
#if K_TOOL_PIVOT
    const v3 pivB = tfpt(tb, V(m.fix_pivot_b[0], m.fix_pivot_b[1], m.fix_pivot_b[2]));   // the tool's base COM (handle)
#else
    const v3 pivB = tb.p;
#endif
    const m3 FA = qmat(frA), FB = qmat(tb.q);
    const v3 c0 = V(FA.m[0][0], FA.m[1][0], FA.m[2][0]), c1 = V(FA.m[0][1], FA.m[1][1], FA.m[2][1]), c2 = V(FA.m[0][2], FA.m[1][2], FA.m[2][2]);
    // The weld's six robot parts, built by the whole wave (lane d: DoF d; coop_robot_row's scheme for
    // six rows at once): every row's Jacobian entry at the pivot, M^-1 J^T from the Jacobians
    // broadcast through LDS, and the parts stored in put_robot's layout; each weld lane then sums
    // its own row's den and rel in DoF order.  (Per lane, a weld row's robot_jac and K_ND^2 M^-1
    // product were the longest chain of the non-contact rows.)
    float (*WJ)[MAXD] = (float (*)[MAXD])&L.u.d.rn[1][0][0];     // [6][MAXD] J, then [6][MAXD] M^-1 J^T
    float (*WM)[MAXD] = WJ + 6;
    {
        const int d = lane;
        const unsigned am = gld(m.anc_mask + (link));
        const int wslot = nrow - 6;
        float j[6], mj[6];
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const v3 lin = r < 3 ? V(r == 0 ? 1.f : 0.f, r == 1 ? 1.f : 0.f, r == 2 ? 1.f : 0.f) : V(0, 0, 0);
            const v3 an = r < 3 ? V(0, 0, 0) : (r == 3 ? c0 : r == 4 ? c1 : c2);
            j[r] = d < MAXD ? jac_entry(m, L, am, d, pivA, lin, an) : 0.f;
            if (d < MAXD) WJ[r][d] = j[r];
        }
        SYNC();
#pragma unroll
        for (int r = 0; r < 6; r++) {
            mj[r] = minv_entry<0, K_ND>(L, WJ[r], d);         // (the weld's robot link: the robot block)
            if (d < MAXD) WM[r][d] = mj[r];
        }
        if (d < 16 * NDL) {
            const bool in = d < MAXD;
#pragma unroll
            for (int r = 0; r < 6; r++) {
                if (wslot + r < MAXNC) {
                    float2 v;
                    v.x = in ? j[r] : 0.f; v.y = in ? mj[r] : 0.f;
                    *(float2 *)(row_rob(m, rows, wslot + r) + (NDL == 2 ? 4 * (d & 15) + 2 * (d >> 4) : 2 * d)) = v;
                }
            }
        }
        SYNC();
    }
    if (kind == 0 || kind == 1 || kind == 2) {
        // J = +-e_dof: M^-1 J^T is a signed column of M^-1
        const float sg = kind == 1 ? -1.f : 1.f;
        float J[MAXD], MJ[MAXD];
#pragma unroll
        for (int d = 0; d < MAXD; d++) { J[d] = d == dof ? sg : 0.f; MJ[d] = sg * L.u.d.Minv[d][dof]; }
        const float den = L.u.d.Minv[dof][dof];
        const float inv = den > BT_DENOM_EPS ? 1.f / den : 1.f;
        const float rel = sg * L.vq[dof];
        float *w = row_rec(m, rows, lane);
        if (kind < 2) {
            put_hdr(w, 0, inv, (-pen * erp / dt - rel) * inv, 0.f, 100.f, lane);
        } else {
            const float q = L.st[S_Q + dof], cur = L.vq[dof];
            const float kp = L.st[S_KP + dof], kd = 1.f;
            const float desired = kp * (L.st[S_QTGT + dof] - q) / dt + cur + kd * (0.f - cur);
            const float mi = L.st[S_MAXIMP + dof];
            put_hdr(w, 0, inv, (desired - rel) * inv, -mi, mi, lane);
        }
        put_free_zero(w + 8); put_free_zero(w + 14);
        put_robot(row_rob(m, rows, lane), J, MJ);
    } else if (kind == 3) {
        v3 lin = V(0, 0, 0);
        float pos;
        v3 jbl, jba;
        if (fix < 3) {
            if (fix == 0) lin.x = 1.f; else if (fix == 1) lin.y = 1.f; else lin.z = 1.f;
            pos = dot(sub(pivA, pivB), lin);
            jbl = scl(lin, -1.f);
            jba = crs(sub(pivB, tb.p), jbl);
        } else {
            m3 rr;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) {
                    float t = 0.f;
                    for (int k = 0; k < 3; k++) t += FA.m[k][a] * FB.m[k][b];
                    rr.m[a][b] = t;
                }
#define ME(i) rr.m[(i) % 3][(i) / 3]
            v3 ang;
            const float fi = ME(2);
            if (fi < 1.f) {
                if (fi > -1.f) ang = V(atan2f(-ME(5), ME(8)), asinf(ME(2)), atan2f(-ME(1), ME(0)));
                else ang = V(-atan2f(ME(3), ME(4)), -1.5707963267948966f, 0.f);
            } else ang = V(atan2f(ME(3), ME(4)), 1.5707963267948966f, 0.f);
#undef ME
            const v3 an = fix == 3 ? c0 : (fix == 4 ? c1 : c2);
            pos = fix == 3 ? ang.x : fix == 4 ? ang.y : ang.z;
            jbl = V(0, 0, 0);
            jba = scl(an, -1.f);
        }
        float den = 0.f, rel = 0.f;
#pragma unroll
        for (int d = 0; d < MAXD; d++) { const float j = WJ[fix][d]; den = fmaf(j, WM[fix][d], den); rel = fmaf(j, L.vq[d], rel); }
#ifdef AVR_COOP_CHECK
        {
            float JA[MAXD], MA[MAXD];
            v3 l2 = V(0, 0, 0), a2 = V(0, 0, 0);
            if (fix < 3) { if (fix == 0) l2.x = 1.f; else if (fix == 1) l2.y = 1.f; else l2.z = 1.f; }
            else a2 = fix == 3 ? c0 : (fix == 4 ? c1 : c2);
            robot_jac(m, L, link, pivA, l2, a2, JA);
            minv_mul_blk<0, K_ND>(L, JA, MA);
            float d2 = 0.f, r2 = 0.f;
            for (int d = 0; d < MAXD; d++) { d2 += JA[d] * MA[d]; r2 += JA[d] * L.vq[d]; }
            int bad = -1;
            for (int d = 0; d < MAXD && bad < 0; d++)
                if (__float_as_int(JA[d]) != __float_as_int(WJ[fix][d]) || __float_as_int(MA[d]) != __float_as_int(WM[fix][d])) bad = d;
            if ((bad >= 0 || __float_as_int(d2) != __float_as_int(den) || __float_as_int(r2) != __float_as_int(rel)) && atomicAdd(&g_coop_check, 1) < 24) {
                const int d = bad < 0 ? 0 : bad;
                printf("weld mismatch fix %d den %a/%a rel %a/%a dof %d J %a/%a MJ %a/%a\n", fix, den, d2, rel, r2, bad, WJ[fix][d], JA[d], WM[fix][d], MA[d]);
            }
        }
#endif
        const float im = 1.f / gld(m.fb_mass + (fb));
        const v3 mbl = scl(jbl, im), mba = iinv_mul(L, fb, jba);
        den += dot(jbl, mbl) + dot(jba, mba);
        const float inv = den > BT_DENOM_EPS ? 1.f / den : 1.f;
        rel += free_dot(L, fb, jbl, jba);
        const float mi = m.fixed_max_imp;
        float *w = row_rec(m, rows, lane);
        put_hdr(w, own_mask(-1, fb), inv, (-pos * erp / dt - rel) * inv, -mi, mi, lane);
        put_free_zero(w + 8);
        put_free(L, fb, w + 14, jbl, jba);
    }
    if (nrow > MAXNC) { if (lane == 0) L.flags |= 16; nrow = MAXNC; }
    if (lane == 0) L.n_nc = nrow;
    return nrow;
}

AVR_DI void plane_space(v3 n, v3 &p, v3 &q) {
    if (fabsf(n.z) > 0.7071067811865475244f) {
        float a = n.y * n.y + n.z * n.z, k = 1.f / sqrtf(a);
        p = V(0, -n.z * k, n.y * k);
        q = V(a * k, -n.x * p.z, n.x * p.y);
    } else {
        float a = n.x * n.x + n.y * n.y, k = 1.f / sqrtf(a);
        p = V(-n.y * k, n.x * k, 0);
        q = V(-n.z * p.y, n.z * p.x, a * k);
    }
}

AVR_DI void body_endpoint(const KModel &m, const EnvLDS &L, int b, int &kind, int &idx) {
    int k = gld(m.body_kind + (b));
    kind = 0; idx = 0;
    if (k == AVR_BODY_ROBOT) { kind = 1; idx = gld(m.body_index + (b)); }
    else if (k == AVR_BODY_FREE) { kind = 2; idx = gld(m.body_index + (b)); }
    else if (k == AVR_BODY_HUMAN) {
        for (int c = 0; c < L.nla - m.nl; c++)     // head-chain link under 'tremor'
            if (m.hc_body[c] == b) { kind = 1; idx = m.nl + c; }
    }
}

// Contact rows: one lane per contact point; contact c owns rows n_nc + c (normal),
// n_nc + n_c + 2c + {0,1} (frictions along btPlaneSpace1 directions) and (K_TORSION, contacts
// whose rolling or spinning coefficient is positive, the t-th of them) n_nc + 3 n_c + 3t + {0,1,2}:
// the torsional rows -- spinning about the normal, rolling about the two friction directions;
// angular-only Jacobians, limits +-coefficient x normal impulse, no positional term
// (btMultiBodyConstraintSolver::addMultiBodyTorsionalFrictionConstraint [ext]).  Their
// coefficients combine the bodies' as btManifoldResult does (roll_A fric_B + roll_B fric_A, clamped
// to 10); a row whose coefficient is 0 (only one of the two positive) is a null record.  The normal
// record's 4th word (unused by the normal resolve) holds t + 1 (0: no torsional rows), so part B
// sweeps only the torsional rows that exist.  Robot parts: 3 slots per robot contact, 6 with
// torsional rows.

// btManifoldResult::calculateCombinedRollingFriction / SpinningFriction [ext]
AVR_DI float torsion_coeff(const float *c, const KModel &m, int ba, int bb) {
    const float x = gld(c + ba) * gld(m.body_friction + bb) + gld(c + bb) * gld(m.body_friction + ba);
    return fminf(fmaxf(x, -10.f), 10.f);
}
// A row's robot part built by the whole wave (lane d: DoF d) instead of by the contact's lane alone:
// the Jacobian entries (jac_entry), M^-1 J^T entry d from the Jacobian broadcast through LDS (the
// sums of minv_mul_blk / minv_mul_add_blk, in their order), den and rel summed over the DoFs in DoF
// order on every lane -- the per-lane builder's roundings, with the robot_jac + M^-1 product chain
// (~K_ND^2 dependent LDS reads and fmas on one lane) cut to ~K_ND.  An env whose contact rows
// hold few robot endpoints (FeedingJaco: one spoon or arm contact against the human, in a wave
// whose other lanes are done) no longer waits for the one lane that builds them.
// lA, lB: the articulated links of endpoints A, B (-1: not articulated); (den, rel) enter holding
// the free A endpoint's part (0 without one) and leave with the robot part added.
// The robot part on the contact's own lane: endpoint A's (articulated link lA, -1: none) Jacobian
// and M^-1 J^T, then endpoint B's (lB) added (minv_mul_add); (den, rel) enter holding the free A
// endpoint's part.  One pair of MAXD arrays live at a time.
AVR_DI void lane_robot_part(const KModel &m, const EnvLDS &L, int lA, int lB, v3 pa, v3 pb, v3 lin, v3 angA, float &den, float &rel,
                            float *J, float *MJ) {
    const v3 nd = scl(lin, -1.f), angB = scl(angA, -1.f);
    if (lA >= 0) {
        robot_jac(m, L, lA, pa, lin, angA, J);
        minv_mul_link(m, L, lA, J, MJ);
#pragma unroll
        for (int d = 0; d < MAXD; d++) { den = fmaf(J[d], MJ[d], den); rel = fmaf(J[d], L.vq[d], rel); }
        if (lB >= 0) {
            // both endpoints on the articulated system (a robot link against a human-chain link):
            // the second endpoint's part is added in registers (minv_mul_add); the read-back of
            // the first from memory cost ~60 us per sub-step (ScratchItch)
            float Jb[MAXD];
            robot_jac(m, L, lB, pb, nd, angB, Jb);
            minv_mul_add(m, L, lB, Jb, J, MJ, den, rel);
        }
    } else {
        robot_jac(m, L, lB, pb, nd, angB, J);
        minv_mul_link(m, L, lB, J, MJ);
#pragma unroll
        for (int d = 0; d < MAXD; d++) { den = fmaf(J[d], MJ[d], den); rel = fmaf(J[d], L.vq[d], rel); }
    }
}
#ifdef AVR_COOP_CHECK
// diagnostic build: the cooperative row against the per-lane one, bit for bit (device printf)
AVR_DI void coop_check(const KModel &m, const EnvLDS &L, const float *wr, int lA, int lB, v3 pa, v3 pb, v3 lin, v3 ang,
                       float den, float rel, float cden, float crel) {
    float J[MAXD], MJ[MAXD];
    lane_robot_part(m, L, lA, lB, pa, pb, lin, ang, den, rel, J, MJ);
    int bad = -1;
    for (int d = 0; d < MAXD && bad < 0; d++) {
        const float *q = wr + (NDL == 2 ? 4 * (d & 15) + 2 * (d >> 4) : 2 * d);
        if (__float_as_int(q[0]) != __float_as_int(J[d]) || __float_as_int(q[1]) != __float_as_int(MJ[d])) bad = d;
    }
    if (bad >= 0 || __float_as_int(den) != __float_as_int(cden) || __float_as_int(rel) != __float_as_int(crel)) {
        if (atomicAdd(&g_coop_check, 1) < 24) {
            const int d = bad < 0 ? 0 : bad;
            const float *q = wr + (NDL == 2 ? 4 * (d & 15) + 2 * (d >> 4) : 2 * d);
            printf("coop mismatch lA %d lB %d den %a/%a rel %a/%a dof %d J %a/%a MJ %a/%a\n", lA, lB, cden, den, crel, rel, bad,
                   q[0], J[d], q[1], MJ[d]);
        }
    }
}
#endif
#ifndef AVR_COOP_ROWS
#define AVR_COOP_ROWS 64     // build a contact-row pass's robot rows wave-cooperatively when at most this many lanes hold one
#endif
AVR_DI void coop_robot_row(const KModel &m, EnvLDS &L, float *X, float *wr, int lA, int lB, v3 pa, v3 pb, v3 lin, v3 ang,
                           float &den, float &rel) {
    const int d = lane_id();
    float *XJ = X, *XM = X + MAXD, *XJ2 = X + 2 * MAXD, *XM2 = X + 3 * MAXD;
    const bool fa = lA >= 0;
    const int lF = fa ? lA : lB;
    const v3 pF = fa ? pa : pb, linF = fa ? lin : scl(lin, -1.f), angF = fa ? ang : scl(ang, -1.f);
    const float jF = d < MAXD ? jac_entry(m, L, gld(m.anc_mask + (lF)), d, pF, linF, angF) : 0.f;
    if (d < MAXD) XJ[d] = jF;
    SYNC();
    float mF = lF < m.nl ? minv_entry<0, K_ND>(L, XJ, d) : minv_entry<K_ND, MAXD>(L, XJ, d);
    if (d < MAXD) XM[d] = mF;
    SYNC();
#pragma unroll
    for (int k = 0; k < MAXD; k++) { const float j = XJ[k]; den = fmaf(j, XM[k], den); rel = fmaf(j, L.vq[k], rel); }
    float J = jF;
    if (fa && lB >= 0) {                     // the second articulated endpoint (minv_mul_add)
        const float jS = d < MAXD ? jac_entry(m, L, gld(m.anc_mask + (lB)), d, pb, scl(lin, -1.f), scl(ang, -1.f)) : 0.f;
        if (d < MAXD) XJ2[d] = jS;
        SYNC();
        const bool rs = lB < m.nl;
        const float sS = rs ? minv_entry<0, K_ND>(L, XJ2, d) : minv_entry<K_ND, MAXD>(L, XJ2, d);
        if (d < MAXD) XM2[d] = sS;
        SYNC();
        if (rs) {
#pragma unroll
            for (int i = 0; i < K_ND; i++) { const float x = XJ2[i]; den = fmaf(x, XM2[i], den); rel = fmaf(x, L.vq[i], rel); }
        } else {
#pragma unroll
            for (int i = K_ND; i < MAXD; i++) { const float x = XJ2[i]; den = fmaf(x, XM2[i], den); rel = fmaf(x, L.vq[i], rel); }
        }
        if (rs ? d < K_ND : d >= K_ND && d < MAXD) mF += sS;
        J = jF + jS;
    }
    // put_robot's layout, one (J, M^-1 J^T) pair per lane
    if (d < 16 * NDL) {
        const bool in = d < MAXD;
        float2 v;
        v.x = in ? J : 0.f; v.y = in ? mF : 0.f;
        *(float2 *)(wr + (NDL == 2 ? 4 * (d & 15) + 2 * (d >> 4) : 2 * d)) = v;
    }
    SYNC();                                  // (X is reused by the next row)
}
static_assert(sizeof(((EnvLDS *)0)->u.d.rn) >= 4 * MAXD * sizeof(float), "cooperative row scratch");
static_assert(sizeof(((EnvLDS *)0)->u.d.rn) - sizeof(((EnvLDS *)0)->u.d.rn[0]) >= 12 * MAXD * sizeof(float), "weld row scratch");

AVR_DI int build_contact_rows(const KModel &m, EnvLDS &L, const float *gcp, float *rows, int n_nc, float dt) {
    const int lane = lane_id();
    const int ncp = (int)L.st[S_TASK + T_NCP];
    const float erp = m.erp;
    int nrob = n_nc;                                 // robot parts: nc rows first, then 3 (6) per robot contact
    int nt = 0;                                      // contacts with torsional rows so far
    for (int base = 0; base < ncp; base += 64) {
        const int i = base + lane;
        const bool act = i < ncp;
        int kA = 0, iA = 0, kB = 0, iB = 0;
        const float *c = gcp + AVR_CP_WORDS * (act ? i : 0);
        int sa = (int)c[AVR_CP_SA], sb = (int)c[AVR_CP_SB];
        int ba = gld(m.shape_body + (sa)), bb = gld(m.shape_body + (sb));
        body_endpoint(m, L, ba, kA, iA);
        body_endpoint(m, L, bb, kB, iB);
        const bool rob = kA == 1 || kB == 1;
#if K_TORSION
        const float spin = torsion_coeff(m.body_spinning, m, ba, bb), roll = torsion_coeff(m.body_rolling, m, ba, bb);
        const bool trs = act && (spin > 0.f || roll > 0.f);
#else
        constexpr bool trs = false;
#endif
        const int nrow = trs ? 6 : 3;
        // robot slots: an inclusive scan of each lane's slot count
        const int wgt = act && rob ? nrow : 0;
        int incl = wgt;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const int slot0 = nrob + incl - wgt;
        nrob += __shfl(incl, 63, 64);
        int ttot;
        const int ti = nt + ballot_prefix(trs, &ttot);
        nt += ttot;
        // (inactive lanes run on contact 0's data, ncp > 0 here: every lane takes part in the
        // wave-cooperative robot rows)
        tf ta = ldtf(L.btf[ba]), tb = ldtf(L.btf[bb]);
        v3 pa = tfpt(ta, ld3(c + AVR_CP_LA)), pb = tfpt(tb, ld3(c + AVR_CP_LB));
        v3 n = ld3(c + AVR_CP_N);
        v3 t1, t2;
        plane_space(n, t1, t2);
        v3 rA = sub(pa, ta.p), rB = sub(pb, tb.p);
        float fric = fminf(gld(m.body_friction + (ba)) * gld(m.body_friction + (bb)), 10.f);
        const int info = own_mask(kA == 2 ? iA : -1, kB == 2 ? iB : -1);
        float imA = kA == 2 ? 1.f / gld(m.fb_mass + (iA)) : 0.f, imB = kB == 2 ? 1.f / gld(m.fb_mass + (iB)) : 0.f;
        float rlim1 = 0.f;                           // the first friction row's residual limit
        const int kmax = __ballot(act && trs) ? 6 : 3;
#pragma unroll 1
        for (int k = 0; k < kmax; k++) {
            bool live = act && k < nrow;
            const int kd = k < 3 ? k : k - 3;
            v3 dir = kd == 0 ? n : (kd == 1 ? t1 : t2);
            const int slot = rob ? slot0 + k : -1;
            float *w = row_crec(rows, k == 0 ? i : k < 3 ? ncp + 2 * i + (k - 1) : 3 * ncp + 3 * ti + (k - 3));
            float den = 0.f, rel = 0.f;
#if K_TORSION
            // torsional rows (k >= 3): angular axis dir, no linear part
            const bool tor = k >= 3;
            const float tcoef = k == 3 ? spin : roll;
            if (live && tor && !(tcoef > 0.f)) {  // null record: no endpoint, inv = rhs = coefficient = 0
#pragma unroll
                for (int q = 0; q < CRW; q++) w[q] = 0.f;
                live = false;
            }
            const v3 lin = tor ? V(0, 0, 0) : dir, angA = tor ? dir : V(0, 0, 0);
#else
            constexpr bool tor = false;
            const float tcoef = 0.f;
            const v3 lin = dir, angA = V(0, 0, 0);
#endif
            // the robot part (J, M^-1 J^T) goes to the row buffer endpoint by endpoint (the second
            // robot endpoint, if any, adds to the first's): one pair of MAXD arrays live at a time
            float *wr = rob ? row_rob(m, rows, slot) : nullptr;
            const v3 nd = scl(lin, -1.f), angB = scl(angA, -1.f);
            if (live) {
                if (kA == 2) {
                    v3 ja = add(crs(rA, lin), angA), ma = iinv_mul(L, iA, ja), ml = scl(lin, imA);
                    den += dot(lin, ml) + dot(ja, ma);
                    rel += free_dot(L, iA, lin, ja);
                    put_free(L, iA, w + 4, lin, ja);
                } else put_free_zero(w + 4);
            }
            const unsigned long long rq = __ballot(live && rob);
            if (rq && __popcll(rq) <= AVR_COOP_ROWS) {
                float *X = &L.u.d.rn[0][0][0];       // (the RNEA temporaries are dead)
                for (unsigned long long q = rq; q; q &= q - 1ull) {
                    const int src = __builtin_ctzll(q);
                    const int lA = __builtin_amdgcn_readlane(kA == 1 ? iA : -1, src), lB = __builtin_amdgcn_readlane(kB == 1 ? iB : -1, src);
                    const int sl = __builtin_amdgcn_readlane(slot, src);
                    const v3 spa = V(rdl_f(pa.x, src), rdl_f(pa.y, src), rdl_f(pa.z, src));
                    const v3 spb = V(rdl_f(pb.x, src), rdl_f(pb.y, src), rdl_f(pb.z, src));
                    const v3 sln = V(rdl_f(lin.x, src), rdl_f(lin.y, src), rdl_f(lin.z, src));
                    const v3 san = V(rdl_f(angA.x, src), rdl_f(angA.y, src), rdl_f(angA.z, src));
                    float cden = rdl_f(den, src), crel = rdl_f(rel, src);
                    coop_robot_row(m, L, X, row_rob(m, rows, sl), lA, lB, spa, spb, sln, san, cden, crel);
#ifdef AVR_COOP_CHECK
                    if (lane == src) coop_check(m, L, row_rob(m, rows, sl), lA, lB, pa, pb, lin, angA, den, rel, cden, crel);
#endif
                    if (lane == src) { den = cden; rel = crel; }
                }
            } else if (live && rob) {
                float J[MAXD], MJ[MAXD];
                lane_robot_part(m, L, kA == 1 ? iA : -1, kB == 1 ? iB : -1, pa, pb, lin, angA, den, rel, J, MJ);
                put_robot(wr, J, MJ);
            }
            if (!live) continue;
            if (kB == 2) {
                v3 jb = add(crs(rB, nd), angB), mb = iinv_mul(L, iB, jb), ml = scl(nd, imB);
                den += dot(nd, ml) + dot(jb, mb);
                rel += free_dot(L, iB, nd, jb);
                put_free(L, iB, w + 10, nd, jb);
            } else put_free_zero(w + 10);
            float inv = den > BT_DENOM_EPS ? 1.f / den : 1.f;
            float rhs = -rel * inv;
            if (k == 0) {
                float pen = c[AVR_CP_DIST];
                float velerr = -rel, poserr = 0.f;
                if (pen > 0.f) velerr -= pen / dt;
                else poserr = -pen * erp / dt;
                rhs = (poserr + velerr) * inv;
            }
            const float rlim = BT_RESIDUAL_SQRT * inv;
            const int tword = K_TORSION && k == 0 && trs ? (ti + 1) << 2 : 0;    // (K_TORSION: MAXF 1, own bits 0-1)
            w[0] = k == 2 ? rlim1 : __int_as_float(info | tword | ((slot + 1) << CI_SLOT)); w[1] = inv; w[2] = rhs;
            w[3] = tor ? tcoef : k == 1 ? fric : rlim;
            if (k == 1) rlim1 = rlim;
#if B4_FPAIR
            if (k == 2) {
                // the friction unit's coupling c = J_2 M^-1 J_1^T (its second row's 4th header word,
                // where the first row keeps the friction coefficient): part B resolves the second
                // row with J_2.dv + delta_1 c instead of re-reading the velocities row 1 changed.
                // In part B's mass-normalised coordinates: the two rows' free parts dotted, plus the
                // second row's J against the first's M^-1 J^T (this lane's own stores, read back)
                const float *w1 = row_crec(rows, ncp + 2 * i);
                float cc = 0.f;
#pragma unroll
                for (int q = 4; q < CRW; q++) cc = fmaf(w1[q], w[q], cc);
                if (rob) {
                    const float *r1 = row_rob(m, rows, slot0 + 1), *r2 = row_rob(m, rows, slot0 + 2);
#pragma unroll
                    for (int q = 0; q < 16 * NDL; q++) cc = fmaf(r2[2 * q], r1[2 * q + 1], cc);
                }
                w[3] = cc;
            }
#endif
        }
    }
    if (lane == 0) { L.n_c = ncp; L.n_t = nt; }
    return nrob;
}

// --------------------------------------------------------------------------- one sub-step
// A sub-step is four kernels: avr_substep_pairs_kernel (forward kinematics, body frames,
// broadphase, shape-pair list), avr_narrowphase_kernel (one lane per listed shape pair, across
// all envs), avr_substep_a_kernel (the rare pairs that need the wave-cooperative narrowphase,
// then manifold update, unconstrained velocities, constraint rows) and avr_substep_b4_kernel
// (PGS + integration).  What crosses the kernel boundaries goes
// through the per-env collision scratch (m.cscr), the workspace (m.ws) and the row buffer
// (m.rows).
AVR_DI bool substep_a(const KModel &m, EnvLDS &L, float dt, float *gst, float *ws, float *rows, const float *cs) {
    const int lane = lane_id();
    PROF_START(ps);
    // (the body and link frames from the pair kernel and the previous contact pool were staged
    // by load_a)
    PROF_STOP(0, ps);
    collide_contacts(m, L, cs, gst + S_CP);
    PROF_STOP(13, ps);
#ifdef AVR_LDS_POISON   // (the dynamics overlay the contact update's storage: re-poison it)
    for (int i = lane; i < (int)(sizeof(L.u) / 4); i += 64) ((float *)&L.u)[i] = __int_as_float(-1);
    SYNC();
#endif
    // unconstrained velocities
    bool ok = robot_mass_matrix(m, L);
    PROF_START(pbias);
    robot_bias(m, L);
    PROF_STOP(27, pbias);
    if (lane < MAXD) {                      // qdd = -M^-1 h, one lane per DoF
        float s = 0.f;
        for (int k = 0; k < L.nda; k++) s -= L.u.d.Minv[lane][k] * L.h[k];
        L.qdd[lane] = s;
    }
    SYNC();
    const float vmax = m.max_vel;
    // every DoF slot is written: the row builders sum J[d] * vq[d] over all MAXD slots, and a
    // slot left over from another kernel's LDS (NaN bit patterns included) would turn those
    // zero-Jacobian terms into NaN (0 * NaN) -- inactive slots (d >= nda) hold 0
    if (lane < MAXD) {
        const float v = L.st[S_QD + lane] + dt * L.qdd[lane];
        L.vq[lane] = lane < L.nda ? clampf(v, -vmax, vmax) : 0.f;
    }
    const float k1l = m.lin_damp, k1a = m.ang_damp;
    if (lane < m.nf) {
        int f = lane;
        const float *fb = L.st + S_FREE + AVR_FB_WORDS * f;
        v3 v = ld3(fb + 7), om = ld3(fb + 10);
        qt q = ldq(fb + 3);
        float mass = gld(m.fb_mass + (f));
        v3 I = gld3(m.fb_inertia + 4 * f), g = gld3(m.fb_gravity + 4 * f);
        v3 Iw = inertia_mul(q, I, om);
        v3 F = sub(scl(g, mass), scl(v, mass * (k1l + k1l * len(v))));
        v3 T = sub(scl(Iw, -(k1a + k1a * len(om))), crs(om, Iw));
        v3 nv = add(v, scl(F, dt / mass));
        v3 nw = add(om, scl(inertia_inv_mul(q, I, T), dt));
        st3(L.fv[f], clamp3(nv, vmax));
        st3(L.fw[f], clamp3(nw, vmax));
        // world inverse inertia R diag(1/I) R^T
        m3 R = qmat(q);
        float inv[3] = {I.x > 0.f ? 1.f / I.x : 0.f, I.y > 0.f ? 1.f / I.y : 0.f, I.z > 0.f ? 1.f / I.z : 0.f};
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) L.Iinv[f][3 * a + b] = R.m[a][0] * inv[0] * R.m[b][0] + R.m[a][1] * inv[1] * R.m[b][1] + R.m[a][2] * inv[2] * R.m[b][2];
        L.gsc[f][0] = 1.f / sqrtf(mass);
        L.gsc[f][1] = sqrtf(inv[0]); L.gsc[f][2] = sqrtf(inv[1]); L.gsc[f][3] = sqrtf(inv[2]);
    }
    SYNC();
    PROF_STOP(6, ps);
    const int n_nc = build_noncontact_rows(m, L, rows, dt);
    PROF_STOP(7, ps);
    const int n_rob = build_contact_rows(m, L, gst + S_CP, rows, n_nc, dt);
    SYNC();
    PROF_STOP(8, ps);
    // hand-over to part B
    if (lane == 0) {
        ws[WS_NNC] = __int_as_float(n_nc); ws[WS_NC] = __int_as_float(L.n_c); ws[WS_NROB] = __int_as_float(n_rob);
        ws[WS_NT] = __int_as_float(K_TORSION ? L.n_t : 0);
    }
    if (lane < MAXD) ws[WS_VQ + lane] = lane < L.nda ? L.vq[lane] : 0.f;
    if (lane < m.nf) {
        st3(ws + WS_FV + 4 * lane, ld3(L.fv[lane]));
        st3(ws + WS_FW + 4 * lane, ld3(L.fw[lane]));
    }
    return ok;
}

// --------------------------------------------------------------------------- task glue
#if AVR_TASK == AVR_TASK_FEEDING
AVR_DI void mouth_target(const KModel &m, EnvLDS &L) {
    tf t = ldtf(L.st + S_HUMAN + 7 * m.head_slot);
    int g = (int)L.st[S_TASK + T_GENDER];
    v3 p = tfpt(t, gld3(m.mouth[g]));
    SYNC();
    if (lane_id() == 0) st3(L.st + S_TASK + T_TARGET, p);
    SYNC();
}

// sum of normalForce over contact points whose body pair satisfies `sel`, and their count
// sel: 0 robot-human, 1 spoon-human, 2 body X vs body Y, 3 body X vs human
AVR_DI float contact_sum(const KModel &m, const EnvLDS &L, const float *gcp, int sel, int X, int Y, int &count) {
    const int lane = lane_id();
    int n = (int)L.st[S_TASK + T_NCP];
    float s = 0.f;
    int c = 0;
    for (int i = lane; i < n; i += 64) {
        const float *cp = gcp + AVR_CP_WORDS * i;
        int ba = gld(m.shape_body + ((int)cp[AVR_CP_SA])), bb = gld(m.shape_body + ((int)cp[AVR_CP_SB]));
        int ka = gld(m.body_kind + (ba)), kb = gld(m.body_kind + (bb));
        bool hit;
        if (sel == 0) hit = (ka == AVR_BODY_ROBOT && kb == AVR_BODY_HUMAN) || (kb == AVR_BODY_ROBOT && ka == AVR_BODY_HUMAN);
        else if (sel == 1) hit = (ba == m.spoon_body && kb == AVR_BODY_HUMAN) || (bb == m.spoon_body && ka == AVR_BODY_HUMAN);
        else if (sel == 2) hit = (ba == X && bb == Y) || (ba == Y && bb == X);
        else hit = (ba == X && kb == AVR_BODY_HUMAN) || (bb == X && ka == AVR_BODY_HUMAN);
        if (hit) { s += cp[AVR_CP_IMP] / m.time_step; c++; }
    }
    // deterministic reduction: sequential order over lanes via shuffles
    float tot = 0.f;
    int ctot = 0;
    for (int k = 0; k < 64; k++) { tot += __shfl(s, k, 64); ctot += __shfl(c, k, 64); }
    count = ctot;
    return tot;
}

AVR_DI void observe(const KModel &m, EnvLDS &L, float spoon_force, float *obs_out) {
    robot_fk(m, L);
    if (lane_id() == 0) {
        v3 torso = ld3(L.cm[m.torso_link]);
        const float *sp = L.st + S_FREE + AVR_FB_WORDS * m.spoon_free;
        v3 spos = ld3(sp);
        v3 tgt = ld3(L.st + S_TASK + T_TARGET);
        const float *h = L.st + S_HUMAN + 7 * m.head_slot;
        int k = 0;
        v3 a = sub(spos, torso);
        obs_out[k++] = a.x; obs_out[k++] = a.y; obs_out[k++] = a.z;
        for (int i = 0; i < 4; i++) obs_out[k++] = sp[3 + i];
        a = sub(spos, tgt);
        obs_out[k++] = a.x; obs_out[k++] = a.y; obs_out[k++] = a.z;
        for (int i = 0; i < m.n_arm; i++) obs_out[k++] = L.st[S_Q + m.arm_dofs[i]];
        a = sub(ld3(h), torso);
        obs_out[k++] = a.x; obs_out[k++] = a.y; obs_out[k++] = a.z;
        for (int i = 0; i < 4; i++) obs_out[k++] = h[3 + i];
        obs_out[k++] = spoon_force;
    }
}

#endif  // AVR_TASK_FEEDING

// Philox4x32-10 (Salmon et al. 2011): counter (env, step, j, 0), key (seed lo, seed hi)
// (philox4x32_10, philox_action: avr_math.h)

enum { MODE_STEP = 0, MODE_STEP_RANDOM = 1, MODE_SETTLE = 2, MODE_SUBSTEP = 3 };

// Occupancy request: waves per SIMD the register allocator must leave room for.
#ifndef AVR_WAVES_PER_EU
#define AVR_WAVES_PER_EU 1
#endif
#define AVR_KATTR __attribute__((amdgpu_waves_per_eu(AVR_WAVES_PER_EU)))

#define AVR_ENV_GUARD()                      \
    const int env = env0 + blockIdx.x;       \
    if (env >= n_envs) return;               \
    if (mask && !mask[env]) return;          \
    const KModel &m = *mp;                   \
    (void)m

#if defined(AVR_PROF) || defined(AVR_WAVETIME)
AVR_DI int xcc_id() {   // XCD of the executing CU (HW_REG_XCC_ID, id 20, bits 3:0)
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 0xf);
}
#endif

AVR_DI float *env_ws(const KModel &m, int env) { return m.ws + (size_t)env * WS_WORDS; }
AVR_DI float *env_rows(const KModel &m, int env) { return m.rows + (size_t)env * (size_t)m.rowstride; }

AVR_DI bool env_hdyn(const KModel &m, const float *gst) { return m.hc_n > 0 && gst[S_TASK + T_HDYN] != 0.f; }

// Global -> LDS copies in two halves: g2r issues a lane's loads of words lane, lane + 64, ...
// (NB of them, indices clamped into [0, n), so every load is unconditional), r2l stores them.  A
// plain strided copy loop waits for each load before its store -- one memory round trip per 64
// words -- where the loads of several g2r calls placed ahead of their r2l calls share one.
template <int NB>
AVR_DI void g2r(float (&t)[NB], const float *src, int n) {
    const int lane = lane_id(), l = max(n - 1, 0);
#pragma unroll
    for (int q = 0; q < NB; q++) t[q] = gld(src + min(lane + 64 * q, l));
}
template <int NB>
AVR_DI void r2l(float *dst, const float (&t)[NB], int n) {
    const int lane = lane_id();
#pragma unroll
    for (int q = 0; q < NB; q++)
        if (lane + 64 * q < n) dst[lane + 64 * q] = t[q];
}
#define NB_OF(words) (((words) + 63) / 64)

template <class LT>
AVR_DI void poison_lds(LT &L) {
#ifdef AVR_LDS_POISON   // diagnostic: NaN-fill the env's LDS block so that a read of a word this
                        // kernel did not write shows up (tools/gpu_poison.sh)
    for (int i = lane_id(); i < (int)(sizeof(LT) / 4); i += 64) ((float *)&L)[i] = __int_as_float(-1);
    SYNC();
#else
    (void)L;
#endif
}

template <class LT>
AVR_DI void load_state(const KModel &m, LT &L, const float *gst) {
    const int lane = lane_id();
    poison_lds(L);
    float ts[NB_OF(S_CP)];
    g2r(ts, gst, S_CP);
    r2l(L.st, ts, S_CP);
    if (lane == 0) {
        L.flags = 0;
        L.gender = (int)gst[S_TASK + T_GENDER];
        const bool hd = env_hdyn(m, gst);
        L.nla = hd ? m.nla : m.nl;
        L.nda = hd ? m.nd + m.hc_n : m.nd;
    }
#ifdef AVR_PROF
    if (lane < AVR_PROF_SLOTS) L.prof[lane] = 0;
#endif
    SYNC();
}

// kernel a's inputs -- the state words, the pair kernel's body and link frames, the previous
// contact pool -- with every load in flight before the first LDS store
AVR_DI void load_a(const KModel &m, EnvLDS &L, const float *gst, const float *cs) {
    const int lane = lane_id();
    poison_lds(L);
    const int nold = (int)gst[S_TASK + T_NCP];
    const bool hd = env_hdyn(m, gst);
    const int nla = hd ? m.nla : m.nl;
    float ts[NB_OF(S_CP)], tb[NB_OF(MAXB * 8)], tc[NB_OF(MAXL * 8)], tx[NB_OF(MAXL * 4)], to[NB_OF(MAXL * 4)];
    float tp[NB_OF(K_MAX_CONTACTS * AVR_CP_WORDS)];
    g2r(ts, gst, S_CP);
    g2r(tb, cs + CS_BTF, m.nb * 8);
    g2r(tc, cs + CS_CM, nla * 8);
    g2r(tx, cs + CS_AX, nla * 4);
    g2r(to, cs + CS_ORG, nla * 4);
    g2r(tp, gst + S_CP, nold * AVR_CP_WORDS);
    r2l(L.st, ts, S_CP);
    r2l(&L.btf[0][0], tb, m.nb * 8);
    r2l(&L.cm[0][0], tc, nla * 8);
    r2l(&L.ax[0][0], tx, nla * 4);
    r2l(&L.org[0][0], to, nla * 4);
    r2l(L.u.k.ocp, tp, nold * AVR_CP_WORDS);
    if (lane == 0) {
        L.flags = 0;
        L.gender = (int)L.st[S_TASK + T_GENDER];
        L.nla = nla;
        L.nda = hd ? m.nd + m.hc_n : m.nd;
    }
#ifdef AVR_PROF
    if (lane < AVR_PROF_SLOTS) L.prof[lane] = 0;
#endif
    SYNC();
}

template <class LT>
AVR_DI void prof_flush(const KModel &m, LT &L, int env) {
#ifdef AVR_PROF
    SYNC();
    if (m.prof && lane_id() < AVR_PROF_SLOTS) m.prof[(size_t)env * AVR_PROF_SLOTS + lane_id()] += L.prof[lane_id()];
#else
    (void)m; (void)L; (void)env;
#endif
}

#if AVR_TASK == AVR_TASK_FEEDING
// take_step (env.py:274-337): clip, scale, 5x limit-respecting accumulation, motor targets.
// One thread per env.
__global__ __launch_bounds__(64) void avr_take_step_kernel(const KModel *__restrict__ mp, float *__restrict__ state, const float *__restrict__ act,
                                                           const unsigned char *__restrict__ mask, int mode, long long t, int env0, int n_envs) {
    // XCD-consistent: lane l of block b takes env e - env0 = 512 (b / 8) + (b % 8) + 8 l, which
    // part A runs on the same XCD (see avr_substep_b4_kernel)
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
        asq += a_raw * a_raw;                    // reward_action uses the caller's action (feeding.py:69)
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
    if (env_hdyn(m, st)) {
        // tremor (env.py:327-337): targets target_human_joint_positions + human_tremors with the
        // tremor's sign alternating with self.iteration, gains human_gains, forces human_forces
        // (x human_strength = 1: 'tremor' is not 'weakness')
        const float sg = ((int)st[S_TASK + T_ITER] & 1) ? -1.f : 1.f;
        for (int c = 0; c < m.hc_n; c++) {
            const int d = m.nd + c;
            st[S_QTGT + d] = st[S_HCH + c] + st[S_HCH + K_HC_N + c] * sg;
            st[S_KP + d] = m.human_gain;
            st[S_MAXIMP + d] = m.human_force * m.time_step;
        }
    }
    ws[WS_ASQ] = asq;
}

#endif  // AVR_TASK_FEEDING

// Diagnostic wave timeline (-DAVR_WAVETIME builds only): global 100 MHz stamps at the start and
// end of every wave of the last A / B launch, [2][n_envs][2] u64 in m.prof (tools/wavetime.py).
#ifdef AVR_WAVETIME
#define WT_START() const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime()
#define WT_END(k)                                                                                   \
    do {                                                                                            \
        const unsigned long long wt1 = __builtin_amdgcn_s_memrealtime();                            \
        if (m.prof && lane_id() == 0) {                                                             \
            m.prof[((size_t)(k) * n_envs + env) * 2] = wt0;                                         \
            m.prof[((size_t)(k) * n_envs + env) * 2 + 1] = wt1;                                     \
        }                                                                                           \
    } while (0)
#else
#define WT_START() (void)0
#define WT_END(k) (void)0
#endif

// Sub-step part A1: one 64-lane block per env -- forward kinematics, body frames, broadphase,
// shape-pair list (collide_pairs) into the env's collision scratch.
AVR_DI void pairs_env(const KModel &m, PairsLDS &L, float *__restrict__ state, int env) {
    float *gst = state + (size_t)env * K_STATE_WORDS;
    // the packed shape info, staged in LDS for the pair enumeration (loads issued first, their
    // LDS stores after the kinematics)
    int si[MAXSH / 64];
#pragma unroll
    for (int q = 0; q < MAXSH / 64; q++) {
        const int s = lane_id() + 64 * q;
        si[q] = s < m.ns ? gld(m.shape_info + (s)) : 0;
    }
    load_state(m, L, gst);
    PROF_START(ps);
    robot_fk(m, L);
    PROF_STOP(0, ps);
#pragma unroll
    for (int q = 0; q < MAXSH / 64; q++) L.sinfo[lane_id() + 64 * q] = (unsigned short)si[q];
    float *cs = env_cs(m, env);
    for (int i = lane_id(); i < L.nla * 8; i += 64) cs[CS_CM + i] = (&L.cm[0][0])[i];
    for (int i = lane_id(); i < L.nla * 4; i += 64) { cs[CS_AX + i] = (&L.ax[0][0])[i]; cs[CS_ORG + i] = (&L.org[0][0])[i]; }
    collide_pairs(m, L, cs);
    prof_flush(m, L, env);
}

__global__ __launch_bounds__(64) AVR_KATTR void avr_substep_pairs_kernel(const KModel *__restrict__ mp, float *__restrict__ state,
                                                                         const unsigned char *__restrict__ mask, int env0, int n_envs) {
    __shared__ PairsLDS L;
    AVR_ENV_GUARD();
    pairs_env(m, L, state, env);
}

// Sphere against convex hull (most of the scene's shape pairs: food against the spoon's and the
// bowl's VHACD pieces): the GJK of narrowphase() restated for a point core -- the sphere's
// support point is its centre, so the simplex keeps only the Minkowski vertices and the hull's
// support points -- with the same iteration, tests and closest-point sums.  A lane works one
// pair at a time; a lane whose pair finishes takes the next pair of the list, so a wave runs
// the list's total iteration count rather than 64-lane maxima.
struct PH {
    int k;                  // pair index
    bool sw;                // the sphere is shape B of the pair
    v3 c;                   // sphere centre (its core)
    WShape H;               // the hull
    float ma, mb, thr, maxd2, prev;
    int it;
    v3 v;
    float lam[4];
    SimplexP S;
};

// (selects of values, never of lvalues: a select between two addresses keeps the simplex in
// scratch memory)
AVR_DI v3 sel3(bool c, v3 a, v3 b) { return V(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
AVR_DI WShape selw(bool c, const WShape &a, const WShape &b) {
    WShape r;
    r.kind = c ? a.kind : b.kind; r.nv = c ? a.nv : b.nv; r.vs = c ? a.vs : b.vs; r.tab = c ? a.tab : b.tab;
    r.t.p = sel3(c, a.t.p, b.t.p);
    r.t.q = Q(c ? a.t.q.x : b.t.q.x, c ? a.t.q.y : b.t.q.y, c ? a.t.q.z : b.t.q.z, c ? a.t.q.w : b.t.q.w);
    r.margin = c ? a.margin : b.margin;
    r.he = sel3(c, a.he, b.he);
    return r;
}

// list entry e: (k | ba << 16 | bb << 24, sa | sb << 16)
AVR_DI int2 np_entry(const float *cs, int l) {
    const float2 e = ((const float2 *)(cs + l))[0];
    return make_int2(__float_as_int(e.x), __float_as_int(e.y));
}

AVR_DI void ph_init(const KModel &m, const float *btf, int2 e, PH &P) {
    const int sa = e.y & 0xffff, sb = e.y >> 16;
    const int ba = (e.x >> 16) & 0xff, bb = (e.x >> 24) & 0xff;
    P.k = e.x & 0xffff;
    P.thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
    const WShape A = make_wshape(m, sa, ldtf(btf + 8 * ba)), B = make_wshape(m, sb, ldtf(btf + 8 * bb));
    P.sw = A.kind != AVR_SPHERE;
    P.c = sel3(P.sw, B.t.p, A.t.p);
    P.H = selw(P.sw, A, B);
    P.ma = A.margin;
    P.mb = B.margin;
    const float maxd = P.ma + P.mb + P.thr;
    P.maxd2 = maxd * maxd;
    P.v = sub(A.t.p, B.t.p);
    if (len2(P.v) < 1e-20f) P.v = V(1, 0, 0);
    P.S.n = 0;
    P.prev = BIGF;
    P.it = 0;
    P.lam[0] = 1.f; P.lam[1] = P.lam[2] = P.lam[3] = 0.f;
}

// one GJK iteration; true when the pair is finished, with its narrowphase result (rc 0 no
// contact, 1 contact, 2 cooperative path: penetrating cores need EPA, or the iteration cap)
AVR_DI bool ph_step(const KModel &m, PH &P, int &rc, v3 &nB, v3 &pB, float &dist) {
    const v3 h = support<false>(m, P.H, sel3(P.sw, scl(P.v, -1.f), P.v));
    const v3 sa = sel3(P.sw, h, P.c), sb = sel3(P.sw, P.c, h);
    const v3 wv = sub(sa, sb);
    const float vv = len2(P.v), vw = dot(P.v, wv);
    if (vw > 0.f && vw * vw > vv * P.maxd2) { rc = 0; return true; }       // GJK_FAR
    bool dup = false;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < P.S.n && P.S.w[k].x == wv.x && P.S.w[k].y == wv.y && P.S.w[k].z == wv.z) dup = true;
    bool conv = (dup && P.S.n > 0) || (P.S.n > 0 && vv - vw <= GJK_REL_EPS * vv);
    if (!conv) {
#pragma unroll
        for (int k = 0; k < 4; k++) {       // (value selects: a store at a computed slot would keep the simplex in scratch)
            P.S.w[k] = sel3(k == P.S.n, wv, P.S.w[k]);
            P.S.h[k] = sel3(k == P.S.n, h, P.S.h[k]);
        }
        P.S.n++;
        v3 nv;
        if (simplex_closest(P.S, nv, P.lam)) { rc = 2; return true; }      // penetrating
        const float nvv = len2(nv);
        if (nvv < 1e-14f * (1.f + len2(wv))) { rc = 2; return true; }     // penetrating
        if (nvv >= P.prev) { P.v = nv; conv = true; }
        else {
            P.prev = nvv;
            P.v = nv;
            if (++P.it >= GJK_MAX_IT) { rc = 2; return true; }            // unfinished
            return false;
        }
    }
    // separated: closest points from the simplex weights (as gjk())
    v3 a = V(0, 0, 0), b = V(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < P.S.n) {
            a = add(a, scl(sel3(P.sw, P.S.h[k], P.c), P.lam[k]));
            b = add(b, scl(sel3(P.sw, P.c, P.S.h[k]), P.lam[k]));
        }
    const float cd = len(sub(a, b));
    if (!(cd > 1e-9f)) { rc = 2; return true; }
    const v3 n = scl(sub(a, b), 1.f / cd);
    const float d = cd - P.ma - P.mb;
    if (d > P.thr) { rc = 0; return true; }
    nB = n;
    pB = add(b, scl(n, P.mb));
    dist = d;
    rc = 1;
    return true;
}

AVR_DI void np_store(float *cs, int k, int rc, v3 nB, v3 pB, float d) {
    float4 *o = (float4 *)(cs + CS_RES) + 2 * k;
    o[0] = make_float4(__int_as_float(rc), nB.x, nB.y, nB.z);
    o[1] = make_float4(pB.x, pB.y, pB.z, d);
    if (rc == 2 || rc == 4) cs[CS_COOP] = 1.f;      // (every writer stores the same value)
}

// the listed pairs (n of them) that the lane path left to the wave-cooperative narrowphase (rc 2:
// a big hull without a support table, penetrating cores that need EPA, the lane iteration cap;
// rc 4: a lane GJK that stalled with an open duality gap, rerun in double -- gjk_coop_d): the
// whole wave runs narrowphase<true> on each, E = the env's EPA buffer
//
// EPA budget (cap): an env whose penetrating hull pairs needed more than AVR_COOP_CAP EPAs in
// each of its last AVR_COOP_PERSIST sub-steps (T_COOPN counts them) gets at most AVR_COOP_CAP per
// sub-step from then on -- an arm driven into the wheelchair's hulls produced 21 per sub-step,
// ~1.3 ms of one wave that every env of the launch waited for.  The pairs are visited from a
// rotating start (rot: the env's counter, restarted every gym step); once the budget is spent a
// penetrating pair reports no new point this sub-step and its manifold keeps and refreshes the
// points it holds.  Transient penetrations (food dropped into the spoon at reset) never persist
// that long, so normal envs are never capped; GJK-only pairs are always solved, and with the
// budget unspent the visiting order changes nothing.  Returns the sub-step's EPA demand (solved +
// skipped).
#ifndef AVR_COOP_CAP
#define AVR_COOP_CAP 4
#endif
#ifndef AVR_COOP_PERSIST
#define AVR_COOP_PERSIST 20
#endif
AVR_DI int np_coop(const KModel &m, float *cs, int n, EpaBuf &E, int rot, int budget) {
    const int lane = lane_id();
    // the cooperative pairs of each 64-pair chunk, read once (the stores below rewrite CS_RES)
    unsigned long long bm[MAXSP / 64], bd[MAXSP / 64];
    int nco = 0;
#pragma unroll
    for (int q = 0; q < MAXSP / 64; q++) {
        const int k = 64 * q + lane;
        const int rc = __float_as_int(gld(cs + CS_RES + 8 * (k < n ? k : 0)));
        bm[q] = __ballot(k < n && (rc == 2 || rc == 4));
        bd[q] = __ballot(k < n && rc == 4);
        nco += __popcll(bm[q]);
    }
    const int r0 = nco > 0 ? rot % nco : 0;
    const int budget0 = budget;
    int skipped = 0;
    for (int pass = 0; pass < 2; pass++) {       // cooperative pairs r0 .. nco - 1, then 0 .. r0 - 1
        int jn = 0;
#pragma unroll
        for (int q = 0; q < MAXSP / 64; q++) {
            const int k = 64 * q + lane;
            unsigned long long cm = bm[q];
            while (cm) {
                const int j = __ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const int jj = jn++;
                if ((jj >= r0) != (pass == 0)) continue;
                const int kj = __shfl(k, j, 64);
                const int key = __float_as_int(gld(cs + CS_PAIRS + 2 * kj)), w = __float_as_int(gld(cs + CS_PAIRS + 2 * kj + 1));
                const int sa = key & 0xffff, sb = key >> 16;
                const int ba = (w >> 16) & 0xff, bb = (w >> 24) & 0xff;
                const float thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
                const WShape A = make_wshape(m, sa, ldtf(cs + CS_BTF + 8 * ba)), B = make_wshape(m, sb, ldtf(cs + CS_BTF + 8 * bb));
                v3 n2 = V(0, 0, 0), p2 = V(0, 0, 0);
                float d2 = 0.f;
                int nit, nk;
#ifdef AVR_PROF
                const unsigned long long c0t = __builtin_readcyclecounter();
#endif
                int r2 = narrowphase<true>(m, E, A, B, thr, n2, p2, d2, nit, nk, &budget, (bd[q] >> j) & 1ull);
                if (r2 == 3) { r2 = 0; skipped++; }
#ifdef AVR_PROF
                if (m.prof && lane == 0) {     // cooperative pairs, their GJK iterations, the time they took
                    const unsigned long long dc = __builtin_readcyclecounter() - c0t;
                    unsigned long long *pr = m.prof + (size_t)(cs - m.cscr) / CS_WORDS * AVR_PROF_SLOTS;
                    atomicAdd(pr + 11, 1ull);
                    atomicAdd(pr + 28, (unsigned long long)nit);
                    // by shape kinds: 19 sphere-hull, 20 hull-hull, 21 other; 22 big hull (no support
                    // table); 29 cycles, 30 the slowest pair's cycles
                    const bool ha = A.kind == AVR_HULL, hb = B.kind == AVR_HULL;
                    const bool sph = (A.kind == AVR_SPHERE && hb) || (B.kind == AVR_SPHERE && ha);
                    atomicAdd(pr + (sph ? 19 : (ha && hb) ? 20 : 21), 1ull);
                    if ((A.nv > SMALL_NV && A.tab < 0) || (B.nv > SMALL_NV && B.tab < 0)) atomicAdd(pr + 22, 1ull);
                    atomicAdd(pr + 29, dc);
                    atomicMax(pr + 30, dc);
                }
#endif
                SYNC();
                if (lane == 0) np_store(cs, kj, r2, n2, p2, d2);
                SYNC();
            }
        }
    }
    return budget0 - budget + skipped;
}

// Sub-step part A2: the narrowphase of every listed shape pair across all envs.  A block takes one
// of the two work lists of NP_ENVS envs, concatenated: the sphere-hull list (point-core GJK, a
// lane that finishes a pair takes the next item of the concatenation, so the lanes stay busy
// until the last NP_ENVS-env tail) or the other pairs (one lane per item, narrowphase()).  Pairs
// with a big hull that has no support table, and penetrating pairs that need EPA, are marked rc =
// 2 for the cooperative kernel.  Block b takes list (b / 8) % 2 of the envs
// e = env0 + 8 NP_ENVS (b / 16) + b % 8 + 8 k, k < NP_ENVS: the XCD (b % 8) whose L2 holds their
// pair lists.  Measured at 4096 envs (env groups on): NP_ENVS 1 / 2 / 4 / 8 give 717k / 703k /
// 638k / 527k env-steps/s -- fewer, longer waves hide less latency than the shorter refill tail saves.
#ifndef NP_ENVS
#define NP_ENVS 1
#endif
#ifndef NP_WAVES
#define NP_WAVES 4
#endif
AVR_DI void np_list(const KModel &m, const unsigned char *__restrict__ mask, int eb, int list, int n_envs, float2 *ent, float (*btfs)[MAXB * 8]) {
    const int lane = lane_id();
    // items per env (0 past the end or masked out), prefix over the block's envs
    int pre[NP_ENVS + 1];
    pre[0] = 0;
#pragma unroll
    for (int k = 0; k < NP_ENVS; k++) {
        const int e = eb + 8 * k;
        const bool live = e < n_envs && (!mask || mask[e]);
        pre[k + 1] = pre[k] + (live ? __float_as_int(gld(env_cs(m, live ? e : eb) + (list ? CS_N1 : CS_N0))) : 0);
    }
    const int T = pre[NP_ENVS];
    // item j: env slot k and its position in that env's list (value selects: no indexed register array)
    auto item = [&](int j, float *&cs) {
        int k = 0, off = 0;
#pragma unroll
        for (int q = 1; q < NP_ENVS; q++)
            if (j >= pre[q]) { k = q; off = pre[q]; }
        cs = env_cs(m, eb + 8 * k);
        return j - off;
    };
    auto slot_of = [&](int j) {
        int k = 0;
#pragma unroll
        for (int q = 1; q < NP_ENVS; q++)
            if (j >= pre[q]) k = q;
        return k;
    };
    // the block's list entries (concatenated over its envs) and its envs' body frames, staged in
    // LDS in one round trip: a refill then reads its entry and frames from LDS
#pragma unroll
    for (int k = 0; k < NP_ENVS; k++) {
        const int e = eb + 8 * k;
        const float *ck = env_cs(m, e < n_envs ? e : eb);
        const int nk = pre[k + 1] - pre[k];
        float te[NB_OF(2 * MAXSP)], tb[NB_OF(MAXB * 8)];
        g2r(te, ck + (list ? CS_L1 : CS_L0), 2 * nk);
        g2r(tb, ck + CS_BTF, m.nb * 8);
        r2l((float *)ent + 2 * pre[k], te, 2 * nk);
        r2l(btfs[k], tb, m.nb * 8);
    }
    SYNC();
    auto entry = [&](int j) { const float2 x = ent[j]; return make_int2(__float_as_int(x.x), __float_as_int(x.y)); };
#ifdef AVR_WAVETIME   // [3][eb] (list-0 block, list-1 block) durations in 100 MHz ticks
    struct WtNp {
        const KModel &m; int env, list, n_envs; unsigned long long t0;
        AVR_DI ~WtNp() {
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            if (m.prof && lane_id() == 0) m.prof[((size_t)3 * n_envs + env) * 2 + list] = t1 - t0;
        }
    } wtnp{m, eb, list, n_envs, __builtin_amdgcn_s_memrealtime()};
#endif
#ifdef AVR_PROF   // narrowphase counters (tools/prof_phases.py): slots 32-39, the block's totals at env eb
    unsigned long long *pr = m.prof ? m.prof + (size_t)eb * AVR_PROF_SLOTS : nullptr;
    auto pcount = [&](int slot, long long v) { if (pr && lane == 0 && v) atomicAdd(pr + slot, (unsigned long long)v); };
#endif
    if (list == 0) {
        PH P;
        float *pcs = nullptr;      // the env of the lane's pair
        bool act = lane < T;
        if (act) { (void)item(lane, pcs); ph_init(m, btfs[slot_of(lane)], entry(lane), P); }
        int next = 64;
#ifdef AVR_PROF
        pcount(32, T);
#endif
        while (__ballot(act)) {
#ifdef AVR_PROF
            pcount(34, 1);
            pcount(35, __popcll(__ballot(act)));
#endif
            bool done = false;
            int rc = 0;
            v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
            float d = 0.f;
            if (act) {
                done = ph_step(m, P, rc, nB, pB, d);
                if (done) np_store(pcs, P.k, rc, nB, pB, d);
            }
            const unsigned long long dm = __ballot(done);
            if (done) {
                const int j = next + __popcll(dm & ((1ull << lane) - 1ull));
                act = j < T;
                if (act) { (void)item(j, pcs); ph_init(m, btfs[slot_of(j)], entry(j), P); }
            }
            next += __popcll(dm);
        }
        return;
    }
#ifdef AVR_PROF
    pcount(33, T);
#endif
    for (int c0 = 0; c0 < T; c0 += 64) {
#ifdef AVR_PROF
        int pit = 0, pk = -1;
#endif
        if (c0 + lane < T) {
            float *cs;
            (void)item(c0 + lane, cs);
            const int2 e = entry(c0 + lane);
            const float *bt = btfs[slot_of(c0 + lane)];
            const int k = e.x & 0xffff;
            const int sa = e.y & 0xffff, sb = e.y >> 16;
            const int ba = (e.x >> 16) & 0xff, bb = (e.x >> 24) & 0xff;
            const float thr = fminf(gld(m.body_threshold + (ba)), gld(m.body_threshold + (bb)));
            const WShape A = make_wshape(m, sa, ldtf(bt + 8 * ba)), B = make_wshape(m, sb, ldtf(bt + 8 * bb));
            int rc = 2;
            v3 nB = V(0, 0, 0), pB = V(0, 0, 0);
            float d = 0.f;
            if (!((A.nv > SMALL_NV && A.tab < 0) || (B.nv > SMALL_NV && B.tab < 0))) {
                int nit, nkind;
                rc = narrowphase<false>(m, *(EpaBuf *)cs, A, B, thr, nB, pB, d, nit, nkind);   // (the lane path never touches the EPA buffer)
#ifdef AVR_PROF
                pit = nit; pk = nkind;
#endif
            }
            np_store(cs, k, rc, nB, pB, d);
        }
#ifdef AVR_PROF   // GJK iterations (sum, and the chunk's maximum: what the wave runs), pairs by kind
        int mx = pit;
        for (int o = 32; o; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        int sm = pit;
        for (int o = 32; o; o >>= 1) sm += __shfl_xor(sm, o);
        pcount(36, sm);
        pcount(37, mx);
        pcount(38, __popcll(__ballot(pk == 3)));
        pcount(39, __popcll(__ballot(pk >= 0 && pk < 3)));
#endif
    }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NP_WAVES))) void avr_narrowphase_kernel(const KModel *__restrict__ mp, const unsigned char *__restrict__ mask, int env0,
                                                             int n_envs) {
    const int list = (blockIdx.x >> 3) & 1;
    const int eb = env0 + 8 * NP_ENVS * (blockIdx.x >> 4) + (blockIdx.x & 7);
    if (eb >= n_envs) return;
    __shared__ float2 ent[NP_ENVS * MAXSP];
    __shared__ float btfs[NP_ENVS][MAXB * 8];
    np_list(*mp, mask, eb, list, n_envs, ent, btfs);
}

// AVR_COOP_KERNEL 1: the wave-cooperative pairs run in a kernel of their own between the
// narrowphase and kernel a (one 64-lane block per env, EPA polytope in LDS), so kernel a's
// register budget is its own (the cooperative path needs ~190 VGPRs, kernel a alone ~130: four
// waves per SIMD instead of two).  0: they open kernel a (an env with an EPA delays only itself).
#ifndef AVR_COOP_KERNEL
#define AVR_COOP_KERNEL 0
#endif
#if AVR_COOP_KERNEL
__global__ __launch_bounds__(64) void avr_coop_kernel(const KModel *__restrict__ mp, const unsigned char *__restrict__ mask, int env0, int n_envs) {
    __shared__ EpaBuf E;
    AVR_ENV_GUARD();
    if (gld(env_cs(m, env) + CS_COOP) != 0.f) {
        float *ws = env_ws(m, env);
        const int rot = __float_as_int(gld(ws + WS_COOPROT));
        (void)np_coop(m, env_cs(m, env), __float_as_int(gld(env_cs(m, env) + CS_NSP)), E, rot, 1 << 30);
        if (lane_id() == 0) ws[WS_COOPROT] = __int_as_float(rot + AVR_COOP_CAP);
    }
}
#endif

// Sub-step part A3: one 64-lane block per env, state staged in LDS -- the pairs the narrowphase
// kernel left to the wave-cooperative path (rc 2: EPA, big hulls; 0.2-0.3 per env-step), then
// manifold update, unconstrained velocities, constraint rows.  The cooperative pairs open this
// kernel rather than a kernel of their own: the few envs that have one (an EPA can take ~40 us)
// delay only their own wave, not a whole launch that every env's kernel a waits behind.
AVR_DI void substep_a_env(const KModel &m, EnvLDS &L, float *__restrict__ state, float dt, int env, int n_envs) {
    (void)n_envs;
    WT_START();
    // the pairs left to the wave-cooperative narrowphase, before the prologue claims the LDS (the
    // EPA polytope overlays it).  Most envs have none: the narrowphase kernel's flag says so
    // without a scan of the per-pair results (written only by np_store, rc 2, after the pairs
    // kernel cleared it in this sub-step)
    static_assert(sizeof(EpaBuf) <= sizeof(EnvLDS), "EPA buffer overlay");
#if !AVR_COOP_KERNEL
    float *gst = state + (size_t)env * K_STATE_WORDS;
    const bool persist = gld(gst + S_TASK + T_COOPN) >= (float)AVR_COOP_PERSIST;
    int demand = 0;
    if (gld(env_cs(m, env) + CS_COOP) != 0.f) {
        float *ws = env_ws(m, env);
        const int rot = __float_as_int(gld(ws + WS_COOPROT));
        demand = np_coop(m, env_cs(m, env), __float_as_int(gld(env_cs(m, env) + CS_NSP)), *reinterpret_cast<EpaBuf *>(&L), rot,
                         persist ? AVR_COOP_CAP : 1 << 30);
        if (lane_id() == 0) ws[WS_COOPROT] = __int_as_float(rot + AVR_COOP_CAP);
        SYNC();
    }
#endif
#if AVR_COOP_KERNEL
    float *gst = state + (size_t)env * K_STATE_WORDS;
#endif
    load_a(m, L, gst, env_cs(m, env));
#if !AVR_COOP_KERNEL
    if (lane_id() == 0) {
        L.st[S_TASK + T_COOPN] = demand > AVR_COOP_CAP ? L.st[S_TASK + T_COOPN] + 1.f : 0.f;
        if (persist && demand > AVR_COOP_CAP) L.flags |= 32;
    }
    SYNC();
#endif
    bool ok = substep_a(m, L, dt, gst, env_ws(m, env), env_rows(m, env), env_cs(m, env));
#ifdef AVR_PROF
    if (lane_id() == 0) env_ws(m, env)[WS_XCC] = __int_as_float(xcc_id());
#endif
    if (lane_id() == 0 && !ok) L.flags |= 1;
    SYNC();
    if (lane_id() == 0) L.st[S_TASK + T_FLAGS] = (float)((int)L.st[S_TASK + T_FLAGS] | L.flags);
    SYNC();
    // write back what part A changes in LDS: contact count and flags (the pool itself was
    // written to global memory by collide_contacts)
    if (lane_id() < 16) gst[S_TASK + lane_id()] = L.st[S_TASK + lane_id()];
    prof_flush(m, L, env);
    WT_END(0);
}

__global__ __launch_bounds__(64) AVR_KATTR void avr_substep_a_kernel(const KModel *__restrict__ mp, float *__restrict__ state,
                                                                     const unsigned char *__restrict__ mask, float dt, int env0, int n_envs) {
    __shared__ EnvLDS L;
    AVR_ENV_GUARD();
    substep_a_env(m, L, state, dt, env, n_envs);
}

// ---------------------------------------------------------------------------- part B: PGS solve
// Projected Gauss-Seidel (btMultiBodyConstraintSolver::solveSingleIteration order: non-contact
// rows with the sweep direction alternating per iteration, normal rows, then the two friction
// rows of every contact with a positive normal impulse) and semi-implicit Euler, four envs per
// wavefront.  Lanes 16g .. 16g+15 solve env g of the block; lane sl = lane & 15 of a group holds
// robot DoF sl's and free body sl's velocity increments (MAXD, MAXF <= 16).  A row's J.dv is one
// 16-lane DPP butterfly (row_ror 8, 4, 2, 1: every lane of the row ends with the sum), so the
// four envs' Gauss-Seidel chains advance in lockstep through one instruction stream.  A group
// with fewer rows than the wave's longest sweep runs null rows (inv = rhs = lo = hi = 0, so
// delta = 0 exactly), which leaves its results identical to a solve on its own.
//
// Where the rows come from: the non-contact rows (~20 per env: motors, violated limits, the
// spoon weld) are read from the env's row buffer in global memory (they stay L2-resident); the
// contact rows -- the bulk -- are copied into LDS at kernel entry whenever the block's four
// envs fit (40 KB per block, 4 blocks per CU), otherwise the whole wave reads them from global
// memory too.  Every load is typed by address space (ds_read / global_load, never flat) and a
// lane's choice between real data and the zero block is an address select, never a value
// select: the waits the compiler places for a row then count only that row's loads, and the
// software pipeline's read-ahead (headers 2D rows ahead, the header-dependent parts D ahead)
// stays in flight.
#if B4_PK
struct DV { float rq, rq2; f2v v1, v2, v3; };             // v1 = (vx, wx), v2 = (vy, wy), v3 = (vz, wz)
#else
struct DV { float rq, rq2, vx, vy, vz, wx, wy, wz; };   // rq2: DoF sl + 16 (NDL 2)
#endif

AVR_DI int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Global row data is read with buffer loads through one resource over the whole row buffer
// (uniform base in SGPRs, 32-bit per-lane byte offsets): a null row or a lane with no part to
// read addresses B4_OOB, past the end of the buffer, and the range check returns zeros -- an
// all-zero header is a null row (no endpoint, inv = rhs = lo = hi = 0), a zero part contributes
// nothing.
#define B4_OOB 0x7fff0000
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u3v __attribute__((ext_vector_type(3)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));
AVR_DI f4v bld4(rsrc_t r, int o) { u4v x = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0); return *(f4v *)&x; }
AVR_DI f2v bld2(rsrc_t r, int o) { u2v x = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0); return *(f2v *)&x; }
AVR_DI float bld1(rsrc_t r, int o) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0)); }
#if NDL == 2
typedef f4v rv_t;           // a lane's robot-part words: (J, M^-1 J^T) of DoF sl, then of DoF sl + 16
#define RVB 16              // bytes per lane in a robot part
#define rload bld4
#else
typedef f2v rv_t;           // (J, M^-1 J^T) of DoF sl
#define RVB 8
#define rload bld2
#endif
typedef __attribute__((address_space(3))) rv_t lds_rv;
AVR_DI f4v bld3(rsrc_t r, int o) {
    u3v x = __builtin_amdgcn_raw_buffer_load_b96(r, o, 0, 0);
    f4v y = {__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), 0.f};
    return y;
}

// LDS of a block (40 KB: 4 blocks per CU, all blocks of a 4096-env launch resident): a null
// contact header and a zero block, then the four groups' regions, packed:
//   impulses [n_rows + 2 null slots] | active-contact list [n_c] | contact records [3 n_c][16]
//   | robot parts of robot-contact rows [n_rob - n_nc][32]
// (the last two only when the block's four envs fit).
#ifndef B4_LDSW
#define B4_LDSW 10240    // LDS words per block
#endif
AVR_DI int al4(int x) { return (x + 3) & ~3; }

// this lane's part of a row from the row's ownership mask (2 bits per free body: 1 endpoint A,
// 2 endpoint B, 0 none).  Lanes sl >= MAXF own no free body and read bits 30-31, which every
// header keeps 0 (a contact header's robot slot + 1 sits in bits CI_SLOT..29), so no lane masks
// the slot bits off.
AVR_DI int own_of(int mask) {
    const int sl = lane_id() & 15;
    return (int)__builtin_amdgcn_ubfe((unsigned)mask, sl < MAXF ? 2 * sl : 30, 2);
}
static_assert(2 * MAXF <= CI_SLOT && MAXNC + K_CROWS * K_MAX_CONTACTS < (1 << (30 - CI_SLOT)), "own mask and slot bit fields");

// Row sources.  A sweep step sets a row's addresses with set(R, valid, address, impulse slot)
// from per-lane bases plus a wave-uniform step offset (an invalid step is a null row), reads its
// header D steps early (hdr / hdr3) and its header-dependent parts (parts) after that.  The two
// friction rows of a unit are consecutive records (the second 64 bytes on) with consecutive
// impulse slots: the second row's loads are the first's plus immediate offsets.

// non-contact rows: buffer loads (they stay L2-resident)
struct NcRow { int o; lds_f *ip; f4v h0, h1; float imp; f2v j0, j1, j2; rv_t r; };   // h1: lo, hi, residual limit
struct NcSrc {
    typedef NcRow Row;
    static constexpr bool robot_parts = true;
    rsrc_t rs;
    int eo, ro;                // this env's records / robot parts (byte offsets)
    lds_f *ip0, *nullip;       // impulse slots: row 0, null rows
    AVR_DI void set(Row &R, bool v, int o, lds_f *ip) const { R.o = v ? o : B4_OOB; R.ip = v ? ip : nullip; }
    AVR_DI void hdr(Row &R) const { R.h0 = bld4(rs, R.o); R.h1 = bld3(rs, R.o + 16); R.imp = *R.ip; }
    AVR_DI void parts(Row &R) const {
        const int o = own_of(__float_as_int(R.h0.x));     // endpoint A at word 8, B at word 14
        const int b = o ? R.o + 8 + 24 * o : B4_OOB;
        R.j0 = bld2(rs, b); R.j1 = bld2(rs, b + 8); R.j2 = bld2(rs, b + 16);
        const int slot = __float_as_int(R.h0.y) - 1;
        R.r = rload(rs, slot >= 0 ? ro + slot * (ROBW * 4) + RVB * (lane_id() & 15) : B4_OOB);
    }
};

// non-contact rows staged in LDS (B4_NC_LDS: the PR2 tasks, whose rows are nearly all non-contact
// rows with 24-DoF robot parts), by byte address: a row's o is its record's address + 8, so its
// header is read at o - 8 and o + 8 and its endpoint part w (1 A, 2 B) at o + 24 w; a null row
// reads its header from the zero head (o = LNB_NCNULL); robot part of the row with slot + 1 = s
// at rob + ROBW 4 s (this lane's DoFs), or the zero block
#define LN_HEAD (NDL == 2 ? 80 : 48)   // NDL 2: zero robot parts at words 12-15 and 76-79
#define LNB_NULL 24                // null contact record - 8 (bytes)
#define LNB_ZERO 48                // zero block (bytes)
#define LNB_NCNULL 16              // null non-contact row: header words 2-7 of the zero head
typedef __attribute__((address_space(3))) char lds_c;
struct NcLds {
    typedef NcRow Row;
    static constexpr bool robot_parts = true;
    lds_c *blk;
    int eo;                    // row 0's record address + 8 (bytes)
    unsigned rob;              // robot part of the row with slot + 1 = s: rob + ROBW 4 s (bytes, this lane's DoFs)
    lds_f *ip0, *nullip;       // impulse slots: row 0, null rows
    AVR_DI void set(Row &R, bool v, int o, lds_f *ip) const { R.o = v ? o : LNB_NCNULL; R.ip = v ? ip : nullip; }
    AVR_DI void hdr(Row &R) const {
        R.h0 = *(const lds_f4 *)(blk + R.o - 8);
        const f2v a = *(const lds_f2 *)(blk + R.o + 8);
        R.h1.x = a.x; R.h1.y = a.y; R.h1.z = *(const lds_f *)(blk + R.o + 16);
        R.imp = *R.ip;
    }
    AVR_DI void parts(Row &R) const {
        const int w = own_of(__float_as_int(R.h0.x));
        const lds_f2 *q = (const lds_f2 *)(blk + (w ? R.o + 24 * w : LNB_ZERO));
        R.j0 = q[0]; R.j1 = q[1]; R.j2 = q[2];
        const unsigned sp = (unsigned)__float_as_int(R.h0.y);
        R.r = *(const lds_rv *)(blk + (sp ? rob + ROBW * 4 * sp : LNB_ZERO));
    }
};

// contact rows staged in LDS, by byte address: a row's wb is its record's address - 8, so its
// header is read at wb + 8 and its endpoint part o (1 A, 2 B) at wb + 24 o.  Null rows and zero
// parts come from the block's zero-filled head (LN_HEAD words): the null record's headers at
// words 8-11 and 24-27 (a null friction unit), zero parts at words 12-17 and 28-33, zero robot
// parts at words 12-13 and 44-45.
struct CRowL { unsigned wb; lds_f *ip; f4v h; float imp; f2v j0, j1, j2; rv_t r; };
template <bool RC>             // RC: the block has robot contacts (otherwise no contact row has a robot part)
struct CLds {
    typedef CRowL Row;
    static constexpr bool robot_parts = RC;
    lds_c *blk;
    unsigned cn, cf;           // normal record 0 / friction unit 0 of this group, - 8 (bytes)
    unsigned rob;              // robot part of the row with slot + 1 = s: rob + 128 s (bytes, this lane's DoF)
    lds_f *ipn, *ipf, *nullip; // impulse slots: normal row 0, friction unit 0, null rows
    unsigned ct;               // (K_TORSION) torsional unit 0 of this group, - 8 (bytes)
    lds_f *ipt;                // (K_TORSION) impulse slot of torsional row 0
    AVR_DI void set(Row &R, bool v, unsigned wb, lds_f *ip) const { R.wb = v ? wb : LNB_NULL; R.ip = v ? ip : nullip; }
    AVR_DI void hdr(Row &R) const { R.h = *(const lds_f4 *)(blk + R.wb + 8); R.imp = *R.ip; }
    AVR_DI void hdr3(Row &R) const {   // normal rows: the friction coefficient is not read
        const lds_f *q = (const lds_f *)(blk + R.wb + 8);
        const f2v a = *(const lds_f2 *)q;
        R.h.x = a.x; R.h.y = a.y; R.h.z = q[2];
        R.imp = *R.ip;
    }
    AVR_DI void hdr2(Row &B, const Row &A) const {   // a unit's second row: the first row's residual limit, inv, rhs, its own limit
        B.h = *(const lds_f4 *)(blk + A.wb + 8 + CRW * 4);
        B.imp = A.ip[1];
    }
    AVR_DI unsigned own_b(const Row &R) const { const int o = own_of(__float_as_int(R.h.x)); return o ? R.wb + 24 * o : LNB_ZERO; }
    AVR_DI void own_at(Row &R, unsigned b) const { const lds_f2 *q = (const lds_f2 *)(blk + b); R.j0 = q[0]; R.j1 = q[1]; R.j2 = q[2]; }
    AVR_DI unsigned rob_b(const Row &R) const { const unsigned s = (unsigned)__float_as_int(R.h.x) >> CI_SLOT; return s ? rob + ROBW * 4 * s : LNB_ZERO; }
    AVR_DI rv_t rob_at(unsigned b) const {
        if constexpr (!RC) { (void)b; return rv_t{}; }
        return *(const lds_rv *)(blk + b);
    }
    AVR_DI void parts(Row &R) const { own_at(R, own_b(R)); R.r = rob_at(rob_b(R)); }
    // (K_TORSION) contact c's torsional index + 1 (0: none), its normal record's 4th word
    AVR_DI int tor_of(int c) const { return (int)((unsigned)__float_as_int(*(const lds_f *)(blk + cn + CRW * 4 * c + 8)) >> 2 & 0x3ffffu); }
    AVR_DI void unit_parts(Row &A, Row &B) const {
        const unsigned b = own_b(A), r = rob_b(A);
        own_at(A, b); own_at(B, b + CRW * 4);
        A.r = rob_at(r); B.r = rob_at(r + ROBW * 4);
    }
};

// contact rows, buffer loads (blocks whose four envs do not fit the LDS); a null row or part
// reads at B4_OOB (+ immediate offsets), past the buffer: zeros
struct CRowG { int o; lds_f *ip; f4v h; float imp; f2v j0, j1, j2; rv_t r; };
struct CGlb {
    typedef CRowG Row;
    static constexpr bool robot_parts = true;
    rsrc_t rs;
    int cn, cf;                // normal record 0 / friction unit 0 of this env (byte offsets)
    int rob;                   // robot part of the row with slot + 1 = s: rob + 128 s (this lane's DoF)
    lds_f *ipn, *ipf, *nullip;
    int ct;                    // (K_TORSION) torsional unit 0 of this env (byte offset)
    lds_f *ipt;
    AVR_DI void set(Row &R, bool v, int o, lds_f *ip) const { R.o = v ? o : B4_OOB; R.ip = v ? ip : nullip; }
    AVR_DI void hdr(Row &R) const { R.h = bld4(rs, R.o); R.imp = *R.ip; }
    AVR_DI void hdr3(Row &R) const { R.h = bld3(rs, R.o); R.imp = *R.ip; }
    AVR_DI void hdr2(Row &B, const Row &A) const { B.h = bld4(rs, A.o + CRW * 4); B.imp = A.ip[1]; }
    AVR_DI int own_b(const Row &R) const { const int o = own_of(__float_as_int(R.h.x)); return o ? R.o - 8 + 24 * o : B4_OOB; }
    AVR_DI void own_at(Row &R, int b) const { R.j0 = bld2(rs, b); R.j1 = bld2(rs, b + 8); R.j2 = bld2(rs, b + 16); }
    AVR_DI int rob_b(const Row &R) const { const int s = (int)((unsigned)__float_as_int(R.h.x) >> CI_SLOT); return s ? rob + ROBW * 4 * s : B4_OOB; }
    AVR_DI rv_t rob_at(int b) const { return rload(rs, b); }
    AVR_DI void parts(Row &R) const { own_at(R, own_b(R)); R.r = rob_at(rob_b(R)); }
    AVR_DI int tor_of(int c) const { return (int)((unsigned)__float_as_int(bld1(rs, cn + CRW * 4 * c)) >> 2 & 0x3ffffu); }
    AVR_DI void unit_parts(Row &A, Row &B) const {
        const int b = own_b(A), r = rob_b(A);
        own_at(A, b); own_at(B, b + CRW * 4);
        A.r = rob_at(r); B.r = rob_at(r + ROBW * 4);
    }
};

// sum over the 16 lanes of each DPP row, result in every lane of the row (each rotate folds
// into the add as a DPP source operand)
AVR_DI float row16_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xf, 0xf, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xf, 0xf, true));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xf, 0xf, true));
    return x;
}

// resolve one row with its current impulse; returns the new impulse.  The fused multiply-adds
// are spelled out and nothing else may contract: every unrolled copy of a row resolve (and every
// pipeline depth) then rounds the same way, so an env's results do not depend on which copy
// resolves its rows or on the row counts of the other envs in its wavefront.  With acc, the lanes
// of a row whose impulse change exceeds its residual limit rl (BT_RESIDUAL_SQRT inv: the row has not
// converged, solverResidualThreshold) are or-ed into acc.
template <bool RP, class R>
AVR_DI float go4(const R &X, DV &d, float imp, float inv, float rhs, float lo, float hi, float rl = 0.f, unsigned long long *acc = nullptr) {
#pragma clang fp contract(off)
#if B4_PK
    // the same products and roundings as below, two per packed instruction: parts are stored as
    // (linear, angular) pairs per axis and the velocity increments likewise, so the lo half of
    // the chain is the linear dot product p and the hi half the angular one q
    f2v s = X.j0 * d.v1;
    if (RP) {
        s.y = fmaf(X.r.x, d.rq, s.y);
#if NDL == 2
        s.y = fmaf(X.r.z, d.rq2, s.y);
#endif
    }
    s = __builtin_elementwise_fma(X.j1, d.v2, s);
    s = __builtin_elementwise_fma(X.j2, d.v3, s);
    const float dv = row16_sum(s.x + s.y);
    const float ni = __builtin_amdgcn_fmed3f(imp + fmaf(-dv, inv, rhs), lo, hi);
    const float delta = ni - imp;
    if (acc) *acc |= __ballot(fabsf(delta) > rl);
    const f2v dd = {delta, delta};
    d.v1 = __builtin_elementwise_fma(X.j0, dd, d.v1);
    d.v2 = __builtin_elementwise_fma(X.j1, dd, d.v2);
    d.v3 = __builtin_elementwise_fma(X.j2, dd, d.v3);
    if (RP) d.rq = fmaf(X.r.y, delta, d.rq);
#if NDL == 2
    if (RP) d.rq2 = fmaf(X.r.w, delta, d.rq2);
#endif
    return ni;
#else
    const float p = fmaf(X.j1.x, d.vz, fmaf(X.j0.y, d.vy, X.j0.x * d.vx));
#if NDL == 2
    const float q = RP ? fmaf(X.j2.y, d.wz, fmaf(X.j2.x, d.wy, fmaf(X.r.z, d.rq2, fmaf(X.r.x, d.rq, X.j1.y * d.wx))))
                       : fmaf(X.j2.y, d.wz, fmaf(X.j2.x, d.wy, X.j1.y * d.wx));
#else
    const float q = RP ? fmaf(X.j2.y, d.wz, fmaf(X.j2.x, d.wy, fmaf(X.r.x, d.rq, X.j1.y * d.wx)))
                       : fmaf(X.j2.y, d.wz, fmaf(X.j2.x, d.wy, X.j1.y * d.wx));
#endif
    const float dv = row16_sum(p + q);
    const float ni = __builtin_amdgcn_fmed3f(imp + fmaf(-dv, inv, rhs), lo, hi);
    const float delta = ni - imp;
    if (acc) *acc |= __ballot(fabsf(delta) > rl);
    d.vx = fmaf(X.j0.x, delta, d.vx); d.vy = fmaf(X.j0.y, delta, d.vy); d.vz = fmaf(X.j1.x, delta, d.vz);
    d.wx = fmaf(X.j1.y, delta, d.wx); d.wy = fmaf(X.j2.x, delta, d.wy); d.wz = fmaf(X.j2.y, delta, d.wz);
    if (RP) d.rq = fmaf(X.r.y, delta, d.rq);
#if NDL == 2
    if (RP) d.rq2 = fmaf(X.r.w, delta, d.rq2);
#endif
    return ni;
#endif
}

// A friction unit: its two rows share their bodies, so the second row's J.dv after the first
// row's update is J_2.dv + delta_1 c with c = J_2 M^-1 J_1^T (kernel a stores it in the second
// row's header).  Both dot products are formed from the same velocities side by side, so only the
// scalar correction stays on the dependency chain between the two resolves; the velocities then
// take both rows' increments.  The same Gauss-Seidel step as two go4 calls, rounded differently.
#if B4_FPAIR
template <bool RP, class R>
AVR_DI void go4_pair(const R &A, const R &B, DV &d, float &ia, float &ib, float lim) {
#pragma clang fp contract(off)
    f2v sa = A.j0 * d.v1, sb = B.j0 * d.v1;
    if (RP) {
        sa.y = fmaf(A.r.x, d.rq, sa.y); sb.y = fmaf(B.r.x, d.rq, sb.y);
#if NDL == 2
        sa.y = fmaf(A.r.z, d.rq2, sa.y); sb.y = fmaf(B.r.z, d.rq2, sb.y);
#endif
    }
    sa = __builtin_elementwise_fma(A.j1, d.v2, sa); sb = __builtin_elementwise_fma(B.j1, d.v2, sb);
    sa = __builtin_elementwise_fma(A.j2, d.v3, sa); sb = __builtin_elementwise_fma(B.j2, d.v3, sb);
    const float dva = row16_sum(sa.x + sa.y), dvb0 = row16_sum(sb.x + sb.y);
    const float na = __builtin_amdgcn_fmed3f(ia + fmaf(-dva, A.h.y, A.h.z), -lim, lim);
    const float da = na - ia;
    const float dvb = fmaf(da, B.h.w, dvb0);
    const float nb = __builtin_amdgcn_fmed3f(ib + fmaf(-dvb, B.h.y, B.h.z), -lim, lim);
    const float db = nb - ib;
    const f2v dda = {da, da}, ddb = {db, db};
    d.v1 = __builtin_elementwise_fma(B.j0, ddb, __builtin_elementwise_fma(A.j0, dda, d.v1));
    d.v2 = __builtin_elementwise_fma(B.j1, ddb, __builtin_elementwise_fma(A.j1, dda, d.v2));
    d.v3 = __builtin_elementwise_fma(B.j2, ddb, __builtin_elementwise_fma(A.j2, dda, d.v3));
    if (RP) d.rq = fmaf(B.r.y, db, fmaf(A.r.y, da, d.rq));
#if NDL == 2
    if (RP) d.rq2 = fmaf(B.r.w, db, fmaf(A.r.w, da, d.rq2));
#endif
    ia = na; ib = nb;
}
#endif

// sweep over n (wave-uniform) steps; at(R, j) sets R's addresses for step j (a null row for
// every j past this lane's group's rows).  Software pipeline of depth D: headers 2D steps ahead,
// the header-dependent parts D steps ahead, in a ring of K = 2D + 1 buffers whose slots are
// compile-time after unrolling.  The sweep runs whole rounds of K steps (the last round pads
// with null rows, delta = 0) and issues its read-ahead unconditionally: with no conditional
// load in the loop the compiler's wait counts are exact (a load that may or may not have been
// issued on some path makes it wait for everything).
template <int D, bool H3, class S>
AVR_DI void hdr_of(const S &s, typename S::Row &R) {
    if constexpr (H3) s.hdr3(R);
    else s.hdr(R);
}
template <int D, bool H3, class S, class AT, class GO>
AVR_DI void sweep4(const S &s, int n, const AT &at, const GO &go) {
    if (n <= 0) return;
    constexpr int K = 2 * D + 1;
    typename S::Row R[K];
#pragma unroll
    for (int q = 0; q < 2 * D; q++) { at(R[q], q); hdr_of<D, H3>(s, R[q]); }
#pragma unroll
    for (int q = 0; q < D; q++) s.parts(R[q]);
    for (int j = 0; j < n; j += K) {
#pragma unroll
        for (int q = 0; q < K; q++) {
            at(R[(q + 2 * D) % K], j + q + 2 * D);
            hdr_of<D, H3>(s, R[(q + 2 * D) % K]);
            s.parts(R[(q + D) % K]);
            go(R[q]);
        }
    }
}

// friction unit: the two friction rows of one active contact and that contact's normal impulse
template <class S>
struct Pair4 { typename S::Row a, b; float in; };

#if K_TORSION
// torsional rows (spinning about the normal, rolling about the two friction directions) of the
// active contacts: one flat sweep, step j = row j mod 3 of the j / 3-th active contact; a row
// carries its contact's normal impulse (its limits are +-coefficient x that impulse)
template <class CS>
struct TorRow : CS::Row { float in; };
template <class CS>
struct TorSrc {
    typedef TorRow<CS> Row;
    static constexpr bool robot_parts = CS::robot_parts;
    const CS &cs;
    AVR_DI void hdr(Row &R) const { cs.hdr(R); }
    AVR_DI void parts(Row &R) const { cs.parts(R); }
};
#endif

// the largest of the four groups' values, wave-uniform
AVR_DI int wave_max4(int x) {
    x = max(x, __shfl_xor(x, 16));
    x = max(x, __shfl_xor(x, 32));
    return uni(x);
}

template <int DN, int DC, class NS, class CS>
AVR_DI int pgs4(const KModel &m, const NS &ns, const CS &cs, lds_i *list, lds_i *tlist, int n_nc, int n_c, int nnc_max, int nc_max, DV &d) {
    typedef typename NS::Row NR;
    typedef typename CS::Row CR;
    const int sl = lane_id() & 15;
#if B4_PK
    d.rq = d.rq2 = 0.f; d.v1 = d.v2 = d.v3 = f2v{0.f, 0.f};
#else
    d.rq = d.rq2 = 0.f; d.vx = d.vy = d.vz = d.wx = d.wy = d.wz = 0.f;
#endif
    // normal rows in contact order: record j at cn + 64 j, impulse slot ipn + j
    auto at_n = [&](CR &R, int j) { cs.set(R, j < n_c, cs.cn + CRW * 4 * j, cs.ipn + j); };
    // warm start (normal rows, contact order): delta = cached impulse x warm-start factor, which
    // is also the rows' starting impulse
    sweep4<DC, true>(cs, nc_max, at_n, [&](const CR &R) { (void)go4<CS::robot_parts>(R, d, 0.f, R.h.y, R.h.z, R.imp, R.imp); });
    int units = 0;      // friction units swept (diagnostics)
    // solverResidualThreshold: a group whose rows all stayed within their residual limits in an
    // iteration is done -- its rows are null rows from then on (Bullet leaves that solve group's
    // PGS loop), and the wave leaves the loop once its four groups are done
    bool done = false;
    for (int it = 0; it < m.iters; it++) {
        const int a_nc = done ? 0 : n_nc, a_c = done ? 0 : n_c;         // this iteration's rows
        const int anc_max = wave_max4(a_nc), ac_max = wave_max4(a_c);
        unsigned long long acc = 0ull;      // lanes of groups with a row above its residual limit
        // non-contact rows, the sweep direction alternating per iteration
        const bool fwd = (it & 1) != 0;
        const int r0 = fwd ? 0 : n_nc - 1, sg = fwd ? 1 : -1;
        const int ob = ns.eo + r0 * (RWC * 4);
        lds_f *ib = ns.ip0 + r0;
        sweep4<DN, false>(ns, anc_max, [&](NR &R, int j) { ns.set(R, j < a_nc, ob + sg * j * (RWC * 4), ib + sg * j); },
                          [&](const NR &R) { *R.ip = go4<true>(R, d, R.imp, R.h0.z, R.h0.w, R.h1.x, R.h1.y, R.h1.z, &acc); });
        auto at_na = [&](CR &R, int j) { cs.set(R, j < a_c, cs.cn + CRW * 4 * j, cs.ipn + j); };
        sweep4<DC, false>(cs, ac_max, at_na, [&](const CR &R) { *R.ip = go4<CS::robot_parts>(R, d, R.imp, R.h.y, R.h.z, 0.f, 1e10f, R.h.w, &acc); });
        // active contacts (positive normal impulse) of each group, in contact order
        int t = 0;
        for (int c0 = 0; c0 < ac_max; c0 += 16) {
            const int c = c0 + sl;
            const bool a = c < a_c && cs.ipn[c < a_c ? c : 0] > 0.f;
            const unsigned long long b = __ballot(a);
            const unsigned gm = (unsigned)(b >> (lane_id() & 48)) & 0xffffu;
            if (a) list[t + __popc(gm & ((1u << sl) - 1u))] = c;
            t += __popc(gm);
        }
        const int tmax = wave_max4(t);
        units += tmax;
        if (tmax > 0) {
        // the same depth-DC pipeline over friction units; list entries are read one step before
        // the headers they address
        constexpr int K = 2 * DC + 1;
        Pair4<CS> X[K];
        auto lst = [&](int u) { const int c = list[u < t ? u : 0]; return u < t ? c : -1; };   // (unconditional read)
        auto hdr = [&](Pair4<CS> &Y, int c) {
            cs.set(Y.a, c >= 0, cs.cf + 2 * CRW * 4 * c, cs.ipf + 2 * c);
            cs.hdr(Y.a);
            cs.hdr2(Y.b, Y.a);
            const float x = cs.ipn[max(c, 0)];     // (read unconditionally: no branch in the pipeline)
            Y.in = c >= 0 ? x : 0.f;
        };
        auto go = [&](const Pair4<CS> &Y) {
            const float lim = Y.a.h.w * Y.in;
#if B4_FPAIR
            float ia = Y.a.imp, ib = Y.b.imp;
            go4_pair<CS::robot_parts>(Y.a, Y.b, d, ia, ib, lim);
            Y.a.ip[0] = ia; Y.a.ip[1] = ib;
#else
            Y.a.ip[0] = go4<CS::robot_parts>(Y.a, d, Y.a.imp, Y.a.h.y, Y.a.h.z, -lim, lim, Y.b.h.x, &acc);
            Y.a.ip[1] = go4<CS::robot_parts>(Y.b, d, Y.b.imp, Y.b.h.y, Y.b.h.z, -lim, lim, Y.b.h.w, &acc);
#endif
        };
        // (whole rounds of K units, null units past the end, unconditional read-ahead: sweep4)
        int cn = lst(0);
#pragma unroll
        for (int q = 0; q < 2 * DC; q++) { hdr(X[q], cn); cn = lst(q + 1); }
#pragma unroll
        for (int q = 0; q < DC; q++) cs.unit_parts(X[q].a, X[q].b);
        for (int u0 = 0; u0 < tmax; u0 += K) {
#pragma unroll
            for (int q = 0; q < K; q++) {
                hdr(X[(q + 2 * DC) % K], cn);
                cn = lst(u0 + q + 2 * DC + 1);
                cs.unit_parts(X[(q + DC) % K].a, X[(q + DC) % K].b);
                go(X[q]);
            }
        }
#if K_TORSION
        // torsional rows after the frictions (btMultiBodyConstraintSolver::solveSingleIteration
        // [ext]), for the active contacts that have them, in contact order: their (contact,
        // torsional index) pairs compacted from the active list, then one flat sweep, step j = row
        // j mod 3 of the j / 3-th such contact; a row carries its contact's normal impulse (its
        // limits are +-coefficient x that impulse)
        {
            int tt = 0;
            for (int u0 = 0; u0 < tmax; u0 += 16) {
                const int u = u0 + sl;
                const int cl = list[u < t ? u : 0];
                const int c = u < t ? cl : 0;
                const int tv = cs.tor_of(c);                 // (read unconditionally, record 0 past the list)
                const bool a = u < t && tv > 0;
                const unsigned long long b = __ballot(a);
                const unsigned gm = (unsigned)(b >> (lane_id() & 48)) & 0xffffu;
                if (a) tlist[tt + __popc(gm & ((1u << sl) - 1u))] = c | (tv - 1) << 8;
                tt += __popc(gm);
            }
            int ttmax = tt;
            ttmax = max(ttmax, __shfl_xor(ttmax, 16));
            ttmax = max(ttmax, __shfl_xor(ttmax, 32));
            ttmax = uni(ttmax);
            const TorSrc<CS> ts{cs};
            sweep4<DC, false>(ts, 3 * ttmax, [&](TorRow<CS> &R, int j) {
                const int u = j / 3, k = j - 3 * u;
                const bool v = u < tt;
                const int e = tlist[v ? u : 0];
                const int c = e & 255, ti = e >> 8;
                cs.set(R, v, cs.ct + 3 * CRW * 4 * ti + CRW * 4 * k, cs.ipt + 3 * ti + k);
                const float x = cs.ipn[v ? c : 0];      // (read unconditionally)
                R.in = v ? x : 0.f;
            }, [&](const TorRow<CS> &R) {
                const float lim = R.h.w * R.in;
                *R.ip = go4<CS::robot_parts>(R, d, R.imp, R.h.y, R.h.z, -lim, lim, BT_RESIDUAL_SQRT * R.h.y, &acc);
            });
        }
#endif
        }   // (tmax > 0)
        done = done || ((acc >> (lane_id() & 48)) & 0xffffull) == 0ull;
        if (__ballot(!done) == 0ull) break;
    }
    return units;
}

#ifndef B4_DN
#define B4_DN 2          // pipeline depth, non-contact rows (global memory, L2-resident)
#endif
#ifndef B4_DC
#define B4_DC 1          // pipeline depth, contact rows staged in LDS
#endif
#ifndef B4_DG
#define B4_DG 3          // pipeline depth, contact rows from global memory (blocks that do not fit)
#endif
#ifndef B4_NC_LDS
#define B4_NC_LDS K_PR2  // stage the non-contact rows and every robot part in LDS too (when the four envs fit)
#endif
#ifndef B4_DNL
#define B4_DNL 1         // pipeline depth, non-contact rows staged in LDS
#endif

// Which envs a part-B block solves.  Blocks are dealt round-robin over the 8 XCDs, and part A runs
// env e as block e - env0, so block b's envs are taken from e - env0 = x + 8 k (x = b % 8): the
// envs part A ran on the same XCD, whose rows, workspace and state sit in that XCD's L2 (per-XCD
// L2s are not coherent with each other).  Index order (B4_SORT 0): block j = b / 8 takes k = 4 j ..
// 4 j + 3.  B4_SORT 1: the XCD's envs are taken in chunks of 128 (32 blocks), ordered by their row
// count (n_nc + 3 n_c + 3 n_t, from part A's workspace; ties by k), and block j takes ranks
// 4 (j mod 32) .. + 3 of its chunk.  A wave sweeps as many rows as its longest env, so grouping
// envs of similar length shortens the sum of the waves' lifetimes (the LDS- and register-time the
// step is bound by) by ~12 % on the oracle's FeedingJaco row counts.  An env's
// results do not depend on its wave mates (null rows are exact zeros), so the order changes no
// result bit (fingerprints equal on all three tasks).  Envs beyond n_envs sort last; masked-off
// envs count 0 rows.  Off: measured slower (FeedingJaco 861k -> 820k, part B 0.202 -> 0.266 ms per
// 4096-env launch): grouping the longest envs together pushes their blocks past the LDS share, onto
// the global-row path, and the slowest block sets the launch.
#ifndef B4_SORT
#define B4_SORT 0
#endif
AVR_DI int b4_env(const KModel &m, const unsigned char *__restrict__ mask, int env0, int n_envs, int bidx, int g) {
    const int x = bidx & 7, j = bidx >> 3;
#if B4_SORT
    const int lane = lane_id();
    const int kc = (j >> 5) << 7;                   // the chunk's first k
    unsigned key[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int kk = lane + 64 * h;
        const int e = env0 + x + 8 * (kc + kk);
        unsigned cost = 0xffffffu;                  // no env: last
        if (e < n_envs) {
            cost = 0u;
            if (!mask || mask[e]) {
                const float *ws = env_ws(m, e);
                cost = (unsigned)(__float_as_int(gld(ws + WS_NNC)) + 3 * __float_as_int(gld(ws + WS_NC)) +
                                  (K_TORSION ? 3 * __float_as_int(gld(ws + WS_NT)) : 0));
                cost = min(cost, 0xfffffeu);
            }
        }
        key[h] = (cost << 7) | (unsigned)kk;       // distinct keys
    }
    int rank0 = 0, rank1 = 0;                       // ranks among the chunk's 128 keys
    for (int i = 0; i < 64; i++) {
        const unsigned a = __builtin_amdgcn_readlane(key[0], i), b = __builtin_amdgcn_readlane(key[1], i);
        rank0 += (a < key[0]) + (b < key[0]);
        rank1 += (a < key[1]) + (b < key[1]);
    }
    int pick = 0;
#pragma unroll
    for (int gg = 0; gg < 4; gg++) {
        const int r = 4 * (j & 31) + gg;
        const unsigned long long b0 = __ballot(rank0 == r), b1 = __ballot(rank1 == r);
        const int kk = b0 ? __builtin_ctzll(b0) : 64 + __builtin_ctzll(b1);
        if (g == gg) pick = kk;
    }
    return env0 + x + 8 * (kc + pick);
#else
    (void)m; (void)mask; (void)n_envs;
    return env0 + 32 * j + x + 8 * g;
#endif
}

AVR_DI void substep_b4_block(const KModel &m, float *__restrict__ state, const unsigned char *__restrict__ mask, float dt, int frame_end,
                             int env0, int n_envs, int bidx, lds_f *blk) {
#ifdef AVR_WAVETIME
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int lane = lane_id(), sl = lane & 15, g = lane >> 4;
    const int env = b4_env(m, mask, env0, n_envs, bidx, g);     // (XCD-consistent; see b4_env)
    const bool live = env < n_envs && (!mask || mask[env]);
    const int ev = live ? env : env0;
    const gfp wsg = (gfp)env_ws(m, ev);
    float *st = state + (size_t)ev * K_STATE_WORDS;
    const int n_nc = live ? __float_as_int(wsg[WS_NNC]) : 0, n_c = live ? __float_as_int(wsg[WS_NC]) : 0;
    const int n_rob = live ? __float_as_int(wsg[WS_NROB]) : 0;
    const int n_t = live && K_TORSION ? __float_as_int(wsg[WS_NT]) : 0;       // contacts with torsional rows
    const int n_cr = 3 * n_c + 3 * n_t;                                        // contact records
    const int n_rows = n_nc + n_cr, n_rc = max(n_rob - n_nc, 0);
    auto wmax = [&](int x) { x = max(x, __shfl_xor(x, 16)); x = max(x, __shfl_xor(x, 32)); return uni(x); };
    const int nnc_max = wmax(n_nc), nc_max = wmax(n_c);
    // the row buffer of every env as one buffer resource; this env's records at byte eo
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(m.rows, 0, m.rows_envs * m.rowstride * 4, 0x00020000);
    const int eo = ev * m.rowstride * 4, ro = eo + m.rowcap * RWC * 4;
#ifdef AVR_LDS_POISON   // diagnostic: NaN-fill the block's LDS (see load_state)
    for (int i = lane; i < B4_LDSW; i += 64) blk[i] = __int_as_float(-1);
    SYNC();
#endif
    // pack the groups' regions; stage every row (B4_NC_LDS) or the contact rows when all four fit
    const int szA = al4(n_rows + 2) + (K_TORSION ? 2 : 1) * al4(n_c), szB = n_cr * CRW + n_rc * ROBW;
#if B4_NC_LDS
    const int szF = szB + n_nc * (RWC + ROBW);
    const int f0 = __shfl(szA + szF, 0), f1 = __shfl(szA + szF, 16), f2 = __shfl(szA + szF, 32), f3 = __shfl(szA + szF, 48);
    const bool full = uni(f0 + f1 + f2 + f3) <= B4_LDSW - LN_HEAD && !m.b4_global;
#else
    const int f0 = 0, f1 = 0, f2 = 0;
    constexpr bool full = false;
#endif
    const int t0 = __shfl(szA + szB, 0), t1 = __shfl(szA + szB, 16), t2 = __shfl(szA + szB, 32), t3 = __shfl(szA + szB, 48);
    const bool in_lds = full || (uni(t0 + t1 + t2 + t3) <= B4_LDSW - LN_HEAD && !m.b4_global);
    int base;
    if (full) base = g == 0 ? 0 : g == 1 ? f0 : g == 2 ? f0 + f1 : f0 + f1 + f2;
    else if (in_lds) base = g == 0 ? 0 : g == 1 ? t0 : g == 2 ? t0 + t1 : t0 + t1 + t2;
    else {
        const int a0 = __shfl(szA, 0), a1 = __shfl(szA, 16), a2 = __shfl(szA, 32);
        base = g == 0 ? 0 : g == 1 ? a0 : g == 2 ? a0 + a1 : a0 + a1 + a2;
    }
    base += LN_HEAD;
    lds_f *imp = blk + base;
    lds_i *list = (lds_i *)(imp + al4(n_rows + 2));
    lds_i *tlist = list + al4(n_c);     // (K_TORSION) active contacts with torsional rows
    // LDS regions: contact records at cw, then (full) the non-contact records at nw, then the
    // robot parts at rw (full: every slot's; otherwise the robot-contact slots')
    const int cw = base + szA, nw = cw + n_cr * CRW, rw = full ? nw + n_nc * RWC : nw;
    // starting impulses: non-contact rows and frictions 0, normal rows the cached impulse x the
    // warm-start factor; null slots 0.  The cached impulses are loaded here and stored after the
    // staging loads below have been issued (one memory round trip for both).
    const gfp cpool = (gfp)(st + S_CP);
    float wimp[K_MAX_CONTACTS / 16];
#pragma unroll
    for (int q = 0; q < K_MAX_CONTACTS / 16; q++) wimp[q] = cpool[AVR_CP_WORDS * min(sl + 16 * q, max(n_c - 1, 0)) + AVR_CP_IMP];
    for (int r = sl; r < n_rows + 2; r += 16) {
        const int c = r - n_nc;
        if (!(c >= 0 && c < n_c)) imp[r] = 0.f;
    }
    for (int i = lane; i < LN_HEAD; i += 64) blk[i] = 0.f;        // null rows, zero parts
    if (in_lds) {   // contact records, (full) non-contact records, robot parts: 8 loads in flight per lane
        const int n4r = n_cr * (CRW / 4), n4n = full ? n_nc * (RWC / 4) : 0, n4s = (full ? n_rob : n_rc) * (ROBW / 4);
        const int n4a = n4r + n4n, n4 = n4a + n4s, so = full ? ro : ro + n_nc * ROBW * 4;
        const int m4 = wmax(n4);
        lds_f4 *l0 = (lds_f4 *)(blk + cw);
        for (int b = 0; b < m4; b += 8 * 16) {
            f4v t[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int i = b + 16 * q + sl;
                t[q] = bld4(rs, i < n4r ? eo + CR_BASE * 4 + 16 * i : i < n4a ? eo + 16 * (i - n4r) : (i < n4 ? so + 16 * (i - n4a) : B4_OOB));
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int i = b + 16 * q + sl;
                if (i < n4) l0[i] = t[q];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < K_MAX_CONTACTS / 16; q++)
        if (sl + 16 * q < n_c) imp[n_nc + sl + 16 * q] = wimp[q] * m.warmstart;
    SYNC();
    // impulse slots: rows 0 .. n_rows - 1 (non-contact, normal, friction pairs), then 2 null slots
    lds_f *const ipn = imp + n_nc, *const ipf = ipn + n_c, *const ipt = ipf + 2 * n_c, *const nullip = imp + n_rows;
    NcSrc ns{rs, eo, ro, imp, nullip};
    DV d;
    int units, rcb = 0;
#if B4_NC_LDS
    if (full) {
        // every row from LDS: robot part of the row with slot + 1 = s at rw + (s - 1) ROBW words
        const unsigned cn = 4 * cw - 8, cf = cn + 4 * CRW * n_c, ct = cf + 8 * CRW * n_c, rob = 4 * (rw - ROBW) + RVB * sl;
        const NcLds nl{(lds_c *)blk, 4 * nw + 8, rob, imp, nullip};
        if (wmax(n_rc) > 0) {
            CLds<true> cs{(lds_c *)blk, cn, cf, rob, ipn, ipf, nullip, ct, ipt};
            units = pgs4<B4_DNL, B4_DC>(m, nl, cs, list, tlist, n_nc, n_c, nnc_max, nc_max, d);
            rcb = 1;
        } else {
            CLds<false> cs{(lds_c *)blk, cn, cf, rob, ipn, ipf, nullip, ct, ipt};
            units = pgs4<B4_DNL, B4_DC>(m, nl, cs, list, tlist, n_nc, n_c, nnc_max, nc_max, d);
        }
    } else
#endif
    if (in_lds) {
        // byte addresses: records - 8; robot part of slot s at rw + (s - n_nc) ROBW + 2 sl words
        const unsigned cn = 4 * cw - 8, cf = cn + 4 * CRW * n_c, ct = cf + 8 * CRW * n_c, rob = 4 * (rw - (n_nc + 1) * ROBW) + RVB * sl;
        if (wmax(n_rc) > 0) {
            CLds<true> cs{(lds_c *)blk, cn, cf, rob, ipn, ipf, nullip, ct, ipt};
            units = pgs4<B4_DN, B4_DC>(m, ns, cs, list, tlist, n_nc, n_c, nnc_max, nc_max, d);
            rcb = 1;
        } else {
            CLds<false> cs{(lds_c *)blk, cn, cf, rob, ipn, ipf, nullip, ct, ipt};
            units = pgs4<B4_DN, B4_DC>(m, ns, cs, list, tlist, n_nc, n_c, nnc_max, nc_max, d);
        }
    } else {
        const int cn = eo + CR_BASE * 4, cf = cn + 4 * CRW * n_c, ct = cf + 8 * CRW * n_c, rob = ro - ROBW * 4 + RVB * sl;
        CGlb cs{rs, cn, cf, rob, ipn, ipf, nullip, ct, ipt};
        units = pgs4<B4_DN, B4_DG>(m, ns, cs, list, tlist, n_nc, n_c, nnc_max, nc_max, d);
    }
    (void)units; (void)rcb;
    // normal impulses back to the manifold points (warm start + normalForce)
    for (int c = sl; c < n_c; c += 16) st[S_CP + AVR_CP_WORDS * c + AVR_CP_IMP] = imp[n_nc + c];
#ifdef AVR_WAVETIME   // block timeline at its group-0 env: [1][env] (start, end); [2][env] (sweep lengths, LDS path, friction units)
    {
        const unsigned long long wt1 = __builtin_amdgcn_s_memrealtime();
        const int e0 = env0 + 32 * (bidx >> 3) + (bidx & 7);
        if (m.prof && lane == 0 && e0 < n_envs) {
            m.prof[((size_t)1 * n_envs + e0) * 2] = wt0;
            m.prof[((size_t)1 * n_envs + e0) * 2 + 1] = wt1;
            m.prof[((size_t)2 * n_envs + e0) * 2] = (unsigned long long)nnc_max | (unsigned long long)nc_max << 16 | (unsigned long long)in_lds << 32;
            m.prof[((size_t)2 * n_envs + e0) * 2 + 1] = (unsigned long long)wmax(n_rows) | (unsigned long long)units << 16 | (unsigned long long)rcb << 40 | (unsigned long long)xcc_id() << 44;
        }
    }
#endif
    if (!live) return;
    const float *ws = env_ws(m, ev);
    // owner lane f: mass-normalised increments back to (dv, dw) (see put_free)
#if B4_PK
    struct { float vx, vy, vz, wx, wy, wz; } dl = {d.v1.x, d.v2.x, d.v3.x, d.v1.y, d.v2.y, d.v3.y};
#else
    DV &dl = d;
#endif
    if (sl < m.nf) {
        const qt q = ldq(st + S_FREE + AVR_FB_WORDS * sl + 3);
        const v3 I = gld3(m.fb_inertia + 4 * sl);
        const float rs = 1.f / sqrtf(gld(m.fb_mass + (sl)));
        const v3 sd = V(sqrtf(I.x > 0.f ? 1.f / I.x : 0.f), sqrtf(I.y > 0.f ? 1.f / I.y : 0.f), sqrtf(I.z > 0.f ? 1.f / I.z : 0.f));
        const v3 w = qrot(q, V(dl.wx * sd.x, dl.wy * sd.y, dl.wz * sd.z));
        dl.vx *= rs; dl.vy *= rs; dl.vz *= rs;
        dl.wx = w.x; dl.wy = w.y; dl.wz = w.z;
    }
    const float vmax = m.max_vel;
    const int nda = env_hdyn(m, st) ? m.nd + m.hc_n : m.nd;
#pragma unroll
    for (int k = 0; k < NDL; k++) {
        const int dof = sl + 16 * k;
        if (dof < nda) {
            float v = clampf(ws[WS_VQ + dof] + (k == 0 ? d.rq : d.rq2), -vmax, vmax);
            float q = st[S_Q + dof] + dt * v;
            if (frame_end && dof >= m.nd) {
                // enforce_hard_human_joint_limits (env.py:389-410): resetJointState onto the limit, qd = 0
#if K_CHAIN_LIMITS_IN_STATE
                const float lo = st[S_HCH + 2 * K_HC_N + (dof - m.nd)], hi = st[S_HCH + 3 * K_HC_N + (dof - m.nd)];
#else
                const float lo = gld(m.hc_lower + (dof - m.nd)), hi = gld(m.hc_upper + (dof - m.nd));
#endif
                if (q < lo) { q = lo; v = 0.f; }
                else if (q > hi) { q = hi; v = 0.f; }
            }
            st[S_QD + dof] = v;
            st[S_Q + dof] = q;
        }
    }
    if (sl < m.nf) {
        float *fb = st + S_FREE + AVR_FB_WORDS * sl;
        v3 v = clamp3(add(ld3(ws + WS_FV + 4 * sl), V(dl.vx, dl.vy, dl.vz)), vmax);
        v3 om = clamp3(add(ld3(ws + WS_FW + 4 * sl), V(dl.wx, dl.wy, dl.wz)), vmax);
        st3(fb + 7, v);
        st3(fb + 10, om);
        st3(fb, add(ld3(fb), scl(v, dt)));
        float ang = len(om);
        if (ang * dt > BT_ANGULAR_MOTION_THRESHOLD) ang = (0.5f * 1.5707963267948966f) / dt;
        v3 ax;
        if (ang < 0.001f) ax = scl(om, 0.5f * dt - (dt * dt * dt) * 0.020833333333f * ang * ang);
        else ax = scl(om, sinf(0.5f * ang * dt) / ang);
        qt dq = Q(ax.x, ax.y, ax.z, cosf(ang * dt * 0.5f));
        stq(fb + 3, qnorm(qmul(dq, ldq(fb + 3))));
    }
}

__global__ __launch_bounds__(64) void avr_substep_b4_kernel(const KModel *__restrict__ mp, float *__restrict__ state,
                                                            const unsigned char *__restrict__ mask, float dt, int frame_end, int env0,
                                                            int n_envs) {
    __shared__ f4v b4l[B4_LDSW / 4];
    substep_b4_block(*mp, state, mask, dt, frame_end, env0, n_envs, blockIdx.x, (lds_f *)(lds_f4 *)b4l);
}



#if AVR_TASK == AVR_TASK_FEEDING
// Task glue after the frames: update_targets (feeding.py:345-349), iteration count,
// get_total_force (83-90), get_food_rewards (92-121), _get_obs (123-142), reward (56-77),
// TimeLimit; SETTLE mode: target + reset observation only.  NaN guard for every mode.
__global__ __launch_bounds__(64) void avr_task_kernel(const KModel *__restrict__ mp, float *__restrict__ state, float *__restrict__ obs,
                                                      float *__restrict__ rew, unsigned char *__restrict__ done, float *__restrict__ info,
                                                      const unsigned char *__restrict__ mask, int mode, int env0, int n_envs) {
    __shared__ EnvLDS L;
    AVR_ENV_GUARD();
    const int lane = lane_id();
    float *gst = state + (size_t)env * K_STATE_WORDS;
    const float *gcp = gst + S_CP;
    load_state(m, L, gst);
    PROF_START(ptask);
    if (L.nla > m.nl) robot_fk(m, L);    // head pose after the last sub-step (update_targets)
    mouth_target(m, L);
    if (mode == MODE_SETTLE) {
        if (obs) observe(m, L, 0.f, obs + (size_t)env * K_OBS_DIM);
    } else if (mode == MODE_STEP || mode == MODE_STEP_RANDOM) {
        if (lane == 0) L.st[S_TASK + T_ITER] += 1.f;
        SYNC();
        int dummy;
        float robot_force = contact_sum(m, L, gcp, 0, 0, 0, dummy);
        float spoon_force = contact_sum(m, L, gcp, 1, 0, 0, dummy);
        float food_reward = 0.f, hit_reward = 0.f, mouth_vel = 0.f;
        int alive = (int)L.st[S_TASK + T_ALIVE], hit = (int)L.st[S_TASK + T_HIT];
        float succ = L.st[S_TASK + T_SUCCESS];
        v3 tgt = ld3(L.st + S_TASK + T_TARGET);
        for (int k = 0; k < m.n_food; k++) {
            if (!(alive >> k & 1)) continue;
            float *fb = L.st + S_FREE + AVR_FB_WORDS * (m.food_free0 + k);
            v3 fp = ld3(fb);
            int fbody = m.food_body0 + k;
            if (len(sub(tgt, fp)) < 0.02f) {
                food_reward += 20.f;
                succ += 1.f;
                mouth_vel += len(ld3(fb + 7));
                alive &= ~(1 << k);
                SYNC();
                if (lane == 0) st3(fb, V(1500.f + 10.f * k, 1500.f, 1500.f));
                SYNC();
                continue;
            }
            int ctab, cbowl, chum;
            contact_sum(m, L, gcp, 2, fbody, m.table_body, ctab);
            contact_sum(m, L, gcp, 2, fbody, m.bowl_body, cbowl);
            if (fp.z < 0.5f || ctab > 0 || cbowl > 0) {
                food_reward -= 5.f;
                alive &= ~(1 << k);
                continue;
            }
            contact_sum(m, L, gcp, 3, fbody, 0, chum);
            if (chum > 0 && !(hit >> k & 1)) { hit |= 1 << k; hit_reward -= 1.f; }
        }
        SYNC();
        if (lane == 0) {
            L.st[S_TASK + T_ALIVE] = (float)alive;
            L.st[S_TASK + T_HIT] = (float)hit;
            L.st[S_TASK + T_SUCCESS] = succ;
        }
        SYNC();
        const float *sp = L.st + S_FREE + AVR_FB_WORDS * m.spoon_free;
        float ee_vel = len(ld3(sp + 7));
        observe(m, L, spoon_force, obs + (size_t)env * K_OBS_DIM);
        float prefs = m.w_velocity * (-ee_vel) + m.w_force_nontarget * (-robot_force) +
                      m.w_high_forces * (spoon_force < 10.f ? 0.f : -spoon_force) + m.w_food_hit * hit_reward +
                      m.w_food_velocities * (-mouth_vel);
        float dist = len(sub(tgt, ld3(sp)));
        float asq = env_ws(m, env)[WS_ASQ];
        float r = m.w_distance * (-dist) + m.w_action * (-asq) + m.w_food * food_reward + prefs;
        if (lane == 0) {
            rew[env] = r;
            int itn = (int)L.st[S_TASK + T_ITER];
            done[env] = (unsigned char)(itn >= m.max_steps);
            info[(size_t)env * AVR_INFO_DIM + 0] = robot_force + spoon_force;
            info[(size_t)env * AVR_INFO_DIM + 1] = succ >= (float)m.n_food * m.task_success_threshold ? 1.f : 0.f;
        }
    }
    SYNC();
    // NaN guard + flags, then write the state back
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
    PROF_STOP(12, ptask);
    prof_flush(m, L, env);
}

#else
#include "avr_glue_scratch.hip"
#endif  // AVR_TASK

// state[e] = src[e] for the envs whose mask byte is set (masked reset upload)
__global__ void avr_copy_masked_kernel(float *state, const float *src, const unsigned char *mask, int n_envs) {
    const int e = blockIdx.x;
    if (e >= n_envs || !mask[e]) return;
    for (int i = threadIdx.x; i < K_STATE_WORDS; i += blockDim.x) state[(size_t)e * K_STATE_WORDS + i] = src[(size_t)e * K_STATE_WORDS + i];
}
hipError_t avr_launch_copy_masked(float *state, const float *src, const unsigned char *mask, int n_envs, hipStream_t st) {
    if (n_envs <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_copy_masked_kernel, dim3(n_envs), dim3(256), 0, st, state, src, mask, n_envs);
    return hipGetLastError();
}

__global__ void avr_random_actions_kernel(unsigned long long seed, int env_offset, long long t, float *act, int n_envs, int n_arm) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_envs * K_ACT_DIM) return;
    int e = i / K_ACT_DIM, j = i % K_ACT_DIM;
    act[i] = j < n_arm ? philox_action(seed, env_offset + e, t, j) : 0.f;
}

// host-side launch helpers (used by avr_capi.hip)
// One gym step / settle / single sub-step as a sequence of kernels on `stream`:
//   take_step -> frame_skip x nsub x (substep_a, substep_b) -> task      (STEP, STEP_RANDOM)
//   t frames x nsub x (substep_a, substep_b) -> task (settle obs)        (SETTLE)
//   substep_a, substep_b with dt = bit-cast(t)                           (SUBSTEP)
// envs [env0, env1) of the handle; n_envs arguments of the kernels are the end bound env1
hipError_t avr_launch_step(const KModel *h_m, const KModel *d_m, float *state, const float *act, float *obs, float *rew,
                                      unsigned char *done, float *info, const unsigned char *mask, int mode, long long t, int env0,
                                      int env1, hipStream_t stream, avr_evlog *log) {
    const int n_envs = env1 - env0;
    if (n_envs <= 0) return hipSuccess;
    const int nsub = h_m->nsub > 0 ? h_m->nsub : 1;
    const float dt = h_m->time_step / (float)nsub;
    auto mark = [&](int kind) {
        if (log && log->n < log->cap && hipEventRecord(log->ev[log->n], stream) == hipSuccess) log->kind[log->n++] = kind;
    };
    // frame_end: the sub-step closes a gym frame (stepSimulation) and B applies
    // enforce_hard_human_joint_limits (env.py:342-343); the reset's settle frames do not
    auto sub = [&](float h, int frame_end) {
        mark(AVR_K_PAIRS);
        hipLaunchKernelGGL(avr_substep_pairs_kernel, dim3(n_envs), dim3(64), 0, stream, d_m, state, mask, env0, env1);
        mark(AVR_K_NARROW);
        hipLaunchKernelGGL(avr_narrowphase_kernel, dim3(16 * ((n_envs + 8 * NP_ENVS - 1) / (8 * NP_ENVS))), dim3(64), 0, stream, d_m, mask, env0, env1);
#if AVR_COOP_KERNEL
        mark(AVR_K_COOP);
        hipLaunchKernelGGL(avr_coop_kernel, dim3(n_envs), dim3(64), 0, stream, d_m, mask, env0, env1);
#endif
        mark(AVR_K_A);
        hipLaunchKernelGGL(avr_substep_a_kernel, dim3(n_envs), dim3(64), 0, stream, d_m, state, mask, h, env0, env1);
        mark(AVR_K_B);
        hipLaunchKernelGGL(avr_substep_b4_kernel, dim3(8 * ((n_envs + 31) / 32)), dim3(64), 0, stream, d_m, state, mask, h, frame_end, env0, env1);
    };
    if (mode == MODE_SUBSTEP) {
        float h;
        std::memcpy(&h, &t, sizeof(float));
        sub(h, 0);
        mark(-1);
        return hipGetLastError();
    }
    if (mode == MODE_SETTLE) {
        for (long long f = 0; f < t; f++)
            for (int k = 0; k < nsub; k++) sub(dt, 0);
    } else {
        mark(AVR_K_TAKE);
        hipLaunchKernelGGL(avr_take_step_kernel, dim3(8 * ((n_envs + 511) / 512)), dim3(64), 0, stream, d_m, state, act, mask, mode, t, env0, env1);
        for (int f = 0; f < h_m->frame_skip; f++)
            for (int k = 0; k < nsub; k++) sub(dt, k == nsub - 1);
    }
    mark(AVR_K_TASK);
    hipLaunchKernelGGL(avr_task_kernel, dim3(n_envs), dim3(64), 0, stream, d_m, state, obs, rew, done, info, mask, mode, env0, env1);
#if AVR_TASK == AVR_TASK_BEDBATH
    if (mode == MODE_STEP || mode == MODE_STEP_RANDOM)      // stalled closest-distance pairs (avr_glue_bedbath.hip)
        hipLaunchKernelGGL(avr_bb_stall_kernel, dim3(n_envs), dim3(64), 0, stream, d_m, state, rew, mask, env0, env1);
#endif
    mark(-1);
    return hipGetLastError();
}

__global__ void avr_set_step_kernel(long long *dst, long long t) { *dst = t; }
hipError_t avr_launch_set_step(long long *dst, long long t, hipStream_t stream) {
    hipLaunchKernelGGL(avr_set_step_kernel, dim3(1), dim3(1), 0, stream, dst, t);
    return hipGetLastError();
}
// a rollout step's counters for one env group: its step index t and its slot k in the rollout
__global__ void avr_set_step2_kernel(long long *dt, long long t, long long *dk, long long k) {
    if (threadIdx.x == 0) *dt = t;
    else *dk = k;
}
hipError_t avr_launch_set_step2(long long *dt, long long t, long long *dk, long long k, hipStream_t stream) {
    hipLaunchKernelGGL(avr_set_step2_kernel, dim3(1), dim3(2), 0, stream, dt, t, dk, k);
    return hipGetLastError();
}
// a rollout graph's step: the group's step index and slot advance by one (in stream order, before
// the step's take_step reads them)
__global__ void avr_step_advance_kernel(long long *dt, long long *dk) {
    if (threadIdx.x == 0) *dt += 1;
    else *dk += 1;
}
hipError_t avr_launch_step_advance(long long *dt, long long *dk, hipStream_t stream) {
    hipLaunchKernelGGL(avr_step_advance_kernel, dim3(1), dim3(2), 0, stream, dt, dk);
    return hipGetLastError();
}
// a stacked rollout: envs [env0, env1)'s outputs of the step just taken, from the handle's output
// buffers to slot *kslot of the caller's [n][E][...] arrays (one thread per env and word)
__global__ __launch_bounds__(256) void avr_rollout_copy_kernel(const long long *__restrict__ kslot, const float *__restrict__ obs, const float *__restrict__ rew,
                                                               const unsigned char *__restrict__ done, const float *__restrict__ info, float *__restrict__ o_obs,
                                                               float *__restrict__ o_rew, unsigned char *__restrict__ o_done, float *__restrict__ o_info,
                                                               int env0, int env1, int E) {
    constexpr int W = K_OBS_DIM + AVR_INFO_DIM + 2;
    const long long k = *kslot;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int env = env0 + i / W, w = i % W;
    if (env >= env1) return;
    const size_t o = (size_t)k * E + env;
    if (w < K_OBS_DIM) o_obs[o * K_OBS_DIM + w] = obs[(size_t)env * K_OBS_DIM + w];
    else if (w < K_OBS_DIM + AVR_INFO_DIM) o_info[o * AVR_INFO_DIM + (w - K_OBS_DIM)] = info[(size_t)env * AVR_INFO_DIM + (w - K_OBS_DIM)];
    else if (w == K_OBS_DIM + AVR_INFO_DIM) o_rew[o] = rew[env];
    else o_done[o] = done[env];
}
hipError_t avr_launch_rollout_copy(const long long *kslot, const float *obs, const float *rew, const unsigned char *done, const float *info, float *o_obs,
                                   float *o_rew, unsigned char *o_done, float *o_info, int env0, int env1, int E, hipStream_t stream) {
    constexpr int W = K_OBS_DIM + AVR_INFO_DIM + 2;
    const int n = (env1 - env0) * W;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_rollout_copy_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, kslot, obs, rew, done, info, o_obs, o_rew, o_done, o_info,
                       env0, env1, E);
    return hipGetLastError();
}

hipError_t avr_launch_random_actions(unsigned long long seed, int env_offset, long long t, float *act, int n_envs, int n_arm,
                                                hipStream_t stream) {
    int n = n_envs * K_ACT_DIM;
    hipLaunchKernelGGL(avr_random_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, seed, env_offset, t, act, n_envs, n_arm);
    return hipGetLastError();
}

// [vgprs, 0, lds bytes, scratch bytes] of each kernel of a step: pairs, narrowphase, a, b4, task
hipError_t avr_kernel_attrs(int *out20) {
    const void *k[5] = {(const void *)avr_substep_pairs_kernel, (const void *)avr_narrowphase_kernel, (const void *)avr_substep_a_kernel,
                        (const void *)avr_substep_b4_kernel, (const void *)avr_task_kernel};
    for (int i = 0; i < 5; i++) {
        hipFuncAttributes a;
        hipError_t e = hipFuncGetAttributes(&a, k[i]);
        if (e != hipSuccess) return e;
        out20[4 * i + 0] = a.numRegs;
        out20[4 * i + 1] = 0;
        out20[4 * i + 2] = (int)a.sharedSizeBytes;
        out20[4 * i + 3] = (int)a.localSizeBytes;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------- state queries
// (avr_get_q / avr_get_link_pose / avr_get_contact_summary, include/avr.h)
__global__ void avr_get_q_kernel(const float *__restrict__ state, float *__restrict__ q, float *__restrict__ qd, int nd, int n_envs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_envs * nd) return;
    const int e = i / nd, j = i - e * nd;
    if (q) q[i] = state[(size_t)e * K_STATE_WORDS + S_Q + j];
    if (qd) qd[i] = state[(size_t)e * K_STATE_WORDS + S_QD + j];
}

// COM frame of articulated link `link` (< 0: the robot base) by forward kinematics on the current
// joint positions, one block per env
__global__ __launch_bounds__(64) void avr_link_pose_kernel(const KModel *__restrict__ mp, float *__restrict__ state, float *__restrict__ out, int link,
                                                           int n_envs) {
    __shared__ PairsLDS L;
    const int env = blockIdx.x;
    if (env >= n_envs) return;
    const KModel &m = *mp;
    load_state(m, L, state + (size_t)env * K_STATE_WORDS);
    robot_fk(m, L);
    if (lane_id() == 0) {
#if K_RBASE_IN_STATE
        const tf t = link < 0 ? ldtf(L.st + S_RBASE) : ldtf(L.cm[link]);
#else
        const tf t = link < 0 ? tf{V(m.base[0], m.base[1], m.base[2]), Q(m.base[3], m.base[4], m.base[5], m.base[6])} : ldtf(L.cm[link]);
#endif
        float *o = out + (size_t)env * 7;
        o[0] = t.p.x; o[1] = t.p.y; o[2] = t.p.z; o[3] = t.q.x; o[4] = t.q.y; o[5] = t.q.z; o[6] = t.q.w;
    }
}

// {points, sum normalForce, robot-human, tool-human} of each env's contact pool
__global__ void avr_contact_summary_kernel(const KModel *__restrict__ mp, const float *__restrict__ state, float *__restrict__ out, int n_envs) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= n_envs) return;
    const KModel &m = *mp;
    const float *st = state + (size_t)env * K_STATE_WORDS;
    const int n = (int)st[S_TASK + T_NCP];
    float all = 0.f, rh = 0.f, th = 0.f;
    for (int i = 0; i < n; i++) {
        const float *cp = st + S_CP + AVR_CP_WORDS * i;
        const int ba = m.shape_body[(int)cp[AVR_CP_SA]], bb = m.shape_body[(int)cp[AVR_CP_SB]];
        const int ka = m.body_kind[ba], kb = m.body_kind[bb];
        const float f = cp[AVR_CP_IMP] / m.time_step;
        const bool ha = ka == AVR_BODY_HUMAN, hb = kb == AVR_BODY_HUMAN;
        const bool ra = ka == AVR_BODY_ROBOT || ka == AVR_BODY_RSTATIC, rb = kb == AVR_BODY_ROBOT || kb == AVR_BODY_RSTATIC;
        all += f;
        if ((ra && hb) || (rb && ha)) rh += f;
        if ((ba == m.tool_body && hb) || (bb == m.tool_body && ha)) th += f;
    }
    float *o = out + (size_t)env * 4;
    o[0] = (float)n; o[1] = all; o[2] = rh; o[3] = th;
}

// per-env health flags (T_FLAGS word: bit0 NaN / failed factorisation, bit1 contact pool full, ...)
__global__ void avr_get_flags_kernel(const float *__restrict__ state, int *__restrict__ out, int n_envs) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n_envs) out[e] = (int)state[(size_t)e * K_STATE_WORDS + S_TASK + T_FLAGS];
}

hipError_t avr_launch_get_flags(const float *state, int *out, int n_envs, hipStream_t st) {
    if (n_envs <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_get_flags_kernel, dim3((n_envs + 255) / 256), dim3(256), 0, st, state, out, n_envs);
    return hipGetLastError();
}

hipError_t avr_launch_get_q(const float *state, float *q, float *qd, int nd, int n_envs, hipStream_t st) {
    const int n = nd * n_envs;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(avr_get_q_kernel, dim3((n + 255) / 256), dim3(256), 0, st, state, q, qd, nd, n_envs);
    return hipGetLastError();
}
hipError_t avr_launch_link_pose(const KModel *d_m, float *state, float *out, int link, int n_envs, hipStream_t st) {
    hipLaunchKernelGGL(avr_link_pose_kernel, dim3(n_envs), dim3(64), 0, st, d_m, state, out, link, n_envs);
    return hipGetLastError();
}
hipError_t avr_launch_contact_summary(const KModel *d_m, const float *state, float *out, int n_envs, hipStream_t st) {
    hipLaunchKernelGGL(avr_contact_summary_kernel, dim3((n_envs + 63) / 64), dim3(64), 0, st, d_m, state, out, n_envs);
    return hipGetLastError();
}

