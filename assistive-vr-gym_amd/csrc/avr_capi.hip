// avr_capi.hip -- body of the C-ABI of libavr.so (include/avr.h) for one task: device arenas, scene
// upload, launches.  Included once per task inside that task's namespace (avr_task_*.hip); the
// extern "C" entry points in avr_api.cpp dispatch to it by the handle's task.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>
#include <cstring>
#include <cmath>

#include "../../include/avr.h"

#define AVR_MAX_GROUPS 8
#define AVR_GRAPH_SLOTS 4
#define AVR_ROLL_CHUNK 16      // steps per rollout graph replay (avr_rollout_random_device)

struct avr_sim {
    avr_config cfg;
    KModel km;          // host copy
    KModel *d_km;       // device copy (the kernel reads the scene description through it)
    hipStream_t stream;
    std::vector<void *> allocs;
    float *d_state;
    float *d_stage;     // [n_envs][STATE_WORDS] host-upload staging (masked resets)
    uint8_t *d_mask;    // [n_envs]
    float *d_act, *d_obs, *d_rew, *d_info;
    unsigned char *d_done;
    char err[512];
    // env groups on their own streams: group g's launch sequence runs concurrently with the
    // others', so latency-bound PGS waves of one group share the CUs with compute-bound
    // collision waves of another (envs are independent; fork/join events keep the handle's
    // stream the single point of ordering for callers)
    int ngroups;
    hipStream_t gstream[AVR_MAX_GROUPS];
    hipEvent_t fork_ev, join_ev[AVR_MAX_GROUPS];
    avr_evlog evlog;                       // per-kernel timing (avr_profile_kernels)
    std::vector<hipEvent_t> ev;
    std::vector<int> evkind;
    double kt_ms[AVR_K_KINDS];
    long long kt_n[AVR_K_KINDS];
    float *d_query;                        // device scratch of the state queries (avr_get_*)
    size_t qcap;
    float *d_ik;                           // device scratch of avr_reset_ik (targets, restart draws, ok bytes)
    size_t ikcap;
    float *d_bs;                           // device scratch of avr_base_search (draws, goals, per-attempt results)
    size_t bscap;
    // the step's launch sequence (every group's launches and the fork / join events) captured
    // once as a HIP graph and replayed.  A graph reads its actions from the handle's own d_act
    // (a caller's action buffer is copied there in stream order first), so it is keyed only by
    // the output buffers and the mode: one executable graph per key, a few keys cached (least
    // recently used evicted).  The take-step nodes read the step counter from km.step_t, written
    // in stream order before each replay; an executable graph is never edited.
    int use_graph;
    struct GraphSlot { hipGraph_t graph; hipGraphExec_t gexec; const void *key[5]; unsigned long long used; };
    GraphSlot gslot[AVR_GRAPH_SLOTS];
    // rollouts (avr_rollout_random_device): graphs of AVR_ROLL_CHUNK steps (and of one step, for
    // the remainder) in which every env group runs all its steps back to back on its own branch,
    // with its own step counter advanced on the device before each step; the branches are
    // forked and joined once per replay, not after every step
    struct RollSlot {
        hipGraph_t graph[2]; hipGraphExec_t gexec[2];                                       // branches: [chunk, 1 step]
        hipGraph_t pgraph[2][2][AVR_MAX_GROUPS]; hipGraphExec_t pgexec[2][2][AVR_MAX_GROUPS];  // per group: [chunk, 1 step][copy][group]
        const void *key[8];
        unsigned long long used;
    };
    RollSlot rslot[AVR_GRAPH_SLOTS];
    unsigned long long gclock;
    long long n_captures;                  // diagnostics (avr_graph_captures)
};

// Every entry point runs on the handle's device and restores the caller's current device on
// return: scratch buffers allocated lazily (hipMalloc) land on the handle's GPU whatever device
// the caller (or another handle, or torch) made current.
struct DevGuard {
    // makes device d current for the call and restores the caller's; an out-of-range d (a handle
    // whose avr_create failed) is left alone, and a failed switch does not leave its error behind
    // for the next hipGetLastError of a launch check
    int prev = -1;
    explicit DevGuard(int d) {
        int n = 0, cur = -1;
        if (d < 0 || hipGetDeviceCount(&n) != hipSuccess || d >= n || hipGetDevice(&cur) != hipSuccess) { (void)hipGetLastError(); return; }
        if (cur == d) return;
        if (hipSetDevice(d) == hipSuccess) prev = cur;
        else (void)hipGetLastError();
    }
    ~DevGuard() {
        if (prev >= 0 && hipSetDevice(prev) != hipSuccess) (void)hipGetLastError();
    }
};

static int fail(avr_sim *s, int code, const char *fmt, ...) {
    if (s) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(s->err, sizeof(s->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(s, x)                                                                      \
    do {                                                                                  \
        hipError_t _e = (x);                                                              \
        if (_e != hipSuccess) return fail((s), -3, "%s: %s", #x, hipGetErrorString(_e)); \
    } while (0)

template <typename T>
static int upload(avr_sim *s, const std::vector<T> &h, const T **out) {
    void *d = nullptr;
    size_t n = h.size() ? h.size() : 1;
    HIPCHK(s, hipMalloc(&d, n * sizeof(T)));
    s->allocs.push_back(d);
    if (h.size()) HIPCHK(s, hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = (const T *)d;
    return 0;
}

static std::vector<float> cvt(const double *p, size_t n, int stride_in = 1, int stride_out = 1, int count = -1) {
    if (count < 0) {
        std::vector<float> v(n);
        for (size_t i = 0; i < n; i++) v[i] = (float)p[i];
        return v;
    }
    std::vector<float> v((size_t)count * stride_out, 0.f);
    for (int i = 0; i < count; i++)
        for (int k = 0; k < stride_in; k++) v[(size_t)i * stride_out + k] = (float)p[(size_t)i * stride_in + k];
    return v;
}

static std::vector<int> ivec(const int32_t *p, size_t n) { return std::vector<int>(p, p + n); }

// host (double) transform helpers for precomputed static geometry; quaternions are x y z w
static void hq_mul(const double *a, const double *b, double *o) {
    double r[4] = {a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1], a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0],
                   a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3], a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]};
    for (int i = 0; i < 4; i++) o[i] = r[i];
}
static void hq_mat(const double *q, double R[3][3]) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    R[0][0] = 1 - 2 * (y * y + z * z); R[0][1] = 2 * (x * y - z * w); R[0][2] = 2 * (x * z + y * w);
    R[1][0] = 2 * (x * y + z * w); R[1][1] = 1 - 2 * (x * x + z * z); R[1][2] = 2 * (y * z - x * w);
    R[2][0] = 2 * (x * z - y * w); R[2][1] = 2 * (y * z + x * w); R[2][2] = 1 - 2 * (x * x + y * y);
}

// world AABB of shape s on a static body: aabb_of(body * shape_pose, center, half) as in the kernel
static void static_shape_aabb(const avr_model_desc *d, int s, float *out8) {
    const int b = d->shape_body[s];
    const double *bp = d->st_pose + 7 * d->body_index[b];
    const double *sp = d->shape_pose + 7 * s;
    double R[3][3], q[4], p[3];
    hq_mat(bp + 3, R);
    for (int i = 0; i < 3; i++) p[i] = bp[i] + R[i][0] * sp[0] + R[i][1] * sp[1] + R[i][2] * sp[2];
    hq_mul(bp + 3, sp + 3, q);
    double T[3][3];
    hq_mat(q, T);
    const double *c = d->shape_aabb + 6 * s, *h = c + 3;
    for (int i = 0; i < 3; i++) {
        double cw = p[i] + T[i][0] * c[0] + T[i][1] * c[1] + T[i][2] * c[2];
        double hw = fabs(T[i][0]) * h[0] + fabs(T[i][1]) * h[1] + fabs(T[i][2]) * h[2];
        out8[i] = (float)(cw - hw);
        out8[4 + i] = (float)(cw + hw);
    }
    out8[3] = out8[7] = 0.f;
}

// pose arrays: [n][pos3 + quat4] -> [n][8]
static std::vector<float> poses(const double *pos, const double *quat, int n) {
    std::vector<float> v((size_t)n * 8, 0.f);
    for (int i = 0; i < n; i++) {
        for (int k = 0; k < 3; k++) v[8 * i + k] = (float)pos[3 * i + k];
        for (int k = 0; k < 4; k++) v[8 * i + 3 + k] = (float)quat[4 * i + k];
    }
    return v;
}


int avr_create(const avr_config *cfg, const avr_model_desc *d, avr_sim **out) {
    if (!cfg || !d || !out) return -1;
    *out = nullptr;
    avr_sim *s = new avr_sim();
    memset(s->err, 0, sizeof(s->err));
    s->cfg = *cfg;
    if (cfg->n_envs <= 0) { int r = fail(s, -1, "n_envs must be > 0"); *out = s; return r; }
    if (cfg->flags & AVR_CFG_RESERVED_MASK) { int r = fail(s, -1, "avr_config.flags 0x%x: no flag is defined", (unsigned)cfg->flags); *out = s; return r; }
    const int hc = d->hc_n > 0 ? d->hc_n : 0;
    if (d->task != AVR_TASK) { int r = fail(s, -2, "model task %d does not match this instantiation (%d)", (int)d->task, (int)AVR_TASK); *out = s; return r; }
    if (d->n_dof != K_ND) { int r = fail(s, -2, "model has %d robot DoFs, this instantiation %d", (int)d->n_dof, (int)K_ND); *out = s; return r; }
    if (d->n_links + hc > K_MAX_LINKS || d->n_dof + hc > K_MAX_DOF || d->n_free > K_MAX_FREE || d->n_human > K_MAX_HUMAN ||
        d->n_bodies > MAXB || d->n_pairs > 65535 || d->n_shapes > MAXSH || d->n_arm > K_ACT_DIM || hc > K_HC_N || hc > AVR_DESC_HC ||
        d->n_free < 1 || d->robot_gravity[0] != 0.0 || d->robot_gravity[1] != 0.0 || d->robot_gravity[2] != 0.0) {
        int r = fail(s, -2, "model exceeds compiled capacities");
        *out = s;
        return r;
    }
    for (int b = 0; b < d->n_bodies; b++)
        if (d->body_shape_count[b] > 128 || d->body_shape_count[b] < 0) {
            // the pair kernel's culled child lists (candA / candB) hold 128 entries
            int r = fail(s, -2, "body %d has %d shapes (> 128)", b, (int)d->body_shape_count[b]);
            *out = s;
            return r;
        }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) { int r = fail(s, -4, "no HIP device available (%s)", hipGetErrorString(e)); *out = s; return r; }
    if (cfg->device < 0 || cfg->device >= ndev) { int r = fail(s, -4, "device %d out of range (%d devices)", cfg->device, ndev); *out = s; return r; }
    *out = s;
    DevGuard dg(cfg->device);
    {
        int cur = -1;
        HIPCHK(s, hipGetDevice(&cur));
        if (cur != cfg->device) return fail(s, -4, "hipSetDevice(%d) failed", cfg->device);
    }
    HIPCHK(s, hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    {
        // default: one group per 1024 envs, at most 4 (4096 envs: 600k -> 680k env-steps/s, the
        // groups' kernels fill each other's launch tails; 4 streams stay within the runtime's
        // default of 4 hardware queues, past which streams share queues and serialise).
        // AVR_ENV_GROUPS=1..8 overrides.
        const char *g = getenv("AVR_ENV_GROUPS");
        int ng = g ? atoi(g) : std::min(4, std::max(1, cfg->n_envs / 1024));
        if (ng < 1) ng = 1;
        if (ng > AVR_MAX_GROUPS) ng = AVR_MAX_GROUPS;
        if (ng > cfg->n_envs) ng = cfg->n_envs;
        s->ngroups = ng;
        const char *gr = getenv("AVR_GRAPH");
        s->use_graph = gr ? atoi(gr) : 1;

        HIPCHK(s, hipEventCreateWithFlags(&s->fork_ev, hipEventDisableTiming));
        for (int i = 1; i < ng; i++) {      // (group 0 runs on the handle's stream)
            HIPCHK(s, hipStreamCreateWithFlags(&s->gstream[i], hipStreamNonBlocking));
            HIPCHK(s, hipEventCreateWithFlags(&s->join_ev[i], hipEventDisableTiming));
        }
    }
    KModel &k = s->km;
    memset(&k, 0, sizeof(k));
    int nl = d->n_links, nb = d->n_bodies, ns = d->n_shapes;
    k.nl = nl; k.nd = d->n_dof; k.nf = d->n_free; k.nb = nb; k.ns = ns; k.np = d->n_pairs; k.nh = d->n_human;
    // articulated link tables: robot links, then the tremor head/neck chain (avr_kmodel.h)
    const int nla = nl + hc;
    k.nla = nla; k.hc_n = hc; k.np_base = hc > 0 ? d->n_pairs_base : d->n_pairs;
    std::vector<int> par(nla), jt(nla), dofv(nla), hasl(nla);
    std::vector<float> jorig((size_t)2 * nla * 8, 0.f), com((size_t)2 * nla * 8, 0.f), axis((size_t)nla * 4, 0.f),
        inert((size_t)2 * nla * 4, 0.f), mass((size_t)2 * nla, 0.f), lo(nla), hi(nla);
    for (int i = 0; i < nl; i++) {
        par[i] = d->rl_parent[i]; jt[i] = d->rl_jtype[i]; dofv[i] = d->rl_dof[i]; hasl[i] = d->rl_has_limit[i];
        lo[i] = (float)d->rl_lower[i]; hi[i] = (float)d->rl_upper[i];
        for (int q = 0; q < 3; q++) axis[4 * i + q] = (float)d->rl_axis[3 * i + q];
        for (int g = 0; g < 2; g++) {
            const size_t o = (size_t)g * nla + i;
            for (int q = 0; q < 3; q++) {
                jorig[8 * o + q] = (float)d->rl_jpos[3 * i + q];
                com[8 * o + q] = (float)d->rl_com_pos[3 * i + q];
                inert[4 * o + q] = (float)d->rl_inertia[3 * i + q];
            }
            for (int q = 0; q < 4; q++) {
                jorig[8 * o + 3 + q] = (float)d->rl_jquat[4 * i + q];
                com[8 * o + 3 + q] = (float)d->rl_com_quat[4 * i + q];
            }
            mass[o] = (float)d->rl_mass[i];
        }
    }
    for (int c = 0; c < hc; c++) {
        const int i = nl + c;
        par[i] = c == 0 ? -2 : i - 1; jt[i] = AVR_J_REVOLUTE; dofv[i] = d->n_dof + c; hasl[i] = 1;
        lo[i] = (float)d->hc_lower[c]; hi[i] = (float)d->hc_upper[c];
        for (int q = 0; q < 3; q++) axis[4 * i + q] = (float)d->hc_axis[c][q];
        for (int g = 0; g < 2; g++) {
            const size_t o = (size_t)g * nla + i;
            for (int q = 0; q < 3; q++) {
                jorig[8 * o + q] = (float)d->hc_jpos[g][c][q];
                inert[4 * o + q] = (float)d->hc_inertia[g][c][q];
            }
            jorig[8 * o + 6] = 1.f;   // identity joint frame rotation
            com[8 * o + 6] = 1.f;     // COM frame == link frame (human_creation.py: inertial offsets 0)
            mass[o] = (float)d->hc_mass[g][c];
        }
        k.hc_slot[c] = d->hc_slot[c]; k.hc_body[c] = d->hc_body[c];
        k.hc_lower[c] = lo[i]; k.hc_upper[c] = hi[i];
    }
    k.hc_parent_slot = d->hc_parent_slot;
    k.human_gain = (float)d->human_gain; k.human_force = (float)d->human_force;
    for (int q = 0; q < 3; q++) {
        k.hc_grav[q] = (float)d->human_gravity[q];
        k.fix_pivot_b[q] = (float)d->fix_pivot_b[q];
        k.tool_tip[q] = (float)d->tool_tip[q];
        k.torso_com[q] = (float)d->torso_com[q];
    }
    k.tool_handle_shapes = d->tool_handle_shapes;
    k.w_tool_force = (float)d->w_tool_force; k.w_scratch = (float)d->w_scratch;
    int r;
#if AVR_TASK == AVR_TASK_BEDBATH
    {
        bool okt = d->bb_targets != nullptr;
        for (int g = 0; g < 2; g++)
            okt = okt && d->bb_ntgt[g][0] >= 0 && d->bb_ntgt[g][1] >= 0 && d->bb_ntgt[g][0] + d->bb_ntgt[g][1] <= AVR_BB_MAX_TARGETS &&
                  d->bb_ntgt[g][0] + d->bb_ntgt[g][1] <= 6 * 24;
        for (int q = 0; q < 2; q++) okt = okt && d->bb_limb_slots[q] >= 0 && d->bb_limb_slots[q] < d->n_human;
        for (int q = 0; q < 3; q++) okt = okt && d->bb_joint_slots[q] >= 0 && d->bb_joint_slots[q] < d->n_human;
        if (!okt) return fail(s, -2, "BedBathing: wipe targets / limb slots out of range");
        std::vector<float4> tg(2 * AVR_BB_MAX_TARGETS);
        for (int i = 0; i < 2 * AVR_BB_MAX_TARGETS; i++)
            tg[i] = make_float4((float)d->bb_targets[4 * i], (float)d->bb_targets[4 * i + 1], (float)d->bb_targets[4 * i + 2], (float)d->bb_targets[4 * i + 3]);
        if ((r = upload(s, tg, &k.bb_tgt))) return r;
        for (int g = 0; g < 2; g++) { k.bb_ntgt[g][0] = d->bb_ntgt[g][0]; k.bb_ntgt[g][1] = d->bb_ntgt[g][1]; }
        for (int q = 0; q < 2; q++) k.bb_limb_slot[q] = d->bb_limb_slots[q];
        for (int q = 0; q < 3; q++) k.bb_joint_slot[q] = d->bb_joint_slots[q];
        k.w_wipe = (float)d->w_wipe;
        k.closest_distance = (float)d->closest_distance;
    }
#endif
    if ((r = upload(s, par, &k.rl_parent))) return r;
    if ((r = upload(s, jt, &k.rl_jtype))) return r;
    if ((r = upload(s, dofv, &k.rl_dof))) return r;
    if ((r = upload(s, hasl, &k.rl_has_limit))) return r;
    if ((r = upload(s, jorig, &k.rl_jorig))) return r;
    if ((r = upload(s, com, &k.rl_com))) return r;
    if ((r = upload(s, axis, &k.rl_axis))) return r;
    if ((r = upload(s, inert, &k.rl_inertia))) return r;
    if ((r = upload(s, mass, &k.rl_mass))) return r;
    if ((r = upload(s, lo, &k.rl_lower))) return r;
    if ((r = upload(s, hi, &k.rl_upper))) return r;
    for (int i = 0; i < 7; i++) k.base[i] = (float)d->robot_base[i];
    if ((r = upload(s, cvt(d->fb_mass, d->n_free), &k.fb_mass))) return r;
    if ((r = upload(s, cvt(d->fb_inertia, 0, 3, 4, d->n_free), &k.fb_inertia))) return r;
    if ((r = upload(s, cvt(d->fb_gravity, 0, 3, 4, d->n_free), &k.fb_gravity))) return r;
    if ((r = upload(s, cvt(d->st_pose, 0, 7, 8, d->n_static), &k.st_pose))) return r;
    if ((r = upload(s, ivec(d->body_kind, nb), &k.body_kind))) return r;
    if ((r = upload(s, ivec(d->body_index, nb), &k.body_index))) return r;
    if ((r = upload(s, ivec(d->body_shape_start, nb), &k.body_shape_start))) return r;
    if ((r = upload(s, ivec(d->body_shape_count, nb), &k.body_shape_count))) return r;
    if ((r = upload(s, ivec(d->body_flags, nb), &k.body_flags))) return r;
    if ((r = upload(s, cvt(d->body_friction, nb), &k.body_friction))) return r;
    if ((r = upload(s, cvt(d->body_threshold, nb), &k.body_threshold))) return r;
    {
        // rolling / spinning friction per body (ABI 5; NULL: none)
        std::vector<float> zr(nb, 0.f);
        if ((r = upload(s, d->body_rolling ? cvt(d->body_rolling, nb) : zr, &k.body_rolling))) return r;
        if ((r = upload(s, d->body_spinning ? cvt(d->body_spinning, nb) : zr, &k.body_spinning))) return r;
#if !K_TORSION
        for (int b = 0; b < nb; b++)
            if ((d->body_rolling && d->body_rolling[b] != 0.0) || (d->body_spinning && d->body_spinning[b] != 0.0))
                return fail(s, -2, "body %d has rolling / spinning friction: this instantiation has no torsional rows", b);
#endif
    }
    if ((r = upload(s, cvt(d->body_aabb, (size_t)nb * 12), &k.body_aabb))) return r;
    if ((r = upload(s, ivec(d->shape_kind, ns), &k.shape_kind))) return r;
    if ((r = upload(s, ivec(d->shape_body, ns), &k.shape_body))) return r;
    if ((r = upload(s, ivec(d->shape_gender, ns), &k.shape_gender))) return r;
    if ((r = upload(s, ivec(d->shape_hull, (size_t)ns * 4), &k.shape_hull))) return r;
    if ((r = upload(s, cvt(d->shape_pose, 0, 7, 8, ns), &k.shape_pose))) return r;
    if ((r = upload(s, cvt(d->shape_param, (size_t)ns * 4), &k.shape_param))) return r;
    if ((r = upload(s, cvt(d->shape_margin, ns), &k.shape_margin))) return r;
    {
        std::vector<float> a((size_t)ns * 8, 0.f);
        for (int i = 0; i < ns; i++) {
            for (int q = 0; q < 3; q++) a[8 * i + q] = (float)d->shape_aabb[6 * i + q];
            for (int q = 0; q < 3; q++) a[8 * i + 4 + q] = (float)d->shape_aabb[6 * i + 3 + q];
        }
        if ((r = upload(s, a, &k.shape_aabb))) return r;
    }
    {
        std::vector<float4> hv((size_t)d->n_hull_verts);
        for (int i = 0; i < d->n_hull_verts; i++)
            hv[i] = make_float4((float)d->hull_verts[3 * i], (float)d->hull_verts[3 * i + 1], (float)d->hull_verts[3 * i + 2], 0.f);
        if ((r = upload(s, hv, &k.hull_verts))) return r;
        // support tables for the large hulls (exact sub-linear support queries, avr_hulltab.cpp)
        std::vector<int> stab(ns, -1);
        std::vector<int2> cells;
        std::vector<float4> cand;
        const int G = AVR_TAB_G, nc = 6 * G * G;
        // hulls with more than tab_min vertices get a table (AVR_TAB_MIN_NV overrides it for experiments)
        int tab_min = AVR_TAB_MIN_NV;
        if (const char *e = getenv("AVR_TAB_MIN_NV")) tab_min = atoi(e);
        for (int i = 0; i < ns; i++) {
            const int vs = d->shape_hull[4 * i], nvh = d->shape_hull[4 * i + 1];
            if (d->shape_kind[i] != AVR_HULL || nvh <= tab_min) continue;
            std::vector<float> pv((size_t)nvh * 3);
            for (int q = 0; q < nvh; q++) { pv[3 * q] = hv[vs + q].x; pv[3 * q + 1] = hv[vs + q].y; pv[3 * q + 2] = hv[vs + q].z; }
            std::vector<int32_t> cl((size_t)2 * nc);
            const int tot = avr_hull_support_table(pv.data(), nvh, G, cl.data(), nullptr, 0);
            if (tot < 0) return fail(s, -2, "support table for shape %d failed", i);
            std::vector<int32_t> ix((size_t)tot);
            avr_hull_support_table(pv.data(), nvh, G, cl.data(), ix.data(), tot);
            stab[i] = (int)cells.size();
            const int base = (int)cand.size();
            for (int c = 0; c < nc; c++) cells.push_back(make_int2(base + cl[2 * c], cl[2 * c + 1]));
            for (int q = 0; q < tot; q++) {
                const float4 v = hv[vs + ix[q]];
                float w;
                std::memcpy(&w, &ix[q], sizeof w);
                cand.push_back(make_float4(v.x, v.y, v.z, w));
            }
        }
        if (cells.empty()) { cells.push_back(make_int2(0, 0)); cand.push_back(make_float4(0.f, 0.f, 0.f, 0.f)); }
        if ((r = upload(s, stab, &k.shape_tab))) return r;
        if ((r = upload(s, cells, &k.tab_cell))) return r;
        if ((r = upload(s, cand, &k.tab_vert))) return r;
    }
    {
        // child AABB cache slots for the non-static shapes; static shapes get host-computed AABBs
        std::vector<int> cidx(ns, -1);
        std::vector<float> saabb((size_t)ns * 8, 0.f);
        int nc = 0;
        for (int i = 0; i < ns; i++) {
            if (d->body_kind[d->shape_body[i]] == AVR_BODY_STATIC) static_shape_aabb(d, i, &saabb[8 * (size_t)i]);
            else cidx[i] = nc++;
        }
        if (nc > MAXCC) return fail(s, -2, "model has %d non-static shapes > MAXCC %d", nc, MAXCC);
        if ((r = upload(s, cidx, &k.shape_cidx))) return r;
        if ((r = upload(s, saabb, &k.static_saabb))) return r;
        // packed per-shape and per-candidate-pair records: one load each in the pair kernel
        std::vector<int> sinfo(ns);
        for (int i = 0; i < ns; i++) sinfo[i] = (cidx[i] + 1) | ((d->shape_gender[i] + 1) << 9) | (d->shape_kind[i] << 11);
        if ((r = upload(s, sinfo, &k.shape_info))) return r;
        std::vector<int4> prec(d->n_pairs > 0 ? d->n_pairs : 1);
        for (int p = 0; p < d->n_pairs; p++) {
            const int ba = d->pair_a[p], bb = d->pair_b[p];
            const int na = d->body_shape_count[ba], nbs = d->body_shape_count[bb];
            const int bare = (d->body_flags[ba] & 1) && (d->body_flags[bb] & 1);
            prec[p] = make_int4(ba | (bb << 16), d->body_shape_start[ba] | (na << 16), d->body_shape_start[bb] | (nbs << 16),
                                bare | ((na == 1 && nbs == 1) ? 2 : 0));
        }
        if ((r = upload(s, prec, &k.pair_rec))) return r;
    }
    if ((r = upload(s, ivec(d->pair_a, d->n_pairs), &k.pair_a))) return r;
    if ((r = upload(s, ivec(d->pair_b, d->n_pairs), &k.pair_b))) return r;
    k.n_arm = d->n_arm;
    for (int i = 0; i < 8; i++) { k.arm_dofs[i] = d->arm_dofs[i]; k.arm_lower[i] = (float)d->arm_lower[i]; k.arm_upper[i] = (float)d->arm_upper[i]; }
    for (int i = d->n_arm; i < 8; i++) { k.arm_lower[i] = -1e10f; k.arm_upper[i] = 1e10f; }
    k.n_finger = d->n_finger;
    for (int i = 0; i < 4; i++) k.finger_dofs[i] = d->finger_dofs[i];
    k.tool_link = d->tool_link; k.torso_link = d->torso_link; k.head_slot = d->head_slot;
    k.spoon_free = d->spoon_free; k.bowl_free = d->bowl_free; k.food_free0 = d->food_free0; k.n_food = d->n_food;
    k.table_body = d->table_body; k.bowl_body = d->bowl_body; k.spoon_body = d->spoon_body; k.food_body0 = d->food_body0;
    k.tool_body = d->spoon_body;     // the tool on the fixed constraint (spoon / scratcher)
    for (int i = 0; i < 7; i++) k.tool_offset[i] = (float)d->tool_offset[i];
    for (int g = 0; g < 2; g++)
        for (int i = 0; i < 3; i++) k.mouth[g][i] = (float)d->mouth_offset[g][i];
    k.time_step = (float)d->time_step;
    k.nsub = d->num_sub_steps; k.frame_skip = d->frame_skip; k.iters = d->solver_iterations; k.max_steps = d->max_episode_steps;
    k.erp = (float)d->erp; k.warmstart = (float)d->warmstart; k.lin_damp = (float)d->linear_damping; k.ang_damp = (float)d->angular_damping;
    k.max_vel = (float)d->max_coord_vel; k.robot_gain = (float)d->robot_gain; k.robot_force = (float)d->robot_force;
    k.fixed_max_imp = (float)(d->fixed_max_force * d->time_step);
    k.w_distance = (float)d->w_distance; k.w_action = (float)d->w_action; k.w_food = (float)d->w_food;
    k.w_velocity = (float)d->w_velocity; k.w_force_nontarget = (float)d->w_force_nontarget; k.w_high_forces = (float)d->w_high_forces;
    k.w_food_hit = (float)d->w_food_hit; k.w_food_velocities = (float)d->w_food_velocities;
    k.task_success_threshold = (float)d->task_success_threshold;
    k.seed = cfg->seed;
    k.env_offset = cfg->env_offset;
    for (int i = 0; i < K_MAX_DOF; i++) k.dof_link[i] = 0;
    for (int l = 0; l < nla; l++)
        if (dofv[l] >= 0) k.dof_link[dofv[l]] = l;
    for (int l = 0; l < nla; l++) {
        unsigned mask = 0;
        for (int q = l; q >= 0; q = par[q]) mask |= 1u << q;
        k.anc_mask[l] = mask;
    }
    for (int l = 0; l < nla; l++) {
        unsigned dm = 0;
        for (int q = 0; q < nla; q++)
            if ((k.anc_mask[q] >> l) & 1u) dm |= 1u << q;
        k.desc_mask[l] = dm;
    }
    // tree levels (parents precede children in DFS order): the kinematics passes run level by level
    k.nlev = 0;
    for (int l = 0; l < nla; l++) {
        k.rl_level[l] = par[l] < 0 ? 0 : k.rl_level[par[l]] + 1;
        if (k.rl_level[l] + 1 > k.nlev) k.nlev = k.rl_level[l] + 1;
    }
    size_t E = (size_t)cfg->n_envs;
    // per-env constraint-row scratch (written and read inside each sub-step)
    k.rowcap = MAXNC + K_CROWS * K_MAX_CONTACTS;
    // records [rowcap][20] then robot parts [rowcap][32]; part B reads the whole row buffer
    // through one buffer resource with 32-bit byte offsets below B4_OOB (avr_kernel.hip)
    k.rowstride = (RWC + ROBW) * k.rowcap;
    k.rows_envs = (int)E;
    k.b4_global = getenv("AVR_B4_GLOBAL") && getenv("AVR_B4_GLOBAL")[0] == '1';
    if (E * (size_t)k.rowstride * sizeof(float) >= 0x7fff0000ull) {
        int r = fail(s, -2, "n_envs %d exceeds the row-buffer addressing limit (%d per handle)", cfg->n_envs, (int)(0x7fff0000ull / (k.rowstride * sizeof(float))));
        return r;
    }
    {
        float *rows = nullptr;
        HIPCHK(s, hipMalloc(&rows, E * (size_t)k.rowstride * sizeof(float)));
        s->allocs.push_back(rows);
        // diagnostic: NaN-fill the row scratch so that a read of a word no kernel wrote shows
        if (getenv("AVR_DEBUG_NANFILL")) HIPCHK(s, hipMemset(rows, 0xFF, E * (size_t)k.rowstride * sizeof(float)));
        k.rows = rows;
        float *ws = nullptr;
        HIPCHK(s, hipMalloc(&ws, E * 128 * sizeof(float)));
        HIPCHK(s, hipMemset(ws, 0, E * 128 * sizeof(float)));
        s->allocs.push_back(ws);
        k.ws = ws;
        float *cscr = nullptr;
        HIPCHK(s, hipMalloc(&cscr, E * (size_t)CS_WORDS * sizeof(float)));
        HIPCHK(s, hipMemset(cscr, 0, E * (size_t)CS_WORDS * sizeof(float)));
        s->allocs.push_back(cscr);
        k.cscr = cscr;
    }
    {
        long long *st = nullptr;      // per env group: the step index (take_step) and, in a rollout, the step's slot
        HIPCHK(s, hipMalloc(&st, 2 * AVR_MAX_GROUPS * sizeof(long long)));
        HIPCHK(s, hipMemset(st, 0, 2 * AVR_MAX_GROUPS * sizeof(long long)));
        s->allocs.push_back(st);
        k.step_t = st;
    }
    HIPCHK(s, hipMalloc(&s->d_km, sizeof(KModel)));
    HIPCHK(s, hipMemcpy(s->d_km, &s->km, sizeof(KModel), hipMemcpyHostToDevice));
    HIPCHK(s, hipMalloc(&s->d_state, E * K_STATE_WORDS * sizeof(float)));
    HIPCHK(s, hipMemset(s->d_state, 0, E * K_STATE_WORDS * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_act, E * K_ACT_DIM * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_obs, E * K_OBS_DIM * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_rew, E * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_done, E));
    HIPCHK(s, hipMalloc(&s->d_info, E * AVR_INFO_DIM * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_stage, E * K_STATE_WORDS * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_mask, E));
    return 0;
}


// env group g's first env (boundaries on multiples of 32 envs, one part-B block's share)
static int group_bound(const avr_sim *s, int g) {
    const int E = s->cfg.n_envs;
    return g >= s->ngroups ? E : std::min(E, (int)(((long long)E * g / s->ngroups + 16) / 32 * 32));
}

// one launch sequence over all envs: on the handle's stream (1 group, or while per-kernel
// timing is on), else split into env groups (boundaries on multiples of 32 envs, one part-B
// block's share) whose sequences run concurrently: group 0 on the handle's stream itself, the
// others forked from it and joined back (ngroups streams in all, within the device's hardware
// queues)
static hipError_t run_step_direct(avr_sim *s, float *state, const float *act, float *obs, float *rew, unsigned char *done, float *info,
                                  const unsigned char *mask, int mode, long long t) {
    const int E = s->cfg.n_envs;
    if (s->ngroups <= 1 || s->evlog.cap)
        return avr_launch_step(&s->km, s->d_km, state, act, obs, rew, done, info, mask, mode, t, 0, E, s->stream,
                               s->evlog.cap ? &s->evlog : nullptr);
    auto bound = [&](int g) { return group_bound(s, g); };
    hipError_t e = hipEventRecord(s->fork_ev, s->stream);
    if (e != hipSuccess) return e;
    for (int g = 1; g < s->ngroups; g++) {
        if ((e = hipStreamWaitEvent(s->gstream[g], s->fork_ev, 0)) != hipSuccess) return e;
        if ((e = avr_launch_step(&s->km, s->d_km, state, act, obs, rew, done, info, mask, mode, t, bound(g), bound(g + 1), s->gstream[g], nullptr)) !=
            hipSuccess)
            return e;
        if ((e = hipEventRecord(s->join_ev[g], s->gstream[g])) != hipSuccess) return e;
    }
    if ((e = avr_launch_step(&s->km, s->d_km, state, act, obs, rew, done, info, mask, mode, t, 0, bound(1), s->stream, nullptr)) != hipSuccess) return e;
    for (int g = 1; g < s->ngroups; g++)
        if ((e = hipStreamWaitEvent(s->stream, s->join_ev[g], 0)) != hipSuccess) return e;
    return hipSuccess;
}

static void drop_roll(avr_sim::RollSlot &r) {
    for (int c = 0; c < 2; c++) {
        if (r.gexec[c]) (void)hipGraphExecDestroy(r.gexec[c]);
        if (r.graph[c]) (void)hipGraphDestroy(r.graph[c]);
        r.gexec[c] = nullptr; r.graph[c] = nullptr;
        for (int p = 0; p < 2; p++)
            for (int g = 0; g < AVR_MAX_GROUPS; g++) {
                if (r.pgexec[c][p][g]) (void)hipGraphExecDestroy(r.pgexec[c][p][g]);
                if (r.pgraph[c][p][g]) (void)hipGraphDestroy(r.pgraph[c][p][g]);
                r.pgexec[c][p][g] = nullptr; r.pgraph[c][p][g] = nullptr;
            }
    }
    memset(r.key, 0, sizeof(r.key));
    r.used = 0;
}

static void drop_graph(avr_sim::GraphSlot &g) {
    if (g.gexec) (void)hipGraphExecDestroy(g.gexec);
    if (g.graph) (void)hipGraphDestroy(g.graph);
    g.gexec = nullptr; g.graph = nullptr;
    memset(g.key, 0, sizeof(g.key));
    g.used = 0;
}

// a gym step (modes 0 / 1, no mask, no per-kernel timing) replays a captured launch sequence;
// everything else launches directly.  Mode 0's actions are first copied (stream-ordered,
// device to device) into the handle's d_act, which every graph reads: a caller that hands a new
// action buffer each step (a policy's output tensor) replays the same graph.
static hipError_t run_step(avr_sim *s, float *state, const float *act, float *obs, float *rew, unsigned char *done, float *info,
                           const unsigned char *mask, int mode, long long t) {
    if (!s->use_graph || mask || s->evlog.cap || (mode != 0 && mode != 1) || state != s->d_state)
        return run_step_direct(s, state, act, obs, rew, done, info, mask, mode, t);
    hipError_t e;
    if (mode == 0 && act != s->d_act) {
        if (!act) return hipErrorInvalidValue;
        if ((e = hipMemcpyAsync(s->d_act, act, (size_t)s->cfg.n_envs * K_ACT_DIM * sizeof(float), hipMemcpyDeviceToDevice, s->stream)) != hipSuccess)
            return e;
    }
    const void *key[5] = {obs, rew, done, info, (const void *)(size_t)(mode + 1)};
    avr_sim::GraphSlot *g = nullptr;
    for (auto &x : s->gslot)
        if (x.gexec && memcmp(key, x.key, sizeof(key)) == 0) g = &x;
    if (!g) {
        // a free slot, else the least recently used one (after the stream has drained: no replay
        // of the graph being destroyed may still be in flight)
        for (auto &x : s->gslot)
            if (!x.gexec && !g) g = &x;
        if (!g) {
            g = &s->gslot[0];
            for (auto &x : s->gslot)
                if (x.used < g->used) g = &x;
            if ((e = hipStreamSynchronize(s->stream)) != hipSuccess) return e;
            drop_graph(*g);
        }
        if ((e = hipStreamBeginCapture(s->stream, hipStreamCaptureModeRelaxed)) != hipSuccess) return e;
        hipError_t el = run_step_direct(s, state, mode == 0 ? s->d_act : nullptr, obs, rew, done, info, nullptr, mode, -1);
        if ((e = hipStreamEndCapture(s->stream, &g->graph)) != hipSuccess) return e;
        if (el != hipSuccess) { drop_graph(*g); return el; }
        if ((e = hipGraphInstantiate(&g->gexec, g->graph, nullptr, nullptr, 0)) != hipSuccess) { drop_graph(*g); return e; }
        memcpy(g->key, key, sizeof(key));
        s->n_captures++;
    }
    g->used = ++s->gclock;
    // the step counter goes to device memory in stream order (an executable graph is never edited
    // while an earlier replay of it may still run)
    if ((e = avr_launch_set_step(s->km.step_t, t, s->stream)) != hipSuccess) return e;
    return hipGraphLaunch(g->gexec, s->stream);
}

int avr_destroy(avr_sim *s) {
    if (!s) return -1;
    DevGuard dg(s->cfg.device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto &x : s->gslot) drop_graph(x);
    for (auto &x : s->rslot) drop_roll(x);
    for (void *p : s->allocs) (void)hipFree(p);
    if (s->d_state) (void)hipFree(s->d_state);
    if (s->d_km) (void)hipFree(s->d_km);
    if (s->d_act) (void)hipFree(s->d_act);
    if (s->d_obs) (void)hipFree(s->d_obs);
    if (s->d_rew) (void)hipFree(s->d_rew);
    if (s->d_done) (void)hipFree(s->d_done);
    if (s->d_info) (void)hipFree(s->d_info);
    if (s->d_stage) (void)hipFree(s->d_stage);
    if (s->d_mask) (void)hipFree(s->d_mask);
    if (s->d_query) (void)hipFree(s->d_query);
    if (s->d_ik) (void)hipFree(s->d_ik);
    if (s->d_bs) (void)hipFree(s->d_bs);
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    for (int i = 0; i < s->ngroups; i++) {
        if (s->gstream[i]) (void)hipStreamDestroy(s->gstream[i]);
        if (s->join_ev[i]) (void)hipEventDestroy(s->join_ev[i]);
    }
    if (s->fork_ev) (void)hipEventDestroy(s->fork_ev);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return 0;
}

const char *avr_last_error(avr_sim *s) { return s ? s->err : "null handle"; }
void *avr_stream(avr_sim *s) { return s ? (void *)s->stream : nullptr; }
void *avr_state_device_ptr(avr_sim *s) { return s ? (void *)s->d_state : nullptr; }
int32_t avr_n_envs(avr_sim *s) { return s ? s->cfg.n_envs : 0; }
int32_t avr_env_groups(avr_sim *s) { return s ? s->ngroups : 0; }

#define CHECK_SIM(s)                         \
    if (!(s) || !(s)->d_state) return -1;    \
    DevGuard dev_guard_((s)->cfg.device)

int64_t avr_graph_captures(avr_sim *s) { return s ? s->n_captures : -1; }

int avr_set_state(avr_sim *s, const float *h) {
    CHECK_SIM(s);
    HIPCHK(s, hipMemcpyAsync(s->d_state, h, (size_t)s->cfg.n_envs * K_STATE_WORDS * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

// Masked upload: the whole host array and the mask go up once, a copy kernel moves the
// selected env rows (one transfer instead of one per env).
static int upload_masked(avr_sim *s, const uint8_t *mask, const float *h) {
    const size_t E = (size_t)s->cfg.n_envs;
    HIPCHK(s, hipMemcpyAsync(s->d_stage, h, E * K_STATE_WORDS * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(s->d_mask, mask, E, hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, avr_launch_copy_masked(s->d_state, s->d_stage, s->d_mask, s->cfg.n_envs, s->stream));
    return 0;
}

int avr_set_state_masked(avr_sim *s, const uint8_t *mask, const float *h) {
    CHECK_SIM(s);
    if (!mask) return avr_set_state(s, h);
    if (upload_masked(s, mask, h)) return -2;
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_reset(avr_sim *s, const uint8_t *mask, const float *h, int32_t n_frames, float *host_obs) {
    CHECK_SIM(s);
    const size_t E = (size_t)s->cfg.n_envs;
    std::vector<uint8_t> all;
    if (!mask) { all.assign(E, 1); mask = all.data(); }
    if (!h) return fail(s, -1, "avr_reset: host_state is NULL");
    if (n_frames < 0) return fail(s, -1, "avr_reset: n_frames < 0");
    if (upload_masked(s, mask, h)) return -2;
    HIPCHK(s, run_step(s, s->d_state, nullptr, s->d_obs, s->d_rew, s->d_done, s->d_info, s->d_mask, 2, n_frames));
    if (host_obs) {
        std::vector<float> o(E * K_OBS_DIM);
        HIPCHK(s, hipMemcpyAsync(o.data(), s->d_obs, E * K_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(s, hipStreamSynchronize(s->stream));
        for (size_t e = 0; e < E; e++)
            if (mask[e]) memcpy(host_obs + e * K_OBS_DIM, o.data() + e * K_OBS_DIM, K_OBS_DIM * sizeof(float));
    }
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_get_state(avr_sim *s, float *h) {
    CHECK_SIM(s);
    HIPCHK(s, hipMemcpyAsync(h, s->d_state, (size_t)s->cfg.n_envs * K_STATE_WORDS * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_settle(avr_sim *s, int32_t n_frames, float *host_obs) {
    CHECK_SIM(s);
    HIPCHK(s, run_step(s, s->d_state, nullptr, s->d_obs, s->d_rew, s->d_done, s->d_info, nullptr, 2, n_frames));
    if (host_obs) HIPCHK(s, hipMemcpyAsync(host_obs, s->d_obs, (size_t)s->cfg.n_envs * K_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_substep(avr_sim *s, float dt) {
    CHECK_SIM(s);
    long long t = 0;
    memcpy(&t, &dt, sizeof(float));
    HIPCHK(s, run_step(s, s->d_state, nullptr, s->d_obs, s->d_rew, s->d_done, s->d_info, nullptr, 3, t));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_step_device(avr_sim *s, const float *d_act, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info) {
    CHECK_SIM(s);
    HIPCHK(s, run_step(s, s->d_state, d_act, d_obs, d_rew, d_done, d_info, nullptr, 0, 0));
    return 0;
}

int avr_step_random_device(avr_sim *s, int64_t t, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info) {
    CHECK_SIM(s);
    // (negative step indices are reserved: the graph-captured take-step reads the counter from
    // device memory when its argument is negative)
    if (t < 0) return fail(s, -1, "avr_step_random_device: step index %lld < 0", (long long)t);
    HIPCHK(s, run_step(s, s->d_state, nullptr, d_obs ? d_obs : s->d_obs, d_rew ? d_rew : s->d_rew, d_done ? d_done : s->d_done,
                              d_info ? d_info : s->d_info, nullptr, 1, t));
    return 0;
}

// n device-random steps t0 .. t0 + n - 1 (avr_step_random_device's actions and results).  With
// stacked = 0 every step writes the given buffers (the last step's outputs remain); with stacked = 1
// step k writes slot k of [n][n_envs][...] arrays.  The steps run as graph replays in which each
// env group runs AVR_ROLL_CHUNK steps (one step for the remainder) back to back, each step first
// advancing the group's own step counter and slot on the device, so the groups are not joined
// after every step: a group that finishes a step early starts the next while the others finish
// theirs (envs are independent; every step of every env is computed as by n
// avr_step_random_device calls, bit for bit).  Asynchronous; the handle's stream holds the rollout.
// rollout replays, two ways (avr_rollout_random_device):
//  - branches: a graph of AVR_ROLL_CHUNK steps per group branch, forked and joined once per replay;
//  - per group: each group's own graph of AVR_ROLL_CHUNK steps replayed on its own stream (two
//    alternating copies), joined once per rollout.
// Measured (tools/gpu_r5_t18.sh, gpu_r5_t19_exp.sh): FeedingJaco 840k (branches) vs 884k (per group)
// env-steps/s; ScratchItch 1.36M vs 0.74M and BedBathing 1.77M vs 1.09M -- separately launched graphs
// dispatch at the direct-launch rate, which the PR2 tasks' short steps (22 launches per group) cannot
// hide.  Per group for FeedingJaco, branches otherwise; AVR_ROLLOUT=branches|groups overrides.
static bool per_group_rollout(const avr_sim *s) {
    const char *e = getenv("AVR_ROLLOUT");
    if (e && !strcmp(e, "branches")) return false;
    if (e && !strcmp(e, "groups")) return true;
    (void)s;
    return AVR_TASK == AVR_TASK_FEEDING;
}

static int rollout_branches(avr_sim *s, int64_t t0, int32_t n, float *o, float *r, uint8_t *dn, float *in, int32_t stacked, const void *const *key) {
    const size_t E = (size_t)s->cfg.n_envs;
    avr_sim::RollSlot *rs = nullptr;
    for (auto &x : s->rslot)
        if (x.gexec[0] && memcmp(key, x.key, sizeof(x.key)) == 0) rs = &x;
    if (!rs) {
        for (auto &x : s->rslot)
            if (!x.gexec[0] && !x.pgexec[0][0][0] && !rs) rs = &x;
        if (!rs) {
            rs = &s->rslot[0];
            for (auto &x : s->rslot)
                if (x.used < rs->used) rs = &x;
            HIPCHK(s, hipStreamSynchronize(s->stream));     // (no replay of the graphs being dropped may still run)
            drop_roll(*rs);
        }
        for (int c = 0; c < 2; c++) {
            const int steps = c == 0 ? AVR_ROLL_CHUNK : 1;
            HIPCHK(s, hipStreamBeginCapture(s->stream, hipStreamCaptureModeRelaxed));
            hipError_t el = hipEventRecord(s->fork_ev, s->stream);
            for (int g = 0; g < s->ngroups && el == hipSuccess; g++) {
                hipStream_t st = g == 0 ? s->stream : s->gstream[g];
                const int e0 = group_bound(s, g), e1 = group_bound(s, g + 1);
                long long *ct = s->km.step_t + g, *ck = s->km.step_t + AVR_MAX_GROUPS + g;
                if (g > 0) el = hipStreamWaitEvent(st, s->fork_ev, 0);
                for (int q = 0; q < steps && el == hipSuccess; q++) {
                    el = avr_launch_step_advance(ct, ck, st);
                    if (el == hipSuccess)
                        el = avr_launch_step(&s->km, s->d_km, s->d_state, nullptr, stacked ? s->d_obs : o, stacked ? s->d_rew : r,
                                             stacked ? s->d_done : dn, stacked ? s->d_info : in, nullptr, 1, -(g + 1), e0, e1, st, nullptr);
                    if (el == hipSuccess && stacked)
                        el = avr_launch_rollout_copy(ck, s->d_obs, s->d_rew, s->d_done, s->d_info, o, r, dn, in, e0, e1, (int)E, st);
                }
                if (g > 0 && el == hipSuccess) el = hipEventRecord(s->join_ev[g], st);
            }
            for (int g = 1; g < s->ngroups && el == hipSuccess; g++) el = hipStreamWaitEvent(s->stream, s->join_ev[g], 0);
            hipError_t e = hipStreamEndCapture(s->stream, &rs->graph[c]);
            if (e == hipSuccess && el == hipSuccess) e = hipGraphInstantiate(&rs->gexec[c], rs->graph[c], nullptr, nullptr, 0);
            if (e != hipSuccess || el != hipSuccess) {
                drop_roll(*rs);
                HIPCHK(s, e != hipSuccess ? e : el);
            }
        }
        memcpy(rs->key, key, sizeof(rs->key));
        s->n_captures++;
    }
    rs->used = ++s->gclock;
    for (int g = 0; g < s->ngroups; g++)      // (in stream order before the replays: the counters are the handle's)
        HIPCHK(s, avr_launch_set_step2(s->km.step_t + g, t0 - 1, s->km.step_t + AVR_MAX_GROUPS + g, -1, s->stream));
    for (int k = 0; k + AVR_ROLL_CHUNK <= n; k += AVR_ROLL_CHUNK) HIPCHK(s, hipGraphLaunch(rs->gexec[0], s->stream));
    for (int k = n / AVR_ROLL_CHUNK * AVR_ROLL_CHUNK; k < n; k++) HIPCHK(s, hipGraphLaunch(rs->gexec[1], s->stream));
    return 0;
}


static int rollout_per_group(avr_sim *s, int64_t t0, int32_t n, float *o, float *r, uint8_t *dn, float *in, int32_t stacked, const void *const *key) {
    const size_t E = (size_t)s->cfg.n_envs;
    avr_sim::RollSlot *rs = nullptr;
    for (auto &x : s->rslot)
        if (x.pgexec[0][0][0] && memcmp(key, x.key, sizeof(x.key)) == 0) rs = &x;
    if (!rs) {
        for (auto &x : s->rslot)
            if (!x.pgexec[0][0][0] && !x.gexec[0] && !rs) rs = &x;
        if (!rs) {
            rs = &s->rslot[0];
            for (auto &x : s->rslot)
                if (x.used < rs->used) rs = &x;
            // only this handle's streams: every rollout joins its groups back into s->stream, and
            // no replay of the graphs being dropped may still run (other handles, torch and RCCL
            // streams on the device are not waited for)
            HIPCHK(s, hipStreamSynchronize(s->stream));
            for (int g = 1; g < s->ngroups; g++) HIPCHK(s, hipStreamSynchronize(s->gstream[g]));
            drop_roll(*rs);
        }
        for (int c = 0; c < 2; c++)
            for (int p = 0; p < 2; p++)
                for (int g = 0; g < s->ngroups; g++) {
                    hipStream_t st = g == 0 ? s->stream : s->gstream[g];
                    const int e0 = group_bound(s, g), e1 = group_bound(s, g + 1);
                    long long *ct = s->km.step_t + g, *ck = s->km.step_t + AVR_MAX_GROUPS + g;
                    HIPCHK(s, hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
                    hipError_t el = hipSuccess;
                    for (int q = 0; q < (c == 0 ? AVR_ROLL_CHUNK : 1) && el == hipSuccess; q++) {
                        el = avr_launch_step_advance(ct, ck, st);
                        if (el == hipSuccess)
                            el = avr_launch_step(&s->km, s->d_km, s->d_state, nullptr, stacked ? s->d_obs : o, stacked ? s->d_rew : r,
                                                 stacked ? s->d_done : dn, stacked ? s->d_info : in, nullptr, 1, -(g + 1), e0, e1, st, nullptr);
                        if (el == hipSuccess && stacked)
                            el = avr_launch_rollout_copy(ck, s->d_obs, s->d_rew, s->d_done, s->d_info, o, r, dn, in, e0, e1, (int)E, st);
                    }
                    hipError_t e = hipStreamEndCapture(st, &rs->pgraph[c][p][g]);
                    if (e == hipSuccess && el == hipSuccess) e = hipGraphInstantiate(&rs->pgexec[c][p][g], rs->pgraph[c][p][g], nullptr, nullptr, 0);
                    if (e != hipSuccess || el != hipSuccess) {
                        drop_roll(*rs);
                        HIPCHK(s, e != hipSuccess ? e : el);
                    }
                }
        memcpy(rs->key, key, sizeof(rs->key));
        s->n_captures++;
    }
    rs->used = ++s->gclock;
    HIPCHK(s, hipEventRecord(s->fork_ev, s->stream));
    for (int g = 0; g < s->ngroups; g++) {
        hipStream_t st = g == 0 ? s->stream : s->gstream[g];
        if (g > 0) HIPCHK(s, hipStreamWaitEvent(st, s->fork_ev, 0));
        HIPCHK(s, avr_launch_set_step2(s->km.step_t + g, t0 - 1, s->km.step_t + AVR_MAX_GROUPS + g, -1, st));
    }
    int rep_ = 0;
    for (int k = 0; k + AVR_ROLL_CHUNK <= n; k += AVR_ROLL_CHUNK, rep_++)
        for (int g = 0; g < s->ngroups; g++) HIPCHK(s, hipGraphLaunch(rs->pgexec[0][rep_ & 1][g], g == 0 ? s->stream : s->gstream[g]));
    for (int k = n / AVR_ROLL_CHUNK * AVR_ROLL_CHUNK; k < n; k++, rep_++)
        for (int g = 0; g < s->ngroups; g++) HIPCHK(s, hipGraphLaunch(rs->pgexec[1][rep_ & 1][g], g == 0 ? s->stream : s->gstream[g]));
    for (int g = 1; g < s->ngroups; g++) {
        HIPCHK(s, hipEventRecord(s->join_ev[g], s->gstream[g]));
        HIPCHK(s, hipStreamWaitEvent(s->stream, s->join_ev[g], 0));
    }
    return 0;
}


int avr_rollout_random_device(avr_sim *s, int64_t t0, int32_t n, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info, int32_t stacked) {
    CHECK_SIM(s);
    if (t0 < 0 || n < 0) return fail(s, -1, "avr_rollout_random_device: t0 %lld / n %d < 0", (long long)t0, n);
    if (n == 0) return 0;
    if (stacked && !(d_obs && d_rew && d_done && d_info)) return fail(s, -1, "avr_rollout_random_device: stacked outputs need all four buffers");
    const size_t E = (size_t)s->cfg.n_envs;
    float *o = d_obs ? d_obs : s->d_obs, *r = d_rew ? d_rew : s->d_rew, *in = d_info ? d_info : s->d_info;
    uint8_t *dn = d_done ? d_done : s->d_done;
    if (!s->use_graph || s->ngroups <= 1 || s->evlog.cap) {
        for (int k = 0; k < n; k++) {
            const size_t q = stacked ? (size_t)k : 0;
            HIPCHK(s, run_step(s, s->d_state, nullptr, o + q * E * K_OBS_DIM, r + q * E, dn + q * E, in + q * E * AVR_INFO_DIM, nullptr, 1, t0 + k));
        }
        return 0;
    }
    // the groups' graphs for these outputs: step outputs straight to the caller's buffers, or
    // (stacked) to the handle's buffers and a copy into slot k
    const void *key[8] = {o, r, dn, in, (const void *)(size_t)(stacked + 1), nullptr, nullptr, nullptr};
    if (per_group_rollout(s)) return rollout_per_group(s, t0, n, o, r, dn, in, stacked, key);
    return rollout_branches(s, t0, n, o, r, dn, in, stacked, key);
}

int avr_random_actions_device(avr_sim *s, int64_t t, float *d_act) {
    CHECK_SIM(s);
    if (t < 0) return fail(s, -1, "avr_random_actions_device: step index %lld < 0", (long long)t);
    HIPCHK(s, avr_launch_random_actions(s->cfg.seed, s->cfg.env_offset, t, d_act, s->cfg.n_envs, s->km.n_arm, s->stream));
    return 0;
}

int avr_step(avr_sim *s, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    CHECK_SIM(s);
    size_t E = (size_t)s->cfg.n_envs;
    HIPCHK(s, hipMemcpyAsync(s->d_act, act, E * K_ACT_DIM * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, run_step(s, s->d_state, s->d_act, s->d_obs, s->d_rew, s->d_done, s->d_info, nullptr, 0, 0));
    HIPCHK(s, hipMemcpyAsync(obs, s->d_obs, E * K_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(rew, s->d_rew, E * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(done, s->d_done, E, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(info, s->d_info, E * AVR_INFO_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_sync(avr_sim *s) {
    CHECK_SIM(s);
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

// Diagnostic builds (-DAVR_PROF): attach a device buffer [n_envs][16] of per-phase cycle counters.
int avr_set_profile_buffer(avr_sim *s, void *d_prof) {
    CHECK_SIM(s);
    s->km.prof = (unsigned long long *)d_prof;
    HIPCHK(s, hipMemcpy(s->d_km, &s->km, sizeof(KModel), hipMemcpyHostToDevice));
    return 0;
}

int avr_kernel_info(avr_sim *s, int32_t *out20) {
    (void)s;
    hipError_t e = avr_kernel_attrs(out20);
    return e == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------ per-kernel timing
// Fold the logged events into per-kind totals (synchronises the stream).
static int drain_evlog(avr_sim *s) {
    if (!s->evlog.cap || !s->evlog.n) return 0;
    HIPCHK(s, hipStreamSynchronize(s->stream));
    for (int i = 0; i + 1 < s->evlog.n; i++) {
        int k = s->evlog.kind[i];
        if (k < 0) continue;
        float ms = 0.f;
        HIPCHK(s, hipEventElapsedTime(&ms, s->evlog.ev[i], s->evlog.ev[i + 1]));
        s->kt_ms[k] += ms;
        s->kt_n[k] += 1;
    }
    s->evlog.n = 0;
    return 0;
}

int avr_profile_kernels(avr_sim *s, int32_t enable) {
    CHECK_SIM(s);
    if (drain_evlog(s)) return -3;
    for (int k = 0; k < AVR_K_KINDS; k++) { s->kt_ms[k] = 0; s->kt_n[k] = 0; }
    if (enable && s->ev.empty()) {
        s->ev.resize(4096);
        s->evkind.resize(4096);
        for (auto &e : s->ev) HIPCHK(s, hipEventCreate(&e));
    }
    s->evlog.ev = s->ev.data();
    s->evlog.kind = s->evkind.data();
    s->evlog.n = 0;
    s->evlog.cap = enable ? (int)s->ev.size() : 0;
    return 0;
}

int avr_kernel_times(avr_sim *s, double *ms8, int64_t *count8) {
    CHECK_SIM(s);
    if (drain_evlog(s)) return -3;
    for (int k = 0; k < AVR_K_KINDS; k++) { ms8[k] = s->kt_ms[k]; count8[k] = s->kt_n[k]; }
    return 0;
}

// ------------------------------------------------------------------ state queries
int32_t avr_n_dof(avr_sim *s) { return s ? s->km.nd + s->km.hc_n : 0; }

// device scratch for the getters: one buffer, grown on demand
static int query_buf(avr_sim *s, size_t floats, float **out) {
    if (floats > s->qcap) {
        if (s->d_query) HIPCHK(s, hipFree(s->d_query));
        s->d_query = nullptr;
        s->qcap = 0;
        HIPCHK(s, hipMalloc(&s->d_query, floats * sizeof(float)));
        s->qcap = floats;
    }
    *out = s->d_query;
    return 0;
}

int avr_get_q(avr_sim *s, float *q, float *qd) {
    CHECK_SIM(s);
    const int nd = avr_n_dof(s), E = s->cfg.n_envs;
    const size_t n = (size_t)nd * E;
    float *d = nullptr;
    if (query_buf(s, 2 * n, &d)) return -3;
    HIPCHK(s, avr_launch_get_q(s->d_state, q ? d : nullptr, qd ? d + n : nullptr, nd, E, s->stream));
    if (q) HIPCHK(s, hipMemcpyAsync(q, d, n * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (qd) HIPCHK(s, hipMemcpyAsync(qd, d + n, n * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_get_link_pose(avr_sim *s, int32_t link, float *out7) {
    CHECK_SIM(s);
    if (!out7) return fail(s, -1, "avr_get_link_pose: out7 is NULL");
    if (link >= s->km.nla) return fail(s, -1, "avr_get_link_pose: link %d out of range (%d articulated links)", (int)link, s->km.nla);
    const int E = s->cfg.n_envs;
    float *d = nullptr;
    if (query_buf(s, (size_t)7 * E, &d)) return -3;
    HIPCHK(s, avr_launch_link_pose(s->d_km, s->d_state, d, link < 0 ? -1 : link, E, s->stream));
    HIPCHK(s, hipMemcpyAsync(out7, d, (size_t)7 * E * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_get_contact_summary(avr_sim *s, float *out4) {
    CHECK_SIM(s);
    if (!out4) return fail(s, -1, "avr_get_contact_summary: out4 is NULL");
    const int E = s->cfg.n_envs;
    float *d = nullptr;
    if (query_buf(s, (size_t)4 * E, &d)) return -3;
    HIPCHK(s, avr_launch_contact_summary(s->d_km, s->d_state, d, E, s->stream));
    HIPCHK(s, hipMemcpyAsync(out4, d, (size_t)4 * E * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

int avr_get_flags(avr_sim *s, int32_t *flags) {
    CHECK_SIM(s);
    if (!flags) return fail(s, -1, "avr_get_flags: flags is NULL");
    const int E = s->cfg.n_envs;
    float *d = nullptr;
    if (query_buf(s, (size_t)E, &d)) return -3;
    HIPCHK(s, avr_launch_get_flags(s->d_state, (int *)d, E, s->stream));
    HIPCHK(s, hipMemcpyAsync(flags, d, (size_t)E * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

// ------------------------------------------------------------------ device reset IK
int avr_reset_ik(avr_sim *s, const uint8_t *mask, const float *h, const float *target7, const float *init, const float *alt4, int32_t restarts,
                 int32_t iters, float tol, const float *keepout8, int32_t n_frames, float *host_obs, uint8_t *host_ok) {
    CHECK_SIM(s);
#if AVR_TASK != AVR_TASK_FEEDING
    (void)mask; (void)h; (void)target7; (void)init; (void)alt4; (void)restarts; (void)iters; (void)tol; (void)keepout8; (void)n_frames; (void)host_obs; (void)host_ok;
    return fail(s, -1, "avr_reset_ik: this task resets through avr_reset (host IK)");
#else
    const size_t E = (size_t)s->cfg.n_envs;
    const int na = s->km.n_arm;
    if (!h || !target7 || !init) return fail(s, -1, "avr_reset_ik: host_state, target7 and init must be given");
    if (restarts < 1 || iters < 1 || n_frames < 0 || !(tol > 0.f)) return fail(s, -1, "avr_reset_ik: restarts, iters >= 1, n_frames >= 0, tol > 0");
    if (na < 1 || na > 8) return fail(s, -1, "avr_reset_ik: %d arm DoFs (1..8 supported)", na);
    std::vector<uint8_t> all;
    if (!mask) { all.assign(E, 1); mask = all.data(); }
    const size_t nt = E * 7, ni = E * (size_t)restarts * na, nq = alt4 ? E * (size_t)restarts * 4 : 0, need = nt + ni + nq + (E + 3) / 4;
    if (need > s->ikcap) {
        if (s->d_ik) HIPCHK(s, hipFree(s->d_ik));
        s->d_ik = nullptr;
        s->ikcap = 0;
        HIPCHK(s, hipMalloc(&s->d_ik, need * sizeof(float)));
        s->ikcap = need;
    }
    float *d_t = s->d_ik, *d_i = s->d_ik + nt, *d_q = alt4 ? s->d_ik + nt + ni : nullptr;
    unsigned char *d_ok = (unsigned char *)(s->d_ik + nt + ni + nq);
    if (upload_masked(s, mask, h)) return -2;
    HIPCHK(s, hipMemcpyAsync(d_t, target7, nt * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(d_i, init, ni * sizeof(float), hipMemcpyHostToDevice, s->stream));
    if (alt4) HIPCHK(s, hipMemcpyAsync(d_q, alt4, nq * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemsetAsync(d_ok, 0, E, s->stream));
    HIPCHK(s, avr_launch_reset_ik(s->d_km, s->d_state, s->d_mask, d_t, d_i, d_q, restarts, iters, tol, keepout8, d_ok, (int)E, s->stream));
    if (n_frames > 0) HIPCHK(s, run_step(s, s->d_state, nullptr, s->d_obs, s->d_rew, s->d_done, s->d_info, s->d_mask, 2, n_frames));
    std::vector<float> o;
    if (host_obs) {
        o.resize(E * K_OBS_DIM);
        HIPCHK(s, hipMemcpyAsync(o.data(), s->d_obs, E * K_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    }
    std::vector<uint8_t> okh;
    if (host_ok) {
        okh.resize(E);
        HIPCHK(s, hipMemcpyAsync(okh.data(), d_ok, E, hipMemcpyDeviceToHost, s->stream));
    }
    HIPCHK(s, hipStreamSynchronize(s->stream));
    for (size_t e = 0; e < E; e++) {
        if (!mask[e]) continue;
        if (host_obs) memcpy(host_obs + e * K_OBS_DIM, o.data() + e * K_OBS_DIM, K_OBS_DIM * sizeof(float));
        if (host_ok) host_ok[e] = okh[e];
    }
    return 0;
#endif
}

// ------------------------------------------------------------------ robot self-contact query
int avr_robot_self_contact(avr_sim *s, int32_t n, const float *q, int32_t *out) {
    CHECK_SIM(s);
    if (n < 0 || (n > 0 && (!q || !out))) return fail(s, -1, "avr_robot_self_contact: n >= 0, q and out must be given");
    if (n == 0) return 0;
    const size_t nd = (size_t)(s->km.nd + s->km.hc_n);
    struct Buf { void *p = nullptr; ~Buf() { if (p) (void)hipFree(p); } } buf;     // (freed on every return)
    HIPCHK(s, hipMalloc(&buf.p, (size_t)n * (nd * sizeof(float) + sizeof(int))));
    float *d_q = (float *)buf.p;
    int *d_o = (int *)(d_q + (size_t)n * nd);
    HIPCHK(s, hipMemcpyAsync(d_q, q, (size_t)n * nd * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, avr_launch_self_contact(s->d_km, s->d_state, d_q, d_o, (int)n, s->stream));
    HIPCHK(s, hipMemcpyAsync(out, d_o, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

// ------------------------------------------------------------------ narrowphase query (test hook)
int avr_narrowphase_query(avr_sim *s, int32_t n, const int32_t *pairs, const float *poses14, float thr, float *out8) {
    CHECK_SIM(s);
    if (n < 0 || (n > 0 && (!pairs || !poses14 || !out8))) return fail(s, -1, "avr_narrowphase_query: n >= 0, pairs, poses14 and out8 must be given");
    for (int32_t i = 0; i < 2 * n; i++)
        if (pairs[i] < 0 || pairs[i] >= s->km.ns) return fail(s, -1, "avr_narrowphase_query: shape %d out of range", (int)pairs[i]);
    if (n == 0) return 0;
    struct Buf { void *p = nullptr; ~Buf() { if (p) (void)hipFree(p); } } buf;
    HIPCHK(s, hipMalloc(&buf.p, (size_t)n * (2 * sizeof(int) + 22 * sizeof(float))));
    int *d_p = (int *)buf.p;
    float *d_x = (float *)(d_p + 2 * (size_t)n), *d_o = d_x + 14 * (size_t)n;
    HIPCHK(s, hipMemcpyAsync(d_p, pairs, 2 * (size_t)n * sizeof(int), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(d_x, poses14, 14 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, avr_launch_np_query(s->d_km, d_p, d_x, thr, d_o, (int)n, s->stream));
    HIPCHK(s, hipMemcpyAsync(out8, d_o, 8 * (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}

// ------------------------------------------------------------------ device base-pose search (PR2 tasks)
int avr_base_search(avr_sim *s, int32_t n, int32_t attempts, const float *base7, const float *rest, const float *tstart3, const float *goals9,
                    int32_t iters, float tol, int32_t *best, uint8_t *ok, float *q_arm, float *res4) {
    CHECK_SIM(s);
#if !K_PR2
    (void)n; (void)attempts; (void)base7; (void)rest; (void)tstart3; (void)goals9; (void)iters; (void)tol; (void)best; (void)ok; (void)q_arm; (void)res4;
    return fail(s, -1, "avr_base_search: the PR2 tasks' base-pose search (this task has a fixed robot base)");
#else
    const int na = s->km.n_arm;
    if (n < 0 || attempts < 1 || iters < 1 || !(tol > 0.f)) return fail(s, -1, "avr_base_search: n >= 0, attempts, iters >= 1, tol > 0");
    if (!base7 || !rest || !tstart3 || !goals9 || !best || !ok || !q_arm) return fail(s, -1, "avr_base_search: NULL buffer");
    if (na < 1 || na > 8) return fail(s, -1, "avr_base_search: %d arm DoFs (1..8 supported)", na);
    if (n == 0) return 0;
    const size_t N = (size_t)n, M = N * (size_t)attempts;
    // layout (floats): base7 [M][7], rest [M][na], tstart [N][3], goals [N][9], res [M][4], q [M][na], best [N] (int), ok [N] (bytes)
    const size_t o_b = 0, o_r = o_b + 7 * M, o_t = o_r + M * na, o_g = o_t + 3 * N, o_res = (o_g + 9 * N + 3) & ~(size_t)3, o_q = o_res + 4 * M,
                 o_best = o_q + M * na, o_ok = o_best + N, need = o_ok + (N + 3) / 4 + 1;
    if (need > s->bscap) {
        if (s->d_bs) HIPCHK(s, hipFree(s->d_bs));
        s->d_bs = nullptr;
        s->bscap = 0;
        HIPCHK(s, hipMalloc(&s->d_bs, need * sizeof(float)));
        s->bscap = need;
    }
    float *d = s->d_bs;
    HIPCHK(s, hipMemcpyAsync(d + o_b, base7, 7 * M * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(d + o_r, rest, M * na * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(d + o_t, tstart3, 3 * N * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(d + o_g, goals9, 9 * N * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, avr_launch_base_search(&s->km, s->d_km, d + o_b, d + o_r, d + o_t, d + o_g, attempts, iters, tol, (float4 *)(d + o_res), d + o_q,
                                     (int *)(d + o_best), (unsigned char *)(d + o_ok), n, s->stream));
    std::vector<float> q(M * na);
    HIPCHK(s, hipMemcpyAsync(best, d + o_best, N * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(ok, d + o_ok, N, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(q.data(), d + o_q, M * na * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (res4) HIPCHK(s, hipMemcpyAsync(res4, d + o_res, 4 * M * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    for (size_t e = 0; e < N; e++) {
        const int b = best[e];
        if (b < 0 || b >= attempts) return fail(s, -3, "avr_base_search: bad pick %d for env %d", b, (int)e);
        memcpy(q_arm + e * na, q.data() + (e * attempts + b) * na, na * sizeof(float));
    }
    return 0;
#endif
}
