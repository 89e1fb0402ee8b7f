// avr_api.cpp -- the extern "C" entry points of libavr.so (include/avr.h).  A handle records its
// task (avr_model_desc.task) and forwards every call to that task's instantiation of the C-ABI
// body (avr_capi.hip inside namespace avr_feeding / avr_scratch / avr_bedbath, see avr_task_tu.h).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>

#include "../../include/avr.h"
#include "../../include/avr_dressing.h"

#define AVR_TASK_DECLS(NS)                                                                                         \
    namespace NS {                                                                                                 \
    struct avr_sim;                                                                                                \
    int avr_create(const avr_config *cfg, const avr_model_desc *d, avr_sim **out);                                  \
    int avr_destroy(avr_sim *s);                                                                                   \
    const char *avr_last_error(avr_sim *s);                                                                        \
    void *avr_stream(avr_sim *s);                                                                                  \
    void *avr_state_device_ptr(avr_sim *s);                                                                        \
    int32_t avr_n_envs(avr_sim *s);                                                                                \
    int32_t avr_env_groups(avr_sim *s);                                                                            \
    int64_t avr_graph_captures(avr_sim *s);                                                                        \
    int32_t avr_n_dof(avr_sim *s);                                                                                 \
    int avr_set_state(avr_sim *s, const float *h);                                                                 \
    int avr_set_state_masked(avr_sim *s, const uint8_t *mask, const float *h);                                     \
    int avr_reset(avr_sim *s, const uint8_t *mask, const float *h, int32_t n_frames, float *host_obs);             \
    int avr_get_state(avr_sim *s, float *h);                                                                       \
    int avr_settle(avr_sim *s, int32_t n_frames, float *host_obs);                                                 \
    int avr_substep(avr_sim *s, float dt);                                                                         \
    int avr_step_device(avr_sim *s, const float *d_act, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info); \
    int avr_step_random_device(avr_sim *s, int64_t t, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info);  \
    int avr_rollout_random_device(avr_sim *s, int64_t t0, int32_t n, float *d_obs, float *d_rew, uint8_t *d_done,   \
                                  float *d_info, int32_t stacked);                                                 \
    int avr_random_actions_device(avr_sim *s, int64_t t, float *d_act);                                            \
    int avr_step(avr_sim *s, const float *act, float *obs, float *rew, uint8_t *done, float *info);                \
    int avr_sync(avr_sim *s);                                                                                      \
    int avr_set_profile_buffer(avr_sim *s, void *d_prof);                                                          \
    int avr_kernel_info(avr_sim *s, int32_t *out20);                                                               \
    int avr_profile_kernels(avr_sim *s, int32_t enable);                                                           \
    int avr_kernel_times(avr_sim *s, double *ms8, int64_t *count8);                                                \
    int avr_get_q(avr_sim *s, float *q, float *qd);                                                                \
    int avr_get_link_pose(avr_sim *s, int32_t link, float *out7);                                                  \
    int avr_get_contact_summary(avr_sim *s, float *out4);                                                          \
    int avr_get_flags(avr_sim *s, int32_t *flags);                                                                 \
    int avr_reset_ik(avr_sim *s, const uint8_t *mask, const float *h, const float *target7, const float *init,      \
                     const float *alt4, int32_t restarts, int32_t iters, float tol, const float *keepout8,          \
                     int32_t n_frames, float *host_obs, uint8_t *host_ok);                                         \
    int avr_robot_self_contact(avr_sim *s, int32_t n, const float *q, int32_t *out);                               \
    int avr_narrowphase_query(avr_sim *s, int32_t n, const int32_t *pairs, const float *poses14, float thr,         \
                              float *out8);                                                                        \
    int avr_base_search(avr_sim *s, int32_t n, int32_t attempts, const float *base7, const float *rest,            \
                        const float *tstart3, const float *goals9, int32_t iters, float tol, int32_t *best,         \
                        uint8_t *ok, float *q_arm, float *res4);                                                   \
    }

AVR_TASK_DECLS(avr_feeding)
AVR_TASK_DECLS(avr_scratch)
AVR_TASK_DECLS(avr_bedbath)
AVR_TASK_DECLS(avr_dressing)

struct avr_sim {
    int32_t task;
    void *impl;          // avr_feeding::avr_sim, avr_scratch::avr_sim or avr_bedbath::avr_sim
    char err[256];       // dispatch-level errors (no impl yet)
};

#define DISPATCH_ANY(s, call)                                                                 \
    do {                                                                                      \
        if ((s)->task == AVR_TASK_SCRATCH) {                                                  \
            avr_scratch::avr_sim *h = (avr_scratch::avr_sim *)(s)->impl;                      \
            return call;                                                                      \
        }                                                                                     \
        if ((s)->task == AVR_TASK_BEDBATH) {                                                  \
            avr_bedbath::avr_sim *h = (avr_bedbath::avr_sim *)(s)->impl;                      \
            return call;                                                                      \
        }                                                                                     \
        if ((s)->task == AVR_TASK_DRESSING) {                                                 \
            avr_dressing::avr_sim *h = (avr_dressing::avr_sim *)(s)->impl;                    \
            return call;                                                                      \
        }                                                                                     \
        avr_feeding::avr_sim *h = (avr_feeding::avr_sim *)(s)->impl;                          \
        return call;                                                                          \
    } while (0)
#define DISPATCH(s, call)                                                                     \
    do {                                                                                      \
        if (!(s) || !(s)->impl) return -1;                                                    \
        DISPATCH_ANY(s, call);                                                                \
    } while (0)

extern "C" {

int32_t avr_abi_version(void) { return AVR_ABI_VERSION; }
int32_t avr_state_words(void) { return AVR_STATE_WORDS; }
int32_t avr_task_state_words(int32_t task) {
    return task == AVR_TASK_FEEDING ? AVR_STATE_WORDS : (task == AVR_TASK_SCRATCH || task == AVR_TASK_BEDBATH) ? AVR_SI_STATE_WORDS
         : task == AVR_TASK_DRESSING ? AVR_DR_STATE_WORDS : -1;
}
int32_t avr_task_obs_dim(int32_t task) {
    return task == AVR_TASK_FEEDING ? AVR_OBS_DIM : task == AVR_TASK_SCRATCH ? AVR_SI_OBS_DIM : task == AVR_TASK_BEDBATH ? AVR_BB_OBS_DIM
         : task == AVR_TASK_DRESSING ? AVR_DR_OBS_DIM : -1;
}
int32_t avr_task_act_dim(int32_t task) {
    return task == AVR_TASK_FEEDING ? AVR_ACT_DIM : (task == AVR_TASK_SCRATCH || task == AVR_TASK_BEDBATH || task == AVR_TASK_DRESSING) ? AVR_SI_ACT_DIM : -1;
}
int32_t avr_task(avr_sim *s) { return s ? s->task : -1; }

int avr_create(const avr_config *cfg, const avr_model_desc *d, avr_sim **out) {
    if (!cfg || !d || !out) return -1;
    *out = nullptr;
    avr_sim *s = new (std::nothrow) avr_sim();
    if (!s) return -1;
    s->task = d->task;
    s->impl = nullptr;
    s->err[0] = 0;
    *out = s;
    int r;
    if (d->task == AVR_TASK_FEEDING) {
        avr_feeding::avr_sim *h = nullptr;
        r = avr_feeding::avr_create(cfg, d, &h);
        s->impl = h;
    } else if (d->task == AVR_TASK_SCRATCH) {
        avr_scratch::avr_sim *h = nullptr;
        r = avr_scratch::avr_create(cfg, d, &h);
        s->impl = h;
    } else if (d->task == AVR_TASK_BEDBATH) {
        avr_bedbath::avr_sim *h = nullptr;
        r = avr_bedbath::avr_create(cfg, d, &h);
        s->impl = h;
    } else if (d->task == AVR_TASK_DRESSING) {
        avr_dressing::avr_sim *h = nullptr;
        r = avr_dressing::avr_create(cfg, d, &h);
        s->impl = h;
    } else {
        snprintf(s->err, sizeof(s->err), "unknown task %d in avr_model_desc.task", (int)d->task);
        return -2;
    }
    return r;
}

int avr_destroy(avr_sim *s) {
    if (!s) return -1;
    int r = 0;
    if (s->impl) {
        if (s->task == AVR_TASK_SCRATCH) r = avr_scratch::avr_destroy((avr_scratch::avr_sim *)s->impl);
        else if (s->task == AVR_TASK_BEDBATH) r = avr_bedbath::avr_destroy((avr_bedbath::avr_sim *)s->impl);
        else if (s->task == AVR_TASK_DRESSING) r = avr_dressing::avr_destroy((avr_dressing::avr_sim *)s->impl);
        else r = avr_feeding::avr_destroy((avr_feeding::avr_sim *)s->impl);
    }
    delete s;
    return r;
}

const char *avr_last_error(avr_sim *s) {
    if (!s) return "null handle";
    if (!s->impl) return s->err;
    DISPATCH_ANY(s, avr_last_error(h));
}

void *avr_stream(avr_sim *s) {
    if (!s || !s->impl) return nullptr;
    DISPATCH_ANY(s, avr_stream(h));
}
void *avr_state_device_ptr(avr_sim *s) {
    if (!s || !s->impl) return nullptr;
    DISPATCH_ANY(s, avr_state_device_ptr(h));
}

int32_t avr_n_envs(avr_sim *s) { if (!s || !s->impl) return 0; DISPATCH(s, avr_n_envs(h)); }
int32_t avr_env_groups(avr_sim *s) { if (!s || !s->impl) return 0; DISPATCH(s, avr_env_groups(h)); }
int32_t avr_n_dof(avr_sim *s) { if (!s || !s->impl) return 0; DISPATCH(s, avr_n_dof(h)); }
int64_t avr_graph_captures(avr_sim *s) { if (!s || !s->impl) return -1; DISPATCH(s, avr_graph_captures(h)); }
int avr_set_state(avr_sim *s, const float *p) { DISPATCH(s, avr_set_state(h, p)); }
int avr_get_state(avr_sim *s, float *p) { DISPATCH(s, avr_get_state(h, p)); }
int avr_set_state_masked(avr_sim *s, const uint8_t *m, const float *p) { DISPATCH(s, avr_set_state_masked(h, m, p)); }
int avr_settle(avr_sim *s, int32_t n, float *o) { DISPATCH(s, avr_settle(h, n, o)); }
int avr_reset(avr_sim *s, const uint8_t *m, const float *p, int32_t n, float *o) { DISPATCH(s, avr_reset(h, m, p, n, o)); }
int avr_step(avr_sim *s, const float *a, float *o, float *r, uint8_t *d, float *i) { DISPATCH(s, avr_step(h, a, o, r, d, i)); }
int avr_step_device(avr_sim *s, const float *a, float *o, float *r, uint8_t *d, float *i) { DISPATCH(s, avr_step_device(h, a, o, r, d, i)); }
int avr_step_random_device(avr_sim *s, int64_t t, float *o, float *r, uint8_t *d, float *i) { DISPATCH(s, avr_step_random_device(h, t, o, r, d, i)); }
int avr_rollout_random_device(avr_sim *s, int64_t t0, int32_t n, float *o, float *r, uint8_t *d, float *i, int32_t stacked) {
    DISPATCH(s, avr_rollout_random_device(h, t0, n, o, r, d, i, stacked));
}
int avr_random_actions_device(avr_sim *s, int64_t t, float *a) { DISPATCH(s, avr_random_actions_device(h, t, a)); }
int avr_substep(avr_sim *s, float dt) { DISPATCH(s, avr_substep(h, dt)); }
int avr_sync(avr_sim *s) { DISPATCH(s, avr_sync(h)); }
int avr_kernel_info(avr_sim *s, int32_t *o) { DISPATCH(s, avr_kernel_info(h, o)); }
int avr_profile_kernels(avr_sim *s, int32_t e) { DISPATCH(s, avr_profile_kernels(h, e)); }
int avr_kernel_times(avr_sim *s, double *ms, int64_t *n) { DISPATCH(s, avr_kernel_times(h, ms, n)); }
int avr_set_profile_buffer(avr_sim *s, void *p) { DISPATCH(s, avr_set_profile_buffer(h, p)); }
int avr_get_q(avr_sim *s, float *q, float *qd) { DISPATCH(s, avr_get_q(h, q, qd)); }
int avr_get_link_pose(avr_sim *s, int32_t link, float *o) { DISPATCH(s, avr_get_link_pose(h, link, o)); }
int avr_get_contact_summary(avr_sim *s, float *o) { DISPATCH(s, avr_get_contact_summary(h, o)); }
int avr_get_flags(avr_sim *s, int32_t *f) { DISPATCH(s, avr_get_flags(h, f)); }
int avr_reset_ik(avr_sim *s, const uint8_t *m, const float *p, const float *t7, const float *init, const float *alt4, int32_t r, int32_t it,
                 float tol, const float *box8, int32_t n, float *o, uint8_t *ok) {
    DISPATCH(s, avr_reset_ik(h, m, p, t7, init, alt4, r, it, tol, box8, n, o, ok));
}
int avr_robot_self_contact(avr_sim *s, int32_t n, const float *q, int32_t *out) { DISPATCH(s, avr_robot_self_contact(h, n, q, out)); }
int avr_narrowphase_query(avr_sim *s, int32_t n, const int32_t *pairs, const float *poses14, float thr, float *out8) {
    DISPATCH(s, avr_narrowphase_query(h, n, pairs, poses14, thr, out8));
}
int avr_base_search(avr_sim *s, int32_t n, int32_t a, const float *b7, const float *rest, const float *t3, const float *g9, int32_t it, float tol,
                    int32_t *best, uint8_t *ok, float *q, float *res4) {
    DISPATCH(s, avr_base_search(h, n, a, b7, rest, t3, g9, it, tol, best, ok, q, res4));
}

}  // extern "C"
