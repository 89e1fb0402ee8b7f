// avr_math.h -- small fp32 vector/quaternion helpers for the gfx950 step kernel.
// Quaternions are (x, y, z, w) as in PyBullet.
#pragma once
#include <hip/hip_runtime.h>

#define AVR_DI __device__ __forceinline__

struct v3 { float x, y, z; };
struct qt { float x, y, z, w; };
struct tf { v3 p; qt q; };

AVR_DI v3 V(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
AVR_DI v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
AVR_DI v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
AVR_DI v3 scl(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
AVR_DI float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
AVR_DI v3 crs(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
AVR_DI float len2(v3 a) { return dot(a, a); }
AVR_DI float len(v3 a) { return sqrtf(dot(a, a)); }
AVR_DI v3 ld3(const float *p) { return V(p[0], p[1], p[2]); }
AVR_DI void st3(float *p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
AVR_DI qt Q(float x, float y, float z, float w) { qt r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
AVR_DI qt ldq(const float *p) { return Q(p[0], p[1], p[2], p[3]); }
AVR_DI void stq(float *p, qt a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; }
AVR_DI qt qmul(qt a, qt b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
             a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
AVR_DI qt qconj(qt a) { return Q(-a.x, -a.y, -a.z, a.w); }
AVR_DI v3 qrot(qt q, v3 v) {
    v3 u = V(q.x, q.y, q.z);
    v3 t = scl(crs(u, v), 2.0f);
    return add(add(v, scl(t, q.w)), crs(u, t));
}
AVR_DI qt qnorm(qt q) {
    float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Q(q.x / n, q.y / n, q.z / n, q.w / n);
}
AVR_DI qt qaxis(v3 a, float ang) {
    float s = sinf(0.5f * ang);
    return Q(a.x * s, a.y * s, a.z * s, cosf(0.5f * ang));
}
AVR_DI tf tfmul(tf a, tf b) { tf r; r.p = add(a.p, qrot(a.q, b.p)); r.q = qmul(a.q, b.q); return r; }
AVR_DI v3 tfpt(tf a, v3 p) { return add(a.p, qrot(a.q, p)); }
AVR_DI v3 tfinvpt(tf a, v3 p) { return qrot(qconj(a.q), sub(p, a.p)); }
AVR_DI tf ldtf(const float *p) { tf r; r.p = ld3(p); r.q = ldq(p + 3); return r; }
AVR_DI void sttf(float *p, tf t) { st3(p, t.p); stq(p + 3, t.q); }
AVR_DI v3 inertia_mul(qt q, v3 I, v3 v) {
    v3 l = qrot(qconj(q), v);
    return qrot(q, V(I.x * l.x, I.y * l.y, I.z * l.z));
}
AVR_DI v3 inertia_inv_mul(qt q, v3 I, v3 v) {
    v3 l = qrot(qconj(q), v);
    return qrot(q, V(I.x > 0.f ? l.x / I.x : 0.f, I.y > 0.f ? l.y / I.y : 0.f, I.z > 0.f ? l.z / I.z : 0.f));
}
AVR_DI float clampf(float x, float lo, float hi) { return fminf(hi, fmaxf(lo, x)); }
AVR_DI v3 clamp3(v3 a, float m) { return V(clampf(a.x, -m, m), clampf(a.y, -m, m), clampf(a.z, -m, m)); }

// 3x3 rotation from quaternion (row-major m[r][c])
struct m3 { float m[3][3]; };
AVR_DI m3 qmat(qt q) {
    m3 r;
    float x = q.x, y = q.y, z = q.z, w = q.w;
    r.m[0][0] = 1 - 2 * (y * y + z * z); r.m[0][1] = 2 * (x * y - z * w); r.m[0][2] = 2 * (x * z + y * w);
    r.m[1][0] = 2 * (x * y + z * w); r.m[1][1] = 1 - 2 * (x * x + z * z); r.m[1][2] = 2 * (y * z - x * w);
    r.m[2][0] = 2 * (x * z - y * w); r.m[2][1] = 2 * (y * z + x * w); r.m[2][2] = 1 - 2 * (x * x + y * y);
    return r;
}

// ---- wave-level helpers (wave64) ----
AVR_DI int lane_id() { return (int)(threadIdx.x & 63u); }   // lane within the wavefront
// exclusive prefix count of `pred` over lanes < lane, and total
AVR_DI int ballot_prefix(bool pred, int *total) {
    unsigned long long b = __ballot(pred);
    *total = __popcll(b);
    unsigned long long below = (lane_id() == 0) ? 0ull : (b & ((1ull << lane_id()) - 1ull));
    return __popcll(below);
}
AVR_DI float wave_sum(float x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
AVR_DI float rdl_f(float x, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); }
// argmax with lowest-index tie break; returns winning index in all lanes
AVR_DI int wave_argmax(float v, int idx) {
    for (int o = 32; o > 0; o >>= 1) {
        float ov = __shfl_xor(v, o, 64);
        int oi = __shfl_xor(idx, o, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    return idx;
}

// Philox4x32-10 (the synthetic action stream, examples/random_actions.py semantics): action j of
// env `env` at step t ~ U(-1, 1), keyed by (seed, env, t); _lib.random_actions is the host mirror
AVR_DI void philox4x32_10(unsigned c[4], unsigned k0, unsigned k1) {
    for (int r = 0; r < 10; r++) {
        unsigned long long p0 = (unsigned long long)0xD2511F53u * c[0];
        unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c[2];
        unsigned h0 = (unsigned)(p0 >> 32), l0 = (unsigned)p0;
        unsigned h1 = (unsigned)(p1 >> 32), l1 = (unsigned)p1;
        unsigned n0 = h1 ^ c[1] ^ k0, n1 = l1, n2 = h0 ^ c[3] ^ k1, n3 = l0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

AVR_DI float philox_action(unsigned long long seed, int env, long long t, int j) {
    unsigned c[4] = {(unsigned)env, (unsigned)t, (unsigned)(j >> 2), (unsigned)((unsigned long long)t >> 32)};
    philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32));
    unsigned x = c[j & 3];
    return (float)(x >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
}
