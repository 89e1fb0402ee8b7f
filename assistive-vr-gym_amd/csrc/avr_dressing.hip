// avr_dressing.hip -- DressingJaco-v0 (BASELINE configs[4]) on gfx950: one kernel launch per gym step.
// A build-defined task (include/avr_dressing.h): the reference holds only its
// hooks -- the cloth spheres (human_creation.py:90-95,136-141), the dressing-force preference
// (env.py:433-434) and Util.sleeve_on_arm_reward (util.py:179-252).  The CPU checker is
// oracle/avr_oracle_dressing.c (same algorithm, fp64 / fp32).
//
// One 64-lane wavefront per env, the whole env step in one launch: take_step for the 7 arm joints,
// then 5 frames x 2 robot sub-steps x 10 cloth sub-steps.  Lane l owns particles l and l + 64 (rings
// l / 16 and 4 + l / 16); their positions and velocities stay in registers, and each sub-step
// publishes the positions and velocities to LDS (4 KB per env) for the neighbours' spring forces:
// 12 springs per particle (structural, shear, bending), gravity, air drag, penalty contact with the
// left arm's two capsules and four spheres, semi-implicit Euler; ring 0 (lanes 0-15's first
// particle) follows the tool frame, interpolated across the robot sub-step.  The tool frame is the
// Jaco's forward kinematics, evaluated by every lane (wave-uniform values).  The task glue
// (sleeve_on_arm_reward, reward, obs) follows on the same wave.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/avr.h"
#include "../../include/avr_dressing.h"

// No implicit contraction in this file: every multiply and add rounds on its own unless it is an
// explicit fmaf, in the order the fp32 oracle (oracle/avr_oracle_dressing.c) writes it with the same
// fused multiply-adds at the same sites (FMA there), so the kernel and the fp32 oracle round alike
// and the sleeve matches it to the last bits (tests/test_dressing.py).  The fused sites are the cloth
// sub-step's hot arithmetic: the spring and contact dot products, the force accumulation, the
// segment projection and the integration.
#pragma clang fp contract(off)

namespace avr_dressing {
#include "avr_math.h"

#define DR_NP AVR_DR_NP
#define DR_NS AVR_DR_SEGS
#define DR_NR AVR_DR_RINGS
#define DR_MAXL 20
#define DR_W AVR_DR_STATE_WORDS

struct DrModel {
    int nl, tool, arm_dof[7];
    int parent[DR_MAXL], jtype[DR_MAXL], dof[DR_MAXL], ajoint[DR_MAXL];   // ajoint: arm joint (0..6) of the link's DoF, -1 none
    float jpos[DR_MAXL][4], jquat[DR_MAXL][4], axis[DR_MAXL][4], compos[DR_MAXL][4], comquat[DR_MAXL][4];
    float base_p[4], base_q[4], lower[8], upper[8];
    float ring[DR_NS][4];            // the held cuff's particles in the tool frame
    float l_ring, l_ring2, l_sh, pmass;   // spring rest lengths and particle mass, rounded as the fp32 oracle's
    int chain_n, chain[DR_MAXL];     // the tool link's chain, root first (the reset IK's kinematics)
    int col[7];                      // chain position of arm joint c's link (Jacobian column c)
    unsigned long long seed;
    int env_offset;
};

enum { DR_MODE_STEP = 0, DR_MODE_STEP_RANDOM = 1, DR_MODE_OBS = 2 };

// COM frames of the tool link and of link 0: lane 0 walks the chain (link frames in LDS, parents
// first), every lane then reads the two frames (wave-uniform values)
struct FkLds { float4 lp[DR_MAXL], lq[DR_MAXL], out[3]; float2 sc[8]; };
AVR_DI void dr_fk(const DrModel &m, const float *q7, v3 &tool_p, qt &tool_q, v3 &torso, FkLds &F) {
    // the arm joints' half-angle sines and cosines, one joint per lane side by side (the double
    // sin / cos are the FK's long latency; lane 0's chain walk below then only reads them)
    if (threadIdx.x < 7) {
        float qa = 0.f;
#pragma unroll
        for (int i = 0; i < 7; i++)
            if (i == (int)threadIdx.x) qa = q7[i];
        const float h = qa * 0.5f;
        // (double sin / cos rounded once to float: what the fp32 oracle's sin() of a float returns)
        F.sc[threadIdx.x] = make_float2((float)sin((double)h), (float)cos((double)h));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 0; i < m.nl; i++) {
            const int p = m.parent[i];
            const float4 a = p < 0 ? make_float4(m.base_p[0], m.base_p[1], m.base_p[2], 0.f) : F.lp[p];
            const float4 b = p < 0 ? make_float4(m.base_q[0], m.base_q[1], m.base_q[2], m.base_q[3]) : F.lq[p];
            const v3 pp = V(a.x, a.y, a.z);
            const qt pq = Q(b.x, b.y, b.z, b.w);
            const v3 tp = add(pp, qrot(pq, ld3(m.jpos[i])));
            qt tq = qmul(pq, ldq(m.jquat[i]));
            if (m.jtype[i] == AVR_J_REVOLUTE) {
                const int aj = m.ajoint[i];
                const float2 c = aj >= 0 ? F.sc[aj] : make_float2(0.f, 1.f);     // (sin 0, cos 0)
                const float sn = c.x;
                tq = qmul(tq, Q(m.axis[i][0] * sn, m.axis[i][1] * sn, m.axis[i][2] * sn, c.y));
            }
            F.lp[i] = make_float4(tp.x, tp.y, tp.z, 0.f);
            F.lq[i] = make_float4(tq.x, tq.y, tq.z, tq.w);
        }
        const float4 a = F.lp[m.tool], b = F.lq[m.tool], c = F.lp[0], d = F.lq[0];
        const qt lq = Q(b.x, b.y, b.z, b.w), l0 = Q(d.x, d.y, d.z, d.w);
        const v3 tp = add(V(a.x, a.y, a.z), qrot(lq, ld3(m.compos[m.tool])));
        const qt tq = qmul(lq, ldq(m.comquat[m.tool]));
        const v3 to = add(V(c.x, c.y, c.z), qrot(l0, ld3(m.compos[0])));
        F.out[0] = make_float4(tp.x, tp.y, tp.z, 0.f);
        F.out[1] = make_float4(tq.x, tq.y, tq.z, tq.w);
        F.out[2] = make_float4(to.x, to.y, to.z, 0.f);
    }
    __syncthreads();
    const float4 a = F.out[0], b = F.out[1], c = F.out[2];
    tool_p = V(a.x, a.y, a.z);
    tool_q = Q(b.x, b.y, b.z, b.w);
    torso = V(c.x, c.y, c.z);
    __syncthreads();
}

// the fused forms (the oracle's dotF / axpyF / lenF): x.y first as a product, then y and z fused in
AVR_DI float dotF(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
AVR_DI float lenF(v3 a) { return sqrtf(dotF(a, a)); }
AVR_DI v3 axpyF(v3 a, float s, v3 y) { return V(fmaf(a.x, s, y.x), fmaf(a.y, s, y.y), fmaf(a.z, s, y.z)); }   // y + a s

AVR_DI v3 seg_closest(v3 a, v3 b, v3 x) {
    const v3 ab = sub(b, a);
    const float l2 = dotF(ab, ab);
    float t = l2 > 0.f ? dotF(sub(x, a), ab) / l2 : 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);
    return axpyF(ab, t, a);
}

AVR_DI v3 dr_contact(v3 x, v3 v, v3 c, float r) {
    const v3 d = sub(x, c);
    const float d2 = dotF(d, d);
    const float cr = r + (float)AVR_DR_THICK;
    // |d| >= r + thickness exactly (the fused form's sign is the exact one): sqrt(d2) then rounds
    // to >= cr and pen <= 0, so the result is the zero vector the full test returns -- without the
    // square root (a wave whose particles are all clear of the shape skips it)
    if (fmaf(-cr, cr, d2) >= 0.f) return V(0, 0, 0);
    const float dist = sqrtf(d2);
    const float pen = cr - dist;
    if (!(pen > 0.f) || !(dist > 1e-9f)) return V(0, 0, 0);
    const v3 n = scl(d, 1.f / dist);
    const float vn = dotF(v, n);
    const float f = fmaf((float)AVR_DR_K_CONTACT, pen, -((float)AVR_DR_C_CONTACT * fminf(vn, 0.f)));
    return scl(n, f);
}

__constant__ int c_nb_dk[12] = {0, 0, 1, -1, 1, 1, -1, -1, 0, 0, 2, -2};
__constant__ int c_nb_dj[12] = {1, -1, 0, 0, 1, -1, 1, -1, 2, -2, 0, 0};

// force on free particle i (ring k = i / NS >= 1) from the published positions / velocities
AVR_DI v3 dr_force(const DrModel &M, int i, v3 x, v3 v, const float4 *X, const float4 *Vv, const float *geo, float &fc_mag) {
    const float m = M.pmass;
    const float L_ring = M.l_ring, L_ax = (float)AVR_DR_SPACING, L_ring2 = M.l_ring2, L_sh = M.l_sh;
    const int k = i / DR_NS, j = i % DR_NS;
    v3 f = V(0, 0, (float)AVR_DR_GRAVITY * m);
    f = sub(f, scl(v, (float)AVR_DR_AIR));
#pragma unroll
    for (int s = 0; s < 12; s++) {
        const int kk = k + c_nb_dk[s];
        if (kk < 0 || kk >= DR_NR) continue;
        const int jj = (j + c_nb_dj[s] + DR_NS) % DR_NS;
        const int o = kk * DR_NS + jj;
        const float ks = s < 4 ? (float)AVR_DR_K_STRUCT : s < 8 ? (float)AVR_DR_K_SHEAR : (float)AVR_DR_K_BEND;
        const float L0 = s < 2 ? L_ring : s < 4 ? L_ax : s < 8 ? L_sh : s < 10 ? L_ring2 : 2.f * L_ax;
        const float4 xo = X[o], vo = Vv[o];
        const v3 d = sub(V(xo.x, xo.y, xo.z), x);
        const float l = lenF(d);
        if (!(l > 1e-9f)) continue;
        const v3 u = scl(d, 1.f / l);
        const float fs = fmaf(ks, l - L0, (float)AVR_DR_DAMP * dotF(sub(V(vo.x, vo.y, vo.z), v), u));
        f = axpyF(u, fs, f);
    }
    v3 fc = V(0, 0, 0);
    // a capsule whose bounding sphere (segment midpoint, half length + radius + thickness, widened
    // by 0.1 %: far above the rounding of the exact path) the particle is clear of contributes the
    // zero vector: the projection's division and the square root are skipped
    const bool far0 = dotF(sub(x, ld3(geo + 30)), sub(x, ld3(geo + 30))) > geo[33];
    const bool far1 = dotF(sub(x, ld3(geo + 34)), sub(x, ld3(geo + 34))) > geo[37];
    fc = add(fc, far0 ? V(0, 0, 0) : dr_contact(x, v, seg_closest(ld3(geo + 12), ld3(geo + 15), x), geo[18]));
    fc = add(fc, far1 ? V(0, 0, 0) : dr_contact(x, v, seg_closest(ld3(geo + 19), ld3(geo + 22), x), geo[25]));
    fc = add(fc, dr_contact(x, v, ld3(geo + 9), geo[26]));
    fc = add(fc, dr_contact(x, v, ld3(geo + 0), geo[27]));
    fc = add(fc, dr_contact(x, v, ld3(geo + 3), geo[28]));
    fc = add(fc, dr_contact(x, v, ld3(geo + 6), geo[29]));
    fc_mag = lenF(fc);
    return add(f, fc);
}

AVR_DI qt qnlerp(qt a, qt b, float s) {
    if (a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w < 0.f) b = Q(-b.x, -b.y, -b.z, -b.w);
    const qt r = Q(a.x + (b.x - a.x) * s, a.y + (b.y - a.y) * s, a.z + (b.z - a.z) * s, a.w + (b.w - a.w) * s);
    // (1 / sqrt in double, rounded once to float: the fp32 oracle's `1 / sqrt(x)` of a float x is
    // a double expression -- a float sqrt then a float division would round twice)
    const float n = (float)(1.0 / sqrt((double)(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w)));
    return Q(r.x * n, r.y * n, r.z * n, r.w * n);
}

// Util.line_intersects_triangle (util.py:179-186)
AVR_DI float svol(v3 a, v3 b, v3 c, v3 d) { return (1.f / 6.f) * dot(crs(sub(b, a), sub(c, a)), sub(d, a)); }
AVR_DI int sgnf(float x) { return (x > 0.f) - (x < 0.f); }
AVR_DI bool line_tri(v3 p0, v3 p1, v3 p2, v3 q0, v3 q1) {
    if (sgnf(svol(q0, p0, p1, p2)) != sgnf(svol(q1, p0, p1, p2))) {
        const int a = sgnf(svol(q0, q1, p0, p1)), b = sgnf(svol(q0, q1, p1, p2)), c = sgnf(svol(q0, q1, p2, p0));
        return a == b && b == c;
    }
    return false;
}
AVR_DI v3 nrm(v3 a) { return scl(a, 1.f / len(a)); }

// Util.sleeve_on_arm_reward (util.py:188-252) on the sleeve's two triangles (ring 0's and the last
// ring's particles 0, 5, 10): {forearm_in, upperarm_in, distance_along_forearm, distance_along_upperarm}
AVR_DI void dr_sleeve_on_arm(const float4 *X, const float *geo, float *out, v3 &hand_end, v3 &elbow_end, v3 &shoulder_end, v3 &center) {
    const v3 sh = ld3(geo), el = ld3(geo + 3), wr = ld3(geo + 6);
    hand_end = add(wr, scl(scl(sub(wr, el), 1.f / len(sub(wr, el))), geo[26] * 2.f));
    elbow_end = add(el, scl(scl(sub(el, wr), 1.f / len(sub(wr, el))), geo[28]));
    shoulder_end = add(sh, scl(scl(sub(sh, el), 1.f / len(sub(sh, el))), geo[27]));
    const int tj[3] = {0, 5, 10};
    v3 P[6];
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const float4 a = X[tj[t]], b = X[(DR_NR - 1) * DR_NS + tj[t]];
        P[t] = V(a.x, a.y, a.z);
        P[3 + t] = V(b.x, b.y, b.z);
    }
#pragma unroll
    for (int seg = 0; seg < 2; seg++) {
        const v3 a = seg == 0 ? hand_end : elbow_end, b = seg == 0 ? elbow_end : shoulder_end;
        const v3 o = seg == 0 ? elbow_end : shoulder_end;
        const v3 normal = nrm(seg == 0 ? sub(hand_end, elbow_end) : sub(elbow_end, shoulder_end));
        const v3 tangent = nrm(crs(V(1, 1, 0), normal));
        const v3 binormal = nrm(crs(tangent, normal));
        bool tp = false, tn = false, bp = false, bn = false;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const float t = dot(tangent, sub(P[k], o)), bb = dot(binormal, sub(P[k], o));
            tp |= t > 0.f; tn |= t < 0.f; bp |= bb > 0.f; bn |= bb < 0.f;
        }
        const bool i1 = line_tri(P[0], P[1], P[2], a, b), i2 = line_tri(P[3], P[4], P[5], a, b);
        out[seg] = (tp && tn && bp && bn && (i1 || i2)) ? 1.f : 0.f;
    }
    v3 c = V(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 6; k++) c = add(c, P[k]);
    center = scl(c, 1.f / 6.f);
    out[2] = len(sub(center, hand_end));
    out[3] = len(sub(center, el));
}

__global__ __launch_bounds__(64) void avr_dress_step_kernel(const DrModel *__restrict__ mp, float *__restrict__ state,
                                                            const float *__restrict__ act, const unsigned char *__restrict__ mask, int mode,
                                                            long long t, float *__restrict__ obs, float *__restrict__ rew,
                                                            unsigned char *__restrict__ done, float *__restrict__ info, int n_envs) {
    __shared__ float4 X[DR_NP], Vv[DR_NP];
    __shared__ float red[DR_NP];
    __shared__ float4 Qc[AVR_DR_CSUB];         // the cuff's orientation at each cloth sub-step of a robot sub-step
    __shared__ FkLds fk;
    const int env = blockIdx.x;
    if (env >= n_envs || (mask && !mask[env])) return;
    const DrModel &m = *mp;
    const int lane = threadIdx.x;
    float *st = state + (size_t)env * DR_W;
    float geo[38];
#pragma unroll
    for (int i = 0; i < 30; i++) geo[i] = st[AVR_DR_S_GEO + i];
    // the two capsules' bounding spheres (dr_force's prefilter): midpoint, squared radius
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const v3 a = ld3(geo + 12 + 7 * c), b = ld3(geo + 15 + 7 * c);
        const v3 mid = scl(add(a, b), 0.5f);
        const float R = (0.5f * len(sub(b, a)) + geo[18 + 7 * c] + (float)AVR_DR_THICK) * 1.001f + 1e-6f;
        geo[30 + 4 * c] = mid.x; geo[31 + 4 * c] = mid.y; geo[32 + 4 * c] = mid.z; geo[33 + 4 * c] = R * R;
    }
    float q[7], qt_[7];
#pragma unroll
    for (int i = 0; i < 7; i++) { q[i] = st[AVR_DR_S_Q + i]; qt_[i] = st[AVR_DR_S_QT + i]; }
    float asq = 0.f;
    if (mode != DR_MODE_OBS) {
        // take_step (env.py:274-337) for the arm joints: clip, x0.05, limit-respecting accumulation
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const float a_raw = mode == DR_MODE_STEP_RANDOM ? philox_action(m.seed, m.env_offset + env, t, i) : act[(size_t)env * 7 + i];
            asq += a_raw * a_raw;
            float a = fminf(fmaxf(a_raw, -1.f), 1.f) * 0.05f;
            float qn = q[i];
            for (int it = 0; it < AVR_DR_FRAME_SKIP; it++) {
                if (qn + a < m.lower[i]) a = 0.f;
                if (qn + a > m.upper[i]) a = 0.f;
                qn += a;
            }
            qt_[i] = qn;
        }
    }
    // this lane's particles
    const int i0 = lane, i1 = lane + 64;
    v3 x0 = ld3(st + AVR_DR_S_X + 4 * i0), x1 = ld3(st + AVR_DR_S_X + 4 * i1);
    v3 v0 = ld3(st + AVR_DR_S_V + 4 * i0), v1 = ld3(st + AVR_DR_S_V + 4 * i1);
    v3 tp0 = ld3(st + AVR_DR_S_TOOL), torso;
    qt tq0 = ldq(st + AVR_DR_S_TOOL + 3);
    const bool pinned = i0 < DR_NS;             // ring 0: lanes 0..15's first particle
    const v3 ringl = ld3(m.ring[i0 & (DR_NS - 1)]);
    const float dtc = (float)AVR_DR_FRAME / (AVR_DR_RSUB * AVR_DR_CSUB);
    const float minv_dt = dtc / m.pmass;
    float ftot = st[AVR_DR_S_TASK + AVR_DR_T_FORCE], speed = 0.f;
    const int frames = mode == DR_MODE_OBS ? 0 : AVR_DR_FRAME_SKIP;
    for (int f = 0; f < frames; f++)
        for (int r = 0; r < AVR_DR_RSUB; r++) {
#pragma unroll
            for (int i = 0; i < 7; i++) q[i] = q[i] + (float)AVR_DR_KP * (qt_[i] - q[i]);
            v3 tp1;
            qt tq1;
            dr_fk(m, q, tp1, tq1, torso, fk);
            // the cuff orientations of the robot sub-step's cloth sub-steps, one per lane, side by
            // side: the normalisation's double-precision square root and division run once per cloth
            // sub-step in parallel, not on the pinned lanes' path of every cloth sub-step (the values
            // are the same; the barrier at the top of the cloth sub-step publishes them)
            if (lane < AVR_DR_CSUB) {
                const qt qq = qnlerp(tq0, tq1, (float)(lane + 1) / AVR_DR_CSUB);
                Qc[lane] = make_float4(qq.x, qq.y, qq.z, qq.w);
            }
            for (int cs = 0; cs < AVR_DR_CSUB; cs++) {
                X[i0] = make_float4(x0.x, x0.y, x0.z, 0.f);
                X[i1] = make_float4(x1.x, x1.y, x1.z, 0.f);
                Vv[i0] = make_float4(v0.x, v0.y, v0.z, 0.f);
                Vv[i1] = make_float4(v1.x, v1.y, v1.z, 0.f);
                __syncthreads();
                float fm0 = 0.f, fm1 = 0.f;
                const v3 F0 = pinned ? V(0, 0, 0) : dr_force(m, i0, x0, v0, X, Vv, geo, fm0);
                const v3 F1 = dr_force(m, i1, x1, v1, X, Vv, geo, fm1);
                // the dressing forces' sum over the free particles, at the step's last cloth sub-step
                // (summed in particle order, as the oracle's loop)
                const bool last = f == frames - 1 && r == AVR_DR_RSUB - 1 && cs == AVR_DR_CSUB - 1;
                if (last) { red[i0] = fm0; red[i1] = fm1; }
                __syncthreads();
                if (pinned) {
                    const float s = (float)(cs + 1) / AVR_DR_CSUB;
                    const v3 p = add(tp0, scl(sub(tp1, tp0), s));
                    const float4 qv = Qc[cs];
                    const qt qq = Q(qv.x, qv.y, qv.z, qv.w);
                    const v3 tg = add(p, qrot(qq, ringl));
                    v0 = scl(sub(tg, x0), 1.f / dtc);
                    x0 = tg;
                } else {
                    v0 = axpyF(F0, minv_dt, v0);
                    x0 = axpyF(v0, dtc, x0);
                }
                v1 = axpyF(F1, minv_dt, v1);
                x1 = axpyF(v1, dtc, x1);
                if (last) {
                    float s = 0.f;
                    for (int k = DR_NS; k < DR_NP; k++) s += red[k];
                    ftot = s;
                }
                __syncthreads();
            }
            speed = len(sub(tp1, tp0)) / ((float)AVR_DR_FRAME / AVR_DR_RSUB);
            tp0 = tp1;
            tq0 = tq1;
        }
    {
        v3 tpx;
        qt tqx;
        dr_fk(m, q, tpx, tqx, torso, fk);
    }
    X[i0] = make_float4(x0.x, x0.y, x0.z, 0.f);
    X[i1] = make_float4(x1.x, x1.y, x1.z, 0.f);
    __syncthreads();
    st3(st + AVR_DR_S_X + 4 * i0, x0); st3(st + AVR_DR_S_X + 4 * i1, x1);
    st3(st + AVR_DR_S_V + 4 * i0, v0); st3(st + AVR_DR_S_V + 4 * i1, v1);
    // task glue (every lane computes the same values; lane 0 writes)
    float so[4];
    v3 hand_end, elbow_end, shoulder_end, center;
    dr_sleeve_on_arm(X, geo, so, hand_end, elbow_end, shoulder_end, center);
    float *T = st + AVR_DR_S_TASK;
    const float iter = T[AVR_DR_T_ITER] + (mode == DR_MODE_OBS ? 0.f : 1.f);
    const float r_dress = so[0] > 0.f ? so[2] + (so[1] > 0.f ? so[3] : 0.f) : 0.f;
    const float r_dist = -len(sub(tp0, shoulder_end));
    const float reward = (float)AVR_DR_W_DISTANCE * r_dist + (float)AVR_DR_W_ACTION * (-asq) + (float)AVR_DR_W_DRESS * r_dress +
                         (float)AVR_DR_W_VELOCITY * (-speed) + (float)AVR_DR_W_FORCE * (-ftot);
    // non-finite guard over the particles (every lane checks its two), the joints and the tool
    bool bad = !(isfinite(x0.x) && isfinite(x0.y) && isfinite(x0.z) && isfinite(x1.x) && isfinite(x1.y) && isfinite(x1.z) && isfinite(v0.x) &&
                 isfinite(v0.y) && isfinite(v0.z) && isfinite(v1.x) && isfinite(v1.y) && isfinite(v1.z));
    bad = __any(bad);
    for (int i = 0; i < 7; i++) bad = bad || !isfinite(q[i]);
    bad = bad || !isfinite(reward);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 7; i++) { st[AVR_DR_S_Q + i] = q[i]; st[AVR_DR_S_QT + i] = qt_[i]; }
        st3(st + AVR_DR_S_TOOL, tp0);
        stq(st + AVR_DR_S_TOOL + 3, tq0);
        T[AVR_DR_T_ITER] = iter;
        T[AVR_DR_T_FORCE] = ftot;
        T[AVR_DR_T_FOREARM] = so[0];
        T[AVR_DR_T_SUCCESS] = so[1];
        if (bad) T[AVR_DR_T_FLAGS] = (float)((int)T[AVR_DR_T_FLAGS] | 1);
        rew[env] = mode == DR_MODE_OBS ? 0.f : reward;
        done[env] = iter >= (float)AVR_DR_MAX_STEPS;
        info[2 * (size_t)env] = ftot;
        info[2 * (size_t)env + 1] = so[1];
    }
    if (lane < AVR_DR_OBS_DIM) {
        const v3 a0 = sub(tp0, torso), a1 = sub(center, hand_end), a2 = sub(center, elbow_end), a3 = sub(center, shoulder_end);
        const float ov[AVR_DR_OBS_DIM] = {a0.x, a0.y, a0.z, tq0.x, tq0.y, tq0.z, tq0.w, a1.x, a1.y, a1.z, a2.x, a2.y,
                                          a2.z, a3.x, a3.y, a3.z, q[0], q[1], q[2], q[3], q[4], q[5], q[6], ftot};
        float o = 0.f;
#pragma unroll
        for (int k = 0; k < AVR_DR_OBS_DIM; k++)
            if (k == lane) o = ov[k];
        obs[(size_t)env * AVR_DR_OBS_DIM + lane] = o;
    }
}

// ------------------------------------------------------------------------------------------ reset IK
// The reset's inverse kinematics on the device (the host restatement, avr/reset_dressing.py
// ik_batch, is the checker): damped least squares of the tool link's COM frame towards the start
// pose, per restart from its own random joint vector (util.py:34-105 ik_random_restarts: the
// first restart whose pose meets the tolerance is kept -- |dp| < tol and |dq| < tol or
// np.isclose(|dq|, 2, atol=tol), util.py:49 -- else the restart closest to the target position,
// util.py:51-54).  Each iteration: J (6 x 7, the arm joints' columns), (J J^T + 1e-4 I) y = e by
// Cholesky, q += J^T y clipped to the limits; a restart stops once its position error and rotation
// angle are below res (calculateInverseKinematics' residual threshold role).  One block per env,
// lane r runs restart r (serial FK of the tool chain in registers); then the block writes the arm,
// its motor targets, the tool frame and the sleeve in its rest shape (ring k centred k * spacing
// along -z of the tool frame, avr/reset_dressing.py cloth_rest).
// the tool COM frame and, per arm joint a, its joint origin and world axis (the Jacobian's
// columns); the chain loop is unrolled to its capacity so every array index is a constant
AVR_DI void ik_fk(const DrModel &m, const float *q7, v3 &cp, qt &cq, v3 *ORa, v3 *AXa) {
    v3 p = ld3(m.base_p);
    qt q = ldq(m.base_q);
    for (int c = 0; c < m.chain_n; c++) {
        const int i = m.chain[c];
        const v3 tp = add(p, qrot(q, ld3(m.jpos[i])));
        qt tq = qmul(q, ldq(m.jquat[i]));
        const v3 ax = qrot(tq, ld3(m.axis[i]));
        const int aj = m.ajoint[i];
        float qa = 0.f;
#pragma unroll
        for (int k = 0; k < 7; k++)
            if (aj == k) { qa = q7[k]; ORa[k] = tp; AXa[k] = ax; }
        if (m.jtype[i] == AVR_J_REVOLUTE) {
            const float h = 0.5f * qa, sn = sinf(h);
            tq = qmul(tq, Q(m.axis[i][0] * sn, m.axis[i][1] * sn, m.axis[i][2] * sn, cosf(h)));
        }
        p = tp;
        q = tq;
    }
    cp = add(p, qrot(q, ld3(m.compos[m.tool])));
    cq = qmul(q, ldq(m.comquat[m.tool]));
}

__global__ __launch_bounds__(64) void avr_dress_reset_ik_kernel(const DrModel *__restrict__ mp, float *__restrict__ state, const unsigned char *__restrict__ mask,
                                                                const float *__restrict__ target7, const float *__restrict__ init, int restarts, int iters,
                                                                float tol, unsigned char *__restrict__ ok_out, int n_envs) {
    __shared__ float rq[64][8];      // per restart: q[7], position error
    __shared__ int acc[64];
    __shared__ float pose[8];
    const int env = blockIdx.x, lane = threadIdx.x;
    if (env >= n_envs || (mask && !mask[env])) return;
    const DrModel &m = *mp;
    const float *t7 = target7 + (size_t)env * 7;
    const v3 tpos = V(t7[0], t7[1], t7[2]);
    const qt tq = Q(t7[3], t7[4], t7[5], t7[6]);
    const float res = 1e-6f, lam = 1e-4f;
    if (lane < restarts) {
        float q[7];
#pragma unroll
        for (int k = 0; k < 7; k++) q[k] = init[((size_t)env * restarts + lane) * 7 + k];
        v3 OR[7], AX[7];
        v3 cp;
        qt cq;
        for (int it = 0; it <= iters; it++) {
            ik_fk(m, q, cp, cq, OR, AX);
            const v3 ep = sub(tpos, cp);
            qt dq = qmul(tq, Q(-cq.x, -cq.y, -cq.z, cq.w));
            if (dq.w < 0.f) dq = Q(-dq.x, -dq.y, -dq.z, -dq.w);
            const float sv = sqrtf(dq.x * dq.x + dq.y * dq.y + dq.z * dq.z);
            const float ang = 2.f * atan2f(sv, dq.w);
            if ((len(ep) < res && ang < res) || it == iters) break;
            const v3 er = sv > 1e-12f ? scl(V(dq.x, dq.y, dq.z), ang / sv) : V(0, 0, 0);
            float J[6][7];
#pragma unroll
            for (int c = 0; c < 7; c++) {
                const v3 a = AX[c], l = crs(a, sub(cp, OR[c]));
                J[0][c] = l.x; J[1][c] = l.y; J[2][c] = l.z; J[3][c] = a.x; J[4][c] = a.y; J[5][c] = a.z;
            }
            float Am[6][6], e[6] = {ep.x, ep.y, ep.z, er.x, er.y, er.z};
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = 0; j <= i; j++) {
                    float t = i == j ? lam : 0.f;
#pragma unroll
                    for (int c = 0; c < 7; c++) t += J[i][c] * J[j][c];
                    Am[i][j] = t;
                }
            // Cholesky A = L L^T (lower, in place), then L L^T y = e
#pragma unroll
            for (int j = 0; j < 6; j++) {
                float d = Am[j][j];
#pragma unroll
                for (int k = 0; k < j; k++) d -= Am[j][k] * Am[j][k];
                d = sqrtf(fmaxf(d, 1e-30f));
                Am[j][j] = d;
#pragma unroll
                for (int i = j + 1; i < 6; i++) {
                    float t = Am[i][j];
#pragma unroll
                    for (int k = 0; k < j; k++) t -= Am[i][k] * Am[j][k];
                    Am[i][j] = t / d;
                }
            }
#pragma unroll
            for (int i = 0; i < 6; i++) {
                float t = e[i];
#pragma unroll
                for (int k = 0; k < i; k++) t -= Am[i][k] * e[k];
                e[i] = t / Am[i][i];
            }
#pragma unroll
            for (int i = 5; i >= 0; i--) {
                float t = e[i];
#pragma unroll
                for (int k = i + 1; k < 6; k++) t -= Am[k][i] * e[k];
                e[i] = t / Am[i][i];
            }
#pragma unroll
            for (int c = 0; c < 7; c++) {
                float st = 0.f;
#pragma unroll
                for (int i = 0; i < 6; i++) st += J[i][c] * e[i];
                q[c] = fminf(fmaxf(q[c] + st, m.lower[c]), m.upper[c]);
            }
        }
        ik_fk(m, q, cp, cq, OR, AX);
        const float pe = len(sub(tpos, cp));
        const float qd = sqrtf((tq.x - cq.x) * (tq.x - cq.x) + (tq.y - cq.y) * (tq.y - cq.y) + (tq.z - cq.z) * (tq.z - cq.z) + (tq.w - cq.w) * (tq.w - cq.w));
        acc[lane] = pe < tol && (qd < tol || fabsf(qd - 2.f) <= tol + 1e-5f * 2.f);
#pragma unroll
        for (int k = 0; k < 7; k++) rq[lane][k] = q[k];
        rq[lane][7] = pe;
    }
    __syncthreads();
    if (lane == 0) {
        int pick = -1;
        for (int r = 0; r < restarts && pick < 0; r++)
            if (acc[r]) pick = r;
        const bool good = pick >= 0;
        if (!good) {
            pick = 0;
            for (int r = 1; r < restarts; r++)
                if (rq[r][7] < rq[pick][7]) pick = r;
        }
        float *st = state + (size_t)env * DR_W;
        float q[7];
        for (int k = 0; k < 7; k++) { q[k] = rq[pick][k]; st[AVR_DR_S_Q + k] = q[k]; st[AVR_DR_S_QT + k] = q[k]; }
        v3 OR[7], AX[7], cp;
        qt cq;
        ik_fk(m, q, cp, cq, OR, AX);
        st3(st + AVR_DR_S_TOOL, cp);
        stq(st + AVR_DR_S_TOOL + 3, cq);
        pose[0] = cp.x; pose[1] = cp.y; pose[2] = cp.z; pose[3] = cq.x; pose[4] = cq.y; pose[5] = cq.z; pose[6] = cq.w;
        ok_out[env] = good;
    }
    __syncthreads();
    const v3 cp = V(pose[0], pose[1], pose[2]);
    const qt cq = Q(pose[3], pose[4], pose[5], pose[6]);
    float *st = state + (size_t)env * DR_W;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int i = lane + 64 * h, k = i / DR_NS, j = i % DR_NS;
        const v3 x = add(cp, qrot(cq, V(m.ring[j][0], m.ring[j][1], -(float)k * (float)AVR_DR_SPACING)));
        float *px = st + AVR_DR_S_X + 4 * i, *pv = st + AVR_DR_S_V + 4 * i;
        px[0] = x.x; px[1] = x.y; px[2] = x.z; px[3] = 0.f;
        pv[0] = 0.f; pv[1] = 0.f; pv[2] = 0.f; pv[3] = 0.f;
    }
}

__global__ void avr_dress_copy_masked_kernel(float *state, const float *src, const unsigned char *mask, int n_envs) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (size_t)n_envs * DR_W && mask[i / DR_W]) state[i] = src[i];
}

__global__ void avr_dress_random_actions_kernel(unsigned long long seed, int env_offset, long long t, float *act, int n_envs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_envs * 7) act[i] = philox_action(seed, env_offset + i / 7, t, i % 7);
}

__global__ void avr_dress_get_q_kernel(const float *state, float *q, float *qd, int n_envs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_envs * 7) return;
    if (q) q[i] = state[(size_t)(i / 7) * DR_W + AVR_DR_S_Q + i % 7];
    if (qd) qd[i] = 0.f;
}

__global__ void avr_dress_get_flags_kernel(const float *state, int *out, int n_envs) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n_envs) out[e] = (int)state[(size_t)e * DR_W + AVR_DR_S_TASK + AVR_DR_T_FLAGS];
}

// ------------------------------------------------------------------------------------------ C-ABI body
struct avr_sim {
    avr_config cfg;
    DrModel hm;
    DrModel *d_m;
    hipStream_t stream;
    float *d_state, *d_stage, *d_act, *d_obs, *d_rew, *d_info, *d_query;
    float *d_ik;                 // reset IK inputs: target frames [E][7], then restarts [E][R][7] (grow-only)
    size_t ik_cap;
    unsigned char *d_ok;
    unsigned char *d_done, *d_mask;
    hipEvent_t ev0, ev1;
    int prof;
    double kt_ms;
    long long kt_n;
    char err[512];
};

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
#define CHECK_SIM(s)                      \
    if (!(s) || !(s)->d_state) return -1; \
    DevGuard dev_guard_((s)->cfg.device)

int avr_create(const avr_config *cfg, const avr_model_desc *d, avr_sim **out) {
    if (!cfg || !d || !out) return -1;
    avr_sim *s = new avr_sim();
    memset(s->err, 0, sizeof(s->err));
    s->cfg = *cfg;
    *out = s;
    if (cfg->n_envs <= 0) return fail(s, -1, "n_envs must be > 0");
    if (cfg->flags & AVR_CFG_RESERVED_MASK) return fail(s, -1, "avr_config.flags 0x%x: no flag is defined", (unsigned)cfg->flags);
    if (d->task != AVR_TASK_DRESSING) return fail(s, -2, "model task %d is not DressingJaco", (int)d->task);
    if (d->n_links > DR_MAXL || d->n_arm != 7 || d->tool_link < 0 || d->tool_link >= d->n_links) return fail(s, -2, "DressingJaco: the Jaco chain exceeds the compiled capacities");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(s, -4, "no HIP device available");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(s, -4, "device %d out of range (%d devices)", cfg->device, ndev);
    DevGuard dg(cfg->device);
    DrModel &m = s->hm;
    memset(&m, 0, sizeof(m));
    m.nl = d->n_links;
    m.tool = d->tool_link;
    for (int i = 0; i < 7; i++) {
        m.arm_dof[i] = d->arm_dofs[i];
        m.lower[i] = (float)d->arm_lower[i];
        m.upper[i] = (float)d->arm_upper[i];
    }
    for (int i = 0; i < m.nl; i++) {
        m.parent[i] = d->rl_parent[i]; m.jtype[i] = d->rl_jtype[i]; m.dof[i] = d->rl_dof[i];
        m.ajoint[i] = -1;
        for (int k = 0; k < 7; k++)
            if (d->rl_dof[i] >= 0 && d->arm_dofs[k] == d->rl_dof[i]) m.ajoint[i] = k;
        for (int k = 0; k < 3; k++) {
            m.jpos[i][k] = (float)d->rl_jpos[3 * i + k];
            m.axis[i][k] = (float)d->rl_axis[3 * i + k];
            m.compos[i][k] = (float)d->rl_com_pos[3 * i + k];
        }
        for (int k = 0; k < 4; k++) {
            m.jquat[i][k] = (float)d->rl_jquat[4 * i + k];
            m.comquat[i][k] = (float)d->rl_com_quat[4 * i + k];
        }
    }
    {
        int rev[DR_MAXL], n = 0;
        for (int k = m.tool; k >= 0 && n < DR_MAXL; k = m.parent[k]) rev[n++] = k;
        m.chain_n = n;
        for (int c = 0; c < n; c++) m.chain[c] = rev[n - 1 - c];
        for (int a = 0; a < 7; a++) {
            m.col[a] = -1;
            for (int c = 0; c < n; c++)
                if (m.ajoint[m.chain[c]] == a) m.col[a] = c;
            if (m.col[a] < 0) return fail(s, -2, "DressingJaco: arm joint %d is not on the tool link's chain", a);
        }
    }
    for (int k = 0; k < 3; k++) m.base_p[k] = (float)d->robot_base[k];
    for (int k = 0; k < 4; k++) m.base_q[k] = (float)d->robot_base[3 + k];
    // the cuff ring, rest lengths and particle mass rounded exactly as the fp32 oracle computes them
    // (float operands, double sin / cos / sqrt rounded to float; avr_oracle_dressing.c cloth_substep
    // and env_step)
    {
        const float pi = (float)3.14159265358979323846, rad = (float)AVR_DR_RADIUS, L_ax = (float)AVR_DR_SPACING;
        for (int j = 0; j < DR_NS; j++) {
            const float th = 2 * pi * j / DR_NS;
            m.ring[j][0] = (float)((double)rad * cos((double)th));
            m.ring[j][1] = (float)((double)rad * sin((double)th));
        }
        m.l_ring = (float)((double)(2 * rad) * sin((double)(pi / DR_NS)));
        m.l_ring2 = (float)((double)(2 * rad) * sin((double)(2 * pi / DR_NS)));
        const float ls2 = m.l_ring * m.l_ring + L_ax * L_ax;
        m.l_sh = (float)sqrt((double)ls2);
        m.pmass = (float)AVR_DR_MASS / DR_NP;
    }
    m.seed = cfg->seed;
    m.env_offset = cfg->env_offset;
    const size_t E = (size_t)cfg->n_envs;
    HIPCHK(s, hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    HIPCHK(s, hipMalloc(&s->d_m, sizeof(DrModel)));
    HIPCHK(s, hipMemcpy(s->d_m, &m, sizeof(DrModel), hipMemcpyHostToDevice));
    HIPCHK(s, hipMalloc(&s->d_state, E * DR_W * sizeof(float)));
    HIPCHK(s, hipMemset(s->d_state, 0, E * DR_W * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_stage, E * DR_W * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_act, E * 7 * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_obs, E * AVR_DR_OBS_DIM * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_rew, E * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_info, E * 2 * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_query, E * 7 * 2 * sizeof(float)));
    HIPCHK(s, hipMalloc(&s->d_done, E));
    HIPCHK(s, hipMalloc(&s->d_mask, E));
    HIPCHK(s, hipMalloc(&s->d_ok, E));
    HIPCHK(s, hipEventCreate(&s->ev0));
    HIPCHK(s, hipEventCreate(&s->ev1));
    return 0;
}

int avr_destroy(avr_sim *s) {
    if (!s) return -1;
    DevGuard dg(s->cfg.device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    void *ptrs[] = {s->d_m, s->d_state, s->d_stage, s->d_act, s->d_obs, s->d_rew, s->d_info, s->d_query, s->d_done, s->d_mask, s->d_ik, s->d_ok};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return 0;
}

const char *avr_last_error(avr_sim *s) { return s ? s->err : "null handle"; }
void *avr_stream(avr_sim *s) { return s ? (void *)s->stream : nullptr; }
void *avr_state_device_ptr(avr_sim *s) { return s ? (void *)s->d_state : nullptr; }
int32_t avr_n_envs(avr_sim *s) { return s ? s->cfg.n_envs : 0; }
int32_t avr_env_groups(avr_sim *s) { return s ? 1 : 0; }
int32_t avr_n_dof(avr_sim *s) { return s ? 7 : 0; }
int64_t avr_graph_captures(avr_sim *s) { return s ? 0 : -1; }

static hipError_t launch(avr_sim *s, const float *act, const unsigned char *mask, int mode, long long t, float *obs, float *rew, unsigned char *done,
                         float *info) {
    if (s->prof) (void)hipEventRecord(s->ev0, s->stream);
    hipLaunchKernelGGL(avr_dress_step_kernel, dim3(s->cfg.n_envs), dim3(64), 0, s->stream, s->d_m, s->d_state, act, mask, mode, t, obs, rew, done, info,
                       s->cfg.n_envs);
    hipError_t e = hipGetLastError();
    if (s->prof && e == hipSuccess) {
        (void)hipEventRecord(s->ev1, s->stream);
        if (hipEventSynchronize(s->ev1) == hipSuccess) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, s->ev0, s->ev1) == hipSuccess) { s->kt_ms += ms; s->kt_n++; }
        }
    }
    return e;
}

int avr_set_state(avr_sim *s, const float *h) {
    CHECK_SIM(s);
    HIPCHK(s, hipMemcpyAsync(s->d_state, h, (size_t)s->cfg.n_envs * DR_W * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_get_state(avr_sim *s, float *h) {
    CHECK_SIM(s);
    HIPCHK(s, hipMemcpyAsync(h, s->d_state, (size_t)s->cfg.n_envs * DR_W * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
static int upload_masked(avr_sim *s, const uint8_t *mask, const float *h) {
    const size_t E = (size_t)s->cfg.n_envs;
    HIPCHK(s, hipMemcpyAsync(s->d_stage, h, E * DR_W * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(s->d_mask, mask, E, hipMemcpyHostToDevice, s->stream));
    const size_t n = E * DR_W;
    hipLaunchKernelGGL(avr_dress_copy_masked_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream, s->d_state, s->d_stage, s->d_mask,
                       s->cfg.n_envs);
    HIPCHK(s, hipGetLastError());
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
    if (!h) return fail(s, -1, "avr_reset: host_state is NULL");
    if (n_frames != 0) return fail(s, -1, "avr_reset: DressingJaco has no settle frames");
    std::vector<uint8_t> all;
    if (!mask) { all.assign(E, 1); mask = all.data(); }
    if (upload_masked(s, mask, h)) return -2;
    HIPCHK(s, launch(s, nullptr, s->d_mask, DR_MODE_OBS, 0, s->d_obs, s->d_rew, s->d_done, s->d_info));
    if (host_obs) {
        std::vector<float> o(E * AVR_DR_OBS_DIM);
        HIPCHK(s, hipMemcpyAsync(o.data(), s->d_obs, o.size() * sizeof(float), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(s, hipStreamSynchronize(s->stream));
        for (size_t e = 0; e < E; e++)
            if (mask[e]) memcpy(host_obs + e * AVR_DR_OBS_DIM, o.data() + e * AVR_DR_OBS_DIM, AVR_DR_OBS_DIM * sizeof(float));
    }
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_settle(avr_sim *s, int32_t n_frames, float *host_obs) {
    CHECK_SIM(s);
    if (n_frames != 0) return fail(s, -1, "avr_settle: DressingJaco has no settle frames (0 = observe)");
    HIPCHK(s, launch(s, nullptr, nullptr, DR_MODE_OBS, 0, s->d_obs, s->d_rew, s->d_done, s->d_info));
    if (host_obs)
        HIPCHK(s, hipMemcpyAsync(host_obs, s->d_obs, (size_t)s->cfg.n_envs * AVR_DR_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_substep(avr_sim *s, float dt) { (void)dt; return fail(s, -1, "avr_substep: not defined for DressingJaco"); }
int avr_step_device(avr_sim *s, const float *d_act, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info) {
    CHECK_SIM(s);
    HIPCHK(s, launch(s, d_act, nullptr, DR_MODE_STEP, 0, d_obs, d_rew, d_done, d_info));
    return 0;
}
int avr_step_random_device(avr_sim *s, int64_t t, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info) {
    CHECK_SIM(s);
    if (t < 0) return fail(s, -1, "avr_step_random_device: step index %lld < 0", (long long)t);
    HIPCHK(s, launch(s, nullptr, nullptr, DR_MODE_STEP_RANDOM, t, d_obs ? d_obs : s->d_obs, d_rew ? d_rew : s->d_rew, d_done ? d_done : s->d_done,
                     d_info ? d_info : s->d_info));
    return 0;
}
// (avr_rollout_random_device: one launch per step, step k's outputs to slot k when stacked)
int avr_rollout_random_device(avr_sim *s, int64_t t0, int32_t n, float *d_obs, float *d_rew, uint8_t *d_done, float *d_info, int32_t stacked) {
    CHECK_SIM(s);
    if (t0 < 0 || n < 0) return fail(s, -1, "avr_rollout_random_device: t0 %lld / n %d < 0", (long long)t0, n);
    if (stacked && !(d_obs && d_rew && d_done && d_info)) return fail(s, -1, "avr_rollout_random_device: stacked outputs need all four buffers");
    const size_t E = (size_t)s->cfg.n_envs;
    float *o = d_obs ? d_obs : s->d_obs, *r = d_rew ? d_rew : s->d_rew, *in = d_info ? d_info : s->d_info;
    uint8_t *dn = d_done ? d_done : s->d_done;
    for (int k = 0; k < n; k++) {
        const size_t q = stacked ? (size_t)k : 0;
        HIPCHK(s, launch(s, nullptr, nullptr, DR_MODE_STEP_RANDOM, t0 + k, o + q * E * AVR_DR_OBS_DIM, r + q * E, dn + q * E, in + q * E * AVR_INFO_DIM));
    }
    return 0;
}
int avr_random_actions_device(avr_sim *s, int64_t t, float *d_act) {
    CHECK_SIM(s);
    if (t < 0) return fail(s, -1, "avr_random_actions_device: step index %lld < 0", (long long)t);
    const int n = s->cfg.n_envs * 7;
    hipLaunchKernelGGL(avr_dress_random_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, s->stream, s->cfg.seed, s->cfg.env_offset, t, d_act,
                       s->cfg.n_envs);
    HIPCHK(s, hipGetLastError());
    return 0;
}
int avr_step(avr_sim *s, const float *act, float *obs, float *rew, uint8_t *done, float *info) {
    CHECK_SIM(s);
    const size_t E = (size_t)s->cfg.n_envs;
    HIPCHK(s, hipMemcpyAsync(s->d_act, act, E * 7 * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, launch(s, s->d_act, nullptr, DR_MODE_STEP, 0, s->d_obs, s->d_rew, s->d_done, s->d_info));
    HIPCHK(s, hipMemcpyAsync(obs, s->d_obs, E * AVR_DR_OBS_DIM * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(rew, s->d_rew, E * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(done, s->d_done, E, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(info, s->d_info, E * 2 * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_sync(avr_sim *s) {
    CHECK_SIM(s);
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_set_profile_buffer(avr_sim *s, void *p) { (void)p; return fail(s, -1, "no phase-timer build for DressingJaco"); }
int avr_kernel_info(avr_sim *s, int32_t *out20) {
    (void)s;
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, (const void *)avr_dress_step_kernel) != hipSuccess) return -3;
    for (int i = 0; i < 20; i++) out20[i] = 0;
    // the one kernel of the step, reported in part B's slot (index 3)
    out20[12] = a.numRegs; out20[14] = (int)a.sharedSizeBytes; out20[15] = (int)a.localSizeBytes;
    return 0;
}
int avr_profile_kernels(avr_sim *s, int32_t enable) {
    CHECK_SIM(s);
    s->prof = enable != 0;
    s->kt_ms = 0; s->kt_n = 0;
    return 0;
}
int avr_kernel_times(avr_sim *s, double *ms8, int64_t *count8) {
    CHECK_SIM(s);
    for (int k = 0; k < 8; k++) { ms8[k] = 0; count8[k] = 0; }
    ms8[2] = s->kt_ms; count8[2] = s->kt_n;          // (part B's slot: avr_dress_step_kernel)
    return 0;
}
int avr_get_q(avr_sim *s, float *q, float *qd) {
    CHECK_SIM(s);
    const int E = s->cfg.n_envs;
    hipLaunchKernelGGL(avr_dress_get_q_kernel, dim3((E * 7 + 255) / 256), dim3(256), 0, s->stream, s->d_state, s->d_query, s->d_query + E * 7, E);
    HIPCHK(s, hipGetLastError());
    if (q) HIPCHK(s, hipMemcpyAsync(q, s->d_query, (size_t)E * 7 * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (qd) HIPCHK(s, hipMemcpyAsync(qd, s->d_query + E * 7, (size_t)E * 7 * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_get_link_pose(avr_sim *s, int32_t link, float *out7) {
    (void)link; (void)out7;
    return fail(s, -1, "avr_get_link_pose: the tool frame is in the state block (AVR_DR_S_TOOL)");
}
int avr_get_contact_summary(avr_sim *s, float *out4) { (void)out4; return fail(s, -1, "avr_get_contact_summary: not defined for DressingJaco"); }
int avr_get_flags(avr_sim *s, int32_t *flags) {
    CHECK_SIM(s);
    if (!flags) return fail(s, -1, "avr_get_flags: flags is NULL");
    const int E = s->cfg.n_envs;
    hipLaunchKernelGGL(avr_dress_get_flags_kernel, dim3((E + 255) / 256), dim3(256), 0, s->stream, s->d_state, (int *)s->d_query, E);
    HIPCHK(s, hipGetLastError());
    HIPCHK(s, hipMemcpyAsync(flags, s->d_query, (size_t)E * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    return 0;
}
int avr_narrowphase_query(avr_sim *s, int32_t n, const int32_t *pairs, const float *poses14, float thr, float *out8) {
    (void)n; (void)pairs; (void)poses14; (void)thr; (void)out8;
    return fail(s, -1, "avr_narrowphase_query: DressingJaco has no rigid collision model");
}
int avr_robot_self_contact(avr_sim *s, int32_t n, const float *q, int32_t *out) {
    (void)n; (void)q; (void)out;
    return fail(s, -1, "avr_robot_self_contact: DressingJaco's robot is kinematic (no robot collision model)");
}
int avr_reset_ik(avr_sim *s, const uint8_t *mask, const float *h, const float *target7, const float *init, const float *alt4, int32_t restarts,
                 int32_t iters, float tol, const float *keepout8, int32_t n_frames, float *host_obs, uint8_t *host_ok) {
    CHECK_SIM(s);
    const size_t E = (size_t)s->cfg.n_envs;
    if (!h || !target7 || !init) return fail(s, -1, "avr_reset_ik: host_state, target7 and init are required");
    if (alt4 || keepout8) return fail(s, -1, "avr_reset_ik: DressingJaco's robot is kinematic (no self-contact screening, no keep-out box)");
    if (n_frames != 0) return fail(s, -1, "avr_reset_ik: DressingJaco has no settle frames");
    if (restarts < 1 || restarts > 64) return fail(s, -1, "avr_reset_ik: restarts %d outside 1..64", (int)restarts);
    if (iters < 0) return fail(s, -1, "avr_reset_ik: iters %d < 0", (int)iters);
    std::vector<uint8_t> all;
    if (!mask) { all.assign(E, 1); mask = all.data(); }
    const size_t need = E * 7 + E * (size_t)restarts * 7;
    if (need > s->ik_cap) {
        if (s->d_ik) HIPCHK(s, hipFree(s->d_ik));
        s->d_ik = nullptr;
        HIPCHK(s, hipMalloc(&s->d_ik, need * sizeof(float)));
        s->ik_cap = need;
    }
    if (upload_masked(s, mask, h)) return -2;
    HIPCHK(s, hipMemcpyAsync(s->d_ik, target7, E * 7 * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemcpyAsync(s->d_ik + E * 7, init, E * (size_t)restarts * 7 * sizeof(float), hipMemcpyHostToDevice, s->stream));
    HIPCHK(s, hipMemsetAsync(s->d_ok, 0, E, s->stream));
    hipLaunchKernelGGL(avr_dress_reset_ik_kernel, dim3(s->cfg.n_envs), dim3(64), 0, s->stream, s->d_m, s->d_state, s->d_mask, s->d_ik, s->d_ik + E * 7,
                       (int)restarts, (int)iters, tol, s->d_ok, s->cfg.n_envs);
    HIPCHK(s, hipGetLastError());
    HIPCHK(s, launch(s, nullptr, s->d_mask, DR_MODE_OBS, 0, s->d_obs, s->d_rew, s->d_done, s->d_info));
    std::vector<float> o(E * AVR_DR_OBS_DIM);
    std::vector<uint8_t> ok(E);
    HIPCHK(s, hipMemcpyAsync(o.data(), s->d_obs, o.size() * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipMemcpyAsync(ok.data(), s->d_ok, E, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    for (size_t e = 0; e < E; e++)
        if (mask[e]) {
            if (host_obs) memcpy(host_obs + e * AVR_DR_OBS_DIM, o.data() + e * AVR_DR_OBS_DIM, AVR_DR_OBS_DIM * sizeof(float));
            if (host_ok) host_ok[e] = ok[e];
        }
    return 0;
}
int avr_base_search(avr_sim *s, int32_t n, int32_t attempts, const float *base7, const float *rest, const float *tstart3, const float *goals9,
                    int32_t iters, float tol, int32_t *best, uint8_t *ok, float *q_arm, float *res4) {
    (void)n; (void)attempts; (void)base7; (void)rest; (void)tstart3; (void)goals9; (void)iters; (void)tol; (void)best; (void)ok; (void)q_arm; (void)res4;
    return fail(s, -1, "avr_base_search: DressingJaco has a fixed robot base");
}
}  // namespace avr_dressing
