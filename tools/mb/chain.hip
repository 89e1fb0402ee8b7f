// Microbenchmark: cycles per dependent step of the instruction chains a part-B row resolve is made
// of (one wave alone on its SIMD, clock64 around the loop).  hipcc --offload-arch=gfx950 -O3
// tools/mb/chain.hip -o /tmp/chain && /tmp/chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dpp(float x, int ctl) {
    switch (ctl) {
    case 8: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, true));
    case 4: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xf, 0xf, true));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xf, 0xf, true));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xf, 0xf, true));
    }
}
__device__ __forceinline__ float row16(float x) { x += dpp(x, 8); x += dpp(x, 4); x += dpp(x, 2); x += dpp(x, 1); return x; }

#define N 256
// 0: dependent fma chain; 1: dependent pk_fma chain; 2: dependent add_dpp chain; 3: row16 + fma;
// 4: the go4 arithmetic chain (packed, as avr_kernel.hip B4_PK); 5: the same unpacked;
// 6: 4 independent fma chains; 7: 4 independent pk chains; 8: dependent ds_read chain
template <int mode>
__global__ __launch_bounds__(64) void k(float *out, long long *cyc, float b, float c) {
#pragma clang fp contract(off)
    __shared__ int lds[1024];
    const int l = threadIdx.x;
    for (int i = l; i < 1024; i += 64) lds[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    float x = l * 1e-3f, y = x + 1.f, z = x + 2.f, w = x + 3.f;
    f2 p = {x, y}, q = {z, w}, r = {y, z}, s = {w, x};
    f2 j0 = {b, c}, j1 = {c, b}, j2 = {b, b};
    int ix = l;
    long long t0 = clock64();
    for (int it = 0; it < N; it++) {
        switch (mode) {   // (compile-time: no branch in the timed loop)
        case 0:
#pragma unroll
            for (int u = 0; u < 16; u++) x = __builtin_fmaf(x, b, c);
            break;
        case 1:
#pragma unroll
            for (int u = 0; u < 16; u++) p = __builtin_elementwise_fma(p, j0, j1);
            break;
        case 2:
#pragma unroll
            for (int u = 0; u < 16; u++) x += dpp(x, 8 >> (u & 3));
            break;
        case 3:
#pragma unroll
            for (int u = 0; u < 4; u++) x = __builtin_fmaf(row16(x), b, c);
            break;
        case 4:
#pragma unroll
            for (int u = 0; u < 4; u++) {   // p, q, r: velocities (v1, v2, v3); j0..j2 parts
                f2 sm = j0 * p;
                sm = __builtin_elementwise_fma(j1, q, sm);
                sm = __builtin_elementwise_fma(j2, r, sm);
                const float dv = row16(sm.x + sm.y);
                const float ni = __builtin_amdgcn_fmed3f(y + __builtin_fmaf(-dv, b, c), -1.f, 1.f);
                const float d = ni - y;
                y = ni;
                const f2 dd = {d, d};
                p = __builtin_elementwise_fma(j0, dd, p);
                q = __builtin_elementwise_fma(j1, dd, q);
                r = __builtin_elementwise_fma(j2, dd, r);
            }
            break;
        case 5:
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const float pp = __builtin_fmaf(j1.x, p.y, __builtin_fmaf(j0.y, q.x, j0.x * p.x));
                const float qq = __builtin_fmaf(j2.y, r.y, __builtin_fmaf(j2.x, r.x, j1.y * q.y));
                const float dv = row16(pp + qq);
                const float ni = __builtin_amdgcn_fmed3f(y + __builtin_fmaf(-dv, b, c), -1.f, 1.f);
                const float d = ni - y;
                y = ni;
                p.x = __builtin_fmaf(j0.x, d, p.x); q.x = __builtin_fmaf(j0.y, d, q.x); p.y = __builtin_fmaf(j1.x, d, p.y);
                q.y = __builtin_fmaf(j1.y, d, q.y); r.x = __builtin_fmaf(j2.x, d, r.x); r.y = __builtin_fmaf(j2.y, d, r.y);
            }
            break;
        case 6:
#pragma unroll
            for (int u = 0; u < 4; u++) { x = __builtin_fmaf(x, b, c); y = __builtin_fmaf(y, b, c); z = __builtin_fmaf(z, b, c); w = __builtin_fmaf(w, b, c); }
            break;
        case 7:
#pragma unroll
            for (int u = 0; u < 4; u++) { p = __builtin_elementwise_fma(p, j0, j1); q = __builtin_elementwise_fma(q, j0, j1); r = __builtin_elementwise_fma(r, j0, j1); s = __builtin_elementwise_fma(s, j0, j1); }
            break;
        case 8:
#pragma unroll
            for (int u = 0; u < 16; u++) ix = lds[ix];
            break;
        case 9:   // go4 chain with the row-16 sum replaced by a 2-step (row_ror 8, 4) + 2 quad_perm sum
#pragma unroll
            for (int u = 0; u < 4; u++) {
                f2 sm = j0 * p;
                sm = __builtin_elementwise_fma(j1, q, sm);
                sm = __builtin_elementwise_fma(j2, r, sm);
                float t = sm.x + sm.y;
                t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xb1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
                t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x4e, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
                t += dpp(t, 4);
                t += dpp(t, 8);
                const float ni = __builtin_amdgcn_fmed3f(y + __builtin_fmaf(-t, b, c), -1.f, 1.f);
                const float d = ni - y;
                y = ni;
                const f2 dd = {d, d};
                p = __builtin_elementwise_fma(j0, dd, p);
                q = __builtin_elementwise_fma(j1, dd, q);
                r = __builtin_elementwise_fma(j2, dd, r);
            }
            break;
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * 64 + l] = x + y + z + w + p.x + p.y + q.x + q.y + r.x + r.y + s.x + s.y + (float)ix;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *out; long long *cyc;
    const int nb = 1024;
    (void)hipMalloc(&out, nb * 64 * 4); (void)hipMalloc(&cyc, nb * 8);
    const char *nm[] = {"fma dep", "pk_fma dep", "add_dpp dep", "row16+fma", "go4 packed", "go4 unpacked", "4x fma indep", "4x pk_fma indep", "ds_read dep", "go4 quad_perm sum"};
    const int per[] = {16, 16, 16, 4, 4, 4, 16, 16, 16, 4};
    void (*ks[])(float *, long long *, float, float) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>};
    for (int mode = 0; mode < 10; mode++) {
        for (int blocks : {1, 1024}) {
            long long h[1024];
            double best = 1e30;
            for (int rep = 0; rep < 3; rep++) {
                hipLaunchKernelGGL(ks[mode], dim3(blocks), dim3(64), 0, 0, out, cyc, 0.999f, 1e-4f);
                (void)hipDeviceSynchronize();
                (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
                double m = 0; for (int i = 0; i < blocks; i++) m += h[i]; m /= blocks;
                if (m < best) best = m;
            }
            printf("%-20s blocks %4d: %.1f cycles per step\n", nm[mode], blocks, best / (N * per[mode]));
        }
    }
    return 0;
}
