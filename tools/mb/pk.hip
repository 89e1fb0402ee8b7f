#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_fma(float *out, long long *cyc, int n, float b, float c) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;

    long long t0 = clock64();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a0 = __builtin_fmaf(a0, b, c); a1 = __builtin_fmaf(a1, b, c); a2 = __builtin_fmaf(a2, b, c); a3 = __builtin_fmaf(a3, b, c);
            a4 = __builtin_fmaf(a4, b, c); a5 = __builtin_fmaf(a5, b, c); a6 = __builtin_fmaf(a6, b, c); a7 = __builtin_fmaf(a7, b, c);
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void k_pk(float *out, long long *cyc, int n, float bx, float by, float cx, float cy) {
    f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const f2 b = {bx, by}, c = {cx, cy};
    long long t0 = clock64();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a0 = __builtin_elementwise_fma(a0, b, c); a1 = __builtin_elementwise_fma(a1, b, c);
            a2 = __builtin_elementwise_fma(a2, b, c); a3 = __builtin_elementwise_fma(a3, b, c);
        }
    }
    long long t1 = clock64();
    f2 s = a0 + a1 + a2 + a3;
    out[blockIdx.x * 64 + threadIdx.x] = s.x + s.y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    float *o; long long *c; hipMalloc(&o, 1 << 20); hipMalloc(&c, 8192);
    long long h[1024];
    int n = 4096;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_fma, dim3(1024), dim3(64), 0, 0, o, c, n, 0.999f, 0.001f); hipDeviceSynchronize();
        hipMemcpy(h, c, 8 * 1024, hipMemcpyDeviceToHost);
        double s = 0; for (int i = 0; i < 1024; i++) s += h[i];
        printf("fma: %.2f clock64 ticks per instruction (1 wave/SIMD, 1024 blocks), 8 fma/iter x 8\n", s / 1024 / (n * 64.0));
        hipLaunchKernelGGL(k_pk, dim3(1024), dim3(64), 0, 0, o, c, n, 0.999f, 0.998f, 0.001f, 0.002f); hipDeviceSynchronize();
        hipMemcpy(h, c, 8 * 1024, hipMemcpyDeviceToHost);
        s = 0; for (int i = 0; i < 1024; i++) s += h[i];
        printf("pk_fma: %.2f clock64 ticks per instruction (2 fma each)\n", s / 1024 / (n * 32.0));
    }
    return 0;
}
