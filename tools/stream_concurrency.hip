// Stream concurrency probe: N non-blocking streams each launch K back-to-back kernels of B
// one-wave blocks (with L bytes of LDS each) that spin for ~T microseconds (s_memrealtime, 100 MHz); prints the wall time
// per round for N = 1..8.  Perfect concurrency keeps it at K x T; serialisation grows it with N.
//   hipcc --offload-arch=gfx950 -O2 tools/stream_concurrency.hip -o tools/stream_concurrency
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void spin(unsigned long long ticks, int *sink) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int x = threadIdx.x;
    lds[threadIdx.x] = x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525 + 1013904223;
    if (x == 0x7fffffff) sink[blockIdx.x] = x + lds[(threadIdx.x + 1) & 63];          // keeps the loop; practically never stores
}

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 256;       // blocks per launch
    const int K = argc > 2 ? atoi(argv[2]) : 20;        // launches per stream per round
    const double T = argc > 3 ? atof(argv[3]) : 50.0;   // spin per launch, microseconds
    const int LDSB = argc > 4 ? atoi(argv[4]) : 256;    // dynamic LDS bytes per block
    int *sink;
    CHK(hipMalloc(&sink, 4 * 65536));
    hipStream_t st[8];
    for (int i = 0; i < 8; i++) CHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    const unsigned long long ticks = (unsigned long long)(T * 100.0);   // 100 MHz realtime counter
    for (int n = 1; n <= 8; n++) {
        double best = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            CHK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < K; k++)
                for (int s = 0; s < n; s++) spin<<<B, 64, LDSB, st[s]>>>(ticks, sink);
            CHK(hipDeviceSynchronize());
            double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (us < best) best = us;
        }
        printf("streams %d blocks %d lds %d launches/stream %d spin %.0f us: round %.0f us (ideal %.0f)\n", n, B, LDSB, K, T, best, K * T);
    }
    CHK(hipFree(sink));
    return 0;
}
