// Diagnostic: dependent-kernel floor inside a hipGraph chain (replayed), vs work per kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_empty(double* p) { if (p == nullptr) p[threadIdx.x] = 0; }
__global__ void k_touch(double* p, long n) {   // writes n doubles
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) p[e] += 1.0;
}
int main() {
    double* buf; (void)hipMalloc(&buf, 64 << 20);
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int CH = 100;
    for (int mode = 0; mode < 5; ++mode) {
        long n = mode == 0 ? 0 : mode == 1 ? 1024 : mode == 2 ? (512 << 10) : mode == 3 ? (4 << 20) / 8 * 8 : (8 << 20);
        int grid = mode == 0 ? 1 : mode == 1 ? 4 : 1024;
        hipGraph_t g; hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < CH; ++i) {
            if (mode == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, buf);
            else hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, s, buf, n);
        }
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphLaunch(ge, s); (void)hipStreamSynchronize(s);
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a, s);
        for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(b, s); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("graph chain: %s  %7.2f us per kernel (bytes touched %ld)\n",
               mode == 0 ? "empty 1 WG    " : "touch kernel  ", ms * 1e3 / (10 * CH), n * 8);
    }
    return 0;
}
