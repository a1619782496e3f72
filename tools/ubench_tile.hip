// Diagnostic micro-benchmark (not part of libmfgp.so): latency of the pieces on the
// k_chol_step critical path, each run REPS times inside ONE single-workgroup launch
// and timed with s_memtime (shader clock) + hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;

template <int NB, int WHAT>
__global__ __launch_bounds__(256) void k_bench(const double* Ag, double* out, long long* cyc, int reps) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem; double* R = A + E; double* B = R + E; double* dg = B + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    long long t0 = 0, t1 = 0;
    Acc<NB> acc; acc_zero(acc);
    for (int it = 0; it < reps; ++it) {
        tile_load<NB>(A, Ag, NB);
        tile_load<NB>(B, Ag, NB);
        __syncthreads();
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        if (WHAT == 0) tile_potrf_inv<NB>(A, R, dg, &bad);
        if (WHAT == 1) { tile_mma<NB, false, true>(acc, A, B, 1.0); __syncthreads(); }
        if (WHAT == 2) { __syncthreads(); }
        if (WHAT == 3) { for (int k = 0; k < NB; ++k) __syncthreads(); }
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / (reps - 2);
    acc_store(acc, out, NB);
    if (WHAT == 0) tile_store<NB>(out, NB, R);
}

template <int NB, int WHAT>
void run(const char* name, const double* dA, double* dO, long long* dc) {
    const int reps = 50;
    size_t sm = sizeof(double) * (3 * NB * (NB + 2) + NB + 2);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    long long c; hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-28s NB=%d  %8lld shader-clk/iter (s_memtime)   %.3f us/iter (event, incl. 2 tile loads)\n", name, NB, c,
           ms * 1e3 / reps);
}

int main() {
    const int NBm = 64;
    double* h = (double*)malloc(sizeof(double) * NBm * NBm);
    for (int nb : {32, 64}) {
        for (int i = 0; i < nb; ++i)
            for (int j = 0; j < nb; ++j) h[i * nb + j] = (i == j ? nb : 0.0) + 1.0 / (1.0 + i + j);
        double *dA, *dO; long long* dc;
        hipMalloc(&dA, sizeof(double) * nb * nb); hipMalloc(&dO, sizeof(double) * nb * nb); hipMalloc(&dc, 8);
        hipMemcpy(dA, h, sizeof(double) * nb * nb, hipMemcpyHostToDevice);
        if (nb == 32) {
            run<32, 0>("tile_potrf_inv", dA, dO, dc); run<32, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<32, 2>("1 barrier + loads", dA, dO, dc); run<32, 3>("NB barriers", dA, dO, dc);
        } else {
            run<64, 0>("tile_potrf_inv", dA, dO, dc); run<64, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<64, 2>("1 barrier + loads", dA, dO, dc); run<64, 3>("NB barriers", dA, dO, dc);
        }
        hipFree(dA); hipFree(dO); hipFree(dc);
    }
    return 0;
}
