// Diagnostic micro-benchmark (not part of libmfgp.so): latency of the pieces on the
// k_chol_step critical path, each run REPS times inside ONE single-workgroup launch
// and timed with s_memtime (shader clock) + hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
static double prev[64 * 64];
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
        __shared__ long long st[2];
        if (WHAT == 5) tile_potrf_inv_w2(A, R, dg, &bad, reinterpret_cast<int*>(dg + NB + 1));
        if (WHAT == 4) { tile_potrf_inv_b8<NB>(A, R, dg, &bad, st); if (threadIdx.x == 0 && it == reps - 1) { cyc[1] = st[0]; cyc[2] = st[1]; } }
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) { cyc[0] = (t1 - t0) / (reps - 2); if (WHAT == 4) { cyc[3] = t1; } }
    acc_store(acc, out, NB);
    if (WHAT == 0 || WHAT == 4 || WHAT == 5) tile_store<NB>(out, NB, R);
}

template <int NB, int WHAT>
void run(const char* name, const double* dA, double* dO, long long* dc) {
    const int reps = 50;
    size_t sm = sizeof(double) * (3 * NB * (NB + 2) + NB + 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    long long c; hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    if (WHAT == 4) { long long cc[4]; hipMemcpy(cc, dc, sizeof(cc), hipMemcpyDeviceToHost);
        printf("    last iter: factor-phase end -> diag-inv end %lld clk, diag-inv end -> t1 %lld clk\n", cc[2] - cc[1], cc[3] - cc[2]); }
    if (WHAT == 0 || WHAT == 4 || WHAT == 5) {
        static double cur[64 * 64];
        hipMemcpy(cur, dO, sizeof(double) * NB * NB, hipMemcpyDeviceToHost);
        printf("    D[0][0]=%.6f D[1][0]=%.6f D[1][1]=%.6f D[31][0]=%.6e D[0][1]=%.3e D[31][31]=%.6f\n", cur[0], cur[NB], cur[NB+1], cur[31*NB], cur[1], cur[31*NB+31]);
        if (WHAT != 0) {
            double e = 0;
            for (int i = 0; i < NB * NB; ++i) e = fmax(e, fabs(cur[i] - prev[i]));
            printf("    max |D - D_pivot| = %.3e\n", e);
        } else memcpy(prev, cur, sizeof(double) * NB * NB);
    }
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
        hipMalloc(&dA, sizeof(double) * nb * nb); hipMalloc(&dO, sizeof(double) * nb * nb); hipMalloc(&dc, 64);
        hipMemcpy(dA, h, sizeof(double) * nb * nb, hipMemcpyHostToDevice);
        if (nb == 32) {
            run<32, 0>("tile_potrf_inv", dA, dO, dc); run<32, 4>("tile_potrf_inv_b8", dA, dO, dc); run<32, 5>("tile_potrf_inv_w2", dA, dO, dc); run<32, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<32, 2>("1 barrier + loads", dA, dO, dc); run<32, 3>("NB barriers", dA, dO, dc);
        } else {
            run<64, 0>("tile_potrf_inv", dA, dO, dc); run<64, 4>("tile_potrf_inv_b8", dA, dO, dc); run<64, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<64, 2>("1 barrier + loads", dA, dO, dc); run<64, 3>("NB barriers", dA, dO, dc);
        }
        hipFree(dA); hipFree(dO); hipFree(dc);
    }
    return 0;
}
