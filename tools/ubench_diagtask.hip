// Diagnostic: the k_chol_step diagonal task (panel product, trailing update, tile factor,
// stores) on one workgroup, global operands L2-hot, per-phase s_memtime stamps.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;
constexpr int NB = 32;
__global__ __launch_bounds__(256) void k_diag(const double* Aik, const double* Aij, const double* Dk, double* Dout,
                                              double* ldiag, long long* st, int reps) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ds = smem; double* T0 = Ds + E; double* Pi = T0 + E; double* Pj = Pi + E; double* dg = Pj + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    long long acc_t[6] = {0, 0, 0, 0, 0, 0};
    for (int it = 0; it < reps; ++it) {
        __syncthreads();
        long long t0 = __builtin_amdgcn_s_memtime();
        tile_load<NB>(Ds, Dk, NB);
        tile_load<NB>(T0, Aik, NB);
        Acc<NB> cij;
        acc_load(cij, Aij, NB);
        __syncthreads();
        long long t1 = __builtin_amdgcn_s_memtime();
        Acc<NB> acc; acc_zero(acc);
        tile_mma<NB, false, true>(acc, T0, Ds, 1.0);
        acc_to_lds(acc, Pi);
        __syncthreads();
        long long t2 = __builtin_amdgcn_s_memtime();
        acc = cij;
        tile_mma<NB, false, true>(acc, Pi, Pi, -1.0);
        acc_to_lds(acc, T0);
        __syncthreads();
        long long t3 = __builtin_amdgcn_s_memtime();
        tile_potrf_inv<NB>(T0, Pj, dg, &bad);
        long long t4 = __builtin_amdgcn_s_memtime();
        tile_store<NB>(Dout, NB, Pj);
        for (int r = threadIdx.x; r < NB; r += NTHREADS) ldiag[r] = dg[r];
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        long long t5 = __builtin_amdgcn_s_memtime();
        if (it > 0) { acc_t[0] += t1 - t0; acc_t[1] += t2 - t1; acc_t[2] += t3 - t2; acc_t[3] += t4 - t3; acc_t[4] += t5 - t4; acc_t[5] += t5 - t0; }
    }
    if (threadIdx.x == 0) for (int q = 0; q < 6; ++q) st[q] = acc_t[q] / (reps - 1);
}
int main() {
    const int n = NB * NB;
    double h[3 * n];
    for (int i = 0; i < NB; ++i) for (int j = 0; j < NB; ++j) {
        h[i * NB + j] = 0.01 / (1.0 + i + j);                         // A_ik
        h[n + i * NB + j] = (i == j ? NB : 0.0) + 1.0 / (1.0 + i + j); // A_ij (SPD)
        h[2 * n + i * NB + j] = (i == j) ? 1.0 : 0.0;                  // D_k
    }
    double *d, *o, *ld; long long* st;
    (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&o, 8 * n); (void)hipMalloc(&ld, 8 * NB); (void)hipMalloc(&st, 64);
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    size_t sm = sizeof(double) * (4 * TileCfg<NB>::ELEMS + NB + 2);
    hipLaunchKernelGGL(k_diag, dim3(1), dim3(256), sm, 0, d, d + n, d + 2 * n, o, ld, st, 20);
    long long s[6]; (void)hipMemcpy(s, st, sizeof(s), hipMemcpyDeviceToHost);
    printf("diag task (clk): loads %lld | P=A_ik D^T %lld | A_ij-=PP^T %lld | factor %lld | stores %lld | total %lld\n",
           s[0], s[1], s[2], s[3], s[4], s[5]);
    return 0;
}
