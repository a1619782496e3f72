// Diagnostic: where the fp32 128 x 128 diagonal-block factor (k32_diag) spends its time.
// Variants of the kernel body on one SPD block: V0 the library kernel, V1 staging only
// (load + store), V2 + the four factor32_w1 sub-factors, V3 + the MFMA panel / trailing stages
// (no inverse blocks).  hipEvent timing over 200 launches each.
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_f32.hip"
#include <stdio.h>
#include <vector>
using namespace mfgp;
using namespace mfgp::f32;

template <int V>
__global__ __launch_bounds__(DIAG_THREADS) void k_var(F32Args a, int k) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;
    float* Ds = As + TB * DLD;
    float* Ts = Ds + TB * DLD;
    float* piv = Ts + 3 * 32 * 33;
    int* bad = reinterpret_cast<int*>(piv + TB);
    int* badw = bad + 1;
    double* R64 = reinterpret_cast<double*>(smem + 2 * TB * DLD + 3 * 32 * 33 + TB + 4);
    double* dg64 = R64 + DIAG_R64;
    double* X64 = reinterpret_cast<double*>(Ts);
    const int w = threadIdx.x >> 6;
    float* Mkk = a.M + row_off(a, k) + (long)k * TB;
    for (int e = threadIdx.x; e < TB * TB / 4; e += DIAG_THREADS) {
        const int r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
        *reinterpret_cast<f32x4*>(As + r * DLD + c4) = *reinterpret_cast<const f32x4*>(Mkk + (long)r * a.ld + c4);
        *reinterpret_cast<f32x4*>(Ds + r * DLD + c4) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if (threadIdx.x == 0) *bad = 0;
    __syncthreads();
    auto T32 = [&](float* base, int i, int j) { return base + 32 * i * DLD + 32 * j; };
    if (V >= 2) {
        for (int s = 0; s < 4; ++s) {
            if (w == 0) factor32_w1(As, Ds, 32 * s, X64, R64, dg64, badw, bad, a.ldiag + k * TB);
            __syncthreads();
            if (V >= 3) {
                for (int i = s + w; i < 4; i += 4) {
                    f32x16 acc = {};
                    mma32_nt(acc, T32(As, i, s), DLD, T32(Ds, s, s), DLD);
                    acc32_store(T32(As, i, s), DLD, acc, 1.0f);
                }
                __syncthreads();
                int t = 0;
                for (int i = s + 1; i < 4; ++i)
                    for (int j = s + 1; j <= i; ++j, ++t) {
                        if (t % 4 != w) continue;
                        f32x16 acc;
                        acc32_load(acc, T32(As, i, j), DLD);
                        f32x16 p = {};
                        mma32_nt(p, T32(As, i, s), DLD, T32(As, j, s), DLD);
                        acc -= p;
                        acc32_store(T32(As, i, j), DLD, acc, 1.0f);
                    }
                __syncthreads();
            }
        }
    }
    float* Dk = a.Dd + (long)k * TB * TB;
    for (int e = threadIdx.x; e < TB * TB / 4; e += DIAG_THREADS) {
        const int r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
        const f32x4 lv = *reinterpret_cast<const f32x4*>(As + r * DLD + c4);
        float* dst = Mkk + (long)r * a.ld + c4;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c4 + q <= r) dst[q] = lv[q];
        *reinterpret_cast<f32x4*>(Dk + r * TB + c4) = *reinterpret_cast<const f32x4*>(Ds + r * DLD + c4);
    }
    (void)piv;
}

template <class K>
static float time_it(K kern, const F32Args& a, const std::vector<float>& h, float* dM) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipMemcpy(dM, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, 0);
        for (int it = 0; it < 40; ++it) kern(a);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms * 1e3f / 40);
    }
    return best;
}

int main() {
    const int n = TB;
    std::vector<float> h(n * n);
    srand(3);
    std::vector<double> x(n * 10);
    for (auto& v : x) v = rand() / (double)RAND_MAX;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double r2 = 0;
            for (int d = 0; d < 10; ++d) r2 += (x[i * 10 + d] - x[j * 10 + d]) * (x[i * 10 + d] - x[j * 10 + d]);
            h[i * n + j] = (float)(exp(-0.5 * r2) + (i == j ? 1e-2 : 0.0));
        }
    float *dM, *dD;
    double* dl;
    int* info;
    (void)hipMalloc(&dM, n * n * 4);
    (void)hipMalloc(&dD, n * n * 4);
    (void)hipMalloc(&dl, n * 8);
    (void)hipMalloc(&info, 4);
    (void)hipMemset(info, 0, 4);
    F32Args a{};
    a.M = dM; a.ld = n; a.T = 1; a.Dd = dD; a.ldiag = dl; a.info = info; a.n = n;
    f32_lds_attributes();
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_var<1>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)DIAG_SMEM);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_var<2>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)DIAG_SMEM);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_var<3>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)DIAG_SMEM);
    const float t0 = time_it([](const F32Args& a) { hipLaunchKernelGGL(k32_diag, dim3(1), dim3(DIAG_THREADS), DIAG_SMEM, 0, a, 0); }, a, h, dM);
    const float t1 = time_it([](const F32Args& a) { hipLaunchKernelGGL(k_var<1>, dim3(1), dim3(DIAG_THREADS), DIAG_SMEM, 0, a, 0); }, a, h, dM);
    const float t2 = time_it([](const F32Args& a) { hipLaunchKernelGGL(k_var<2>, dim3(1), dim3(DIAG_THREADS), DIAG_SMEM, 0, a, 0); }, a, h, dM);
    const float t3 = time_it([](const F32Args& a) { hipLaunchKernelGGL(k_var<3>, dim3(1), dim3(DIAG_THREADS), DIAG_SMEM, 0, a, 0); }, a, h, dM);
    printf("k32_diag %.1f us | staging only %.1f | + 4 x factor32_w1 %.1f | + panel/trailing MFMA %.1f (inverse = rest)\n",
           t0, t1, t2, t3);
    return 0;
}
