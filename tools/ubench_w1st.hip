// Diagnostic: per-round issue stamps of the single-wave factor (tools/ubench_w1.hip harness).
#include <hip/hip_runtime.h>
__device__ long long g_w1st[32];
#define W1_STAMP(i) do { W1_SCHED_BARRIER(); if (threadIdx.x == 0) g_w1st[i] = __builtin_amdgcn_s_memtime(); W1_SCHED_BARRIER(); } while (0)
#define main main_w1
#include "ubench_w1.hip"
#undef main
int main() {
    main_w1();
    long long h[32];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_w1st), sizeof(h));
    printf("round: publish->reads-issued+rwork | LDL..A-mfma issued | off-chain -> next publish\n");
    for (int k = 0; k < 8; ++k)
        printf("  K=%d  %5lld | %5lld | %5lld\n", k, h[3 * k + 1] - h[3 * k], h[3 * k + 2] - h[3 * k + 1],
               k < 7 ? h[3 * k + 3] - h[3 * k + 2] : 0LL);
    printf("  total rounds %lld clk\n", h[23] - h[0]);
    return 0;
}
