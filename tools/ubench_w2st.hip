// Diagnostic: issue stamps of the two-wave factor (tools/ubench_w1.hip harness).
#include <hip/hip_runtime.h>
__device__ long long g_w2st[32];
#define W2_STAMP(i) do { __builtin_amdgcn_sched_barrier(0); if ((threadIdx.x & 63) == 0) g_w2st[i] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define main main_w1
#include "ubench_w1.hip"
#undef main
int main() {
    main_w1();
    long long h[32];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_w2st), sizeof(h));
    printf("K   wave0 round start | wave1 round start (clk from wave0 K=0)\n");
    for (int k = 0; k < 8; ++k) printf("%d  %6lld | %6lld\n", k, h[k] - h[0], h[8 + k] - h[0]);
    printf("wave0 end %lld, wave1 rounds end %lld\n", h[16] - h[0], h[17] - h[0]);
    return 0;
}
