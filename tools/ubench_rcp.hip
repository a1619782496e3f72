// Diagnostic: accuracy of v_rcp_f64 (raw and with 1 Newton step) vs correctly rounded 1/x.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
__global__ void k(const double* x, double* r0, double* r1, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a = x[i];
    double r = __builtin_amdgcn_rcp(a);
    r0[i] = r;
    double e = fma(-a, r, 1.0);
    r1[i] = fma(r, e, r);
}
int main() {
    const int n = 1 << 20;
    double* h = (double*)malloc(8 * n); double* g0 = (double*)malloc(8 * n); double* g1 = (double*)malloc(8 * n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = ldexp(1.0 + (double)(s >> 11) / 9007199254740992.0, (int)(s % 60) - 30); }
    double *dx, *d0, *d1; (void)hipMalloc(&dx, 8 * n); (void)hipMalloc(&d0, 8 * n); (void)hipMalloc(&d1, 8 * n);
    (void)hipMemcpy(dx, h, 8 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, n);
    (void)hipMemcpy(g0, d0, 8 * n, hipMemcpyDeviceToHost); (void)hipMemcpy(g1, d1, 8 * n, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0;
    for (int i = 0; i < n; ++i) { double t = 1.0 / h[i]; e0 = fmax(e0, fabs(g0[i] - t) / fabs(t)); e1 = fmax(e1, fabs(g1[i] - t) / fabs(t)); }
    printf("v_rcp_f64 max rel err: raw %.3e, 1 Newton %.3e (ulp = %.3e)\n", e0, e1, ldexp(1.0, -52));
}
