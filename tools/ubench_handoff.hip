// Diagnostic: dependent-load latency of the load flavours the k_chol_flow hand-offs can use,
// against working sets that live in L2 (1 MB), in the MALL (64 MB) and in HBM (1 GB).
//   plain   : global_load (cached in L1/L2)
//   agent   : __hip_atomic_load relaxed, agent scope (ld_coherent: global_load ... sc1)
//   buf_sc1 : raw_buffer_load aux 16 (op_load_pub's 16-B loads)
// One lane chases a random cyclic permutation with a 256-B stride; ns per load from
// s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

template <int MODE>
__global__ void k_chase(const long long* buf, long long start, int steps, long long* out) {
    if (threadIdx.x != 0) return;
    long long idx = start;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<long long*>(buf), (short)0, 0x7fffffff, 0x00020000);
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int s = 0; s < steps; ++s) {
        if (MODE == 0) idx = buf[idx];
        else if (MODE == 1) idx = __hip_atomic_load(const_cast<long long*>(buf + idx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else {
            // buffer offsets are 32-bit: the 1 GB set still fits (< 2 GB)
            const unsigned lo = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(idx * 8), 0, 16);
            idx = (long long)lo;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = idx;
    out[1] = t1 - t0;
}

int main() {
    const size_t sizes[3] = {1u << 20, 64u << 20, 1u << 30};
    const char* names[3] = {"1 MB (L2)", "64 MB (MALL)", "1 GB (HBM)"};
    long long* d;
    long long* o;
    (void)hipMalloc(&d, sizes[2]);
    (void)hipMalloc(&o, 16);
    srand(1);
    for (int z = 0; z < 3; ++z) {
        const size_t nslot = sizes[z] / 256;          // one element per 256 B
        std::vector<long long> perm(nslot), h(nslot * 32, 0);
        for (size_t i = 0; i < nslot; ++i) perm[i] = (long long)i;
        for (size_t i = nslot - 1; i > 0; --i) std::swap(perm[i], perm[(size_t)rand() % (i + 1)]);
        for (size_t i = 0; i < nslot; ++i) h[perm[i] * 32] = perm[(i + 1) % nslot] * 32;
        (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
        const int steps = 4000;
        long long r[2];
        for (int m = 0; m < 3; ++m) {
            // 1 MB: rep 0 warms the whole set into L2; larger sets: every (mode, rep) chases a
            // fresh part of the cycle, so only the caches that hold the whole set can hit
            for (int rep = 0; rep < 2; ++rep) {
                const long long st = perm[z == 0 ? 0 : ((size_t)(2 * m + rep + 1) * 5000) % nslot] * 32;
                if (m == 0) hipLaunchKernelGGL(k_chase<0>, dim3(1), dim3(64), 0, 0, d, st, steps, o);
                if (m == 1) hipLaunchKernelGGL(k_chase<1>, dim3(1), dim3(64), 0, 0, d, st, steps, o);
                if (m == 2) hipLaunchKernelGGL(k_chase<2>, dim3(1), dim3(64), 0, 0, d, st, steps, o);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
            printf("%-14s %-8s %7.1f ns/load\n", names[z], m == 0 ? "plain" : m == 1 ? "agent" : "buf_sc1",
                   r[1] * 10.0 / steps);
        }
    }
    return 0;
}
