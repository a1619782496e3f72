// Diagnostic: hipGraph capture of the fp32 sweep's multi-stream fork / join pattern.
// Round 2 recorded that capturing a three-stream variant of the sweep (in-panel updates split
// between the panel stream and a third stream) "crashed the HIP graph capture"; the variant was not
// kept.  This probe rebuilds the launch / event pattern with small kernels at the Synth counts
// (T = 144 tile columns, panels of W = 6) and captures it in several forms, reporting the first
// failing HIP call of each:
//   two      the shipped lookahead: main + high-priority side stream, one fork / join event pair
//            re-recorded every panel (launch_f32_sweep)
//   three    + a third stream per in-panel update, one event pair reused for every column
//   three_ev the same with a fresh event pair per column
//   three_pr the third stream at the side stream's (high) priority
//   unjoined the third stream's last work never joined back before the capture ends
//   hipcc --offload-arch=gfx950 -O3 tools/graph_capture_probe.hip -o tools/ubench_graph_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <vector>

__global__ void k_work(float* p, int n, int tag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.999f + (float)tag;
}

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("    FAILED %s -> %s (%s)\n", #x, hipGetErrorName(e_), hipGetErrorString(e_)); \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

static int run(const char* mode, float* buf) {
    const bool three = strncmp(mode, "three", 5) == 0 || strcmp(mode, "unjoined") == 0;
    const bool fresh = strcmp(mode, "three_ev") == 0;
    const bool hiprio3 = strcmp(mode, "three_pr") == 0;
    const bool unjoined = strcmp(mode, "unjoined") == 0;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t s, side, third;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&third, hipStreamNonBlocking, hiprio3 ? hi : lo));
    hipEvent_t fork, join, f3, j3;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&f3, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j3, hipEventDisableTiming));
    std::vector<hipEvent_t> evs;
    const int T = 144, W = 6, n = 1 << 16;
    auto launch = [&](hipStream_t st, int tag) { hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, st, buf, n, tag); };
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    int tag = 0;
    auto panel = [&](int k0, int k1, hipStream_t ps) -> int {
        for (int k = k0; k < k1; ++k) {
            launch(ps, ++tag);   // diag
            launch(ps, ++tag);   // panel
            if (k + 1 < k1) {
                if (!three) {
                    launch(ps, ++tag);   // in-panel update
                } else {
                    hipEvent_t a = f3, b = j3;
                    if (fresh) {
                        CK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
                        CK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
                        evs.push_back(a);
                        evs.push_back(b);
                    }
                    CK(hipEventRecord(a, ps));
                    CK(hipStreamWaitEvent(third, a, 0));
                    launch(ps, ++tag);      // column k + 1
                    launch(third, ++tag);   // the rest of the panel's columns
                    CK(hipEventRecord(b, third));
                    if (!(unjoined && k + 2 >= k1)) CK(hipStreamWaitEvent(ps, b, 0));
                }
            }
        }
        return 0;
    };
    if (panel(0, W, s)) return 1;
    for (int k0 = 0; k0 < T; k0 += W) {
        const int k1 = k0 + W < T ? k0 + W : T;
        if (k1 >= T) break;
        const int k2 = k1 + W < T ? k1 + W : T;
        launch(s, ++tag);   // next panel's columns
        if (k2 < T) {
            CK(hipEventRecord(fork, s));
            CK(hipStreamWaitEvent(side, fork, 0));
            launch(s, ++tag);   // trailing update
            if (panel(k1, k2, side)) return 1;
            CK(hipEventRecord(join, side));
            CK(hipStreamWaitEvent(s, join, 0));
        } else if (panel(k1, k2, s)) {
            return 1;
        }
    }
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(s, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    hipGraphExec_t ge = nullptr;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    printf("    ok: %zu nodes, %d kernels, instantiated and replayed 3x\n", nn, tag);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    for (hipEvent_t e : evs) CK(hipEventDestroy(e));
    CK(hipEventDestroy(fork));
    CK(hipEventDestroy(join));
    CK(hipEventDestroy(f3));
    CK(hipEventDestroy(j3));
    CK(hipStreamDestroy(s));
    CK(hipStreamDestroy(side));
    CK(hipStreamDestroy(third));
    return 0;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    float* buf;
    if (hipMalloc(&buf, sizeof(float) << 16) != hipSuccess) return 2;
    (void)hipMemset(buf, 0, sizeof(float) << 16);
    const char* modes[] = {"two", "three", "three_ev", "three_pr", "unjoined"};
    for (const char* m : modes) {
        if (argc > 1 && strcmp(argv[1], m) != 0) continue;
        printf("%s\n", m);
        run(m, buf);
        (void)hipGetLastError();
    }
    return 0;
}
