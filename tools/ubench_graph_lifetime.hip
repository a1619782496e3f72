// Diagnostic: the session-lifetime pattern of the fp32 sweep with the HIP runtime
// alone (no torch, no libmfgp).  Per session k: a new stream s_k; one eager run of the step's launch
// pattern (main stream + the handle's high-priority side stream, one fork / join event pair shared
// by every session, as mfgp_f32.hip launch_f32_sweep); a capture of the same pattern on s_k,
// instantiated, the hipGraph itself destroyed right away (as torch does); then the graph replayed.
// The previous session's graph exec is destroyed at a point set by the mode:
//   reassign       before session k captures (the order of round 5's knob sweep)
//   after          after session k captured, before its first replay
//   nofork         reassign, but the pattern never forks to the side stream
//   samestream     reassign, every session on one stream
//   reassign_free  reassign + a hipFree of a fresh 64 MB buffer before each capture (torch's
//                  empty_cache at torch.cuda.graph entry)
//   reassign_cs    reassign, every capture on ONE capture stream (torch's default capture stream),
//                  the eager runs and the replays on the session's stream s_k
//   after_cs       after, with the capture stream
//   *_af           (suffix) instantiated with hipGraphInstantiateFlagAutoFreeOnLaunch, as torch's
//                  CUDAGraph::capture_end does
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_graph_lifetime.hip -o tools/ubench_graph_lifetime
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

__global__ void k_work(float* p, int n, int tag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.999f + (float)tag;
}

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("FAILED %s -> %s\n", #x, hipGetErrorName(e_));                               \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "reassign";
    const bool fork = strcmp(mode, "nofork") != 0;
    const bool same = strcmp(mode, "samestream") == 0;
    const bool after = strncmp(mode, "after", 5) == 0;
    const bool dofree = strcmp(mode, "reassign_free") == 0;
    const bool cs = strstr(mode, "_cs") != nullptr;
    const bool af = strstr(mode, "_af") != nullptr;
    const int sessions = 8, panels = 20, n = 1 << 16;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t side;
    CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, hi));
    hipEvent_t evf, evj;
    CK(hipEventCreateWithFlags(&evf, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evj, hipEventDisableTiming));
    float* buf;
    CK(hipMalloc(&buf, n * sizeof(float)));
    CK(hipMemset(buf, 0, n * sizeof(float)));
    auto pattern = [&](hipStream_t s) {
        int tag = 0;
        for (int p = 0; p < panels; ++p) {
            hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, s, buf, n, ++tag);
            if (fork) {
                (void)hipEventRecord(evf, s);
                (void)hipStreamWaitEvent(side, evf, 0);
                hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, s, buf, n / 2, ++tag);
                hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, side, buf + n / 2, n / 2, ++tag);
                (void)hipEventRecord(evj, side);
                (void)hipStreamWaitEvent(s, evj, 0);
            }
        }
    };
    hipStream_t one = nullptr, cap = nullptr;
    if (same) CK(hipStreamCreateWithFlags(&one, hipStreamNonBlocking));
    if (cs) CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
    hipGraphExec_t prev = nullptr;
    for (int k = 0; k < sessions; ++k) {
        hipStream_t s = one;
        if (!same) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        pattern(s);                       // eager warm-up
        CK(hipStreamSynchronize(s));
        if (!after && prev) { CK(hipGraphExecDestroy(prev)); prev = nullptr; }
        if (dofree) {
            void* t;
            CK(hipMalloc(&t, 64 << 20));
            CK(hipFree(t));
        }
        hipGraph_t g;
        hipStream_t c = cs ? cap : s;
        if (cs) {   // the capture stream follows the session's work (torch's wait_stream)
            hipEvent_t e;
            CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            CK(hipEventRecord(e, s));
            CK(hipStreamWaitEvent(c, e, 0));
            CK(hipStreamSynchronize(c));
            CK(hipEventDestroy(e));
        }
        CK(hipStreamBeginCapture(c, hipStreamCaptureModeGlobal));
        pattern(c);
        pattern(c);                       // two steps a graph
        CK(hipStreamEndCapture(c, &g));
        hipGraphExec_t ex;
        if (af) CK(hipGraphInstantiateWithFlags(&ex, g, hipGraphInstantiateFlagAutoFreeOnLaunch));
        else CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
        if (after && prev) { CK(hipGraphExecDestroy(prev)); prev = nullptr; }
        printf("session %d: launching\n", k);
        fflush(stdout);
        CK(hipGraphLaunch(ex, s));
        CK(hipGraphLaunch(ex, s));
        CK(hipStreamSynchronize(s));
        printf("session %d: ok\n", k);
        fflush(stdout);
        prev = ex;
    }
    printf("%s: all %d sessions ok\n", mode, sessions);
    return 0;
}
