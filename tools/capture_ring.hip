// The capture pattern that kills the process (VERDICT round 4
// item 4), in plain HIP: no torch, no srpc library.  A stream capture forks
// three streams (in, k, out) off the capturing stream with an event, then
// runs CHUNKS rounds of in -> k -> out joined by events, and, from round
// DEPTH on, makes `in` wait on k's event of round i - DEPTH and/or `k` wait on
// out's event of round i - DEPTH (the ring of a depth-limited pipeline).
//
//   capture_ring <mode>    mode: none | in | k | both | in_work | in_lazy
//
// in_lazy: as `in`, with every event created right before its first record,
// inside the capture (as torch.cuda.Event() does on its first record()).
//
// Prints "captured", "replayed" and exits 0 when the runtime takes the
// pattern; a crash inside hipStreamBeginCapture..EndCapture shows up as a
// signal exit status (the caller runs it as a child process).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 2;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_add(int* p, int n, int v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += v;
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "both";
    const bool lazy = !std::strcmp(mode, "in_lazy");
    const bool in_ring = !std::strcmp(mode, "in") || !std::strcmp(mode, "both") || !std::strcmp(mode, "in_work") || lazy;
    const bool k_ring = !std::strcmp(mode, "k") || !std::strcmp(mode, "both");
    const bool in_work = !std::strcmp(mode, "in_work");  // a kernel on `in` between its wait and its record
    constexpr int kChunks = 8, kDepth = 2, kN = 1 << 16;
    int* buf[kChunks];
    int* inb = nullptr;
    for (auto& b : buf) CK(hipMalloc(&b, kN * sizeof(int)));
    CK(hipMalloc(&inb, kN * sizeof(int)));
    for (auto& b : buf) CK(hipMemset(b, 0, kN * sizeof(int)));
    hipStream_t cur, s_in, s_k, s_out;
    CK(hipStreamCreateWithFlags(&cur, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s_k, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
    hipEvent_t start, ev_in[kChunks], ev_k[kChunks], ev_out[kChunks];
    CK(hipEventCreateWithFlags(&start, hipEventDisableTiming));
    for (int i = 0; i < kChunks && !lazy; ++i) {
        CK(hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_k[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_out[i], hipEventDisableTiming));
    }
    std::printf("mode %s: capturing\n", mode);
    std::fflush(stdout);
    CK(hipStreamBeginCapture(cur, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(start, cur));
    CK(hipStreamWaitEvent(s_in, start, 0));
    CK(hipStreamWaitEvent(s_k, start, 0));
    CK(hipStreamWaitEvent(s_out, start, 0));
    for (int i = 0; i < kChunks; ++i) {
        if (i >= kDepth) {
            if (in_ring) CK(hipStreamWaitEvent(s_in, ev_k[i - kDepth], 0));
            if (k_ring) CK(hipStreamWaitEvent(s_k, ev_out[i - kDepth], 0));
        }
        if (in_work) hipLaunchKernelGGL(k_add, dim3(kN / 256), dim3(256), 0, s_in, inb, kN, 1);
        if (lazy) CK(hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming));
        CK(hipEventRecord(ev_in[i], s_in));
        CK(hipStreamWaitEvent(s_k, ev_in[i], 0));
        hipLaunchKernelGGL(k_add, dim3(kN / 256), dim3(256), 0, s_k, buf[i % kChunks], kN, 1);
        if (lazy) CK(hipEventCreateWithFlags(&ev_k[i], hipEventDisableTiming));
        CK(hipEventRecord(ev_k[i], s_k));
        CK(hipStreamWaitEvent(s_out, ev_k[i], 0));
        hipLaunchKernelGGL(k_add, dim3(kN / 256), dim3(256), 0, s_out, buf[i % kChunks], kN, 2);
        if (lazy) CK(hipEventCreateWithFlags(&ev_out[i], hipEventDisableTiming));
        CK(hipEventRecord(ev_out[i], s_out));
    }
    // (in and k join through out: their last events are waited on there)
    CK(hipStreamWaitEvent(cur, ev_out[kChunks - 1], 0));
    hipGraph_t g;
    CK(hipStreamEndCapture(cur, &g));
    std::printf("mode %s: captured\n", mode);
    std::fflush(stdout);
    hipGraphExec_t x;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, cur));
    CK(hipStreamSynchronize(cur));
    int h = 0;
    CK(hipMemcpy(&h, buf[kChunks - 1], sizeof(int), hipMemcpyDeviceToHost));
    std::printf("mode %s: replayed, value %d (want 3)\n", mode, h);
    return h == 3 ? 0 : 1;
}
