// Which HIP call of the round-4 fence sequence crashes (tools only, never
// part of libsdsp.so).  Each scenario runs in a forked child (the parent never touches
// HIP), prints a marker before every call and reports how the child ended, so a crash
// names the call.  The round-4 sequence (AutoCorrelator block queued on torch's default
// stream, passed to the C ABI as hipStreamLegacy; then get_energy on the handle's own
// stream) is scenario "legacy->stream".
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/fence_probe tools/fence_probe.hip
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define STEP(call)                                                      \
    do {                                                                \
        std::printf("    %s ... ", #call);                              \
        std::fflush(stdout);                                            \
        hipError_t e_ = (call);                                         \
        std::printf("%s\n", hipGetErrorString(e_));                     \
        std::fflush(stdout);                                            \
        if (e_ != hipSuccess) return 2;                                 \
    } while (0)

__global__ void touch(float* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

// rec: the stream the marker is recorded on; wt: the stream that waits on it; then a
// pageable D2H copy and a synchronize on `wt` (get_energy's sequence)
static int scenario(const char* rec_name, const char* wt_name, int reps) {
    hipStream_t own;
    STEP(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
    hipStream_t other;
    STEP(hipStreamCreateWithFlags(&other, hipStreamNonBlocking));
    auto named = [&](const char* s) -> hipStream_t {
        if (!std::strcmp(s, "legacy")) return hipStreamLegacy;
        if (!std::strcmp(s, "null")) return nullptr;
        if (!std::strcmp(s, "other")) return other;
        return own;
    };
    hipStream_t rec = named(rec_name), wt = named(wt_name);
    const int n = 1 << 20;
    float* d;
    STEP(hipMalloc(&d, n * sizeof(float)));
    STEP(hipMemset(d, 0, n * sizeof(float)));
    std::vector<double> host(3);
    hipEvent_t ev;
    STEP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int r = 0; r < reps; ++r) {
        std::printf("  rep %d\n", r);
        hipLaunchKernelGGL(touch, dim3(n / 256), dim3(256), 0, rec, d, n);
        STEP(hipGetLastError());
        STEP(hipEventRecord(ev, rec));
        STEP(hipDeviceSynchronize());  // the test synchronised before get_energy
        STEP(hipStreamWaitEvent(wt, ev, 0));
        STEP(hipMemcpyAsync(host.data(), d, 24, hipMemcpyDeviceToHost, wt));
        STEP(hipStreamSynchronize(wt));
    }
    STEP(hipEventDestroy(ev));
    STEP(hipFree(d));
    return 0;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    const char* cases[][2] = {{"own", "other"}, {"legacy", "own"}, {"null", "own"}, {"own", "legacy"},
                              {"own", "null"}, {"legacy", "legacy"}, {"null", "legacy"}, {"null", "null"}};
    int worst = 0;
    for (auto& c : cases) {
        std::printf("scenario %s->%s\n", c[0], c[1]);
        std::fflush(stdout);
        pid_t pid = fork();
        if (pid == 0) std::_Exit(scenario(c[0], c[1], reps));
        int st = 0;
        waitpid(pid, &st, 0);
        if (WIFSIGNALED(st)) {
            std::printf("RESULT %s->%s: killed by signal %d\n", c[0], c[1], WTERMSIG(st));
            worst = 1;
        } else {
            std::printf("RESULT %s->%s: exit %d\n", c[0], c[1], WEXITSTATUS(st));
            if (WEXITSTATUS(st)) worst = 1;
        }
        std::fflush(stdout);
    }
    std::printf("fence_probe: %s\n", worst ? "at least one scenario failed (see RESULT lines)" : "all scenarios ran");
    return 0;  // a report: the RESULT lines say which scenario ended how
}
