// ipc_reopen.hip -- which HIP IPC export/import pattern fails on this stack (development probe,
// VERDICT r3 "what's weak" 3: hipIpcOpenMemHandle "invalid device pointer" in 2 of 3 runs of the
// first, per-collective IpcComm).  Two processes on one GPU, forked before any HIP call; a
// MAP_SHARED page carries the handles and a step counter.  Per mode, ITERS rounds of: the
// exporter publishes a handle, the importer opens it, copies 1 MiB out of it, checks the bytes,
// closes it; then the exporter may free.  Modes:
//   same      one allocation, re-exported every round (hipIpcGetMemHandle on the same base),
//             imported / closed every round -- the first IpcComm's pattern
//   samehdl   one allocation exported once, the same handle bytes imported / closed every round
//   fresh     a new allocation every round, freed after the importer closed it (VA reuse)
//   keep      a new allocation every round, kept until the end (today's IpcComm on regrowth:
//             each allocation exported once, the importer closes the old one and opens the new)
//   nofree    as same, but the importer never closes between rounds (opens again on an open one)
// Prints, per mode, the rounds that failed and the first error.
//   build: hipcc --offload-arch=gfx950 -O2 -o tools/experiments/ipc_reopen.bin tools/experiments/ipc_reopen.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <vector>

constexpr int kIters = 200;
constexpr size_t kBytes = size_t(1) << 20, kAlloc = size_t(8) << 20;

struct Shared {
    std::atomic<int> step;  // even: exporter's turn, odd: importer's
    std::atomic<int> fails, ok;
    hipIpcMemHandle_t h;
    uint32_t tag;
    char first_err[256];
};

static void wait_step(Shared *s, int v) {
    while (s->step.load(std::memory_order_acquire) != v) usleep(10);
}

__global__ void fill(uint32_t *p, size_t n, uint32_t tag) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        p[i] = tag ^ (uint32_t)i;
}

static void exporter(Shared *s, const char *mode) {
    std::vector<void *> keep;
    void *one = nullptr;
    const bool single = !strcmp(mode, "same") || !strcmp(mode, "samehdl") || !strcmp(mode, "nofree");
    if (single) hipMalloc(&one, kAlloc);
    for (int it = 0; it < kIters; ++it) {
        wait_step(s, 2 * it);
        void *p = one;
        if (!single) hipMalloc(&p, kAlloc);
        const uint32_t tag = 0x1234567u * (it + 1);
        fill<<<256, 256>>>((uint32_t *)p, kBytes / 4, tag);
        hipDeviceSynchronize();
        if (!(it > 0 && !strcmp(mode, "samehdl"))) hipIpcGetMemHandle(&s->h, p);
        s->tag = tag;
        s->step.store(2 * it + 1, std::memory_order_release);
        wait_step(s, 2 * it + 2);
        if (!strcmp(mode, "fresh")) hipFree(p);
        if (!strcmp(mode, "keep")) keep.push_back(p);
    }
    for (void *p : keep) hipFree(p);
    if (one) hipFree(one);
}

static void importer(Shared *s, const char *mode) {
    std::vector<uint32_t> host(kBytes / 4);
    void *dst = nullptr;
    hipMalloc(&dst, kBytes);
    void *prev = nullptr;
    for (int it = 0; it < kIters; ++it) {
        wait_step(s, 2 * it + 1);
        void *p = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&p, s->h, hipIpcMemLazyEnablePeerAccess);
        bool good = e == hipSuccess;
        if (good) {
            e = hipMemcpy(dst, p, kBytes, hipMemcpyDeviceToDevice);
            if (e == hipSuccess) e = hipMemcpy(host.data(), dst, kBytes, hipMemcpyDeviceToHost);
            good = e == hipSuccess;
            for (size_t i = 0; good && i < host.size(); i += 4099) good = host[i] == (s->tag ^ (uint32_t)i);
            if (e == hipSuccess && !good) e = hipErrorUnknown;  // wrong bytes
        }
        if (good) {
            s->ok++;
        } else if (s->fails++ == 0) {
            snprintf(s->first_err, sizeof s->first_err, "round %d: %s", it, hipGetErrorString(e));
        }
        if (p) {
            if (!strcmp(mode, "nofree")) {
                prev = p;  // left open
            } else {
                hipIpcCloseMemHandle(p);
            }
        }
        s->step.store(2 * it + 2, std::memory_order_release);
    }
    (void)prev;
    hipFree(dst);
}

int main(int argc, char **argv) {
    const char *modes[] = {"same", "samehdl", "fresh", "keep", "nofree"};
    for (const char *mode : modes) {
        if (argc > 1 && strcmp(argv[1], mode)) continue;
        Shared *s = (Shared *)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE,
                                   MAP_SHARED | MAP_ANONYMOUS, -1, 0);
        new (s) Shared();
        // the parent never touches HIP: both sides are fresh children
        const pid_t pe = fork();
        if (pe == 0) {
            exporter(s, mode);
            _exit(0);
        }
        const pid_t pi = fork();
        if (pi == 0) {
            importer(s, mode);
            _exit(0);
        }
        int st = 0, st2 = 0;
        waitpid(pi, &st, 0);
        waitpid(pe, &st2, 0);
        printf("%-8s ok %3d fail %3d  child exit %d  %s\n", mode, s->ok.load(), s->fails.load(),
               WIFEXITED(st) ? WEXITSTATUS(st) : -1, s->first_err);
        fflush(stdout);
        munmap(s, sizeof(Shared));
    }
    return 0;
}
