// ipc_group.hip -- the first IpcComm's export / import pattern with P processes on one GPU
// (development probe; ipc_reopen.hip found no failure with two processes).  Every round, every
// rank exports a pointer inside its send allocation (hipMemGetAddressRange base, as that
// IpcComm did), publishes handle + offset in a MAP_SHARED page, meets the others at a barrier,
// opens every peer's handle, copies 256 KiB out of each, checks the bytes, closes them, meets
// them again.  Modes (argv[2]):
//   reexport  one send allocation per rank, re-exported every round (the first IpcComm)
//   grow      the send allocation is freed and allocated larger every 8th round, then
//             re-exported (ensure() growing a scratch buffer between collectives)
//   fresh     freed and allocated again at the same size every 8th round, re-exported
//   keepgrow  a larger allocation every 8th round, the old one kept (never freed while the
//             group lives: today's IpcComm staging), re-exported
//   once      one allocation exported once, every peer opens it once and keeps it (today's)
// usage: ipc_group.bin P mode [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <vector>

constexpr size_t kChunk = size_t(256) << 10;
constexpr int kMax = 16;

struct Slot {
    hipIpcMemHandle_t h;
    uint64_t off;
    uint32_t tag;
};
struct Shared {
    std::atomic<int> arrived, gen, fails, ok;
    Slot slot[kMax];
    char first_err[kMax][200];
};

static void barrier(Shared *s, int P) {
    const int g = s->gen.load();
    if (s->arrived.fetch_add(1) + 1 == P) {
        s->arrived.store(0);
        s->gen.fetch_add(1);
        return;
    }
    while (s->gen.load() == g) usleep(5);
}

__global__ void fill(uint32_t *p, size_t n, uint32_t tag) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        p[i] = tag ^ (uint32_t)i;
}

static void rank_main(Shared *s, int P, int me, const char *mode, int rounds) {
    hipSetDevice(0);
    size_t cap = size_t(4) << 20;
    char *buf = nullptr;
    hipMalloc((void **)&buf, cap);
    std::vector<void *> open_peer(P, nullptr), kept;
    void *dst = nullptr;
    hipMalloc(&dst, kChunk);
    std::vector<uint32_t> host(kChunk / 4);
    const bool once = !strcmp(mode, "once");
    for (int it = 0; it < rounds; ++it) {
        if (it % 8 == 7 && (!strcmp(mode, "grow") || !strcmp(mode, "fresh") ||
                            !strcmp(mode, "keepgrow"))) {
            if (!strcmp(mode, "keepgrow")) kept.push_back(buf);
            else hipFree(buf);
            if (strcmp(mode, "fresh")) cap += size_t(1) << 20;
            hipMalloc((void **)&buf, cap);
        }
        const uint64_t off = (uint64_t)((it * 4096 + me * 65536) % (cap - kChunk)) & ~4095ull;
        const uint32_t tag = 0x9E3779B9u * (uint32_t)(it * kMax + me + 1);
        fill<<<128, 256>>>((uint32_t *)(buf + off), kChunk / 4, tag);
        hipDeviceSynchronize();
        if (!once || it == 0) {
            void *base = nullptr;
            size_t len = 0;
            hipMemGetAddressRange(&base, &len, buf + off);
            hipIpcGetMemHandle(&s->slot[me].h, base);
            s->slot[me].off = (uint64_t)(buf + off - (char *)base);
        } else {
            s->slot[me].off = off;
        }
        s->slot[me].tag = tag;
        barrier(s, P);
        for (int q = 0; q < P; ++q) {
            if (q == me) continue;
            hipError_t e = hipSuccess;
            if (!open_peer[q]) e = hipIpcOpenMemHandle(&open_peer[q], s->slot[q].h,
                                                       hipIpcMemLazyEnablePeerAccess);
            bool good = e == hipSuccess;
            if (good) {
                e = hipMemcpy(dst, (char *)open_peer[q] + s->slot[q].off, kChunk,
                              hipMemcpyDeviceToDevice);
                if (e == hipSuccess) e = hipMemcpy(host.data(), dst, kChunk, hipMemcpyDeviceToHost);
                good = e == hipSuccess;
                for (size_t i = 0; good && i < host.size(); i += 1021)
                    good = host[i] == (s->slot[q].tag ^ (uint32_t)i);
                if (e == hipSuccess && !good) e = hipErrorUnknown;
            }
            if (good) s->ok++;
            else if (s->fails++ < kMax && !s->first_err[me][0])
                snprintf(s->first_err[me], 200, "rank %d round %d peer %d: %s", me, it, q,
                         hipGetErrorString(e));
        }
        hipDeviceSynchronize();
        if (!once)
            for (int q = 0; q < P; ++q)
                if (open_peer[q]) { hipIpcCloseMemHandle(open_peer[q]); open_peer[q] = nullptr; }
        barrier(s, P);
    }
    for (int q = 0; q < P; ++q)
        if (open_peer[q]) hipIpcCloseMemHandle(open_peer[q]);
    barrier(s, P);
    hipFree(buf);
    for (void *k : kept) hipFree(k);
    hipFree(dst);
}

int main(int argc, char **argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 4;
    const char *mode = argc > 2 ? argv[2] : "reexport";
    const int rounds = argc > 3 ? atoi(argv[3]) : 200;
    if (P < 2 || P > kMax) return 2;
    Shared *s = (Shared *)mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE,
                               MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    new (s) Shared();
    std::vector<pid_t> pids;
    for (int r = 0; r < P; ++r) {  // the parent never touches HIP
        const pid_t pid = fork();
        if (pid == 0) {
            rank_main(s, P, r, mode, rounds);
            _exit(0);
        }
        pids.push_back(pid);
    }
    int bad_exit = 0;
    for (pid_t pid : pids) {
        int st = 0;
        waitpid(pid, &st, 0);
        bad_exit += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    }
    printf("P=%d %-9s rounds %d: ok %d fail %d bad_exit %d\n", P, mode, rounds, s->ok.load(),
           s->fails.load(), bad_exit);
    for (int r = 0; r < P; ++r)
        if (s->first_err[r][0]) printf("  %s\n", s->first_err[r]);
    return 0;
}
