// Diagnostic: share a multi-GiB device buffer between two processes with HIP's virtual memory
// API instead of hipIpcOpenMemHandle (which hangs above ~2 GiB on this image).  The buffer
// is hipMemCreate'd in chunks, mapped contiguously in the exporter; each chunk is exported as
// a POSIX fd and passed over a Unix socket (SCM_RIGHTS; pidfd_getfd is not permitted between
// sibling processes here); the importer maps them contiguously and reads both sides of every
// chunk boundary.  fork() happens before any HIP call.
//   hipcc -O2 tools/vmm_probe.cpp -o tools/vmm_probe && tools/vmm_probe 6 1
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "[%s] %s:%d %s: %s\n", who, __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                       \
        }                                                                                       \
    } while (0)

static const char *who = "?";

static hipMemAllocationProp prop_for(int dev)
{
    hipMemAllocationProp p;
    std::memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}

int main(int argc, char **argv)
{
    const double gib = argc > 1 ? std::atof(argv[1]) : 6.0;
    const double chunk_gib = argc > 2 ? std::atof(argv[2]) : 1.0;
    const bool by_ptr = argc > 3 && std::strcmp(argv[3], "ptr") == 0;
    int rt = 0;
    (void)hipRuntimeGetVersion;   // printed by the exporter below
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 3;
    const pid_t child = fork();
    if (child != 0) {   // ------------------------------------------------ exporter
        who = "exporter";
        close(sv[0]);
        hipMemAllocationProp prop = prop_for(0);
        size_t gran = 0;
        CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
        size_t chunk = ((size_t)(chunk_gib * (1ull << 30)) + gran - 1) / gran * gran;
        size_t total = ((size_t)(gib * (1ull << 30)) + chunk - 1) / chunk * chunk;
        const int k = (int)(total / chunk);
        void *base = nullptr;
        CK(hipMemAddressReserve(&base, total, gran, nullptr, 0));
        std::vector<hipMemGenericAllocationHandle_t> h((size_t)k);
        std::vector<int> fds((size_t)k);
        hipMemAccessDesc acc;
        std::memset(&acc, 0, sizeof(acc));
        acc.location.type = hipMemLocationTypeDevice;
        acc.location.id = 0;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        for (int i = 0; i < k; ++i) {
            CK(hipMemCreate(&h[i], chunk, &prop, 0));
            CK(hipMemMap((char *)base + (size_t)i * chunk, chunk, 0, h[i], 0));
            CK(hipMemExportToShareableHandle(&fds[i], h[i], hipMemHandleTypePosixFileDescriptor, 0));
        }
        CK(hipMemSetAccess(base, total, &acc, 1));
        // pattern: each 4-byte word holds its own index (mod 2^32) -> hipMemsetD32 per chunk region
        for (int i = 0; i < k; ++i)
            CK(hipMemsetD32((hipDeviceptr_t)((char *)base + (size_t)i * chunk), 0x11111111u * (unsigned)(i + 1),
                            chunk / 4));
        CK(hipDeviceSynchronize());
        CK(hipRuntimeGetVersion(&rt));
        std::printf("[exporter] HIP runtime %d; %d chunks of %zu bytes (granularity %zu), total %zu\n", rt, k, chunk,
                    gran, total);
        std::fflush(stdout);
        long msg[3] = {(long)getpid(), (long)k, (long)chunk};
        for (int i = 0; i < k; ++i) {   // one message per chunk: the header words + its fd
            struct iovec io = {msg, sizeof(msg)};
            char cbuf[CMSG_SPACE(sizeof(int))];
            std::memset(cbuf, 0, sizeof(cbuf));
            struct msghdr mh;
            std::memset(&mh, 0, sizeof(mh));
            mh.msg_iov = &io;
            mh.msg_iovlen = 1;
            mh.msg_control = cbuf;
            mh.msg_controllen = sizeof(cbuf);
            struct cmsghdr *c = CMSG_FIRSTHDR(&mh);
            c->cmsg_level = SOL_SOCKET;
            c->cmsg_type = SCM_RIGHTS;
            c->cmsg_len = CMSG_LEN(sizeof(int));
            std::memcpy(CMSG_DATA(c), &fds[i], sizeof(int));
            if (sendmsg(sv[1], &mh, 0) != (ssize_t)sizeof(msg)) return 4;
        }
        int status = 0;
        waitpid(child, &status, 0);
        CK(hipMemUnmap(base, total));
        for (auto x : h) CK(hipMemRelease(x));
        CK(hipMemAddressFree(base, total));
        std::printf("[exporter] importer exited %d\n", WIFEXITED(status) ? WEXITSTATUS(status) : -1);
        return WIFEXITED(status) ? WEXITSTATUS(status) : 5;
    }
    // ---------------------------------------------------------------- importer
    who = "importer";
    close(sv[1]);
    long msg[3];
    std::vector<int> rfds;
    do {
        struct iovec io = {msg, sizeof(msg)};
        char cbuf[CMSG_SPACE(sizeof(int))];
        struct msghdr mh;
        std::memset(&mh, 0, sizeof(mh));
        mh.msg_iov = &io;
        mh.msg_iovlen = 1;
        mh.msg_control = cbuf;
        mh.msg_controllen = sizeof(cbuf);
        if (recvmsg(sv[0], &mh, MSG_WAITALL) != (ssize_t)sizeof(msg)) return 6;
        struct cmsghdr *c = CMSG_FIRSTHDR(&mh);
        if (!c || c->cmsg_type != SCM_RIGHTS) return 7;
        int fd;
        std::memcpy(&fd, CMSG_DATA(c), sizeof(int));
        rfds.push_back(fd);
    } while ((long)rfds.size() < msg[1]);
    const int k = (int)msg[1];
    const size_t chunk = (size_t)msg[2];
    const size_t total = chunk * (size_t)k;
    void *base = nullptr;
    CK(hipMemAddressReserve(&base, total, 0, nullptr, 0));
    std::vector<hipMemGenericAllocationHandle_t> h((size_t)k);
    for (int i = 0; i < k; ++i) {
        const int fd = rfds[i];
        int fd_copy = fd;   // "ptr" mode: pass the fd's address (older runtimes read *osHandle)
        CK(hipMemImportFromShareableHandle(&h[i], by_ptr ? (void *)&fd_copy : (void *)(intptr_t)fd,
                                           hipMemHandleTypePosixFileDescriptor));
        CK(hipMemMap((char *)base + (size_t)i * chunk, chunk, 0, h[i], 0));
        close(fd);
        std::printf("[importer] chunk %d mapped\n", i);
        std::fflush(stdout);
    }
    hipMemAccessDesc acc;
    std::memset(&acc, 0, sizeof(acc));
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = 0;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(base, total, &acc, 1));
    // read 64 bytes across every chunk boundary through one contiguous device-to-device copy
    void *local = nullptr;
    CK(hipMalloc(&local, 64));
    int bad = 0;
    for (int i = 1; i < k; ++i) {
        CK(hipMemcpy(local, (char *)base + (size_t)i * chunk - 32, 64, hipMemcpyDeviceToDevice));
        unsigned w[16];
        CK(hipMemcpy(w, local, 64, hipMemcpyDeviceToHost));
        for (int j = 0; j < 16; ++j) {
            const unsigned want = 0x11111111u * (unsigned)((j < 8 ? i - 1 : i) + 1);
            bad += w[j] != want;
        }
    }
    std::printf("[importer] %d chunk boundaries checked, %d bad words\n", k - 1, bad);
    CK(hipMemUnmap(base, total));
    for (auto x : h) CK(hipMemRelease(x));
    CK(hipMemAddressFree(base, total));
    return bad ? 9 : 0;
}
