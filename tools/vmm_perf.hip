// Diagnostic: streaming bandwidth of device memory from hipMalloc vs hipMemCreate/hipMemMap
// (VMM, as exported snapshot slots would use), same copy kernel, cold-ish (1.2 GB buffers).
//   hipcc -O3 --offload-arch=gfx950 tools/vmm_perf.hip -o tools/vmm_perf && tools/vmm_perf
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 2;                                                                    \
        }                                                                                \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(u32x4 *__restrict__ d, const u32x4 *__restrict__ s, long n16)
{
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) d[i] = __builtin_nontemporal_load(s + i);
}

static int vmm_alloc(void **out, size_t bytes, size_t chunk, size_t align)
{
    hipMemAllocationProp p;
    std::memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    size_t total = (bytes + chunk - 1) / chunk * chunk;
    CK(hipMemAddressReserve(out, total, align, nullptr, 0));
    for (size_t off = 0; off < total; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, chunk, &p, 0));
        CK(hipMemMap((char *)*out + off, chunk, 0, h, 0));
    }
    hipMemAccessDesc a;
    std::memset(&a, 0, sizeof(a));
    a.location.type = hipMemLocationTypeDevice;
    a.location.id = 0;
    a.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(*out, total, &a, 1));
    return 0;
}

static double run(void *d, void *s, size_t bytes, int reps)
{
    long n16 = (long)(bytes / 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_copy, dim3((n16 + 255) / 256), dim3(256), 0, 0, (u32x4 *)d, (const u32x4 *)s, n16);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_copy, dim3((n16 + 255) / 256), dim3(256), 0, 0, (u32x4 *)d, (const u32x4 *)s, n16);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return 2.0 * bytes * reps / (ms * 1e-3) / 1e9;
}

int main()
{
    const size_t bytes = (size_t)1200 << 20;
    void *s = nullptr, *d = nullptr;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    std::printf("hipMalloc -> hipMalloc          %.0f GB/s\n", run(d, s, bytes, 20));
    const size_t G = 1ull << 30, M2 = 2ull << 20;
    struct Cfg { const char *name; size_t chunk, align; } cfgs[] = {
        {"VMM 1 GiB chunks, 2 MiB aligned", G, M2}, {"VMM 1 GiB chunks, 1 GiB aligned", G, G},
        {"VMM 2 MiB chunks, 2 MiB aligned", M2, M2}, {"VMM 256 MiB chunks, 4 KiB aligned", 256ull << 20, 4096}};
    for (auto &c : cfgs) {
        void *vs = nullptr, *vd = nullptr;
        if (vmm_alloc(&vs, bytes, c.chunk, c.align) || vmm_alloc(&vd, bytes, c.chunk, c.align)) return 3;
        CK(hipMemset(vs, 1, bytes));
        std::printf("%-32s %.0f GB/s   (hipMalloc src -> VMM dst %.0f, VMM src -> hipMalloc dst %.0f)\n", c.name,
                    run(vd, vs, bytes, 20), run(vd, s, bytes, 20), run(d, vs, bytes, 20));
    }
    return 0;
}
