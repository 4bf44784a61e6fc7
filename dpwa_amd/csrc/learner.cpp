// learner.cpp -- the per-node runtime behind DpwaConnection (dpwa/dpwa.py:54-156) on MI355X.
//
// The reference keeps, per node, an RxThread that serves the latest (state, payload)
// under a lock (conn.py:51-172) and a TxThread that fetches one peer's (state, payload)
// over TCP (conn.py:197-334).  Here a node (learner) owns, on its GPU:
//   slots    two snapshot slots [header 256 B | pad to 4 KiB | payload] -- RxThread.state/payload,
//            double-buffered so a publish never overwrites the slot a peer may be reading
//   staging  one slot-sized buffer receiving a peer's snapshot -- TxThread.peer_payload
//   ctl      the device clock and the averaging coefficients (dpwa_coef)
// and a side stream on which fetches (xGMI pulls for peers on other GPUs) overlap the
// training step.  Nothing here synchronises the host with the device except the explicit
// read/write helpers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <set>
#include <unistd.h>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace {

thread_local std::string g_last_error;

}  // namespace

namespace dpwa {

int set_error(int code, const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace dpwa

using namespace dpwa;

namespace {

constexpr size_t kHeader = sizeof(dpwa_header);
constexpr size_t kPayloadOff = DPWA_SLOT_PAYLOAD_OFFSET;   // [header | pad | payload]
static_assert(kPayloadOff >= kHeader && kPayloadOff % 1024 == 0, "payload offset");
static_assert(sizeof(dpwa_header) == 256, "dpwa_header must be 256 bytes");
constexpr uint64_t kIpcMagic = 0x445057414950430aULL;  // "DPWAIPC\n"

struct IpcBlob {
    hipIpcMemHandle_t handle;   // 64 B
    uint64_t magic;
    int64_t slot_stride;
    int64_t n;
    int32_t dtype;
    int32_t device;
    int32_t pid;
    int32_t vmm;                // 1: the allocation is shared as fds (dpwa_learner_export_fds)
};
static_assert(sizeof(IpcBlob) <= DPWA_IPC_HANDLE_BYTES, "IPC blob too large");

// An exportable device allocation (snapshot slots, relay buffer).  Ordinary allocations come
// from hipMalloc and are shared with hipIpcGetMemHandle / hipIpcOpenMemHandle.  On this ROCm
// stack hipIpcOpenMemHandle never returns for allocations above ~2 GiB (tools/ipc_size_probe.py),
// so allocations from kVmmMinBytes up (or any size with DPWA_VMM=1) are built from hipMemCreate
// chunks mapped contiguously, and shared as one POSIX fd per chunk (hipMemExportToShareableHandle)
// that the peer maps contiguously again (tools/vmm_probe.cpp; streaming rates equal hipMalloc's,
// tools/vmm_perf.hip).
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr size_t kVmmMinBytes = (size_t)3 << 29;     // 1.5 GiB
constexpr size_t kVmmChunk = (size_t)1 << 30;        // 1 GiB per exported chunk
constexpr size_t kVmmAlign = (size_t)2 << 20;

struct DevMem {
    char *ptr = nullptr;
    size_t bytes = 0;                                   // mapped bytes (VMM: chunk multiple)
    size_t chunk = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles;   // VMM chunks; empty: hipMalloc
    bool vmm() const { return !handles.empty(); }
};

hipMemAllocationProp vmm_prop(int device)
{
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = device;
    return p;
}

hipError_t vmm_grant(const DevMem &m, int device)
{
    hipMemAccessDesc a;
    memset(&a, 0, sizeof(a));
    a.location.type = hipMemLocationTypeDevice;
    a.location.id = device;
    a.flags = hipMemAccessFlagsProtReadWrite;
    return hipMemSetAccess(m.ptr, m.bytes, &a, 1);
}

void devmem_free(DevMem &m)
{
    if (!m.ptr) return;
    if (m.vmm()) {
        (void)hipMemUnmap(m.ptr, m.bytes);
        for (auto h : m.handles) (void)hipMemRelease(h);
        (void)hipMemAddressFree(m.ptr, m.bytes);
    } else {
        (void)hipFree(m.ptr);
    }
    m = DevMem();
}

// Maps `n` chunks (VMM handles in h[]) contiguously into a fresh reservation, readable and
// writable from `device`; releases the handles on failure.
hipError_t vmm_map(DevMem &m, std::vector<hipMemGenericAllocationHandle_t> &h, size_t chunk, int device)
{
    m = DevMem();
    const size_t total = chunk * h.size();
    void *va = nullptr;
    hipError_t e = hipMemAddressReserve(&va, total, kVmmAlign, nullptr, 0);
    size_t mapped = 0;
    if (e == hipSuccess) {
        for (; mapped < h.size(); ++mapped)
            if ((e = hipMemMap((char *)va + mapped * chunk, chunk, 0, h[mapped], 0)) != hipSuccess) break;
    }
    m.ptr = (char *)va;
    m.bytes = total;
    m.chunk = chunk;
    if (e == hipSuccess) {
        m.handles = h;
        if ((e = vmm_grant(m, device)) == hipSuccess) return hipSuccess;
    }
    if (va) {
        if (mapped) (void)hipMemUnmap(va, mapped * chunk);
        (void)hipMemAddressFree(va, total);
    }
    for (auto x : h) (void)hipMemRelease(x);
    h.clear();
    m = DevMem();
    return e;
}

bool use_vmm(size_t bytes)
{
    const char *e = getenv("DPWA_VMM");
    if (e && e[0] == '1') return true;
    if (e && e[0] == '0') return false;
    return bytes >= kVmmMinBytes;
}

hipError_t devmem_alloc(DevMem &m, size_t bytes, int device)
{
    m = DevMem();
    if (!use_vmm(bytes)) {
        hipError_t e = hipMalloc(&m.ptr, bytes);
        if (e == hipSuccess) m.bytes = bytes;
        return e;
    }
    const hipMemAllocationProp prop = vmm_prop(device);
    size_t gran = 0;
    hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
    if (e != hipSuccess) return e;
    const size_t unit = std::max(gran, kVmmAlign);
    size_t chunk = std::min(kVmmChunk, round_up(bytes, unit));
    chunk = round_up(chunk, unit);
    const size_t n = (bytes + chunk - 1) / chunk;
    std::vector<hipMemGenericAllocationHandle_t> h;
    for (size_t i = 0; i < n; ++i) {
        hipMemGenericAllocationHandle_t x;
        if ((e = hipMemCreate(&x, chunk, &prop, 0)) != hipSuccess) {
            for (auto y : h) (void)hipMemRelease(y);
            return e;
        }
        h.push_back(x);
    }
    return vmm_map(m, h, chunk, device);
}

// One POSIX fd per chunk of a VMM allocation (the caller closes them).
int devmem_export(const DevMem &m, int *fds, int max_fds, int *n_fds, int64_t *chunk_bytes)
{
    *n_fds = 0;
    if (chunk_bytes) *chunk_bytes = (int64_t)m.chunk;
    if (!m.vmm()) return DPWA_OK;
    if ((int)m.handles.size() > max_fds)
        return set_error(DPWA_ERR_ARG, "export: %zu chunks, room for %d fds", m.handles.size(), max_fds);
    for (size_t i = 0; i < m.handles.size(); ++i) {
        int fd = -1;
        hipError_t e = hipMemExportToShareableHandle(&fd, m.handles[i], hipMemHandleTypePosixFileDescriptor, 0);
        if (e != hipSuccess) {
            for (int j = 0; j < (int)i; ++j) close(fds[j]);
            return set_error(DPWA_ERR_HIP, "hipMemExportToShareableHandle: %s", hipGetErrorString(e));
        }
        fds[i] = fd;
    }
    *n_fds = (int)m.handles.size();
    return DPWA_OK;
}

// Maps a peer's exported chunks (fds from devmem_export, received over a Unix socket) into
// this process, readable and writable from `device`.  The fds stay the caller's.
int devmem_import(DevMem &m, const int *fds, int n_fds, int64_t chunk, size_t need_bytes, int device)
{
    if (n_fds < 1 || chunk <= 0 || (size_t)chunk * (size_t)n_fds < need_bytes)
        return set_error(DPWA_ERR_ARG, "import: %d chunks of %lld bytes for %zu bytes", n_fds, (long long)chunk,
                         need_bytes);
    // How the fd is handed over depends on the runtime in the process (a torch process runs the
    // HIP runtime torch bundles): 7.0 reads the fd through the pointer (and faults on an fd
    // passed as the pointer value), 7.2 takes the fd as the pointer value (and rejects an
    // address as an invalid fd) -- tools/vmm_torch_probe.py, tools/vmm_probe.cpp.
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    const bool fd_by_value = rt >= 70200000;
    std::vector<hipMemGenericAllocationHandle_t> h;
    for (int i = 0; i < n_fds; ++i) {
        hipMemGenericAllocationHandle_t x;
        int fd = fds[i];
        hipError_t e = hipMemImportFromShareableHandle(&x, fd_by_value ? (void *)(intptr_t)fd : (void *)&fd,
                                                       hipMemHandleTypePosixFileDescriptor);
        if (e == hipErrorInvalidValue && fd_by_value)   // a runtime of the older convention
            e = hipMemImportFromShareableHandle(&x, (void *)&fd, hipMemHandleTypePosixFileDescriptor);
        if (e != hipSuccess) {
            for (auto y : h) (void)hipMemRelease(y);
            return set_error(DPWA_ERR_HIP, "hipMemImportFromShareableHandle: %s", hipGetErrorString(e));
        }
        h.push_back(x);
    }
    hipError_t e = vmm_map(m, h, (size_t)chunk, device);
    if (e != hipSuccess) return set_error(DPWA_ERR_HIP, "import: mapping the peer's chunks: %s", hipGetErrorString(e));
    return DPWA_OK;
}

struct Ctl {            // device control block
    double clock[4];    // a ring: a factor reads clock[cur] and writes clock[cur+1]; a
                        // write-through average also writes the next publish's clock+1 into
                        // clock[cur+2], which that publish then selects without a kernel
    dpwa_coef coef;
    int32_t guard_dirty;   // reuse guard: the generation (publish number) of the last publish that found
                           // the parameters changed (kernels.hip k_guard_publish)
    uint32_t guard_hits;   // ... and how many publishes did
    int32_t window_dirty;  // window guard (resident): the generation of the last window found written
    uint32_t window_hits;  // ... and how many windows were
};


// Registry of live learners, so a learner never dereferences a destroyed local peer.
std::mutex g_reg_mu;
std::set<dpwa_learner *> g_live;

class DeviceGuard {
public:
    explicit DeviceGuard(int dev)
    {
        (void)hipGetDevice(&prev_);
        if (prev_ != dev) (void)hipSetDevice(dev);
        dev_ = dev;
    }
    ~DeviceGuard()
    {
        if (prev_ != dev_) (void)hipSetDevice(prev_);
    }

private:
    int prev_ = 0, dev_ = 0;
};

}  // namespace

struct Endpoint {
    int kind = 0;                    // 1 local learner, 2 IPC-mapped
    dpwa_learner *local = nullptr;
    char *base = nullptr;            // slot 0 in this process's address space
    int device = -1;
    int64_t slot_stride = 0;
    int64_t n = 0;
    int32_t dtype = 0;
    DevMem imported;                 // kind 2 through fds (VMM); empty: hipIpc-opened `base`
};

static void close_endpoint(Endpoint &ep)
{
    if (ep.kind != 2 || !ep.base) return;
    if (ep.imported.vmm())
        devmem_free(ep.imported);
    else
        (void)hipIpcCloseMemHandle(ep.base);
    ep.base = nullptr;
}

// A rescue lane: where a fetch re-selected after a timed-out pull goes (conn.py:304-309) -- a
// buffer and a stream of the greatest priority (a hardware queue no stalled normal-priority stream
// shares), so no stalled pull ahead of it can hold it up.  Lanes are made at first use, up to
// kMaxRescueLanes, only while the device keeps kRescueReserve free beyond the new buffer and all
// lanes together stay within 1/kRescueShare of the device's memory (7B bf16: two 14 GB lanes on a
// 288 GB GPU); an allocation that fails caps the count where it is (rescue_cap) instead of failing
// the round.  Lanes beyond the first kKeepRescueLanes are given back once they have been idle for
// kLaneIdleRounds fetch rounds (trim_lanes), so a burst of stalled pulls does not hold HBM outside
// PyTorch's allocator for the rest of the process.
constexpr int kMaxRescueLanes = 8;
constexpr int kKeepRescueLanes = 2;
constexpr uint64_t kLaneIdleRounds = 8;
constexpr size_t kRescueShare = 8;
// fetch_state: a backlog on the caller's stream longer than this no longer defers the timeout (a
// stream that never reaches update_send is stuck, not slow); a probe waits at most kProbeWaitUs
constexpr int64_t kMaxBacklogMs = 60000;
constexpr int64_t kProbeWaitUs = 2000;
constexpr size_t kRescueReserve = (size_t)1 << 30;
struct RescueLane {
    char *buf = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_landed = nullptr;     // its last pull landed
    hipEvent_t ev_done = nullptr;       // the last reader of its buffer is done
    bool used = false;                  // a pull was issued into it
    bool read = false;                  // ev_done recorded
    uint64_t last_round = 0;            // fetch round of its last pull
};

void destroy_lane(RescueLane &r)
{
    if (r.buf) (void)hipFree(r.buf);
    if (r.stream) (void)hipStreamDestroy(r.stream);
    if (r.ev_landed) (void)hipEventDestroy(r.ev_landed);
    if (r.ev_done) (void)hipEventDestroy(r.ev_done);
    r = RescueLane();
}

struct dpwa_learner {
    int device = 0;
    int64_t n = 0;
    int32_t dtype = DPWA_F32;
    dpwa_interp cfg{};
    size_t payload_bytes = 0;
    size_t slot_stride = 0;
    char *slots = nullptr;          // 2 slots (= slot_mem.ptr)
    DevMem slot_mem;
    char *staging = nullptr;        // 1 slot
    Ctl *ctl = nullptr;
    uint64_t version = 0;
    int cur = 0;                        // index of the live clock in ctl->clock (mod 4)
    bool exported = false;
    hipStream_t side = nullptr;
    // Cross-stream ordering is recorded lazily: the stream of every publish / consumption is
    // remembered and an event is recorded (on that stream, at the moment a dependent
    // operation is enqueued) only when the dependent operation runs on a different stream.
    // In the common single-stream loop no event is recorded at all.
    hipEvent_t ev_published[2] = {nullptr, nullptr};
    hipStream_t publish_stream[2] = {nullptr, nullptr};
    bool published[2] = {false, false};
    hipEvent_t ev_issue = nullptr;      // fetch may start (recorded on the caller's stream)
    hipEvent_t ev_fetched = nullptr;    // fetch landed (recorded on the side stream)
    hipEvent_t ev_consumed = nullptr;   // this learner finished reading its fetch source
    hipStream_t consume_stream = nullptr;
    bool consumed_once = false;
    // Fetches of published snapshots (DPWA_FETCH_PUBLISHED: the gossip board) alternate between
    // two staging buffers and are not ordered after the caller's stream: each waits only for
    // the average that last read its buffer (ev_stage_done), so a pull starts at update_send
    // instead of after the caller's queued work, and a peer's read mark is released sooner.
    char *staging_alt = nullptr;        // second staging buffer, allocated at the first such fetch
    hipEvent_t ev_stage_done[2] = {nullptr, nullptr};
    bool stage_read[2] = {false, false};
    // rescue lanes (RescueLane), allocated at first use: a lane whose pull has not landed stays
    // taken and the next re-selected pull takes another, as TxThread keeps re-selecting
    RescueLane rescue[kMaxRescueLanes];
    int rescue_lanes = 0;
    int rescue_cap = kMaxRescueLanes;   // lowered when a lane's allocation fails
    uint64_t fetch_rounds = 0;          // first (non-rescue) pulls issued: the lanes' idle clock
    int64_t fetch_issue_ns = 0;         // host time the fetch in flight was issued (its timeout clock)
    // the fetch in flight waits for ev_issue (the caller's stream at update_send): its deadline runs
    // from when that point is reached, not from the host's enqueue (fetch_state)
    bool issue_evented = false;
    hipStream_t probe_stream = nullptr; // only ever holds ev_probe (fetch_state)
    hipEvent_t ev_probe = nullptr;
    hipStream_t fetch_stream = nullptr; // stream the fetch in flight moves its bytes on
    int stage_next = 0;
    int src_stage = -1;                 // buffer l->src points into: staging 0 / 1, rescue lane 2 + j; -1: none
    hipEvent_t ev_factor = nullptr;     // last factor computation done
    // write-through snapshot: the last average also wrote its result into the slot of the
    // next publish (for the flat buffer `wt_flat`, on stream `wt_stream`)
    int pull_mode = DPWA_PULL_COPY_ENGINE;   // how cross-device fetches move bytes
    int pull_blocks = 512;
    bool loss_f32 = false;              // device loss pointers point at a float32
    bool wt_valid = false;
    bool wt_header = false;             // the write-through average also wrote the next header
    bool header_on_publish = false;     // never write the next header ahead (served to wire peers)
    bool reuse_guard = false;           // check a header-only publish's parameters on the device
    // resident parameters (dpwa_learner_set_resident): they live in slot res_slot's payload and
    // move to the other slot at every average (or relocate)
    bool resident = false;
    int res_slot = 0;
    // window guard (resident, with reuse_guard): each publish checks the payload published last
    // time against the samples saved then and saves the new payload's (kernels.hip k_window_roll);
    // written windows are counted on the device and mirrored into a host-mapped word the next
    // publishes read without waiting
    char *window_sample = nullptr;      // kWindowSampleBytes, allocated at first use
    uint32_t *window_host = nullptr;    // mapped pinned: windows found written (device-written)
    uint32_t *window_host_dev = nullptr;
    const char *window_src = nullptr;   // payload the samples were taken from (NULL: none)
    hipStream_t window_stream = nullptr;    // stream of the last roll
    hipEvent_t ev_window = nullptr;     // orders a roll after the last one on another stream
    int32_t window_gen = 0;
    uint32_t window_reported = 0;
    const void *wt_flat = nullptr;
    hipStream_t wt_stream = nullptr;
    hipEvent_t ev_wt = nullptr;
    // timing of the averaging launches (bench): kernel begin/end events, filled in order
    std::vector<LaunchTiming> timing;
    int timing_used = 0;
    bool timing_armed = false;   // time the next averaging launch (one-shot)
    // timing of copying fetches (bench at N > 1: the pull over xGMI), filled in order
    std::vector<LaunchTiming> fetch_timing;
    int fetch_timing_used = 0;
    // relay transport (multi-link lock-step pulls), see kernels.hip
    bool relay_on = false;
    int relay_world = 0, relay_rank = 0;
    int64_t relay_stripe = 0;
    char *relay_buf = nullptr;               // world x stripe, IPC-exported (= relay_mem.ptr)
    DevMem relay_mem;
    std::vector<const char *> relay_slots;   // per rank: slot 0 base (own or IPC-mapped)
    std::vector<const char *> relay_bufs;    // per rank: relay buffer (own or IPC-mapped)
    std::vector<char *> relay_opened;        // IPC mappings to close
    std::vector<DevMem> relay_imported;      // fd-imported relay buffers to unmap
    hipEvent_t ev_relay = nullptr;           // all relay work of the last round
    bool relay_pending = false;
    // phase 2 deferred into the average (dpwa_learner_relay_phase2 with fuse != 0): the stripes
    // are read where phase 1 left them by the next fused average, or gathered into staging
    // first if the fetch is consumed any other way (relay_materialize)
    bool relay_deferred = false;
    RelayArgs relay_saved{};
    int relay_saved_pick = -1, relay_saved_blocks = 0;
    // host readers of published slots (wire bridge) run on other threads; their stream is created
    // at the first read, under pub_mu
    std::mutex pub_mu;
    hipStream_t read_stream = nullptr;
    hipEvent_t ev_read = nullptr;
    // fetch state
    const char *src = nullptr;          // header of the snapshot to average with
    bool src_copied = false;
    bool have_fetch = false;
    bool have_factor = false;
    dpwa_learner *src_owner = nullptr;  // local peer whose slot is being read (reader tracking)
    int src_slot = -1;
    std::unordered_map<int, Endpoint> peers;
    // learners (local) that read our slot k and must be waited for before rewriting it
    std::mutex readers_mu;
    std::vector<dpwa_learner *> readers[2];
    int32_t *host_status = nullptr;     // pinned mirror of coef.status for non-blocking polls
    int32_t *host_status_dev = nullptr; // its device-side address
};

static char *slot_payload(const dpwa_learner *l, int k)
{
    return l->slots + (size_t)k * l->slot_stride + kPayloadOff;
}

static int64_t now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static bool is_live(dpwa_learner *l)
{
    std::lock_guard<std::mutex> g(g_reg_mu);
    return g_live.count(l) != 0;
}

extern "C" {

const char *dpwa_last_error(void) { return g_last_error.c_str(); }

int dpwa_abi_version(void) { return DPWA_ABI_VERSION; }

int dpwa_lerp_f32(float *param, const float *peer, int64_t n, const dpwa_coef *coef_dev, dpwa_stream_t stream)
{
    if (n < 0 || (n > 0 && (!param || !peer || !coef_dev))) return set_error(DPWA_ERR_ARG, "dpwa_lerp_f32: bad arguments");
    HIP_TRY(launch_lerp(DPWA_F32, param, peer, n, coef_dev, 0.f, 0.f, (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_lerp_bf16(uint16_t *param, const uint16_t *peer, int64_t n, const dpwa_coef *coef_dev,
                   dpwa_stream_t stream)
{
    if (n < 0 || (n > 0 && (!param || !peer || !coef_dev))) return set_error(DPWA_ERR_ARG, "dpwa_lerp_bf16: bad arguments");
    HIP_TRY(launch_lerp(DPWA_BF16, param, peer, n, coef_dev, 0.f, 0.f, (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_lerp_f32_host(float *param, const float *peer, int64_t n, double factor, dpwa_stream_t stream)
{
    if (n < 0 || (n > 0 && (!param || !peer))) return set_error(DPWA_ERR_ARG, "dpwa_lerp_f32_host: bad arguments");
    HIP_TRY(launch_lerp(DPWA_F32, param, peer, n, nullptr, (float)factor, (float)(1.0 - factor), (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_lerp_bf16_host(uint16_t *param, const uint16_t *peer, int64_t n, double factor, dpwa_stream_t stream)
{
    if (n < 0 || (n > 0 && (!param || !peer))) return set_error(DPWA_ERR_ARG, "dpwa_lerp_bf16_host: bad arguments");
    HIP_TRY(launch_lerp(DPWA_BF16, param, peer, n, nullptr, (float)factor, (float)(1.0 - factor), (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_factor(const dpwa_interp *cfg, double *clock_dev, const dpwa_header *peer_header_dev, double loss,
                const double *loss_dev, dpwa_coef *coef_dev, dpwa_stream_t stream)
{
    if (!cfg || !clock_dev || !peer_header_dev || !coef_dev) return set_error(DPWA_ERR_ARG, "dpwa_factor: NULL argument");
    if (cfg->method < 0 || cfg->method > 2) return set_error(DPWA_ERR_ARG, "dpwa_factor: unknown method %d", cfg->method);
    FusedArgs fa{};
    fa.cfg = *cfg;
    fa.clock_in = clock_dev;
    fa.clock_out = clock_dev;
    fa.hdr = peer_header_dev;
    fa.loss_h = loss;
    fa.loss_d = loss_dev;
    fa.coef_out = coef_dev;
    HIP_TRY(launch_factor(fa, (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_average(int32_t dtype, void *param, const void *peer_slot, int64_t n, const dpwa_interp *cfg,
                 double *clock_dev, double loss, dpwa_coef *coef_dev, void *snap_payload, dpwa_stream_t stream,
                 void *start_event, void *stop_event)
{
    if (!cfg || !clock_dev || !coef_dev || !peer_slot || n < 0 || (n > 0 && !param) || dtype_size(dtype) == 0 ||
        (!start_event) != (!stop_event))
        return set_error(DPWA_ERR_ARG, "dpwa_average: bad arguments");
    if (cfg->method < 0 || cfg->method > 2) return set_error(DPWA_ERR_ARG, "dpwa_average: unknown method %d", cfg->method);
    FusedArgs fa{};
    fa.cfg = *cfg;
    fa.clock_in = clock_dev;
    fa.clock_out = clock_dev + 1;
    fa.hdr = (const dpwa_header *)peer_slot;
    fa.loss_h = loss;
    fa.coef_out = coef_dev;
    LaunchTiming t{(hipEvent_t)start_event, (hipEvent_t)stop_event};
    HIP_TRY(launch_average(dtype, param, (const char *)peer_slot + kPayloadOff, n, fa, snap_payload, (hipStream_t)stream,
                           start_event ? &t : nullptr));
    return DPWA_OK;
}

int dpwa_stream_mix(void *const *dst, int nw, const void *const *src, int nr, int64_t nbytes, dpwa_stream_t stream,
                    void *start_event, void *stop_event)
{
    if (!dst || !src || nr < 1 || nr > 2 || nw < 1 || nw > 2 || nbytes < 0 || (nbytes & 15) ||
        (!start_event) != (!stop_event))
        return set_error(DPWA_ERR_ARG, "dpwa_stream_mix: bad arguments");
    StreamMixArgs a{};
    for (int i = 0; i < nr; ++i) a.src[i] = (const char *)src[i];
    for (int j = 0; j < nw; ++j) a.dst[j] = (char *)dst[j];
    for (int i = 0; i < nr; ++i)
        if (!a.src[i] || ((uintptr_t)a.src[i] & 15)) return set_error(DPWA_ERR_ARG, "dpwa_stream_mix: source %d", i);
    for (int j = 0; j < nw; ++j)
        if (!a.dst[j] || ((uintptr_t)a.dst[j] & 15)) return set_error(DPWA_ERR_ARG, "dpwa_stream_mix: destination %d", j);
    a.nbytes = nbytes;
    a.nr = nr;
    a.nw = nw;
    LaunchTiming t{(hipEvent_t)start_event, (hipEvent_t)stop_event};
    HIP_TRY(launch_stream_mix(a, (hipStream_t)stream, start_event ? &t : nullptr));
    return DPWA_OK;
}

int dpwa_learner_create(dpwa_learner **out, int device, int64_t n, int32_t dtype, const dpwa_interp *cfg)
{
    if (!out || n < 0 || !cfg || dtype_size(dtype) == 0) return set_error(DPWA_ERR_ARG, "dpwa_learner_create: bad arguments");
    if (cfg->method < 0 || cfg->method > 2) return set_error(DPWA_ERR_ARG, "dpwa_learner_create: unknown method");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_error(DPWA_ERR_ARG, "dpwa_learner_create: device %d of %d", device, ndev);
    DeviceGuard dg(device);
    dpwa_learner *l = new (std::nothrow) dpwa_learner();
    if (!l) return set_error(DPWA_ERR_NOMEM, "dpwa_learner_create: out of memory");
    l->device = device;
    l->n = n;
    l->dtype = dtype;
    l->cfg = *cfg;
    l->payload_bytes = (size_t)n * dtype_size(dtype);
    l->slot_stride = kPayloadOff + round_up(l->payload_bytes, kPayloadOff);
    hipError_t e = hipSuccess;
    do {
        if ((e = devmem_alloc(l->slot_mem, 2 * l->slot_stride, device)) != hipSuccess) break;
        l->slots = l->slot_mem.ptr;
        if ((e = hipMalloc(&l->staging, l->slot_stride)) != hipSuccess) break;
        if ((e = hipMalloc(&l->ctl, sizeof(Ctl))) != hipSuccess) break;
        if ((e = hipMemset(l->slots, 0, kPayloadOff)) != hipSuccess) break;
        if ((e = hipMemset(l->slots + l->slot_stride, 0, kPayloadOff)) != hipSuccess) break;
        if ((e = hipMemset(l->staging, 0, kPayloadOff)) != hipSuccess) break;
        if ((e = hipMemset(l->ctl, 0, sizeof(Ctl))) != hipSuccess) break;
        if ((e = hipStreamCreateWithFlags(&l->side, hipStreamNonBlocking)) != hipSuccess) break;
        for (auto &ev : l->ev_published)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) break;
        if (e != hipSuccess) break;
        if ((e = hipEventCreate(&l->ev_issue)) != hipSuccess) break;     // timed: the fetch deadline
        if ((e = hipEventCreateWithFlags(&l->ev_fetched, hipEventDisableTiming)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&l->ev_consumed, hipEventDisableTiming)) != hipSuccess) break;
        for (auto &ev : l->ev_stage_done)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) break;
        if (e != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&l->ev_factor, hipEventDisableTiming)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&l->ev_wt, hipEventDisableTiming)) != hipSuccess) break;
        if ((e = hipHostMalloc((void **)&l->host_status, sizeof(int32_t), hipHostMallocMapped)) != hipSuccess) break;
        *l->host_status = 0;
        if ((e = hipHostGetDevicePointer((void **)&l->host_status_dev, l->host_status, 0)) != hipSuccess) break;
        if ((e = hipDeviceSynchronize()) != hipSuccess) break;
    } while (0);
    if (e != hipSuccess) {
        int rc = set_error(DPWA_ERR_HIP, "dpwa_learner_create: %s (slot %zu bytes)", hipGetErrorString(e), l->slot_stride);
        dpwa_learner_destroy(l);
        return rc;
    }
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        g_live.insert(l);
    }
    *out = l;
    return DPWA_OK;
}

int dpwa_learner_destroy(dpwa_learner *l)
{
    if (!l) return DPWA_OK;
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        g_live.erase(l);
        for (dpwa_learner *o : g_live) {   // forget `l` as a reader of anyone's slot
            std::lock_guard<std::mutex> r(o->readers_mu);
            for (auto &v : o->readers) v.erase(std::remove(v.begin(), v.end(), l), v.end());
        }
    }
    DeviceGuard dg(l->device);
    (void)hipDeviceSynchronize();
    for (auto &kv : l->peers) close_endpoint(kv.second);
    if (l->side) (void)hipStreamDestroy(l->side);
    for (auto ev : l->ev_published)
        if (ev) (void)hipEventDestroy(ev);
    if (l->ev_issue) (void)hipEventDestroy(l->ev_issue);
    if (l->ev_probe) (void)hipEventDestroy(l->ev_probe);
    if (l->probe_stream) (void)hipStreamDestroy(l->probe_stream);
    if (l->ev_fetched) (void)hipEventDestroy(l->ev_fetched);
    if (l->ev_consumed) (void)hipEventDestroy(l->ev_consumed);
    for (auto ev : l->ev_stage_done)
        if (ev) (void)hipEventDestroy(ev);
    if (l->staging_alt) (void)hipFree(l->staging_alt);
    for (auto &r : l->rescue) destroy_lane(r);
    if (l->ev_factor) (void)hipEventDestroy(l->ev_factor);
    if (l->ev_wt) (void)hipEventDestroy(l->ev_wt);
    if (l->ev_read) (void)hipEventDestroy(l->ev_read);
    if (l->ev_relay) (void)hipEventDestroy(l->ev_relay);
    if (l->ev_window) (void)hipEventDestroy(l->ev_window);
    if (l->window_sample) (void)hipFree(l->window_sample);
    if (l->window_host) (void)hipHostFree(l->window_host);
    for (auto &t : l->timing) {
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    for (auto &t : l->fetch_timing) {
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    for (char *p : l->relay_opened) (void)hipIpcCloseMemHandle(p);
    for (auto &m : l->relay_imported) devmem_free(m);
    devmem_free(l->relay_mem);
    if (l->read_stream) (void)hipStreamDestroy(l->read_stream);
    if (l->host_status) (void)hipHostFree(l->host_status);
    devmem_free(l->slot_mem);
    if (l->staging) (void)hipFree(l->staging);
    if (l->ctl) (void)hipFree(l->ctl);
    delete l;
    return DPWA_OK;
}

// Local learners that read slot k (two publishes ago) must have finished before it is
// rewritten (WAR); the wait is enqueued on `s` only for readers on another stream.
static int wait_slot_readers(dpwa_learner *l, int k, hipStream_t s)
{
    std::lock_guard<std::mutex> g(l->readers_mu);
    for (dpwa_learner *r : l->readers[k]) {
        if (r->have_fetch && r->src_owner == l && r->src_slot == k)
            return set_error(DPWA_ERR_STATE,
                             "a peer still has an unconsumed fetch of the snapshot slot about to be rewritten "
                             "(publish at most once per round)");
        if (r->consumed_once && r->consume_stream != s) {
            DeviceGuard rg(r->device);
            HIP_TRY(hipEventRecord(r->ev_consumed, r->consume_stream));
            HIP_TRY(hipStreamWaitEvent(s, r->ev_consumed, 0));
        }
    }
    l->readers[k].clear();
    return DPWA_OK;
}

static int relocate_impl(dpwa_learner *l, hipStream_t s);

// ---------------------------------------------------------------- window guard (resident)
// Between update_send and update_wait resident parameters ARE the snapshot peers read (the
// reference snapshots at update_send, pytorch.py:49-53, so a step in that window never reaches a
// peer there).  The adapter catches optimizer steps by version counter; writes through
// `param.data` move none, so with the reuse guard on every publish runs one small kernel
// (kernels.hip k_window_roll): the payload published last time -- its window closed at the
// average, which wrote the other slot, and nothing writes it again before the average after this
// publish -- is compared with the reuse guard's 4,096 sampled words saved when it was published,
// and the new payload's samples are saved.  A written window is counted on the device and
// mirrored into a host-mapped word; a publish that finds the count grown (never waiting for a
// check) fails with DPWA_ERR_STATE before publishing, and the one after proceeds.  Writes that
// change none of the sampled words are not seen.
static int window_alloc(dpwa_learner *l)
{
    if (l->window_sample) return DPWA_OK;
    char *sample = nullptr;
    uint32_t *host = nullptr, *host_dev = nullptr;
    hipEvent_t ev = nullptr;
    hipError_t e = hipMalloc(&sample, kWindowSampleBytes);
    if (e == hipSuccess) e = hipHostMalloc((void **)&host, sizeof(uint32_t), hipHostMallocMapped);
    if (e == hipSuccess) {
        *host = 0;
        e = hipHostGetDevicePointer((void **)&host_dev, host, 0);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (sample) (void)hipFree(sample);
        if (host) (void)hipHostFree(host);
        if (ev) (void)hipEventDestroy(ev);
        return set_error(DPWA_ERR_HIP, "window guard: %s", hipGetErrorString(e));
    }
    l->window_sample = sample;
    l->window_host = host;
    l->window_host_dev = host_dev;
    l->ev_window = ev;
    l->window_reported = 0;
    return DPWA_OK;
}

// Work on `s` that overwrites slot version % 2 -- the payload the window guard's last roll read
// (the one published before the last publish): an average's write-through store or a relocation --
// runs after that roll when the roll went to another stream.
static int wait_window_roll(dpwa_learner *l, hipStream_t s)
{
    if (!l->resident || !l->window_stream || l->window_stream == s) return DPWA_OK;
    HIP_TRY(hipEventRecord(l->ev_window, l->window_stream));
    HIP_TRY(hipStreamWaitEvent(s, l->ev_window, 0));
    return DPWA_OK;
}

// One roll on `s`: check the last window (if any), then sample `cur` (if not NULL).
static int window_roll(dpwa_learner *l, const char *cur, hipStream_t s)
{
    int rc = window_alloc(l);
    if (rc) return rc;
    if (l->window_stream && l->window_stream != s) {
        HIP_TRY(hipEventRecord(l->ev_window, l->window_stream));
        HIP_TRY(hipStreamWaitEvent(s, l->ev_window, 0));
    }
    HIP_TRY(launch_window_roll(l->window_src, cur, (int64_t)l->payload_bytes, l->window_sample, &l->ctl->window_dirty,
                               &l->ctl->window_hits, l->window_host_dev, l->window_gen, (int32_t)(l->version + 1), s));
    l->window_stream = s;
    if (cur) {
        l->window_src = cur;
        l->window_gen = (int32_t)(l->version + 1);
    }
    return DPWA_OK;
}

// Reports written windows counted since the last report; never waits for a check.
static int window_report(dpwa_learner *l)
{
    if (!l->window_host) return DPWA_OK;
    const uint32_t seen = __atomic_load_n(l->window_host, __ATOMIC_ACQUIRE);
    if (seen == l->window_reported) return DPWA_OK;
    const uint32_t newly = seen - l->window_reported;
    l->window_reported = seen;
    return set_error(DPWA_ERR_STATE,
                     "resident parameters were written between update_send and update_wait (%u more window(s); "
                     "through param.data, which moves no version counter): peers may have averaged with a partly "
                     "written snapshot. With resident parameters the loop must run update_send -> update_wait -> "
                     "step", newly);
}

static int publish_impl(dpwa_learner *l, const void *flat, double loss, const double *loss_dev, hipStream_t s,
                        bool reuse)
{
    TraceRange tr(reuse ? "dpwa.learner_publish.reuse" : "dpwa.learner_publish");
    l->timing_armed = false;   // armed for the last round's average, which did not happen
    if (l->resident && l->reuse_guard) {   // the window guard's buffers, before anything is queued
        int rc = window_alloc(l);
        if (rc) return rc;
    }
    const int k = (int)(l->version % 2);   // slot of publish number version+1
    char *slot = l->slots + (size_t)k * l->slot_stride;
    if (l->resident) {
        int rc = window_report(l);
        if (rc) return rc;
        // the parameters are the payload already: publish the header of the slot they are in
        // (after a publish with no average since, they first move on by one copy)
        if (flat != slot_payload(l, l->res_slot))
            return set_error(DPWA_ERR_ARG, "resident learner: publish the parameters where they are "
                                           "(dpwa_learner_resident_params)");
        rc = relocate_impl(l, s);
        if (rc) return rc;
        flat = slot_payload(l, l->res_slot);
        reuse = true;
    }
    const bool header_only = reuse && l->wt_valid && l->wt_flat == flat;
    if (header_only && l->wt_header) {
        // payload, header and clock of this publish were written by the last average: nothing
        // moves (IPC-exported slots still get their system-scope write-back).  Work on `s`
        // after this publish (the next factor reads the clock the average wrote) is ordered
        // after the average.
        if (l->wt_stream != s) {
            HIP_TRY(hipEventRecord(l->ev_wt, l->wt_stream));
            HIP_TRY(hipStreamWaitEvent(s, l->ev_wt, 0));
        }
        if (l->reuse_guard && !l->resident)
            HIP_TRY(launch_guard_payload(slot + kPayloadOff, flat, (int64_t)l->payload_bytes, &l->ctl->guard_dirty,
                                         &l->ctl->guard_hits, (int32_t)(l->version + 1), s));
        if (l->exported) HIP_TRY(launch_release_system(s));
        l->cur = (l->cur + 1) & 3;
    } else if (header_only) {
        // the payload was written by the last average (readers of slot k were waited for then)
        if (l->wt_stream != s) {
            HIP_TRY(hipEventRecord(l->ev_wt, l->wt_stream));
            HIP_TRY(hipStreamWaitEvent(s, l->ev_wt, 0));
        }
        if (l->reuse_guard && !l->resident)
            HIP_TRY(launch_guard_payload(slot + kPayloadOff, flat, (int64_t)l->payload_bytes, &l->ctl->guard_dirty,
                                         &l->ctl->guard_hits, (int32_t)(l->version + 1), s));
        HIP_TRY(launch_publish_header(slot, l->n, l->dtype, &l->ctl->clock[l->cur], loss, loss_dev, l->loss_f32,
                                      l->version + 1, l->exported, s));
    } else {
        if (l->resident) return set_error(DPWA_ERR_STATE, "resident learner: parameters not in the next slot");
        int rc = wait_slot_readers(l, k, s);
        if (rc) return rc;
        HIP_TRY(launch_publish(slot, flat, (int64_t)l->payload_bytes, l->n, l->dtype, &l->ctl->clock[l->cur], loss,
                               loss_dev, l->loss_f32, l->version + 1, l->exported, s));
    }
    l->wt_valid = false;
    l->wt_header = false;
    if (l->resident && l->reuse_guard) {   // the last window's check; this window's samples
        int rc = window_roll(l, (const char *)flat, s);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> g(l->pub_mu);
    l->publish_stream[k] = s;
    l->published[k] = true;
    l->version++;
    return DPWA_OK;
}

int dpwa_learner_publish(dpwa_learner *l, const void *flat, double loss, const double *loss_dev, dpwa_stream_t stream)
{
    if (!l || (!flat && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_publish: NULL argument");
    DeviceGuard dg(l->device);
    return publish_impl(l, flat, loss, loss_dev, (hipStream_t)stream, false);
}

int dpwa_learner_publish_reuse(dpwa_learner *l, const void *flat, double loss, const double *loss_dev,
                               dpwa_stream_t stream)
{
    if (!l || (!flat && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_publish_reuse: NULL argument");
    DeviceGuard dg(l->device);
    return publish_impl(l, flat, loss, loss_dev, (hipStream_t)stream, true);
}

int dpwa_learner_version(const dpwa_learner *l, uint64_t *version)
{
    if (!l || !version) return set_error(DPWA_ERR_ARG, "dpwa_learner_version: NULL argument");
    *version = l->version;
    return DPWA_OK;
}

// peer == l is the self-peer (the learner's own published slot, read like any local peer's)
int dpwa_learner_attach_local(dpwa_learner *l, int peer_id, dpwa_learner *peer)
{
    if (!l || !peer) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_local: bad peer");
    if (peer->n != l->n || peer->dtype != l->dtype)
        return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_local: peer holds %lld elements of dtype %d, this learner %lld of %d",
                         (long long)peer->n, peer->dtype, (long long)l->n, l->dtype);
    if (peer->device != l->device) {
        DeviceGuard dg(l->device);
        int can = 0;
        HIP_TRY(hipDeviceCanAccessPeer(&can, l->device, peer->device));
        if (!can) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_local: device %d cannot access device %d", l->device, peer->device);
        hipError_t e = hipDeviceEnablePeerAccess(peer->device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            return set_error(DPWA_ERR_HIP, "hipDeviceEnablePeerAccess: %s", hipGetErrorString(e));
        (void)hipGetLastError();
        if (peer->slot_mem.vmm()) HIP_TRY(vmm_grant(peer->slot_mem, l->device));   // VMM: per-device access
        peer->exported = true;   // read by another GPU: its publishes release at system scope
    }
    Endpoint ep;
    ep.kind = 1;
    ep.local = peer;
    ep.base = peer->slots;
    ep.device = peer->device;
    ep.slot_stride = (int64_t)peer->slot_stride;
    ep.n = peer->n;
    ep.dtype = peer->dtype;
    l->peers[peer_id] = ep;
    return DPWA_OK;
}

static IpcBlob make_blob(const dpwa_learner *l, const DevMem &m, int64_t stride)
{
    IpcBlob b;
    memset(&b, 0, sizeof(b));
    b.magic = kIpcMagic;
    b.slot_stride = stride;
    b.n = l->n;
    b.dtype = l->dtype;
    b.device = l->device;
    b.pid = (int32_t)getpid();
    b.vmm = m.vmm() ? 1 : 0;
    return b;
}

int dpwa_learner_ipc_handle(dpwa_learner *l, void *handle_out, int64_t handle_len)
{
    if (!l || !handle_out || handle_len < (int64_t)sizeof(IpcBlob))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_ipc_handle: need %zu bytes", sizeof(IpcBlob));
    DeviceGuard dg(l->device);
    IpcBlob b = make_blob(l, l->slot_mem, (int64_t)l->slot_stride);
    if (!b.vmm) HIP_TRY(hipIpcGetMemHandle(&b.handle, l->slots));   // else: fds, dpwa_learner_export_fds
    memset(handle_out, 0, (size_t)handle_len);
    memcpy(handle_out, &b, sizeof(b));
    l->exported = true;   // from now on publishes release at system scope
    return DPWA_OK;
}

int dpwa_learner_export_fds(dpwa_learner *l, int which, int *fds, int max_fds, int *n_fds, int64_t *chunk_bytes)
{
    if (!l || (which != 0 && which != 1) || !n_fds || (max_fds > 0 && !fds) || (which == 1 && !l->relay_on))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_export_fds: bad arguments");
    DeviceGuard dg(l->device);
    const int rc = devmem_export(which == 0 ? l->slot_mem : l->relay_mem, fds, max_fds, n_fds, chunk_bytes);
    if (rc == DPWA_OK) l->exported = true;
    return rc;
}

static int check_blob(const dpwa_learner *l, const void *handle, int64_t handle_len, IpcBlob &b, const char *fn)
{
    if (!handle || handle_len < (int64_t)sizeof(IpcBlob)) return set_error(DPWA_ERR_ARG, "%s: bad handle", fn);
    memcpy(&b, handle, sizeof(b));
    if (b.magic != kIpcMagic) return set_error(DPWA_ERR_ARG, "%s: not a dpwa handle", fn);
    if (b.n != l->n || b.dtype != l->dtype)
        return set_error(DPWA_ERR_ARG, "%s: peer holds %lld elements of dtype %d, this learner %lld of %d", fn,
                         (long long)b.n, b.dtype, (long long)l->n, l->dtype);
    return DPWA_OK;
}

static void set_remote(dpwa_learner *l, int peer_id, const IpcBlob &b, char *base, DevMem &&imported)
{
    auto it = l->peers.find(peer_id);
    if (it != l->peers.end()) close_endpoint(it->second);
    Endpoint ep;
    ep.kind = 2;
    ep.base = base;
    ep.device = b.device;
    ep.slot_stride = b.slot_stride;
    ep.n = b.n;
    ep.dtype = b.dtype;
    ep.imported = std::move(imported);
    l->peers[peer_id] = std::move(ep);
}

int dpwa_learner_attach_ipc(dpwa_learner *l, int peer_id, const void *handle, int64_t handle_len)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_ipc: NULL learner");
    IpcBlob b;
    int rc = check_blob(l, handle, handle_len, b, "dpwa_learner_attach_ipc");
    if (rc) return rc;
    if (b.vmm) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_ipc: the peer shares its slots as fds (dpwa_learner_attach_fds)");
    DeviceGuard dg(l->device);
    void *ptr = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&ptr, b.handle, hipIpcMemLazyEnablePeerAccess));
    set_remote(l, peer_id, b, (char *)ptr, DevMem());
    return DPWA_OK;
}

int dpwa_learner_attach_fds(dpwa_learner *l, int peer_id, const void *handle, int64_t handle_len, const int *fds,
                            int n_fds, int64_t chunk_bytes)
{
    if (!l || !fds) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_fds: bad arguments");
    IpcBlob b;
    int rc = check_blob(l, handle, handle_len, b, "dpwa_learner_attach_fds");
    if (rc) return rc;
    if (!b.vmm) return set_error(DPWA_ERR_ARG, "dpwa_learner_attach_fds: the peer shares a hipIpc handle (dpwa_learner_attach_ipc)");
    DeviceGuard dg(l->device);
    DevMem m;
    if ((rc = devmem_import(m, fds, n_fds, chunk_bytes, 2 * (size_t)b.slot_stride, l->device))) return rc;
    char *base = m.ptr;
    set_remote(l, peer_id, b, base, std::move(m));
    return DPWA_OK;
}

// A free rescue lane: one whose last pull landed (or none issued); *lane = -1 when every lane made
// so far is still pulling.
static int free_lane(dpwa_learner *l, int *lane)
{
    *lane = -1;
    for (int j = 0; j < l->rescue_lanes; ++j) {
        RescueLane &r = l->rescue[j];
        const hipError_t e = r.used ? hipEventQuery(r.ev_landed) : hipSuccess;
        if (e == hipSuccess) {
            *lane = j;
            return DPWA_OK;
        }
        if (e != hipErrorNotReady) return set_error(DPWA_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
    }
    return DPWA_OK;
}

// A free rescue lane, making a new one when every lane is taken and fewer than rescue_cap exist;
// *lane = -1 when none is free and none can be made.  A new lane is built in a local and counted
// only once every resource exists.  Running short of memory (or an allocation failing) is not an
// error of the round: the lane count is capped where it is and the caller waits for a lane to land.
static int rescue_lane(dpwa_learner *l, int *lane)
{
    int rc = free_lane(l, lane);
    if (rc || *lane >= 0 || l->rescue_lanes >= l->rescue_cap) return rc;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < l->slot_stride + kRescueReserve ||
        (size_t)(l->rescue_lanes + 1) * l->slot_stride > total_b / kRescueShare) {
        (void)hipGetLastError();
        l->rescue_cap = l->rescue_lanes;
        return DPWA_OK;
    }
    RescueLane r;
    int least = 0, greatest = 0;
    hipError_t e;
    do {
        if ((e = hipMalloc(&r.buf, l->slot_stride)) != hipSuccess) break;
        if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) != hipSuccess) break;
        if ((e = hipStreamCreateWithPriority(&r.stream, hipStreamNonBlocking, greatest)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&r.ev_landed, hipEventDisableTiming)) != hipSuccess) break;
        e = hipEventCreateWithFlags(&r.ev_done, hipEventDisableTiming);
    } while (0);
    if (e != hipSuccess) {
        destroy_lane(r);
        (void)hipGetLastError();          // clear the sticky error: the round goes on without a new lane
        l->rescue_cap = l->rescue_lanes;
        return DPWA_OK;
    }
    l->rescue[l->rescue_lanes] = r;
    *lane = l->rescue_lanes++;
    return DPWA_OK;
}

// Gives back the lanes beyond the first kKeepRescueLanes, last first, once idle for kLaneIdleRounds
// fetch rounds: their pull landed and the last reader of their buffer is done (event queries, no
// wait).  Called at a round's first pull, the normal path, where it costs one comparison.
static void trim_lanes(dpwa_learner *l)
{
    while (l->rescue_lanes > kKeepRescueLanes) {
        const int j = l->rescue_lanes - 1;
        RescueLane &r = l->rescue[j];
        if (l->fetch_rounds - r.last_round < kLaneIdleRounds || l->src_stage == 2 + j) return;
        if (r.used && hipEventQuery(r.ev_landed) != hipSuccess) break;
        if (r.read && hipEventQuery(r.ev_done) != hipSuccess) break;
        destroy_lane(r);
        l->rescue_lanes--;
    }
    (void)hipGetLastError();   // a not-ready query leaves no error behind
}

int dpwa_learner_fetch(dpwa_learner *l, int peer_id, uint64_t peer_version, int flags, dpwa_stream_t stream)
{
    const int zero_copy = flags & DPWA_FETCH_ZERO_COPY;
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_fetch: NULL learner");
    auto it = l->peers.find(peer_id);
    if (it == l->peers.end()) return set_error(DPWA_ERR_ARG, "dpwa_learner_fetch: peer %d not attached", peer_id);
    if (peer_version == 0) return set_error(DPWA_ERR_STATE, "dpwa_learner_fetch: peer %d has not published", peer_id);
    Endpoint &ep = it->second;
    if (ep.kind == 1 && !is_live(ep.local)) return set_error(DPWA_ERR_STATE, "dpwa_learner_fetch: peer %d was destroyed", peer_id);
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    const int k = (int)((peer_version - 1) % 2);
    const char *peer_slot = ep.base + (size_t)k * (size_t)ep.slot_stride;
    if (ep.kind == 1) {
        // RAW: the peer's publish of that slot must be complete before anyone reads it.
        dpwa_learner *pl = ep.local;
        if (!pl->published[k]) return set_error(DPWA_ERR_STATE, "dpwa_learner_fetch: peer %d slot %d never published", peer_id, k);
        if (pl->publish_stream[k] != s) {
            DeviceGuard pg(pl->device);
            HIP_TRY(hipEventRecord(pl->ev_published[k], pl->publish_stream[k]));
            HIP_TRY(hipStreamWaitEvent(s, pl->ev_published[k], 0));
        }
        std::lock_guard<std::mutex> g(ep.local->readers_mu);
        auto &rv = ep.local->readers[k];
        if (std::find(rv.begin(), rv.end(), l) == rv.end()) rv.push_back(l);
    }
    l->fetch_issue_ns = now_ns();
    l->fetch_stream = l->side;
    l->issue_evented = false;
    if (!(flags & DPWA_FETCH_RESCUE)) {
        l->fetch_rounds++;
        if (l->rescue_lanes > kKeepRescueLanes) trim_lanes(l);
    }
    if (flags & DPWA_FETCH_RESCUE) {
        // re-selected after a timed-out pull: a free lane (its own stream and buffer), ordered
        // after the publish of the snapshot (above, local peers) and after the last reader of the
        // lane's buffer
        int j = -1;
        const int rc = rescue_lane(l, &j);
        if (rc) return rc;
        if (j < 0)
            return set_error(DPWA_ERR_STATE, "dpwa_learner_fetch: all %d rescue lanes are still pulling",
                             l->rescue_lanes);
        RescueLane &r = l->rescue[j];
        if (!(flags & DPWA_FETCH_PUBLISHED)) {
            HIP_TRY(hipEventRecord(l->ev_issue, s));
            HIP_TRY(hipStreamWaitEvent(r.stream, l->ev_issue, 0));
            l->issue_evented = true;
        }
        if (r.read) HIP_TRY(hipStreamWaitEvent(r.stream, r.ev_done, 0));
        const size_t nbytes = kPayloadOff + round_up(l->payload_bytes, 16);
        if (l->pull_mode == DPWA_PULL_KERNEL)
            HIP_TRY(launch_pull(r.buf, peer_slot, (int64_t)nbytes, l->pull_blocks,
                                ep.kind == 2 || ep.device != l->device, r.stream));
        else
            HIP_TRY(hipMemcpyAsync(r.buf, peer_slot, nbytes, hipMemcpyDefault, r.stream));
        HIP_TRY(hipEventRecord(r.ev_landed, r.stream));
        HIP_TRY(hipEventRecord(l->ev_fetched, r.stream));
        r.used = true;
        r.last_round = l->fetch_rounds;
        l->fetch_stream = r.stream;
        l->src = r.buf;
        l->src_copied = true;
        l->src_stage = 2 + j;
    } else if (zero_copy && ep.kind == 1 && ep.device == l->device) {
        l->src = peer_slot;             // read in place; stream order covers the rest
        l->src_copied = false;
        l->src_stage = -1;
    } else if ((flags & DPWA_FETCH_PUBLISHED) && ep.kind == 2) {
        if (!l->staging_alt) {
            HIP_TRY(hipMalloc(&l->staging_alt, l->slot_stride));
            HIP_TRY(hipMemsetAsync(l->staging_alt, 0, kPayloadOff, l->side));
        }
        const int b = l->stage_next;
        l->stage_next ^= 1;
        char *dst = b == 0 ? l->staging : l->staging_alt;
        // WAR: the average that last read this buffer; nothing else on the caller's stream
        if (l->stage_read[b]) HIP_TRY(hipStreamWaitEvent(l->side, l->ev_stage_done[b], 0));
        const size_t nbytes = kPayloadOff + round_up(l->payload_bytes, 16);
        const LaunchTiming *ft = l->fetch_timing_used < (int)l->fetch_timing.size()
                                     ? &l->fetch_timing[l->fetch_timing_used++] : nullptr;
        if (ft) HIP_TRY(hipEventRecord(ft->start, l->side));
        if (l->pull_mode == DPWA_PULL_KERNEL)
            HIP_TRY(launch_pull(dst, peer_slot, (int64_t)nbytes, l->pull_blocks, true, l->side));
        else
            HIP_TRY(hipMemcpyAsync(dst, peer_slot, nbytes, hipMemcpyDefault, l->side));
        if (ft) HIP_TRY(hipEventRecord(ft->stop, l->side));
        HIP_TRY(hipEventRecord(l->ev_fetched, l->side));
        l->src = dst;
        l->src_copied = true;
        l->src_stage = b;
    } else {
        if (l->stage_read[0]) HIP_TRY(hipStreamWaitEvent(l->side, l->ev_stage_done[0], 0));
        HIP_TRY(hipEventRecord(l->ev_issue, s));
        HIP_TRY(hipStreamWaitEvent(l->side, l->ev_issue, 0));
        l->issue_evented = true;
        // WAR on our own staging buffer: the previous average must have consumed it.
        if (l->consumed_once && l->consume_stream != s) {
            HIP_TRY(hipEventRecord(l->ev_consumed, l->consume_stream));
            HIP_TRY(hipStreamWaitEvent(l->side, l->ev_consumed, 0));
        }
        const size_t nbytes = kPayloadOff + round_up(l->payload_bytes, 16);
        const LaunchTiming *ft = l->fetch_timing_used < (int)l->fetch_timing.size()
                                     ? &l->fetch_timing[l->fetch_timing_used++] : nullptr;
        if (ft) HIP_TRY(hipEventRecord(ft->start, l->side));
        if (l->pull_mode == DPWA_PULL_KERNEL)
            HIP_TRY(launch_pull(l->staging, peer_slot, (int64_t)nbytes, l->pull_blocks,
                                ep.kind == 2 || ep.device != l->device, l->side));
        else
            HIP_TRY(hipMemcpyAsync(l->staging, peer_slot, nbytes, hipMemcpyDefault, l->side));
        if (ft) HIP_TRY(hipEventRecord(ft->stop, l->side));
        HIP_TRY(hipEventRecord(l->ev_fetched, l->side));
        l->src = l->staging;
        l->src_copied = true;
        l->src_stage = 0;
    }
    l->src_owner = ep.kind == 1 ? ep.local : nullptr;
    l->src_slot = k;
    l->have_fetch = true;
    return DPWA_OK;
}

static int relay_materialize(dpwa_learner *l);
static hipError_t staging_read(dpwa_learner *l, hipStream_t s);

static FusedArgs fused_args(dpwa_learner *l, double loss, const double *loss_dev)
{
    FusedArgs fa{};
    fa.cfg = l->cfg;
    fa.clock_in = &l->ctl->clock[l->cur];
    fa.clock_out = &l->ctl->clock[(l->cur + 1) & 3];
    fa.hdr = (const dpwa_header *)l->src;
    fa.loss_h = loss;
    fa.loss_d = loss_dev;
    fa.loss_f32 = l->loss_f32 ? 1 : 0;
    fa.coef_out = &l->ctl->coef;
    fa.status_mirror = l->host_status_dev;
    return fa;
}

int dpwa_learner_factor(dpwa_learner *l, double loss, const double *loss_dev, dpwa_stream_t stream)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_factor: NULL learner");
    if (!l->have_fetch) return set_error(DPWA_ERR_STATE, "dpwa_learner_factor: no fetch in flight");
    if (l->have_factor) return set_error(DPWA_ERR_STATE, "dpwa_learner_factor: factor already computed for this fetch");
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = relay_materialize(l);
    if (rc) return rc;
    if (l->src_copied) HIP_TRY(hipStreamWaitEvent(s, l->ev_fetched, 0));   // TxThread.fetch_wait
    HIP_TRY(launch_factor(fused_args(l, loss, loss_dev), s));
    HIP_TRY(hipEventRecord(l->ev_factor, s));
    HIP_TRY(staging_read(l, s));   // a later pull into this staging buffer waits for the header read
    l->consume_stream = s;   // the header has been read on s
    l->consumed_once = true;
    l->cur = (l->cur + 1) & 3;
    l->have_factor = true;
    return DPWA_OK;
}

// The fetched snapshot in staging buffer src_stage has been read by everything enqueued on s.
static hipError_t staging_read(dpwa_learner *l, hipStream_t s)
{
    if (l->src_stage < 0 || !l->src_copied) return hipSuccess;
    if (l->src_stage >= 2) {
        RescueLane &r = l->rescue[l->src_stage - 2];
        r.read = true;
        return hipEventRecord(r.ev_done, s);
    }
    l->stage_read[l->src_stage] = true;
    return hipEventRecord(l->ev_stage_done[l->src_stage], s);
}

static void finish_fetch(dpwa_learner *l)
{
    l->have_fetch = false;
    l->have_factor = false;
    l->src = nullptr;
}

int dpwa_learner_lerp(dpwa_learner *l, void *flat, dpwa_stream_t stream)
{
    if (!l || (!flat && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_lerp: NULL argument");
    if (!l->have_factor) return set_error(DPWA_ERR_STATE, "dpwa_learner_lerp: no factor computed for this fetch");
    if (l->resident)
        return set_error(DPWA_ERR_STATE, "dpwa_learner_lerp: a resident learner averages with dpwa_learner_average");
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(launch_lerp(l->dtype, flat, l->src + kPayloadOff, l->n, &l->ctl->coef, 0.f, 0.f, s));
    HIP_TRY(staging_read(l, s));
    l->wt_valid = false;
    l->consume_stream = s;
    l->consumed_once = true;
    finish_fetch(l);
    return DPWA_OK;
}

// One fused average, split so that several learners' averages can share a dispatch:
// average_prepare orders `s` after everything the kernel reads or overwrites and builds its
// arguments; the caller launches; average_commit does the learner's bookkeeping.
struct AvgPlan {
    void *flat = nullptr;
    const char *peer = nullptr;   // payload averaged with (contiguous source)
    char *snap = nullptr;         // write-through destination
    FusedArgs fa{};
    bool relay = false;           // the relay's phase 2 fused into this average (k_lerp_relay)
    bool write_through = false;
    bool oop = false;             // resident: the result goes to `snap` only
    int snap_slot = -1;
};

static int average_prepare(dpwa_learner *l, void *flat, double loss, const double *loss_dev, hipStream_t s,
                           bool write_through, AvgPlan &p)
{
    if (!l->have_fetch || l->have_factor) return set_error(DPWA_ERR_STATE, "dpwa_learner_average: no fetch in flight");
    p = AvgPlan();
    if (l->resident) {   // read where the parameters are (the published slot), write the next slot
        if (flat != slot_payload(l, l->res_slot))
            return set_error(DPWA_ERR_ARG, "resident learner: average the parameters where they are "
                                           "(dpwa_learner_resident_params)");
        write_through = true;
        p.oop = true;
    }
    p.flat = flat;
    p.write_through = write_through;
    p.fa = fused_args(l, loss, loss_dev);
    if (write_through) {
        const int k = (int)(l->version % 2);   // slot of the next publish
        int rc = wait_slot_readers(l, k, s);
        if (rc) return rc;
        if ((rc = wait_window_roll(l, s))) return rc;
        p.snap = slot_payload(l, k);
        p.snap_slot = k;
        if (l->cfg.method != DPWA_INTERP_LOSS && !l->header_on_publish) {   // peers never read this header's loss
            p.fa.next_header = (dpwa_header *)(p.snap - kPayloadOff);
            p.fa.clock_next = &l->ctl->clock[(l->cur + 2) & 3];
            p.fa.next_version = l->version + 1;
            p.fa.n = l->n;
            p.fa.dtype = l->dtype;
        }
    }
    if (l->relay_deferred && (((uintptr_t)flat | (uintptr_t)p.snap) & 15) == 0) {
        // the relay's phase 2 fused into the average: stripes read where phase 1 left them
        const RelayArgs &a = l->relay_saved;
        p.fa.hdr = (const dpwa_header *)(a.slots[l->relay_saved_pick] + a.slot_off);
        HIP_TRY(hipStreamWaitEvent(s, l->ev_fetched, 0));
        p.relay = true;
    } else {
        int rc = relay_materialize(l);
        if (rc) return rc;
        if (l->src_copied) HIP_TRY(hipStreamWaitEvent(s, l->ev_fetched, 0));   // TxThread.fetch_wait
        p.peer = l->src + kPayloadOff;
    }
    return DPWA_OK;
}

static const LaunchTiming *take_timing(dpwa_learner *l)
{
    if (l->timing_armed && l->timing_used < (int)l->timing.size()) return &l->timing[l->timing_used++];
    return nullptr;
}

static int average_commit(dpwa_learner *l, const AvgPlan &p, hipStream_t s)
{
    if (p.relay) {
        HIP_TRY(hipEventRecord(l->ev_relay, s));   // the next round's barrier waits for these reads
        l->relay_pending = true;
        l->relay_deferred = false;
    } else {
        HIP_TRY(staging_read(l, s));
    }
    l->timing_armed = false;
    l->consume_stream = s;
    l->consumed_once = true;
    l->cur = (l->cur + 1) & 3;
    l->wt_valid = p.write_through;
    l->wt_header = p.fa.next_header != nullptr;
    l->wt_flat = p.flat;
    l->wt_stream = s;
    if (p.oop) {   // the parameters moved into the next publish's slot
        l->res_slot = p.snap_slot;
        l->wt_flat = p.snap;
    }
    finish_fetch(l);
    return DPWA_OK;
}

static int average_launch(dpwa_learner *l, const AvgPlan &p, hipStream_t s)
{
    if (p.relay) {
        HIP_TRY(launch_average_relay(l->dtype, p.flat, l->n, p.fa, p.snap, l->relay_saved, l->relay_saved_pick, s,
                                     take_timing(l), p.oop));
    } else {
        const LaunchTiming *timing = ((uintptr_t)p.flat & 15) == 0 ? take_timing(l) : nullptr;
        HIP_TRY(launch_average(l->dtype, p.flat, p.peer, l->n, p.fa, p.snap, s, timing, p.oop));
    }
    return DPWA_OK;
}

static int average_impl(dpwa_learner *l, void *flat, double loss, const double *loss_dev, hipStream_t s,
                        bool write_through)
{
    TraceRange tr("dpwa.average");
    AvgPlan p;
    int rc = average_prepare(l, flat, loss, loss_dev, s, write_through, p);
    if (rc) return rc;
    if ((rc = average_launch(l, p, s))) return rc;
    return average_commit(l, p, s);
}

// Can plan p join a batched dispatch (k_lerp_batch)?  Contiguous source, 16-B aligned operands.
static bool batchable(const AvgPlan &p)
{
    return !p.relay && ((((uintptr_t)p.flat | (uintptr_t)p.peer | (uintptr_t)p.snap) & 15) == 0);
}

// Launches the batchable plans in groups of the same (dtype, write-through), up to
// kMaxAvgBatch per dispatch, and every other plan on its own.  Timed like a single average:
// the first armed learner of a dispatch lends it its timing pair.
static int launch_plans(dpwa_learner *const *ls, const AvgPlan *plans, const int *idx, int count, hipStream_t s)
{
    std::vector<char> done((size_t)count, 0);
    for (int a = 0; a < count; ++a) {
        if (done[a]) continue;
        const int ia = idx[a];
        dpwa_learner *la = ls[ia];
        const AvgPlan &pa = plans[ia];
        done[a] = 1;
        if (!batchable(pa)) {
            int rc = average_launch(la, pa, s);
            if (rc) return rc;
            continue;
        }
        AvgBatch b{};
        const LaunchTiming *timing = take_timing(la);
        auto add = [&](dpwa_learner *l, const AvgPlan &p) {
            AvgEntry &e = b.e[b.count++];
            e.param = p.flat;
            e.peer = p.peer;
            e.snap = p.snap;
            e.n = l->n;
            e.fa = p.fa;
        };
        add(la, pa);
        for (int c = a + 1; c < count && b.count < kMaxAvgBatch; ++c) {
            const int ic = idx[c];
            if (done[c] || !batchable(plans[ic]) || ls[ic]->dtype != la->dtype ||
                plans[ic].write_through != pa.write_through || plans[ic].oop != pa.oop)
                continue;
            if (!timing) timing = take_timing(ls[ic]);
            add(ls[ic], plans[ic]);
            done[c] = 1;
        }
        HIP_TRY(launch_average_batch(la->dtype, pa.write_through, b, s, timing, pa.oop));
    }
    return DPWA_OK;
}

int dpwa_learner_average(dpwa_learner *l, void *flat, double loss, const double *loss_dev, dpwa_stream_t stream)
{
    if (!l || (!flat && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_average: NULL argument");
    DeviceGuard dg(l->device);
    return average_impl(l, flat, loss, loss_dev, (hipStream_t)stream, false);
}

int dpwa_learner_average_through(dpwa_learner *l, void *flat, double loss, const double *loss_dev,
                                 dpwa_stream_t stream)
{
    if (!l || (!flat && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_average_through: NULL argument");
    DeviceGuard dg(l->device);
    return average_impl(l, flat, loss, loss_dev, (hipStream_t)stream, true);
}

int dpwa_learner_average_many(dpwa_learner *const *ls, void *const *flats, const double *loss,
                              const double *const *loss_dev, const int *write_through, int count, dpwa_stream_t stream)
{
    if (count < 0 || (count > 0 && (!ls || !flats || !loss || !write_through)))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_average_many: bad arguments");
    if (count == 0) return DPWA_OK;
    for (int i = 0; i < count; ++i) {
        if (!ls[i] || (!flats[i] && ls[i]->n > 0))
            return set_error(DPWA_ERR_ARG, "dpwa_learner_average_many: NULL learner or buffer at %d", i);
        if (ls[i]->device != ls[0]->device)
            return set_error(DPWA_ERR_ARG, "dpwa_learner_average_many: learners on devices %d and %d share one stream",
                             ls[0]->device, ls[i]->device);
        for (int j = 0; j < i; ++j)
            if (ls[j] == ls[i]) return set_error(DPWA_ERR_ARG, "dpwa_learner_average_many: learner %d given twice", i);
    }
    DeviceGuard dg(ls[0]->device);
    hipStream_t s = (hipStream_t)stream;
    std::vector<AvgPlan> plans((size_t)count);
    std::vector<int> idx;
    idx.reserve((size_t)count);
    for (int i = 0; i < count; ++i) {
        int rc = average_prepare(ls[i], flats[i], loss[i], loss_dev ? loss_dev[i] : nullptr, s, write_through[i] != 0,
                                 plans[i]);
        if (rc) return rc;   // nothing launched yet for this learner; earlier ones are prepared only
        idx.push_back(i);
    }
    int rc = launch_plans(ls, plans.data(), idx.data(), count, s);
    if (rc) return rc;
    for (int i = 0; i < count; ++i)
        if ((rc = average_commit(ls[i], plans[i], s))) return rc;
    return DPWA_OK;
}

static int average_many_impl(const char *fn, int32_t dtype, const dpwa_average_desc *descs, int count,
                             const dpwa_interp *cfg, dpwa_stream_t stream, void *start_event, void *stop_event,
                             bool oop)
{
    if (count < 1 || count > kMaxAvgBatch || !descs || !cfg || dtype_size(dtype) == 0 || (!start_event) != (!stop_event))
        return set_error(DPWA_ERR_ARG, "%s: bad arguments (1..%d descriptors)", fn, kMaxAvgBatch);
    if (cfg->method < 0 || cfg->method > 2) return set_error(DPWA_ERR_ARG, "%s: unknown method %d", fn, cfg->method);
    AvgBatch b{};
    bool dual = oop;   // an empty entry may pass no buffers at all
    for (int i = 0; i < count; ++i) dual = dual || descs[i].snap_payload != nullptr;
    for (int i = 0; i < count; ++i) {
        const dpwa_average_desc &d = descs[i];
        if ((!d.param && d.n > 0) || !d.peer_slot || !d.clock_dev || !d.coef_dev || d.n < 0 ||
            (d.snap_payload == nullptr && d.n > 0 && dual) ||
            (((uintptr_t)d.param | (uintptr_t)d.peer_slot | (uintptr_t)d.snap_payload) & 15))
            return set_error(DPWA_ERR_ARG, "%s: descriptor %d: NULL, unaligned or mixed write-through", fn, i);
        AvgEntry &e = b.e[b.count++];
        e.param = d.param;
        e.peer = (const char *)d.peer_slot + kPayloadOff;
        e.snap = d.snap_payload;
        e.n = d.n;
        e.fa.cfg = *cfg;
        e.fa.clock_in = d.clock_dev;
        e.fa.clock_out = d.clock_dev + 1;
        e.fa.hdr = (const dpwa_header *)d.peer_slot;
        e.fa.loss_h = d.loss;
        e.fa.coef_out = d.coef_dev;
    }
    LaunchTiming t{(hipEvent_t)start_event, (hipEvent_t)stop_event};
    if (oop && count == 1) {   // one resident average: the single kernel, as a resident learner runs it
        const AvgEntry &e = b.e[0];
        HIP_TRY(launch_average(dtype, e.param, e.peer, e.n, e.fa, e.snap, (hipStream_t)stream,
                               start_event ? &t : nullptr, true));
        return DPWA_OK;
    }
    HIP_TRY(launch_average_batch(dtype, dual, b, (hipStream_t)stream, start_event ? &t : nullptr, oop));
    return DPWA_OK;
}

int dpwa_average_many(int32_t dtype, const dpwa_average_desc *descs, int count, const dpwa_interp *cfg,
                      dpwa_stream_t stream, void *start_event, void *stop_event)
{
    return average_many_impl("dpwa_average_many", dtype, descs, count, cfg, stream, start_event, stop_event, false);
}

int dpwa_average_many_resident(int32_t dtype, const dpwa_average_desc *descs, int count, const dpwa_interp *cfg,
                               dpwa_stream_t stream, void *start_event, void *stop_event)
{
    return average_many_impl("dpwa_average_many_resident", dtype, descs, count, cfg, stream, start_event, stop_event,
                             true);
}

int dpwa_learner_set_header_publish(dpwa_learner *l, int always)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_set_header_publish: NULL learner");
    l->header_on_publish = always != 0;
    return DPWA_OK;
}

int dpwa_learner_set_reuse_guard(dpwa_learner *l, int on)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_set_reuse_guard: NULL learner");
    l->reuse_guard = on != 0;
    l->window_src = nullptr;   // a resident learner's window guard starts afresh at the next publish
    return DPWA_OK;
}

// Moves resident parameters from the published slot into the next publish's slot (a round
// without an average; two publishes in a row).  No-op when they are there already.
static int relocate_impl(dpwa_learner *l, hipStream_t s)
{
    const int k = (int)(l->version % 2);
    if (!l->resident || l->res_slot == k) return DPWA_OK;
    int rc = wait_slot_readers(l, k, s);
    if (rc) return rc;
    if ((rc = wait_window_roll(l, s))) return rc;
    HIP_TRY(launch_copy_payload(slot_payload(l, k), slot_payload(l, l->res_slot), (int64_t)l->payload_bytes, s));
    l->res_slot = k;
    l->wt_valid = true;
    l->wt_header = false;     // the publish writes the header (the clock did not move)
    l->wt_flat = slot_payload(l, k);
    l->wt_stream = s;
    return DPWA_OK;
}

int dpwa_learner_set_resident(dpwa_learner *l, const void *init, dpwa_stream_t stream)
{
    if (!l || (!init && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_set_resident: NULL argument");
    if (l->resident) return set_error(DPWA_ERR_STATE, "dpwa_learner_set_resident: already resident");
    if (l->version != 0 || l->have_fetch)
        return set_error(DPWA_ERR_STATE, "dpwa_learner_set_resident: only before the first publish");
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = wait_slot_readers(l, 0, s);
    if (rc) return rc;
    char *dst = slot_payload(l, 0);
    if (l->payload_bytes && dst != init)
        HIP_TRY(hipMemcpyAsync(dst, init, l->payload_bytes, hipMemcpyDeviceToDevice, s));
    l->resident = true;
    l->res_slot = 0;
    l->wt_valid = true;
    l->wt_header = false;
    l->wt_flat = dst;
    l->wt_stream = s;
    return DPWA_OK;
}

int dpwa_learner_resident_params(dpwa_learner *l, void **params, int *slot)
{
    if (!l || !params) return set_error(DPWA_ERR_ARG, "dpwa_learner_resident_params: NULL argument");
    *params = l->resident ? (void *)slot_payload(l, l->res_slot) : nullptr;
    if (slot) *slot = l->resident ? l->res_slot : -1;
    return DPWA_OK;
}

int dpwa_learner_relocate(dpwa_learner *l, dpwa_stream_t stream)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_relocate: NULL learner");
    if (l->have_fetch) return set_error(DPWA_ERR_STATE, "dpwa_learner_relocate: a fetch is in flight (average it)");
    DeviceGuard dg(l->device);
    return relocate_impl(l, (hipStream_t)stream);
}

int dpwa_learner_window_hits(dpwa_learner *l, uint32_t *hits)
{
    if (!l || !hits) return set_error(DPWA_ERR_ARG, "dpwa_learner_window_hits: NULL argument");
    DeviceGuard dg(l->device);
    *hits = 0;
    if (!l->window_sample) return DPWA_OK;
    if (l->window_src) {   // check the window open now (or closed, not yet checked); keep its samples
        hipStream_t s = l->window_stream;
        HIP_TRY(launch_window_roll(l->window_src, nullptr, (int64_t)l->payload_bytes, l->window_sample,
                                   &l->ctl->window_dirty, &l->ctl->window_hits, l->window_host_dev, l->window_gen, 0,
                                   s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *hits = __atomic_load_n(l->window_host, __ATOMIC_ACQUIRE);
    return DPWA_OK;
}

int dpwa_learner_reuse_guard_hits(dpwa_learner *l, uint32_t *hits)
{
    if (!l || !hits) return set_error(DPWA_ERR_ARG, "dpwa_learner_reuse_guard_hits: NULL argument");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(hits, &l->ctl->guard_hits, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return DPWA_OK;
}

int dpwa_learner_read_snapshot(dpwa_learner *l, void *header_out, void *payload_out, int64_t payload_bytes,
                               uint64_t *version_out)
{
    if (!l || !header_out || !version_out || payload_bytes < 0 || (payload_bytes > 0 && !payload_out))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_read_snapshot: bad arguments");
    if ((size_t)payload_bytes > l->payload_bytes) payload_bytes = (int64_t)l->payload_bytes;
    DeviceGuard dg(l->device);
    for (int attempt = 0; attempt < 8; ++attempt) {
        uint64_t v;
        int k;
        {
            std::lock_guard<std::mutex> g(l->pub_mu);
            v = l->version;
            if (v == 0) {
                *version_out = 0;
                return DPWA_OK;   // nothing published: the reference replies without state
            }
            k = (int)((v - 1) % 2);
            if (!l->read_stream) {   // created at the first host read: no stream (and no hardware
                                     // queue share) for learners nobody reads over the wire
                HIP_TRY(hipEventCreateWithFlags(&l->ev_read, hipEventDisableTiming));
                HIP_TRY(hipStreamCreateWithFlags(&l->read_stream, hipStreamNonBlocking));
            }
            // order after the publish (and everything before it) on the publisher's stream
            HIP_TRY(hipEventRecord(l->ev_read, l->publish_stream[k]));
        }
        HIP_TRY(hipStreamWaitEvent(l->read_stream, l->ev_read, 0));
        const char *slot = l->slots + (size_t)k * l->slot_stride;
        HIP_TRY(hipMemcpyAsync(header_out, slot, kHeader, hipMemcpyDeviceToHost, l->read_stream));
        if (payload_bytes)
            HIP_TRY(hipMemcpyAsync(payload_out, slot + kPayloadOff, (size_t)payload_bytes, hipMemcpyDeviceToHost,
                                   l->read_stream));
        HIP_TRY(hipStreamSynchronize(l->read_stream));
        // a slot is rewritten two publishes later: if that happened meanwhile, read again
        std::lock_guard<std::mutex> g(l->pub_mu);
        if (l->version < v + 2 && ((const dpwa_header *)header_out)->version == v) {
            *version_out = v;
            return DPWA_OK;
        }
    }
    return set_error(DPWA_ERR_STATE, "dpwa_learner_read_snapshot: publishes outran the reader");
}

int dpwa_learner_fetch_host(dpwa_learner *l, const void *header, const void *payload, int64_t payload_bytes,
                            dpwa_stream_t stream)
{
    if (!l || !header || payload_bytes != (int64_t)l->payload_bytes || (payload_bytes > 0 && !payload))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_fetch_host: need a header and %zu payload bytes",
                         l ? l->payload_bytes : (size_t)0);
    DeviceGuard dg(l->device);
    (void)stream;
    // The copy waits only for the last reader of the staging buffer (every consumer of a fetch
    // records ev_stage_done), not for all the work queued on the caller's stream: it starts
    // at once, beside a training step already enqueued.
    if (l->stage_read[0]) HIP_TRY(hipStreamWaitEvent(l->side, l->ev_stage_done[0], 0));
    // Pageable host sources: the calls return once the host bytes have been taken.  A
    // page-locked source is copied asynchronously, so the copy is waited for: either way the
    // caller may reuse its buffer when this returns.
    hipPointerAttribute_t attr{};
    const bool pinned = payload_bytes > 0 && hipPointerGetAttributes(&attr, payload) == hipSuccess &&
                        attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();   // a pageable pointer is "invalid" to hipPointerGetAttributes
    HIP_TRY(hipMemcpyAsync(l->staging, header, kHeader, hipMemcpyHostToDevice, l->side));
    if (payload_bytes)
        HIP_TRY(hipMemcpyAsync(l->staging + kPayloadOff, payload, (size_t)payload_bytes, hipMemcpyHostToDevice, l->side));
    HIP_TRY(hipEventRecord(l->ev_fetched, l->side));
    if (pinned) HIP_TRY(hipEventSynchronize(l->ev_fetched));
    l->src = l->staging;
    l->src_copied = true;
    l->src_stage = 0;
    l->src_owner = nullptr;
    l->src_slot = -1;
    l->have_fetch = true;
    l->have_factor = false;
    return DPWA_OK;
}

int dpwa_learner_relay_enable(dpwa_learner *l, int world, int rank)
{
    if (!l || world < 2 || world > kMaxRelayRanks || rank < 0 || rank >= world)
        return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_enable: bad world/rank");
    if (l->relay_on) return set_error(DPWA_ERR_STATE, "dpwa_learner_relay_enable: already enabled");
    DeviceGuard dg(l->device);
    const int64_t payload16 = (int64_t)round_up(l->payload_bytes, 16);
    l->relay_stripe = (int64_t)round_up((size_t)((payload16 + world - 1) / world), kPayloadOff);
    HIP_TRY(devmem_alloc(l->relay_mem, (size_t)l->relay_stripe * world, l->device));
    l->relay_buf = l->relay_mem.ptr;
    HIP_TRY(hipEventCreateWithFlags(&l->ev_relay, hipEventDisableTiming));
    l->relay_world = world;
    l->relay_rank = rank;
    l->relay_slots.assign((size_t)world, nullptr);
    l->relay_bufs.assign((size_t)world, nullptr);
    l->relay_slots[rank] = l->slots;
    l->relay_bufs[rank] = l->relay_buf;
    l->relay_on = true;
    return DPWA_OK;
}

int dpwa_learner_relay_handle(dpwa_learner *l, void *handle_out, int64_t handle_len)
{
    if (!l || !l->relay_on || !handle_out || handle_len < (int64_t)sizeof(IpcBlob))
        return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_handle: relay not enabled or short buffer");
    DeviceGuard dg(l->device);
    IpcBlob b = make_blob(l, l->relay_mem, l->relay_stripe);
    if (!b.vmm) HIP_TRY(hipIpcGetMemHandle(&b.handle, l->relay_buf));
    memset(handle_out, 0, (size_t)handle_len);
    memcpy(handle_out, &b, sizeof(b));
    l->exported = true;
    return DPWA_OK;
}

static int relay_check(dpwa_learner *l, int rank, int peer_id, const void *relay_handle, int64_t handle_len,
                       IpcBlob &b, Endpoint *&slots_ep, const char *fn)
{
    if (!l || !l->relay_on || rank < 0 || rank >= l->relay_world || rank == l->relay_rank || !relay_handle ||
        handle_len < (int64_t)sizeof(IpcBlob))
        return set_error(DPWA_ERR_ARG, "%s: bad arguments", fn);
    auto it = l->peers.find(peer_id);
    if (it == l->peers.end() || it->second.kind != 2)
        return set_error(DPWA_ERR_STATE, "%s: peer %d's slots are not IPC-attached", fn, peer_id);
    memcpy(&b, relay_handle, sizeof(b));
    if (b.magic != kIpcMagic || b.slot_stride != l->relay_stripe || b.n != l->n || b.dtype != l->dtype)
        return set_error(DPWA_ERR_ARG, "%s: relay buffer of rank %d does not match", fn, rank);
    slots_ep = &it->second;
    return DPWA_OK;
}

int dpwa_learner_relay_attach(dpwa_learner *l, int rank, int peer_id, const void *relay_handle, int64_t handle_len)
{
    IpcBlob b;
    Endpoint *ep = nullptr;
    int rc = relay_check(l, rank, peer_id, relay_handle, handle_len, b, ep, "dpwa_learner_relay_attach");
    if (rc) return rc;
    if (b.vmm) return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_attach: rank %d shares its relay buffer as fds", rank);
    DeviceGuard dg(l->device);
    void *ptr = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&ptr, b.handle, hipIpcMemLazyEnablePeerAccess));
    l->relay_opened.push_back((char *)ptr);
    l->relay_slots[rank] = ep->base;
    l->relay_bufs[rank] = (const char *)ptr;
    return DPWA_OK;
}

int dpwa_learner_relay_attach_fds(dpwa_learner *l, int rank, int peer_id, const void *relay_handle,
                                  int64_t handle_len, const int *fds, int n_fds, int64_t chunk_bytes)
{
    IpcBlob b;
    Endpoint *ep = nullptr;
    int rc = relay_check(l, rank, peer_id, relay_handle, handle_len, b, ep, "dpwa_learner_relay_attach_fds");
    if (rc) return rc;
    if (!b.vmm || !fds) return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_attach_fds: rank %d shares a hipIpc handle", rank);
    DeviceGuard dg(l->device);
    DevMem m;
    if ((rc = devmem_import(m, fds, n_fds, chunk_bytes, (size_t)l->relay_stripe * l->relay_world, l->device))) return rc;
    l->relay_slots[rank] = ep->base;
    l->relay_bufs[rank] = m.ptr;
    l->relay_imported.push_back(std::move(m));
    return DPWA_OK;
}

static int relay_args(dpwa_learner *l, const int32_t *picks_dev, uint64_t version, RelayArgs &a)
{
    for (int r = 0; r < l->relay_world; ++r)
        if (!l->relay_slots[r] || !l->relay_bufs[r])
            return set_error(DPWA_ERR_STATE, "relay: rank %d not attached", r);
    if (version == 0) return set_error(DPWA_ERR_STATE, "relay: nothing published");
    memset(&a, 0, sizeof(a));
    for (int r = 0; r < l->relay_world; ++r) {
        a.slots[r] = l->relay_slots[r];
        a.relays[r] = l->relay_bufs[r];
    }
    a.relay_mine = l->relay_buf;
    a.staging = l->staging;
    a.picks = picks_dev;
    a.slot_off = (int64_t)((version - 1) % 2) * (int64_t)l->slot_stride;
    a.stripe = l->relay_stripe;
    a.payload = (int64_t)round_up(l->payload_bytes, 16);
    a.world = l->relay_world;
    a.rank = l->relay_rank;
    return DPWA_OK;
}

int dpwa_learner_relay_wait(dpwa_learner *l, dpwa_stream_t stream)
{
    if (!l || !l->relay_on) return set_error(DPWA_ERR_STATE, "dpwa_learner_relay_wait: relay not enabled");
    if (l->relay_pending) {
        DeviceGuard dg(l->device);
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, l->ev_relay, 0));
    }
    return DPWA_OK;
}

int dpwa_learner_relay_phase1(dpwa_learner *l, const int32_t *picks_dev, uint64_t version, int blocks,
                              dpwa_stream_t stream)
{
    if (!l || !l->relay_on || !picks_dev || blocks < 1)
        return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_phase1: bad arguments");
    RelayArgs a;
    int rc = relay_args(l, picks_dev, version, a);
    if (rc) return rc;
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipEventRecord(l->ev_issue, s));
    HIP_TRY(hipStreamWaitEvent(l->side, l->ev_issue, 0));
    HIP_TRY(launch_relay(1, a, blocks, l->side));
    HIP_TRY(hipEventRecord(l->ev_relay, l->side));
    l->relay_pending = true;
    return DPWA_OK;
}

// Phase 2 on the side stream: my_pick's stripes gathered into staging.
static int relay_phase2_now(dpwa_learner *l, const RelayArgs &a, int my_pick, int blocks)
{
    if (my_pick >= 0 && l->consumed_once && l->consume_stream) {   // WAR on staging
        HIP_TRY(hipEventRecord(l->ev_consumed, l->consume_stream));
        HIP_TRY(hipStreamWaitEvent(l->side, l->ev_consumed, 0));
    }
    if (my_pick >= 0 && l->stage_read[0]) HIP_TRY(hipStreamWaitEvent(l->side, l->ev_stage_done[0], 0));
    HIP_TRY(launch_relay(2, a, blocks, l->side));
    HIP_TRY(hipEventRecord(l->ev_relay, l->side));
    l->relay_pending = true;
    if (my_pick >= 0) HIP_TRY(hipEventRecord(l->ev_fetched, l->side));
    return DPWA_OK;
}

// A deferred phase 2 whose fetch is consumed other than by the fused average (the split
// update_wait, a copy of the payload, an unaligned buffer): gather into staging now.  The side
// stream is still ordered after phase 1 and the round's barrier.
static int relay_materialize(dpwa_learner *l)
{
    if (!l->relay_deferred) return DPWA_OK;
    l->relay_deferred = false;
    return relay_phase2_now(l, l->relay_saved, l->relay_saved_pick, l->relay_saved_blocks);
}

int dpwa_learner_relay_phase2(dpwa_learner *l, const int32_t *picks_dev, int my_pick, uint64_t version, int blocks,
                              int fuse)
{
    if (!l || !l->relay_on || !picks_dev || blocks < 1 || my_pick >= l->relay_world || my_pick == l->relay_rank)
        return set_error(DPWA_ERR_ARG, "dpwa_learner_relay_phase2: bad arguments");
    RelayArgs a;
    int rc = relay_args(l, picks_dev, version, a);
    if (rc) return rc;
    DeviceGuard dg(l->device);
    l->relay_deferred = false;
    if (fuse && my_pick >= 0) {
        // everything the fused average needs is on the side stream now (phase 1, the barrier)
        HIP_TRY(hipEventRecord(l->ev_fetched, l->side));
        l->relay_saved = a;
        l->relay_saved_pick = my_pick;
        l->relay_saved_blocks = blocks;
        l->relay_deferred = true;
    } else if (!fuse || my_pick >= 0) {
        if ((rc = relay_phase2_now(l, a, my_pick, blocks))) return rc;
    }
    if (my_pick >= 0) {
        l->src = l->staging;
        l->src_copied = true;
        l->src_stage = 0;
        l->src_owner = nullptr;
        l->src_slot = -1;
        l->have_fetch = true;
        l->have_factor = false;
    }
    return DPWA_OK;
}

int dpwa_learner_time_averages(dpwa_learner *l, int capacity)
{
    if (!l || capacity < 0) return set_error(DPWA_ERR_ARG, "dpwa_learner_time_averages: bad arguments");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    for (auto &t : l->timing) {
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    l->timing.clear();
    l->timing_used = 0;
    l->timing_armed = false;
    for (int i = 0; i < capacity; ++i) {
        LaunchTiming t{};
        HIP_TRY(hipEventCreate(&t.start));
        HIP_TRY(hipEventCreate(&t.stop));
        l->timing.push_back(t);
    }
    return DPWA_OK;
}

int dpwa_learner_arm_timing(dpwa_learner *l)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_arm_timing: NULL learner");
    l->timing_armed = true;
    return DPWA_OK;
}

int dpwa_learner_read_average_times(dpwa_learner *l, float *us_out, int max, int *count)
{
    if (!l || !count || (max > 0 && !us_out)) return set_error(DPWA_ERR_ARG, "dpwa_learner_read_average_times: bad arguments");
    DeviceGuard dg(l->device);
    const int k = l->timing_used < max ? l->timing_used : max;
    for (int i = 0; i < k; ++i) {
        HIP_TRY(hipEventSynchronize(l->timing[i].stop));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, l->timing[i].start, l->timing[i].stop));
        us_out[i] = ms * 1000.f;
    }
    *count = k;
    l->timing_used = 0;
    return DPWA_OK;
}

int dpwa_learner_time_fetches(dpwa_learner *l, int capacity)
{
    if (!l || capacity < 0) return set_error(DPWA_ERR_ARG, "dpwa_learner_time_fetches: bad arguments");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    for (auto &t : l->fetch_timing) {
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    l->fetch_timing.clear();
    l->fetch_timing_used = 0;
    for (int i = 0; i < capacity; ++i) {
        LaunchTiming t{};
        HIP_TRY(hipEventCreate(&t.start));
        HIP_TRY(hipEventCreate(&t.stop));
        l->fetch_timing.push_back(t);
    }
    return DPWA_OK;
}

int dpwa_learner_read_fetch_times(dpwa_learner *l, float *us_out, int max, int *count)
{
    if (!l || !count || (max > 0 && !us_out)) return set_error(DPWA_ERR_ARG, "dpwa_learner_read_fetch_times: bad arguments");
    DeviceGuard dg(l->device);
    const int k = l->fetch_timing_used < max ? l->fetch_timing_used : max;
    for (int i = 0; i < k; ++i) {
        HIP_TRY(hipEventSynchronize(l->fetch_timing[i].stop));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, l->fetch_timing[i].start, l->fetch_timing[i].stop));
        us_out[i] = ms * 1000.f;
    }
    *count = k;
    return DPWA_OK;
}

int dpwa_learner_side_stream(dpwa_learner *l, dpwa_stream_t *stream)
{
    if (!l || !stream) return set_error(DPWA_ERR_ARG, "dpwa_learner_side_stream: NULL argument");
    *stream = l->side;
    return DPWA_OK;
}

int dpwa_learner_wait_fetch(dpwa_learner *l, dpwa_stream_t stream)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_wait_fetch: NULL learner");
    if (l->have_fetch && l->src_copied) {
        DeviceGuard dg(l->device);
        int rc = relay_materialize(l);
        if (rc) return rc;
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, l->ev_fetched, 0));
    }
    return DPWA_OK;
}

int dpwa_learner_set_loss_dtype(dpwa_learner *l, int32_t dtype)
{
    if (!l || (dtype != DPWA_F32 && dtype != DPWA_F64)) return set_error(DPWA_ERR_ARG, "dpwa_learner_set_loss_dtype: bad arguments");
    l->loss_f32 = dtype == DPWA_F32;
    return DPWA_OK;
}

int dpwa_learner_set_pull(dpwa_learner *l, int mode, int max_blocks)
{
    if (!l || (mode != DPWA_PULL_COPY_ENGINE && mode != DPWA_PULL_KERNEL) || max_blocks < 1)
        return set_error(DPWA_ERR_ARG, "dpwa_learner_set_pull: bad arguments");
    l->pull_mode = mode;
    l->pull_blocks = max_blocks;
    return DPWA_OK;
}

int dpwa_learner_copy_factor(dpwa_learner *l, double *dst_dev, dpwa_stream_t stream)
{
    if (!l || !dst_dev) return set_error(DPWA_ERR_ARG, "dpwa_learner_copy_factor: NULL argument");
    DeviceGuard dg(l->device);
    HIP_TRY(hipMemcpyAsync(dst_dev, &l->ctl->coef.factor, sizeof(double), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
    return DPWA_OK;
}

int dpwa_learner_copy_fetched(dpwa_learner *l, void *dst_dev, dpwa_stream_t stream)
{
    if (!l || (!dst_dev && l->n > 0)) return set_error(DPWA_ERR_ARG, "dpwa_learner_copy_fetched: NULL argument");
    if (!l->have_fetch || !l->src) return set_error(DPWA_ERR_STATE, "dpwa_learner_copy_fetched: no fetch in flight");
    DeviceGuard dg(l->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = relay_materialize(l);
    if (rc) return rc;
    if (l->src_copied) HIP_TRY(hipStreamWaitEvent(s, l->ev_fetched, 0));
    if (l->payload_bytes)
        HIP_TRY(hipMemcpyAsync(dst_dev, l->src + kPayloadOff, l->payload_bytes, hipMemcpyDeviceToDevice, s));
    HIP_TRY(staging_read(l, s));   // a later pull into this staging buffer waits for this copy
    l->consume_stream = s;   // the staging buffer / peer slot is read on s
    l->consumed_once = true;
    return DPWA_OK;
}

// Milliseconds since the (completed, timing) event `since`, on the device's clock: an event
// recorded now on the probe stream -- a stream that holds nothing else -- and the two timestamps'
// difference.  DPWA_ERR_STATE when the probe does not complete within kProbeWaitUs (its hardware
// queue is held up by another stream mapped to it: no measurement).  The probe stream has the
// normal priority: the greatest-priority hardware queues are left to the rescue lanes (streams are
// dealt round-robin onto a few queues per priority, so a probe there would push a lane onto a
// queue another lane already uses).
static int probe_since(dpwa_learner *l, hipEvent_t since, float *ms)
{
    if (!l->probe_stream) {
        hipStream_t ps = nullptr;
        hipEvent_t pe = nullptr;
        hipError_t e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
        if (e == hipSuccess && (e = hipEventCreate(&pe)) != hipSuccess) (void)hipStreamDestroy(ps);
        if (e != hipSuccess) return set_error(DPWA_ERR_HIP, "probe stream: %s", hipGetErrorString(e));
        l->probe_stream = ps;
        l->ev_probe = pe;
    }
    HIP_TRY(hipEventRecord(l->ev_probe, l->probe_stream));
    const int64_t t0 = now_ns();
    for (;;) {
        const hipError_t q = hipEventQuery(l->ev_probe);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return set_error(DPWA_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(q));
        if (now_ns() - t0 > kProbeWaitUs * 1000) return set_error(DPWA_ERR_STATE, "probe held up");
    }
    HIP_TRY(hipEventElapsedTime(ms, since, l->ev_probe));
    return DPWA_OK;
}

int dpwa_learner_fetch_state(dpwa_learner *l, int64_t timeout_ms, int *state)
{
    if (!l || !state) return set_error(DPWA_ERR_ARG, "dpwa_learner_fetch_state: NULL argument");
    *state = DPWA_FETCH_LANDED;
    if (!l->have_fetch || !l->src_copied || l->relay_deferred) return DPWA_OK;
    DeviceGuard dg(l->device);
    const hipError_t e = hipEventQuery(l->ev_fetched);
    if (e == hipSuccess) return DPWA_OK;
    if (e != hipErrorNotReady) return set_error(DPWA_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
    *state = DPWA_FETCH_IN_FLIGHT;
    if (timeout_ms < 0) return DPWA_OK;
    // The host's enqueue is an upper bound on how long the request has been out: within the
    // timeout by it, the pull is in time.  Past it, a pull ordered after the caller's stream
    // (ev_issue: a local peer's snapshot) is timed from when that stream reached update_send --
    // the reference's socket timeout bounds only the wait for the reply (conn.py:249), and work the
    // caller queued before update_send is not the peer's delay.
    const int64_t waited_ns = now_ns() - l->fetch_issue_ns;
    if (waited_ns < timeout_ms * 1000000LL) return DPWA_OK;
    if (l->issue_evented && waited_ns < (timeout_ms + kMaxBacklogMs) * 1000000LL) {
        const hipError_t q = hipEventQuery(l->ev_issue);
        if (q == hipErrorNotReady) return DPWA_OK;        // the request has not gone out yet
        if (q != hipSuccess) return set_error(DPWA_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(q));
        float ms = 0.f;
        if (probe_since(l, l->ev_issue, &ms) == DPWA_OK && ms >= 0.f) {
            *state = ms >= (float)timeout_ms ? DPWA_FETCH_TIMED_OUT : DPWA_FETCH_IN_FLIGHT;
            return DPWA_OK;
        }
    }
    *state = DPWA_FETCH_TIMED_OUT;
    return DPWA_OK;
}

int dpwa_learner_rescue_free(dpwa_learner *l, int *free_out)
{
    if (!l || !free_out) return set_error(DPWA_ERR_ARG, "dpwa_learner_rescue_free: NULL argument");
    DeviceGuard dg(l->device);
    int lane = -1;
    // makes a lane now if one is needed and can be made: at most one allocation per wait (the
    // node's poll ends as soon as a lane is free); with the lanes at their cap a poll only queries
    const int rc = rescue_lane(l, &lane);
    *free_out = lane >= 0 ? 1 : 0;
    return rc;
}

int dpwa_learner_rescue_lanes(dpwa_learner *l, int *lanes, int *cap)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_rescue_lanes: NULL learner");
    if (lanes) *lanes = l->rescue_lanes;
    if (cap) *cap = l->rescue_cap;
    return DPWA_OK;
}

int dpwa_learner_set_rescue_cap(dpwa_learner *l, int cap)
{
    if (!l || cap < 0) return set_error(DPWA_ERR_ARG, "dpwa_learner_set_rescue_cap: bad arguments");
    l->rescue_cap = std::min(std::max(cap, l->rescue_lanes), kMaxRescueLanes);
    return DPWA_OK;
}

int dpwa_learner_fetch_stream(dpwa_learner *l, dpwa_stream_t *stream)
{
    if (!l || !stream) return set_error(DPWA_ERR_ARG, "dpwa_learner_fetch_stream: NULL argument");
    *stream = l->fetch_stream ? l->fetch_stream : l->side;
    return DPWA_OK;
}

int dpwa_learner_cancel(dpwa_learner *l)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_cancel: NULL learner");
    l->relay_deferred = false;   // nothing reads the stripes: no gather
    finish_fetch(l);
    return DPWA_OK;
}

int dpwa_learner_pointers(dpwa_learner *l, double **clock_dev, dpwa_coef **coef_dev, dpwa_header **staging_header_dev,
                          void **staging_payload_dev)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_pointers: NULL learner");
    if (clock_dev) *clock_dev = &l->ctl->clock[l->cur];
    if (coef_dev) *coef_dev = &l->ctl->coef;
    if (staging_header_dev) *staging_header_dev = (dpwa_header *)l->staging;
    if (staging_payload_dev) *staging_payload_dev = l->staging + kPayloadOff;
    return DPWA_OK;
}

int dpwa_learner_status_word(dpwa_learner *l, int32_t **status_word)
{
    if (!l || !status_word) return set_error(DPWA_ERR_ARG, "dpwa_learner_status_word: NULL argument");
    *status_word = l->host_status;
    return DPWA_OK;
}

int dpwa_learner_read_clock(dpwa_learner *l, double *clock)
{
    if (!l || !clock) return set_error(DPWA_ERR_ARG, "dpwa_learner_read_clock: NULL argument");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(clock, &l->ctl->clock[l->cur], sizeof(double), hipMemcpyDeviceToHost));
    return DPWA_OK;
}

int dpwa_learner_write_clock(dpwa_learner *l, double clock)
{
    if (!l) return set_error(DPWA_ERR_ARG, "dpwa_learner_write_clock: NULL learner");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&l->ctl->clock[l->cur], &clock, sizeof(double), hipMemcpyHostToDevice));
    l->wt_header = false;   // the next header was written from the old clock: publish it anew
    return DPWA_OK;
}

int dpwa_learner_read_coef(dpwa_learner *l, dpwa_coef *coef)
{
    if (!l || !coef) return set_error(DPWA_ERR_ARG, "dpwa_learner_read_coef: NULL argument");
    DeviceGuard dg(l->device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(coef, &l->ctl->coef, sizeof(dpwa_coef), hipMemcpyDeviceToHost));
    return DPWA_OK;
}

int dpwa_learner_poll_status(dpwa_learner *l, int *done, int32_t *status)
{
    if (!l || !done || !status) return set_error(DPWA_ERR_ARG, "dpwa_learner_poll_status: NULL argument");
    DeviceGuard dg(l->device);
    hipError_t e = hipEventQuery(l->ev_factor);
    if (e != hipSuccess && e != hipErrorNotReady) return set_error(DPWA_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
    *done = e == hipSuccess ? 1 : 0;
    // Sticky word: the factor kernel writes only non-OK statuses; reading clears it.
    volatile int32_t *w = l->host_status;
    *status = *w;
    if (*status != DPWA_STATUS_OK) *w = DPWA_STATUS_OK;
    return DPWA_OK;
}

}  // extern "C"
