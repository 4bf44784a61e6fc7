// kernels.hpp -- internal launch API of the HIP kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace dpwa {

// Size in bytes of one element of `dtype`, 0 if unknown.
inline size_t dtype_size(int32_t dtype)
{
    return dtype == DPWA_F32 ? 4 : dtype == DPWA_BF16 ? 2 : 0;
}

// Inputs/outputs of the device factor computation (dpwa.py:139-155).  clock_in and
// clock_out may alias only for the one-thread factor kernel.
struct FusedArgs {
    dpwa_interp cfg;
    const double *clock_in;
    double *clock_out;
    const dpwa_header *hdr;     // the peer's published state
    double loss_h;              // used when loss_d is null
    const double *loss_d;       // a device float64, or a float32 when loss_f32
    int32_t loss_f32;
    dpwa_coef *coef_out;
    int32_t *status_mirror;     // nullable device-visible pinned host word (sticky errors)
    // Write-through averages (the next publish then moves no bytes): the header of the next
    // snapshot {new clock + 1, version, n, dtype; loss NaN -- the peers' factor math reads a
    // peer's loss only under loss interpolation, which keeps the header publish} and that
    // clock into *clock_next.  Null: nothing beyond the average.
    dpwa_header *next_header;
    double *clock_next;
    uint64_t next_version;
    int64_t n;
    int32_t dtype;
};

// Lerp over n elements; coefficients from `coef` (device) or, when coef is null, from (a, b).
hipError_t launch_lerp(int32_t dtype, void *param, const void *peer, int64_t n, const dpwa_coef *coef,
                       float a, float b, hipStream_t s);

// Optional timing of one launch: HIP records the kernel's own begin/end in the two events
// (hipExtLaunchKernelGGL), so the figure excludes the dispatch gaps an event pair around the
// launch would add.
struct LaunchTiming {
    hipEvent_t start, stop;
};

// Fused factor + lerp (one launch); a non-null `snap` also receives the result.  `oop` (the
// resident form): the result goes to `snap` only and `param` is read, never written.
hipError_t launch_average(int32_t dtype, void *param, const void *peer, int64_t n, const FusedArgs &fa,
                          void *snap, hipStream_t s, const LaunchTiming *timing = nullptr, bool oop = false);

// Several fused averages (co-resident learners) in one dispatch: entry i's workgroups follow
// entry i-1's.  Every pointer 16-B aligned; `dual` = every entry writes through (snap non-null).
constexpr int kMaxAvgBatch = 8;
struct AvgEntry {
    void *param;
    const void *peer;    // payload of the snapshot averaged with
    void *snap;          // write-through destination, or null
    int64_t n;
    FusedArgs fa;
};
struct AvgBatch {
    int32_t count;
    // span order over equal-size entries (launcher): 0 one entry after the other, 1 dealt
    // round-robin, 2 XCD-grouped (every entry's span s on XCD s % 8, one after the other: entries
    // that read the same buffer -- resident learners that picked each other -- share it in L2)
    int32_t interleave;
    uint32_t spans;                 // spans per entry (XCD-grouped: equal sizes; the last may be empty)
    uint32_t begin[kMaxAvgBatch];   // first workgroup of each entry (filled by the launcher)
    // a group (k_lerp_pair / k_lerp_group: resident entries of equal size whose reads overlap):
    // the distinct buffers its entries read, src[0..count) the entries' parameters and then the
    // peer snapshots of no entry's parameters; entry i's peer is src[peer_of[i]] (filled by the
    // launcher)
    int8_t peer_of[kMaxAvgBatch];
    const void *src[kMaxAvgBatch];
    AvgEntry e[kMaxAvgBatch];
};
hipError_t launch_average_batch(int32_t dtype, bool dual, const AvgBatch &b, hipStream_t s,
                                const LaunchTiming *timing = nullptr, bool oop = false);

// Factor + clock only (one thread).
hipError_t launch_factor(const FusedArgs &fa, hipStream_t s);

// Snapshot publish: slot header {clock+1, loss, version, n, dtype} + payload copy of `nbytes`.
// `system_release` follows it with a system-scope L2 write-back on every XCD so other
// devices (IPC peers) read the bytes from HBM.
hipError_t launch_publish(char *slot, const void *flat, int64_t nbytes, int64_t n, int32_t dtype,
                          double *clock, double loss, const double *loss_dev, bool loss_f32, uint64_t version,
                          bool system_release, hipStream_t s);
// Local streaming copy of `nbytes` (a resident learner's relocation between its slots).
hipError_t launch_copy_payload(void *dst, const void *src, int64_t nbytes, hipStream_t s);
// Pull of `nbytes` (multiple of 16, 16-B aligned) from a peer's slot into local staging with
// a copy kernel of at most `max_blocks` workgroups.  `remote`: the source is another GPU's
// memory -- the kernel is preceded by a system-scope acquire on every XCD, so no L2 line of
// that memory cached by an earlier round is read.
hipError_t launch_pull(void *dst, const void *src, int64_t nbytes, int max_blocks, bool remote, hipStream_t s);
// Relay (multi-link) pull of a lock-step round; see kernels.hip.  All pointers are in this
// process's address space (IPC-mapped for other ranks).
constexpr int kMaxRelayRanks = 64;
struct RelayArgs {
    const char *slots[kMaxRelayRanks];    // slot 0 of every rank's snapshot allocation
    const char *relays[kMaxRelayRanks];   // every rank's relay buffer
    char *relay_mine;
    char *staging;                        // header + payload destination (phase 2)
    const int32_t *picks;                 // device: the peer every rank averages with, -1 none
    int64_t slot_off;                     // byte offset of this round's slot from slot 0
    int64_t stripe;                       // bytes per stripe (multiple of 16)
    int64_t payload;                      // payload bytes to move (multiple of 16)
    int32_t world, rank;
};
hipError_t launch_relay(int phase, const RelayArgs &a, int blocks_per_part, hipStream_t s);
// The relay's phase 2 fused into the average: the fused average of `param` reading stripe r of
// my_pick's snapshot where phase 1 left it (k_lerp_relay), preceded by a system-scope acquire.
// The header is read from fa.hdr (my_pick's slot).  param / snap 16-B aligned.
hipError_t launch_average_relay(int32_t dtype, void *param, int64_t n, const FusedArgs &fa, void *snap,
                                const RelayArgs &a, int my_pick, hipStream_t s, const LaunchTiming *timing = nullptr,
                                bool oop = false);
// Publish of the header only (the payload was written through by the last average).
hipError_t launch_publish_header(char *slot, int64_t n, int32_t dtype, double *clock, double loss,
                                 const double *loss_dev, bool loss_f32, uint64_t version, bool system_release,
                                 hipStream_t s);

// Reuse guard of a header-only publish: sampled words of `flat` against the snapshot `payload`
// the last average wrote; on a difference the payload is copied from `flat` and *hits += 1
// (*dirty: the verdict, device memory; both written by the device).
// dpwa_stream_mix: the averaging kernels' access mix alone (measurement only).
struct StreamMixArgs {
    const char *src[2];
    char *dst[2];
    int64_t nbytes;   // a multiple of 16
    int32_t nr, nw;
};
hipError_t launch_stream_mix(const StreamMixArgs &a, hipStream_t s, const LaunchTiming *timing);

hipError_t launch_guard_payload(char *payload, const void *flat, int64_t nbytes, int32_t *dirty, uint32_t *hits,
                                int32_t gen, hipStream_t s);

// Window guard of resident parameters (learner.cpp): one launch per publish compares the payload
// published last time (`old`) with the samples saved then -- on a difference stamping *dirty with
// `gen`, counting the window in *hits and mirroring the count into the host-mapped word *host --
// and saves the samples of the payload published now (`cur`) into `sample` (kWindowSampleBytes).
// Payloads 16-B aligned; either may be NULL.
constexpr int64_t kWindowSampleBytes = (4096 + 3) * 16;   // samples, tail bytes, first and last word
hipError_t launch_window_roll(const char *old, const char *cur, int64_t nbytes, char *sample, int32_t *dirty,
                              uint32_t *hits, uint32_t *host, int32_t gen, int32_t cur_gen, hipStream_t s);

// A system-scope L2 write-back on every XCD after the work already on `s` (a publish whose
// bytes were written by an earlier kernel, read by other devices).
hipError_t launch_release_system(hipStream_t s);

// A system-scope release store of one 64-bit word after the work already on `s`.
hipError_t launch_store_u64(uint64_t *p, uint64_t v, hipStream_t s);

}  // namespace dpwa
